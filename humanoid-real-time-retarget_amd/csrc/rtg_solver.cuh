// rtg_solver.cuh -- the retarget solver bodies and kernel templates (included by rtg_solve_*.hip, which
// instantiate disjoint subsets so the heavy kernels compile in parallel).
//
// Work decomposition: one mocap frame per lane.  Frames are independent
// (SURVEY.md §0), every solver step is a short dependent chain of scalar-sized
// math, and a frame's working set (<= 32 input points) fits in VGPRs, so a
// lane solves its frame end-to-end with no cross-lane traffic.  Zero-pose-only
// terms are evaluated once per solver (k_solver_prep) and arrive as a by-value
// kernel argument (SGPR-resident).  The 30-float DOF row of each frame is
// staged through LDS so the block stores one contiguous, dwordx4-coalesced
// tile instead of 64 lanes writing 120-byte-strided rows.
#pragma once
#include "rtg_device.cuh"

namespace rtg {

// ----------------------------------------------------------------------------
// solver constants prep (1 thread): theta0 / phi0 of the four arm maps and the
// gripper denominator, computed with exactly the per-frame device math.
// ----------------------------------------------------------------------------

// ----------------------------------------------------------------------------
// solver bodies.  Each link quaternion is emitted as soon as it is final: its
// DOF (quat_to_dof_pos, transform3d.py:176-183: dof k <-> link k+1, component
// Hu_DOF_AXIS[k]) goes to the block's LDS tile and, if requested, the
// quaternion to local_rot -- so only the few values later steps need (parents,
// wrist fits) stay live in VGPRs.
// ----------------------------------------------------------------------------
struct Emit {
    float *row;                  // LDS row of this frame (30 DOFs)
    float *__restrict__ lr;      // local_rot row (31 x 4) or nullptr
    const uint32_t *__restrict__ ang;   // exp-map angle table (SolverConsts::ang_tab)
    float2 *st;                  // LDS stash of this lane: (w, Hu_DOF_AXIS component) per DOF link, stride sst
    int sst;
    // links 12..18 and 21..27 (DOFs 11..17, 20..26) -> stash slots 0..13
    template <int LINK>
    static constexpr int slot() { return LINK <= 18 ? LINK - 12 : LINK - 14; }
    template <int LINK>
    RTG_DEV void link(Q q) const
    {
        constexpr int k = hu_dof_axis(LINK - 1);
        st[slot<LINK>() * sst] = make_float2(q.w, k == 0 ? q.x : (k == 1 ? q.y : q.z));
        if (lr) st4(lr + 4 * LINK, q);
    }
    template <int LINK>
    RTG_DEV void identity() const   // untouched link: exp-map of the identity is +0
    {
        st[slot<LINK>() * sst] = make_float2(1.0f, 0.0f);
        if (lr) st4(lr + 4 * LINK, qident());
    }
    // The DOF read-out of slots [s0, s0 + n) in one batch: the table loads of all links are in flight together
    // and their arithmetic interleaves, instead of one exposed load latency per link.
    // The slots' exact-path fallbacks (w outside the table or a code-0 entry, rare) share one branch, and inside it
    // one loop (not unrolled: a single copy of the exact path) redoes just those slots.  Same values.
    RTG_DEV void finalize(int s0, int n) const
    {
        uint32_t exact = 0;
#pragma unroll
        for (int j = 0; j < 14; ++j)
            if (j >= s0 && j < s0 + n) {
                const float2 v = st[j * sst];
                const ExpDof e = exp_dof_table_part(v.x, ang);
                exact |= (uint32_t)e.exact << j;
                row[j < 7 ? 11 + j : 13 + j] = exp_dof_finish(e, v.y);
            }
        if (__builtin_expect(exact != 0u, 0)) {
#pragma unroll 1
            for (int j = s0; j < s0 + n; ++j)
                if ((exact >> j) & 1u) {
                    const float2 v = st[j * sst];
                    const float angle = normalize_angle(2.0f * cr_acos(v.x));
                    row[j < 7 ? 11 + j : 13 + j] = angle * (v.y / cr_sqrt(1.0f - v.x * v.x));   // mask holds here
                }
        }
    }
};

RTG_DEV void emit_fixed_links(const Emit &E)
{
#pragma unroll
    for (int k = 0; k < 11; ++k) E.row[k] = 0.0f;
    E.row[29] = 0.0f;
    if (E.lr) {
#pragma unroll
        for (int j = 0; j < 12; ++j) st4(E.lr + 4 * j, qident());
        st4(E.lr + 4 * 19, qident());
        st4(E.lr + 4 * 20, qident());
        st4(E.lr + 4 * 28, qident());
        st4(E.lr + 4 * 29, qident());
        st4(E.lr + 4 * 30, qident());
    }
}

// one arm: shoulder pitch/roll then shoulder yaw / elbow pitch (full_body_pos_retargeter.py:75-93);
// returns quat_mul_four of the four link rotations (the wrist parent chain, :128-136)
template <int L0>
RTG_DEV Q solve_arm(const Emit &E, V upper, V fore, ArmZero zs, ArmZero ze, Q parent)
{
    Q p, r, y, e;
    shoulder_pr(upper, zs, parent, p, r);
    E.link<L0>(p);
    E.link<L0 + 1>(r);
    elbow_py(fore, ze, qmul(qmul(parent, p), r), y, e);
    E.link<L0 + 2>(y);
    E.link<L0 + 3>(e);
    return qmul(qmul(qmul(p, r), y), e);
}

template <int L0>
RTG_DEV void emit_euler_xyz(const Emit &E, Q local)   // quat_in_xyz_axis(q, 'XYZ') -> links L0..L0+2
{
    Q eul[3];
    quat_in_xyz_axis(local, 0, 1, 2, false, eul);
    E.link<L0>(eul[0]);
    E.link<L0 + 1>(eul[1]);
    E.link<L0 + 2>(eul[2]);
}

RTG_DEV float hand_x_mean(Q rot, V h0, const V (&tip)[5])   // gripper x-spread
{
    const float x0 = qrotate(rot, h0).x;
    return mean5(qrotate(rot, tip[0]).x - x0, qrotate(rot, tip[1]).x - x0, qrotate(rot, tip[2]).x - x0,
                 qrotate(rot, tip[3]).x - x0, qrotate(rot, tip[4]).x - x0);
}
// One frame's input rows.  AoS (the reference's layout): the frame's (P, C) row at p.  SoA (RTG_LAYOUT_SOA):
// component planes of the whole batch, element (j, c) of frame f at p[(j C + c) B + f] with p pointing at frame f
// -- a wave's load of one component is 256 contiguous bytes.
template <bool SOA>
struct FV;
template <>
struct FV<false> {
    const float *__restrict__ p;
    RTG_DEV V p3(int j) const { return ld3(p + 3 * j); }
    RTG_DEV Q q4(int j) const { return ld4(p + 4 * j); }
};
template <>
struct FV<true> {
    const float *__restrict__ p;
    int64_t s;
    RTG_DEV V p3(int j) const { return V{p[(3 * j) * s], p[(3 * j + 1) * s], p[(3 * j + 2) * s]}; }
    RTG_DEV Q q4(int j) const { return Q{p[(4 * j) * s], p[(4 * j + 1) * s], p[(4 * j + 2) * s], p[(4 * j + 3) * s]}; }
};
template <bool SOA>
RTG_DEV FV<SOA> frame_view(const float *__restrict__ base, int64_t f, int row_floats, int64_t B);
template <>
RTG_DEV FV<false> frame_view<false>(const float *__restrict__ base, int64_t f, int row_floats, int64_t)
{
    return FV<false>{base + f * row_floats};
}
template <>
RTG_DEV FV<true> frame_view<true>(const float *__restrict__ base, int64_t f, int, int64_t B)
{
    return FV<true>{base + f, B};
}

template <typename View>
RTG_DEV float hand_x_mean(Q rot, const View &H, const int (&idx)[5])
{
    const V tip[5] = {H.p3(idx[0]), H.p3(idx[1]), H.p3(idx[2]), H.p3(idx[3]), H.p3(idx[4])};
    return hand_x_mean(rot, H.p3(0), tip);
}
RTG_DEV float hand_x_mean(Q rot, const float *__restrict__ H, const int (&idx)[5])
{
    return hand_x_mean(rot, FV<false>{H}, idx);
}

// The 32 input points VtrdynFullBodyPosRetargeter reads (body 10,11,13..20; per
// hand 0 + the Kabsch points 2,6,10,14,17 + the tips 4,8,12,16,19).
struct FbpIn {
    V b10, b11, b13, b17, b18, b19, b20, b14, b15, b16;
    V l0, lk[5], lt[5];
    V r0, rk[5], rt[5];
};
RTG_DEV FbpIn load_fbp(const float *__restrict__ b, const float *__restrict__ L, const float *__restrict__ R)
{
    FbpIn I;
    I.b10 = ld3(b + 30); I.b11 = ld3(b + 33); I.b13 = ld3(b + 39); I.b17 = ld3(b + 51);
    I.b18 = ld3(b + 54); I.b19 = ld3(b + 57); I.b20 = ld3(b + 60);
    I.b14 = ld3(b + 42); I.b15 = ld3(b + 45); I.b16 = ld3(b + 48);
    constexpr int kp[5] = {2, 6, 10, 14, 17}, tp[5] = {4, 8, 12, 16, 19};
    I.l0 = ld3(L); I.r0 = ld3(R);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        I.lk[i] = ld3(L + 3 * kp[i]); I.lt[i] = ld3(L + 3 * tp[i]);
        I.rk[i] = ld3(R + 3 * kp[i]); I.rt[i] = ld3(R + 3 * tp[i]);
    }
    return I;
}

// VtrdynFullBodyPosRetargeter.retarget  full_body_pos_retargeter.py:25-217
template <bool PRECISE>
RTG_DEV void solve_full_body_pos(const SolverConsts &C, const FbpIn &I, const Emit &E, float *__restrict__ body_rot)
{
    // _retarget_arm_from_global_translation :61-118
    Q R10;
    {
        const V Mt[3] = {vsub(I.b17, I.b10), vsub(I.b13, I.b10), vsub(I.b11, I.b10)};
        R10 = cal_joint_quat<3>(C.Zt, Mt);
    }
    const Q chainL = solve_arm<12>(E, vsub(I.b19, I.b18), vsub(I.b20, I.b19), C.lsh, C.lel, R10);
    const Q chainR = solve_arm<21>(E, vsub(I.b15, I.b14), vsub(I.b16, I.b15), C.rsh, C.rel, R10);
    // _retarget_wrist_from_global_translation :120-175
    Q WL, WR;
    {
        const V Ml[5] = {vsub(I.lk[0], I.l0), vsub(I.lk[1], I.l0), vsub(I.lk[2], I.l0), vsub(I.lk[3], I.l0),
                         vsub(I.lk[4], I.l0)};
        WL = cal_joint_quat<5>(C.Zl, Ml);
    }
    emit_euler_xyz<16>(E, qmul_norm(qconj(qmul_norm(R10, chainL)), WL));
    {
        const V Mr[5] = {vsub(I.rk[0], I.r0), vsub(I.rk[1], I.r0), vsub(I.rk[2], I.r0), vsub(I.rk[3], I.r0),
                         vsub(I.rk[4], I.r0)};
        WR = cal_joint_quat<5>(C.Zr, Mr);
    }
    emit_euler_xyz<25>(E, qmul_norm(qconj(qmul_norm(R10, chainR)), WR));
    // _retarget_gripper :177-217 -- hand points in the wrist frame (rotate by conj(W))
    const float la = hand_x_mean(qconj(WL), I.l0, I.lt), ra = hand_x_mean(qconj(WR), I.r0, I.rt);
    if (PRECISE) {
        const float ls = clamp_lohi(la / C.orig - 0.5f, 0.0f, 0.5f) / 0.5f;
        const float rs = clamp_lohi(ra / C.orig - 0.5f, 0.0f, 0.5f) / 0.5f;
        E.row[18] = ls * 0.044f; E.row[19] = ls * -0.044f;
        E.row[27] = rs * 0.044f; E.row[28] = rs * -0.044f;
    } else {
        const bool lc = la / C.orig < 0.7f, rc = ra / C.orig < 0.7f;
        E.row[18] = lc ? 0.0f : 0.044f; E.row[19] = lc ? 0.0f : -0.044f;
        E.row[27] = rc ? 0.0f : 0.044f; E.row[28] = rc ? 0.0f : -0.044f;
    }
    if (body_rot) {   // body_global_rotation: identity except rows 10, 14, 39 (:116, :172-173)
        for (int j = 0; j < 59; ++j) st4(body_rot + 4 * j, j == 10 ? R10 : (j == 14 ? WL : (j == 39 ? WR : qident())));
    }
}

// HuUpperBodyFromMocapRetarget.retarget_from_global_translation  retarget_solver.py:40-99
RTG_DEV void solve_upper_body(const SolverConsts &C, const float *__restrict__ x, const Emit &E)
{
    auto pt = [&](int j) {   // coord_transform(dir=[-1,-1,1]) :41
        const V v = ld3(x + 3 * j);
        return V{v.x * -1.0f, v.y * -1.0f, v.z * 1.0f};
    };
    Q R10;
    {
        const V s10 = pt(10);
        const V Mt[3] = {vsub(pt(17), s10), vsub(pt(13), s10), vsub(pt(11), s10)};
        R10 = cal_joint_quat<3>(C.Zt, Mt);
    }
    const V s19 = pt(19), s15 = pt(15);
    solve_arm<12>(E, vsub(s19, pt(18)), vsub(pt(20), s19), C.lsh, C.lel, R10);
    solve_arm<21>(E, vsub(s15, pt(14)), vsub(pt(16), s15), C.rsh, C.rel, R10);
    E.identity<16>(); E.identity<17>(); E.identity<18>();
    E.identity<25>(); E.identity<26>(); E.identity<27>();
    E.row[18] = 0.0f; E.row[19] = 0.0f; E.row[27] = 0.0f; E.row[28] = 0.0f;
}

// VtrdynFullBodyRetargeter.retarget  full_body_retargeter.py:19-177
RTG_DEV void solve_full_body_rot(const SolverConsts &C, const float *__restrict__ q, const float *__restrict__ b,
                                 const float *__restrict__ L, const float *__restrict__ R, const Emit &E)
{
    const Q parL = ld4(q + 17 * 4), parR = ld4(q + 13 * 4);
    const V b19 = ld3(b + 57), b15 = ld3(b + 45);
    const Q chainL = solve_arm<12>(E, vsub(b19, ld3(b + 54)), vsub(ld3(b + 60), b19), C.lsh, C.lel, parL);
    const Q chainR = solve_arm<21>(E, vsub(b15, ld3(b + 42)), vsub(ld3(b + 48), b15), C.rsh, C.rel, parR);
    const Q wl = ld4(q + 20 * 4), wr = ld4(q + 16 * 4);
    emit_euler_xyz<16>(E, qmul_norm(qconj(qmul_norm(parL, chainL)), wl));
    emit_euler_xyz<25>(E, qmul_norm(qconj(qmul_norm(parR, chainR)), wr));
    // _retarget_gripper :145-177 -- rotates by the wrist quaternion itself (not its inverse)
    constexpr int tips[5] = {3, 7, 11, 15, 19};
    const bool lc = hand_x_mean(wl, L, tips) / C.orig < 0.7f, rc = hand_x_mean(wr, R, tips) / C.orig < 0.7f;
    E.row[18] = lc ? 0.0f : 0.044f; E.row[19] = lc ? 0.0f : -0.044f;
    E.row[27] = rc ? 0.0f : 0.044f; E.row[28] = rc ? 0.0f : -0.044f;
}

// Mocap2HuBodyRetargeter.retarget_from_pose  body_retargeter.py:34-81
RTG_DEV void solve_body_rot(const SolverConsts &C, const float *__restrict__ g, const Emit &E)
{
    // cal_local_rotation (kinematics.py:41-63) for the four joints used
    auto local = [&](int j, int p) { return qmul_norm(qconj(ld4(g + 4 * p)), ld4(g + 4 * j)); };
#pragma unroll
    for (int side = 0; side < 2; ++side) {
        const int sh = side == 0 ? 18 : 14, el = side == 0 ? 19 : 15;
        Q s3[3], e3[3];
        quat_in_xyz_axis(local(sh, C.par[side == 0 ? 0 : 1]), 1, 0, 2, false, s3);   // 'YXZ'
        quat_in_xyz_axis(local(el, C.par[side == 0 ? 2 : 3]), 2, 1, 0, false, e3);   // 'ZYX'
        if (side == 0) {
            E.link<12>(s3[0]); E.link<13>(s3[1]); E.link<14>(qmul_norm(e3[0], s3[2]));
            E.link<15>(e3[1]); E.link<16>(e3[2]);
        } else {
            E.link<21>(s3[0]); E.link<22>(s3[1]); E.link<23>(qmul_norm(e3[0], s3[2]));
            E.link<24>(e3[1]); E.link<25>(e3[2]);
        }
    }
    E.identity<17>(); E.identity<18>(); E.identity<26>(); E.identity<27>();
    E.row[18] = 0.0f; E.row[19] = 0.0f; E.row[27] = 0.0f; E.row[28] = 0.0f;
}

// ----------------------------------------------------------------------------
// solver kernel: per-frame body + coalesced DOF tile store
// ----------------------------------------------------------------------------
constexpr int kSolverBlock = 256;

// Fire-and-forget touch of the 128-byte lines covering [p, p + nbytes): one line per lane per instruction, loaded
// by LDS-DMA into a sink slot nobody reads, so no VGPR is held while the line travels.
RTG_DEV void l2_touch(const float *p, int nbytes, float *sink)
{
    const int nlines = (nbytes + 127) >> 7;
    for (int k = threadIdx.x & 63; k < nlines; k += 64)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(p + 32 * k),
                                         (__attribute__((address_space(3))) void *)sink, 4, 0, 0);
}
constexpr int kDofStride = 31;   // LDS row pitch (dwords): odd -> conflict-free ds_write_b32

template <int KIND, bool PRECISE>
__global__ __launch_bounds__(kSolverBlock) void k_retarget(SolverConsts C, const float *__restrict__ in0,
                                                           const float *__restrict__ in1,
                                                           const float *__restrict__ in2,
                                                           const float *__restrict__ in3, int64_t B,
                                                           float *__restrict__ dof, float *__restrict__ local_rot,
                                                           float *__restrict__ body_rot)
{
    __shared__ float sdof[kSolverBlock * kDofStride];
    __shared__ float2 sst[14 * kSolverBlock];
    const int64_t f = (int64_t)blockIdx.x * kSolverBlock + threadIdx.x;
    if (f < B) {
        const Emit E{sdof + threadIdx.x * kDofStride, local_rot ? local_rot + f * 124 : nullptr, C.ang_tab,
                     sst + threadIdx.x, kSolverBlock};
        emit_fixed_links(E);
        if (KIND == RTG_SOLVER_FULL_BODY_POS)
            solve_full_body_pos<PRECISE>(C, load_fbp(in0 + f * 63, in1 + f * 60, in2 + f * 60), E,
                                         body_rot ? body_rot + f * 236 : nullptr);
        else if (KIND == RTG_SOLVER_UPPER_BODY)
            solve_upper_body(C, in0 + f * 63, E);
        else if (KIND == RTG_SOLVER_FULL_BODY_ROT)
            solve_full_body_rot(C, in0 + f * 84, in1 + f * 63, in2 + f * 60, in3 + f * 60, E);
        else
            solve_body_rot(C, in0 + f * 84, E);
        E.finalize(0, 14);
    }
    __syncthreads();
    // coalesced store of the block's contiguous DOF tile: rows [f0, min(B, f0+256)) x 30.
    // f0*120 B is 16-byte aligned, so the tile goes out as dwordx4 (full-line writes).
    const int64_t f0 = (int64_t)blockIdx.x * kSolverBlock;
    const int64_t nrows = (B - f0) < kSolverBlock ? (B - f0) : kSolverBlock;
    const int nvals = (int)nrows * 30;
    float *dst = dof + f0 * 30;
    auto lds_at = [&](int i) {
        const int r = i / 30;
        return sdof[r * kDofStride + (i - r * 30)];
    };
    const int nvec = nvals >> 2;
    for (int v = threadIdx.x; v < nvec; v += kSolverBlock) {
        const int i = v << 2;
        *reinterpret_cast<float4 *>(dst + i) = make_float4(lds_at(i), lds_at(i + 1), lds_at(i + 2), lds_at(i + 3));
    }
    for (int i = (nvec << 2) + threadIdx.x; i < nvals; i += kSolverBlock) dst[i] = lds_at(i);
}

// ----------------------------------------------------------------------------
// Every solver kind, two waves per frame tile.  After the torso fit (or, for the rotation solvers, from the
// start) the two sides are independent (full_body_pos_retargeter.py:70-175, retarget_solver.py:72-99,
// full_body_retargeter.py:60-177, body_retargeter.py:48-81), so waves 2k and 2k+1 of a block take the left
// and the right side of the same 64 frames.  The side is wave-uniform: its constants stay scalar, the branch never diverges, and each
// wave runs the torso fit plus half the frame program -- twice the waves in flight, about half the per-frame
// latency, the same arithmetic per value (so the same bits as the fused body).
// ----------------------------------------------------------------------------
constexpr int kSideFrames = 128;   // frames per 256-thread block

// torso fit R10 (full_body_pos_retargeter.py:69-70 / retarget_solver.py:49-50)
template <typename View, typename Hook = NoHook>
RTG_DEV Q fbp_torso(const SolverConsts &C, const View &b, const Hook &hook = Hook{})
{
    const V b10 = b.p3(10);
    const V Mt[3] = {vsub(b.p3(17), b10), vsub(b.p3(13), b10), vsub(b.p3(11), b10)};
    return cal_joint_quat<3>(C.Zt, Mt, hook);
}
RTG_DEV Q upper_pt_sign(V v) { return Q{v.x * -1.0f, v.y * -1.0f, v.z * 1.0f, 0.0f}; }   // coord_transform :41
template <typename View>
RTG_DEV Q upper_torso(const SolverConsts &C, const View &x)
{
    auto pt = [&](int j) {
        const Q q = upper_pt_sign(x.p3(j));
        return V{q.x, q.y, q.z};
    };
    const V s10 = pt(10);
    const V Mt[3] = {vsub(pt(17), s10), vsub(pt(13), s10), vsub(pt(11), s10)};
    return cal_joint_quat<3>(C.Zt, Mt);
}
// wrist fit W (full_body_pos_retargeter.py:137-140 left, :160-163 right)
template <int SIDE, typename View, typename Hook = NoHook>
RTG_DEV Q fbp_wrist_fit(const SolverConsts &C, const View &H, const Hook &hook = Hook{})
{
    const V h0 = H.p3(0);
    const V M[5] = {vsub(H.p3(2), h0), vsub(H.p3(6), h0), vsub(H.p3(10), h0), vsub(H.p3(14), h0), vsub(H.p3(17), h0)};
    return cal_joint_quat<5>(SIDE ? C.Zr : C.Zl, M, hook);
}

// A side's body points (shoulder, elbow, wrist) and hand points for the gripper (0 and the tips 4,8,12,16,19),
// loaded where the kernel chooses (RTG_PRELOAD_*: next to the other loads of the same rows, so the rows' lines are
// still in L2 -- see DESIGN.md §5 on the re-fetch of evicted rows).
struct ArmPts { V sh, el, wr; };
struct TipPts { V h0, t[5]; };
template <int SIDE, typename View>
RTG_DEV ArmPts load_arm(const View &b)
{
    return ArmPts{b.p3(SIDE ? 14 : 18), b.p3(SIDE ? 15 : 19), b.p3(SIDE ? 16 : 20)};
}
template <typename View>
RTG_DEV TipPts load_tips(const View &H)
{
    return TipPts{H.p3(0), {H.p3(4), H.p3(8), H.p3(12), H.p3(16), H.p3(19)}};
}

// one arm's chain from its points and R10 (full_body_pos_retargeter.py:75-93)
template <int SIDE>
RTG_DEV Q fbp_arm(const SolverConsts &C, const ArmPts &ap, Q R10, const Emit &E)
{
    return solve_arm<SIDE ? 21 : 12>(E, vsub(ap.el, ap.sh), vsub(ap.wr, ap.el), SIDE ? C.rsh : C.lsh,
                                     SIDE ? C.rel : C.lel, R10);
}
template <bool PRECISE, int SIDE, typename Hook = NoHook>
RTG_DEV void fbp_side_after_arm(const SolverConsts &C, const TipPts &tp, Q R10, Q chain, Q W, const Emit &E,
                                float *__restrict__ brow, const Hook &hook = Hook{});
template <bool PRECISE, int SIDE, typename Hook = NoHook>
RTG_DEV void solve_fbp_side(const SolverConsts &C, const ArmPts &ap, const TipPts &tp, Q R10, Q W, const Emit &E,
                            float *__restrict__ brow, const Hook &hook = Hook{})
{
    const Q chain = fbp_arm<SIDE>(C, ap, R10, E);
    hook(2);
    fbp_side_after_arm<PRECISE, SIDE>(C, tp, R10, chain, W, E, brow, hook);
}
// the Euler split of the wrist (:128-136), the gripper (:142-158 / :165-175) and the body_rot rows (:116, :172-173)
template <bool PRECISE, int SIDE, typename Hook>
RTG_DEV void fbp_side_after_arm(const SolverConsts &C, const TipPts &tp, Q R10, Q chain, Q W, const Emit &E,
                                float *__restrict__ brow, const Hook &hook)
{
    constexpr int E0 = SIDE ? 25 : 16, D0 = SIDE ? 27 : 18, WROW = SIDE ? 39 : 14;
    emit_euler_xyz<E0>(E, qmul_norm(qconj(qmul_norm(R10, chain)), W));
    hook(3);
    const float a = hand_x_mean(qconj(W), tp.h0, tp.t);
    if (PRECISE) {
        const float sc = clamp_lohi(a / C.orig - 0.5f, 0.0f, 0.5f) / 0.5f;
        E.row[D0] = sc * 0.044f;
        E.row[D0 + 1] = sc * -0.044f;
    } else {
        const bool closed = a / C.orig < 0.7f;
        E.row[D0] = closed ? 0.0f : 0.044f;
        E.row[D0 + 1] = closed ? 0.0f : -0.044f;
    }
    if (brow) {   // body_global_rotation rows (:116, :172-173): the left wave also writes row 10 and the identities
        st4(brow + 4 * WROW, W);
        if (!SIDE)
            for (int j = 0; j < 59; ++j)
                if (j != 14 && j != 39) st4(brow + 4 * j, j == 10 ? R10 : qident());
    }
}

// HuUpperBodyFromMocapRetarget (retarget_solver.py:40-99), one side: one arm given the torso fit; wrists untouched
template <int SIDE, typename View>
RTG_DEV void solve_upper_side(const SolverConsts &C, const View &x, Q R10, const Emit &E)
{
    auto pt = [&](int j) {   // coord_transform(dir=[-1,-1,1]) :41
        const Q q = upper_pt_sign(x.p3(j));
        return V{q.x, q.y, q.z};
    };
    constexpr int L0 = SIDE ? 21 : 12, E0 = SIDE ? 25 : 16, D0 = SIDE ? 27 : 18;
    constexpr int SH = SIDE ? 14 : 18, EL = SIDE ? 15 : 19, WR = SIDE ? 16 : 20;
    const V sel = pt(EL);
    solve_arm<L0>(E, vsub(sel, pt(SH)), vsub(pt(WR), sel), SIDE ? C.rsh : C.lsh, SIDE ? C.rel : C.lel, R10);
    E.identity<E0>(); E.identity<E0 + 1>(); E.identity<E0 + 2>();
    E.row[D0] = 0.0f; E.row[D0 + 1] = 0.0f;
}

// VtrdynFullBodyRetargeter (full_body_retargeter.py:19-177), one side
template <int SIDE, typename View>
RTG_DEV void solve_full_body_rot_side(const SolverConsts &C, const View &q, const View &b, const View &H,
                                      const Emit &E)
{
    constexpr int L0 = SIDE ? 21 : 12, E0 = SIDE ? 25 : 16, D0 = SIDE ? 27 : 18;
    constexpr int SH = SIDE ? 14 : 18, EL = SIDE ? 15 : 19, WR = SIDE ? 16 : 20, PAR = SIDE ? 13 : 17;
    const Q par = q.q4(PAR);
    const V bel = b.p3(EL);
    const Q chain = solve_arm<L0>(E, vsub(bel, b.p3(SH)), vsub(b.p3(WR), bel), SIDE ? C.rsh : C.lsh,
                                  SIDE ? C.rel : C.lel, par);
    const Q w = q.q4(WR);
    emit_euler_xyz<E0>(E, qmul_norm(qconj(qmul_norm(par, chain)), w));
    constexpr int tips[5] = {3, 7, 11, 15, 19};   // :145-177 rotates by the wrist quaternion itself
    const bool closed = hand_x_mean(w, H, tips) / C.orig < 0.7f;
    E.row[D0] = closed ? 0.0f : 0.044f;
    E.row[D0 + 1] = closed ? 0.0f : -0.044f;
}

// Mocap2HuBodyRetargeter (body_retargeter.py:34-81), one side
template <int SIDE, typename View>
RTG_DEV void solve_body_rot_side(const SolverConsts &C, const View &g, const Emit &E)
{
    auto local = [&](int j, int p) { return qmul_norm(qconj(g.q4(p)), g.q4(j)); };
    constexpr int SH = SIDE ? 14 : 18, EL = SIDE ? 15 : 19, D0 = SIDE ? 27 : 18;
    Q s3[3], e3[3];
    quat_in_xyz_axis(local(SH, C.par[SIDE ? 1 : 0]), 1, 0, 2, false, s3);   // 'YXZ'
    quat_in_xyz_axis(local(EL, C.par[SIDE ? 3 : 2]), 2, 1, 0, false, e3);   // 'ZYX'
    if (SIDE) {
        E.link<21>(s3[0]); E.link<22>(s3[1]); E.link<23>(qmul_norm(e3[0], s3[2]));
        E.link<24>(e3[1]); E.link<25>(e3[2]);
        E.identity<26>(); E.identity<27>();
    } else {
        E.link<12>(s3[0]); E.link<13>(s3[1]); E.link<14>(qmul_norm(e3[0], s3[2]));
        E.link<15>(e3[1]); E.link<16>(e3[2]);
        E.identity<17>(); E.identity<18>();
    }
    E.row[D0] = 0.0f; E.row[D0 + 1] = 0.0f;
}

// A release is per lane, but the hand-over is per wave: the lanes that skipped the work (frames past B) must not
// raise the flag on their own -- the compiler may run their path first (it did: the flag went up before the live
// lanes' writes).  So the flag goes up after a convergent ballot, where the whole wave has rejoined and every
// lane's LDS writes have issued, from one lane, with a release (s_waitcnt lgkmcnt(0) before the store).
RTG_DEV void lds_signal(int *flag)
{
    const uint64_t joined = __builtin_amdgcn_ballot_w64(true);
    if (joined != 0 && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(joined))
        __hip_atomic_store(flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
RTG_DEV void lds_wait(int *flag)
{
    for (int it = 0; it < (1 << 22); ++it) {   // ~0.1 s at s_sleep 1: a bound every wave reaches
        if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) return;
        __builtin_amdgcn_s_sleep(1);
    }
}

template <int KIND, bool PRECISE, bool SOA>
__global__ __launch_bounds__(256, RTG_SIDES_WAVES) void k_solve_sides(SolverConsts C, const float *__restrict__ in0,
                                                     const float *__restrict__ in1, const float *__restrict__ in2,
                                                     const float *__restrict__ in3, int64_t B,
                                                     float *__restrict__ dof, float *__restrict__ local_rot,
                                                     float *__restrict__ body_rot)
{
    __shared__ float sdof[kSideFrames * kDofStride];
    __shared__ float4 storso[kSideFrames];   // the tile's torso fit, handed from the left wave to the right one
    __shared__ float4 sarm_own[(RTG_SIDES_REBALANCE && !RTG_SIDES_FLAGS) ? kSideFrames : 1];
    __shared__ float2 sst[2 * 14 * 64];      // exp-map stash, [tile][slot][lane]
    const int w = threadIdx.x >> 6, side = w & 1;
    const int r = (w >> 1) * 64 + (threadIdx.x & 63);   // tile row
    const int64_t f0 = (int64_t)blockIdx.x * kSideFrames, f = f0 + r;
    const bool live = f < B;
    const Emit E{sdof + r * kDofStride, live && local_rot ? local_rot + f * 124 : nullptr, C.ang_tab,
                 sst + (w >> 1) * 14 * 64 + (threadIdx.x & 63), 64};
#if RTG_EXP_HOT_INPUTS   // measurement knob (tools/build_variants.sh): every tile reads the first block's rows
    const int64_t fi = f & (kSideFrames - 1);
#else
    const int64_t fi = f;
#endif
    auto view = [&](const float *base, int row_floats) { return frame_view<SOA>(base, fi, row_floats, B); };
#if RTG_L2_PREFETCH
    if (KIND == RTG_SOLVER_FULL_BODY_POS && !SOA) {
        __shared__ float sink[64 * 4];
        const int64_t ft = f0 + (w >> 1) * 64, nt = B - ft < 64 ? B - ft : 64;
        if (nt > 0) {
            if (side) l2_touch(in0 + ft * 63, (int)nt * 252, sink + 64 * (w & 3));   // the right arm's body rows
            else l2_touch(in1 + ft * 60, (int)nt * 240, sink + 64 * (w & 3));       // the left hand
        }
    }
#endif
    // the left arm chain, right wave -> left wave.  With flags it shares storso: the right wave reads its R10 from
    // storso[r] before it writes its chain there (same lane, program order), and the left wave reads the chain after
    // the flag -- 2 KiB less LDS, 32.3 KiB per block, so 5 blocks (5 waves / SIMD) fit a CU's 160 KiB
    float4 *const sarm = RTG_SIDES_FLAGS ? storso : sarm_own;
#if RTG_SIDES_FLAGS
    // per tile: [0] R10 ready (left -> right), [1] left chain ready (right -> left), [2] waves done (RTG_SIDES_TILE_STORE)
    __shared__ int sflag[2][3];
    if (KIND == RTG_SOLVER_FULL_BODY_POS && RTG_SIDES_REBALANCE) {
        if (threadIdx.x < 6) (&sflag[0][0])[threadIdx.x] = 0;
        __syncthreads();
    }
#endif
#if RTG_EXP_TIMESTAMPS
    // measurement knob: lane 0 of each wave of every 8th block records the 100 MHz wall clock at the phase
    // boundaries into the body_rot buffer (tools/side_phases.py): 16 slots per wave, 4 waves per block
    float *const tsb = body_rot;
    body_rot = nullptr;
    auto TS = [&](int k) {
        if (tsb && (blockIdx.x & 7) == 0 && (threadIdx.x & 63) == 0) {
            const uint64_t t = wall_clock64();
            uint32_t *o = reinterpret_cast<uint32_t *>(tsb) + 2 * (((blockIdx.x >> 3) * 4 + w) * 16 + k);
            o[0] = (uint32_t)t;
            o[1] = (uint32_t)(t >> 32);
        }
    };
#else
    auto TS = [](int) {};
#endif
    auto hook1 = [&](int k) { TS(1 + k); };    // 1: first fit's A formed (its points loaded), 2: its SVD + R done
    auto hook2 = [&](int k) { TS(10 + k); };   // 10 / 11: the same for the left wave's second fit
    TS(0);
    if (KIND == RTG_SOLVER_FULL_BODY_POS && RTG_SIDES_REBALANCE) {
        // Balanced FULL_BODY_POS: left wave = torso fit, then the left wrist fit, then the left Euler split /
        // gripper; right wave = the right wrist fit, then BOTH arm chains (each needs only R10), then the right
        // Euler split / gripper.  Two barriers hand R10 (left -> right) and the left chain (right -> left) over LDS.
        // RTG_SIDES_FLAGS: the two hand-overs are per-tile LDS flags instead of block barriers, so each wave waits
        // only for what it reads -- the right wave for R10, the left wave for the left chain -- and the left wave
        // starts its wrist fit as soon as its torso fit is out (it idled 8-10 us at the first barrier behind the
        // right wave's wrist fit: tools/side_phases.py, profiles/r03/side_phases_base.json).
        const auto b = view(in0, 63);
        Q R10 = qident(), W = qident();
        ArmPts apL{}, apR{};
        TipPts tp{};   // RTG_PRELOAD_TIPS: the gripper's hand points, loaded with the wrist fit's points
#if RTG_SIDES_FLAGS
        int *const fl = sflag[w >> 1];
#endif
        if (live) {
            if (!side) {
                R10 = fbp_torso(C, b, hook1);
                storso[r] = make_float4(R10.x, R10.y, R10.z, R10.w);
            } else {
                apL = load_arm<0>(b);
                apR = load_arm<1>(b);
                if (RTG_PRELOAD_TIPS) tp = load_tips(view(in2, 60));
                W = fbp_wrist_fit<1>(C, view(in2, 60), hook1);
            }
        }
        TS(3);
#if RTG_SIDES_FLAGS
        if (!side) lds_signal(&fl[0]);   // R10 of this tile is in storso
        else lds_wait(&fl[0]);
#else
        __syncthreads();
#endif
        TS(4);
        Q chain = qident();
        if (side) {
            if (live) {
                const float4 t = storso[r];
                R10 = Q{t.x, t.y, t.z, t.w};
                if (RTG_SIDES_FLAGS == 2) chain = fbp_arm<1>(C, apR, R10, E);   // right arm first: see below
                const Q cl = fbp_arm<0>(C, apL, R10, E);
                sarm[r] = make_float4(cl.x, cl.y, cl.z, cl.w);
            }
#if RTG_SIDES_FLAGS
            // the left chain and its exp-map slots 0-3 are in LDS (RTG_SIDES_FLAGS == 2: the right arm's 7-10 too, so
            // the left wave, which finishes its own program first, can take more of the read-out: RTG_SIDES_FIN_LEFT)
            lds_signal(&fl[1]);
#endif
            if (live && RTG_SIDES_FLAGS != 2) chain = fbp_arm<1>(C, apR, R10, E);
        } else if (live) {
            emit_fixed_links(E);
            if (RTG_PRELOAD_TIPS) tp = load_tips(view(in1, 60));
            W = fbp_wrist_fit<0>(C, view(in1, 60), hook2);
        }
        TS(5);
#if RTG_SIDES_FLAGS
        if (!side) lds_wait(&fl[1]);
#else
        __syncthreads();
#endif
        TS(6);
        if (live) {
            float *brow = body_rot ? body_rot + f * 236 : nullptr;
            if (!RTG_PRELOAD_TIPS) tp = load_tips(view(side ? in2 : in1, 60));
            if (side) {
                fbp_side_after_arm<PRECISE, 1>(C, tp, R10, chain, W, E, brow);
            } else {
                const float4 c = sarm[r];
                fbp_side_after_arm<PRECISE, 0>(C, tp, R10, Q{c.x, c.y, c.z, c.w}, W, E, brow);
            }
        }
        TS(7);
    } else if (KIND == RTG_SOLVER_FULL_BODY_POS || KIND == RTG_SOLVER_UPPER_BODY) {
        // The torso fit is shared by both sides: the left wave fits it while the right wave fits its own hand
        // (FULL_BODY_POS; nothing to overlap for UPPER_BODY), then one block barrier hands R10 over LDS.
        const auto b = view(in0, 63);   // body (FULL_BODY_POS) / mocap points (UPPER_BODY), both (B, 21, 3)
        Q R10 = qident(), W = qident();
        ArmPts ap{};
        TipPts tp{};
        if (live) {
            if (KIND == RTG_SOLVER_FULL_BODY_POS && RTG_PRELOAD_ARM) ap = side ? load_arm<1>(b) : load_arm<0>(b);
            if (!side) {
                R10 = KIND == RTG_SOLVER_FULL_BODY_POS ? fbp_torso(C, b) : upper_torso(C, b);
                storso[r] = make_float4(R10.x, R10.y, R10.z, R10.w);
            } else if (KIND == RTG_SOLVER_FULL_BODY_POS) {
                const auto H = view(in2, 60);
                if (RTG_PRELOAD_TIPS) tp = load_tips(H);
                W = fbp_wrist_fit<1>(C, H);
            }
        }
        __syncthreads();
        if (live) {
            if (side) {
                const float4 t = storso[r];
                R10 = Q{t.x, t.y, t.z, t.w};
            } else {
                emit_fixed_links(E);
            }
            if (KIND == RTG_SOLVER_FULL_BODY_POS) {
                float *brow = body_rot ? body_rot + f * 236 : nullptr;
                if (!RTG_PRELOAD_ARM) ap = side ? load_arm<1>(b) : load_arm<0>(b);
                if (side) {
                    if (!RTG_PRELOAD_TIPS) tp = load_tips(view(in2, 60));
                    solve_fbp_side<PRECISE, 1>(C, ap, tp, R10, W, E, brow);
                } else {
                    const auto H = view(in1, 60);
                    if (RTG_PRELOAD_TIPS) tp = load_tips(H);
                    W = fbp_wrist_fit<0>(C, H);
                    if (!RTG_PRELOAD_TIPS) tp = load_tips(H);
                    solve_fbp_side<PRECISE, 0>(C, ap, tp, R10, W, E, brow);
                }
            } else {
                if (side) solve_upper_side<1>(C, b, R10, E);
                else solve_upper_side<0>(C, b, R10, E);
            }
        }
    } else if (live) {
        if (!side) emit_fixed_links(E);
        if (KIND == RTG_SOLVER_FULL_BODY_ROT) {
            if (side) solve_full_body_rot_side<1>(C, view(in0, 84), view(in1, 63), view(in3, 60), E);
            else solve_full_body_rot_side<0>(C, view(in0, 84), view(in1, 63), view(in2, 60), E);
        } else {
            if (side) solve_body_rot_side<1>(C, view(in0, 84), E);
            else solve_body_rot_side<0>(C, view(in0, 84), E);
        }
    }
    if (live) {
        // exp-map read-out split: slots [0, NL) on the left wave, [NL, 14) on the right.  Balanced FULL_BODY_POS
        // leaves the right wave the heavier side program (two arm chains), so the left wave takes more slots.  The
        // arm slots (0-3 left, 7-10 right) were written before the last barrier, by either wave; the wrist slots are
        // written by their own side's wave after it (4-6 left, 11-13 right), so each wave may read out only slots it
        // wrote itself or the arm slots: NL in [7, 11] (static_assert below).
        constexpr int NL = (KIND == RTG_SOLVER_FULL_BODY_POS && RTG_SIDES_REBALANCE) ? RTG_SIDES_FIN_LEFT : 7;
        static_assert(NL >= 7 && NL <= 11, "RTG_SIDES_FIN_LEFT must keep each wave's wrist slots on that wave");
        // with flags the left wave has only the left chain's slots 0-3 from the right wave (the right arm's 7-10 are
        // written after the flag): it reads exactly [0, 7)
        static_assert(!(KIND == RTG_SOLVER_FULL_BODY_POS && RTG_SIDES_REBALANCE && RTG_SIDES_FLAGS == 1) || NL == 7,
                      "RTG_SIDES_FLAGS == 1 needs RTG_SIDES_FIN_LEFT == 7");
        E.finalize(side ? NL : 0, side ? 14 - NL : NL);
    }
    TS(8);
#if RTG_SIDES_FLAGS && RTG_SIDES_TILE_STORE
    if (KIND == RTG_SOLVER_FULL_BODY_POS && RTG_SIDES_REBALANCE) {
        // The tile's two waves meet at an LDS counter instead of the block barrier: the first to arrive exits (its
        // VGPRs free for the next block, whose LDS already fits beside this one's), the second stores the tile's rows.
        // The side programs are unequal (the left wave runs two SVDs, the right one SVD and both arm chains), so
        // one wave of each tile used to idle at the barrier.  acq_rel: the first wave's sdof writes are visible to
        // the second wave's reads below.
        const int lane = threadIdx.x & 63;
        int prev = 0;
        if (lane == 0)
            prev = __hip_atomic_fetch_add(&sflag[w >> 1][2], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_readfirstlane(prev) == 0) return;   // wave-uniform: lane 0 is active here
        TS(9);
        const int64_t t0 = f0 + (w >> 1) * 64;
        const int64_t nrows = (B - t0) < 64 ? (B - t0) : 64;
        if (nrows <= 0) return;
        const int nvals = (int)nrows * 30;
        float *dst = dof + t0 * 30;   // (f0 + 64 t) * 120 bytes: 16-byte aligned
        const float *src = sdof + (w >> 1) * 64 * kDofStride;
        auto at = [&](int i) {
            const int rr = i / 30;
            return src[rr * kDofStride + (i - rr * 30)];
        };
        const int nvec = nvals >> 2;
        for (int v = lane; v < nvec; v += 64) {
            const int i = v << 2;
            *reinterpret_cast<float4 *>(dst + i) = make_float4(at(i), at(i + 1), at(i + 2), at(i + 3));
        }
        for (int i = (nvec << 2) + lane; i < nvals; i += 64) dst[i] = at(i);
        TS(12);
        return;
    }
#endif
    __syncthreads();
    TS(9);
    const int64_t nrows = (B - f0) < kSideFrames ? (B - f0) : kSideFrames;
    const int nvals = (int)nrows * 30;
    float *dst = dof + f0 * 30;
    auto at = [&](int i) {
        const int rr = i / 30;
        return sdof[rr * kDofStride + (i - rr * 30)];
    };
    const int nvec = nvals >> 2;
    for (int v = threadIdx.x; v < nvec; v += 256) {
        const int i = v << 2;
        *reinterpret_cast<float4 *>(dst + i) = make_float4(at(i), at(i + 1), at(i + 2), at(i + 3));
    }
    for (int i = (nvec << 2) + threadIdx.x; i < nvals; i += 256) dst[i] = at(i);
    TS(12);
}

// ----------------------------------------------------------------------------
// FULL_BODY_POS for small batches (the teleop / config-2 latency path): three waves per 64-frame tile, one per
// Kabsch fit.  The torso fit and the two wrist fits are independent (full_body_pos_retargeter.py:69-70, 137-140,
// 160-163), so they run concurrently; after one barrier the wrist waves each run their side (arm, Euler split,
// gripper) while the torso wave writes the fixed links; the exp-map read-out is split three ways.  A frame's
// critical path loses one SVD against k_solve_sides (which runs the torso and the left wrist fit on one wave).
// The same device functions in the same order per value: the same bits (test_solver_batch_invariance).
// Large batches keep k_solve_sides: there the third wave idles after its fit and costs throughput.
// ----------------------------------------------------------------------------
constexpr int kLatFrames = 64;

template <bool PRECISE, bool SOA>
__global__ __launch_bounds__(192) void k_fbp_latency(SolverConsts C, const float *__restrict__ in0,
                                                     const float *__restrict__ in1, const float *__restrict__ in2,
                                                     int64_t B, float *__restrict__ dof, float *__restrict__ local_rot,
                                                     float *__restrict__ body_rot)
{
    __shared__ float sdof[kLatFrames * kDofStride];
    __shared__ float4 sfit[3][kLatFrames];   // R10, W_left, W_right
    __shared__ float2 sst[14 * kLatFrames];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t f0 = (int64_t)blockIdx.x * kLatFrames, f = f0 + lane;
    const bool live = f < B;
#if RTG_EXP_TIMESTAMPS
    float *const tsb = body_rot;
    body_rot = nullptr;
    auto TS = [&](int k) {
        if (tsb && blockIdx.x == 0 && lane == 0) {
            const uint64_t t = wall_clock64();
            reinterpret_cast<uint32_t *>(tsb)[2 * (16 * w + k)] = (uint32_t)t;
            reinterpret_cast<uint32_t *>(tsb)[2 * (16 * w + k) + 1] = (uint32_t)(t >> 32);
        }
    };
#else
    auto TS = [](int) {};
#endif
    auto hook = [&](int k) { TS(8 + k); };   // 8: A formed, 9: SVD + R done, 10: arm, 11: Euler
    TS(0);
    const Emit E{sdof + lane * kDofStride, live && local_rot ? local_rot + f * 124 : nullptr, C.ang_tab, sst + lane,
                 kLatFrames};
    auto view = [&](const float *base, int row_floats) { return frame_view<SOA>(base, f, row_floats, B); };
    const auto b = view(in0, 63);
    ArmPts ap{};
    TipPts tp{};
    if (live) {
        Q q;
        if (w == 0) {
            q = fbp_torso(C, b, hook);
        } else {
            const auto H = view(w == 1 ? in1 : in2, 60);
            ap = w == 1 ? load_arm<0>(b) : load_arm<1>(b);
            q = w == 1 ? fbp_wrist_fit<0>(C, H, hook) : fbp_wrist_fit<1>(C, H, hook);
            tp = load_tips(H);
        }
        sfit[w][lane] = make_float4(q.x, q.y, q.z, q.w);
    }
    TS(1);
    __syncthreads();
    TS(2);
    if (live) {
        const float4 t = sfit[0][lane];
        const Q R10{t.x, t.y, t.z, t.w};
        float *brow = body_rot ? body_rot + f * 236 : nullptr;
        if (w == 0) {
            emit_fixed_links(E);
        } else {
            const float4 u = sfit[w][lane];
            const Q W{u.x, u.y, u.z, u.w};
            if (w == 1) solve_fbp_side<PRECISE, 0>(C, ap, tp, R10, W, E, brow, hook);
            else solve_fbp_side<PRECISE, 1>(C, ap, tp, R10, W, E, brow, hook);
        }
    }
    TS(3);
    __syncthreads();
    TS(4);
    if (live) E.finalize(w == 0 ? 0 : (w == 1 ? 5 : 10), w == 2 ? 4 : 5);
    TS(5);
    __syncthreads();
    TS(6);
    const int64_t nrows = (B - f0) < kLatFrames ? (B - f0) : kLatFrames;
    const int nvals = (int)nrows * 30;
    float *dst = dof + f0 * 30;
    auto at = [&](int i) {
        const int rr = i / 30;
        return sdof[rr * kDofStride + (i - rr * 30)];
    };
    const int nvec = nvals >> 2;   // f0 * 30 floats = 16-byte aligned (f0 is a multiple of 64)
    for (int v = threadIdx.x; v < nvec; v += 192) {
        const int i = v << 2;
        *reinterpret_cast<float4 *>(dst + i) = make_float4(at(i), at(i + 1), at(i + 2), at(i + 3));
    }
    for (int i = (nvec << 2) + threadIdx.x; i < nvals; i += 192) dst[i] = at(i);
    TS(7);
}

// ----------------------------------------------------------------------------
// FULL_BODY_POS latency kernel, five waves per 64-frame tile (RTG_LATENCY_WAVES = 5).  The arm chain
// (shoulder_pr / elbow_py, full_body_pos_retargeter.py:75-93) needs only the torso fit R10, not the wrist fit, so
// it runs on its own wave as soon as R10 is in LDS -- concurrently with the (longer) wrist SVDs -- instead of after a
// block barrier that waits for all three fits (measured phase split, tools/latency_phases.py: torso fit 6-8 us,
// wrist fits 9-13 us, arm 5-7 us, Euler 3-4 us).
//   wave 0      torso fit -> R10 -> fixed links
//   wave 1, 2   left / right wrist fit -> gripper; then (arm chain ready) Euler split, body_rot rows, exp-maps
//   wave 3, 4   left / right arm points; (R10 ready) arm chain -> LDS; the arm links' exp-maps
// Hand-over is by per-wave LDS flags (release / acquire at workgroup scope): a producer never waits on a consumer,
// and all five waves of a workgroup are resident together, so the waits always end; each also has an iteration
// cap.  Every value is computed by the same device function from the same operands as in k_fbp_latency /
// k_solve_sides: the same bits (test_solver_batch_invariance covers both sizes).
// ----------------------------------------------------------------------------

// one 64-frame tile (frames f0..) by the 320 threads of a workgroup; shared by the batched latency kernel and the
// per-frame server (k_frame_server)
template <bool PRECISE, bool SOA>
RTG_DEV void fbp_latency5_tile(const SolverConsts &C, const float *__restrict__ in0, const float *__restrict__ in1,
                               const float *__restrict__ in2, int64_t B, int64_t f0, float *__restrict__ dof,
                               float *__restrict__ local_rot, float *__restrict__ body_rot)
{
    __shared__ float sdof[kLatFrames * kDofStride];
    __shared__ float4 sfit[kLatFrames];        // R10
    __shared__ float4 schain[2][kLatFrames];   // quat_mul_four of each arm's links (the wrist parent chain)
    __shared__ float2 sst[14 * kLatFrames];
    __shared__ int sflag[3];                   // R10 ready, left arm ready, right arm ready
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t f = f0 + lane;
    const bool live = f < B;
    if (threadIdx.x < 3) sflag[threadIdx.x] = 0;
    __syncthreads();
#if RTG_EXP_TIMESTAMPS
    float *const tsb = body_rot;
    body_rot = nullptr;
    auto TS = [&](int k) {
        if (tsb && blockIdx.x == 0 && lane == 0) {
            const uint64_t t = wall_clock64();
            reinterpret_cast<uint32_t *>(tsb)[2 * (16 * w + k)] = (uint32_t)t;
            reinterpret_cast<uint32_t *>(tsb)[2 * (16 * w + k) + 1] = (uint32_t)(t >> 32);
        }
    };
#else
    auto TS = [](int) {};
#endif
    auto hook = [&](int k) { TS(8 + k); };
    TS(0);
    const Emit E{sdof + lane * kDofStride, live && local_rot ? local_rot + f * 124 : nullptr, C.ang_tab, sst + lane,
                 kLatFrames};
    auto view = [&](const float *base, int row_floats) { return frame_view<SOA>(base, f, row_floats, B); };
    const auto b = view(in0, 63);
    if (w == 0) {
        if (live) {
            const Q q = fbp_torso(C, b, hook);
            sfit[lane] = make_float4(q.x, q.y, q.z, q.w);
        }
        lds_signal(&sflag[0]);
        TS(1);
        if (live) emit_fixed_links(E);
        TS(2);
    } else if (w >= 3) {
        const int side = w - 3;
        ArmPts ap{};
        if (live) ap = side ? load_arm<1>(b) : load_arm<0>(b);
        TS(1);
        lds_wait(&sflag[0]);
        TS(2);
        if (live) {
            const float4 t = sfit[lane];
            const Q R10{t.x, t.y, t.z, t.w};
            const V up = vsub(ap.el, ap.sh), fo = vsub(ap.wr, ap.el);
            const Q ch = side ? solve_arm<21>(E, up, fo, C.rsh, C.rel, R10) : solve_arm<12>(E, up, fo, C.lsh, C.lel, R10);
            schain[side][lane] = make_float4(ch.x, ch.y, ch.z, ch.w);
        }
        lds_signal(&sflag[1 + side]);
        TS(3);
        if (live) E.finalize(side ? 7 : 0, 4);
        TS(4);
    } else {
        const int side = w - 1;
        const auto H = view(side ? in2 : in1, 60);
        Q W = qident();
        TipPts tp{};
        if (live) {
            W = side ? fbp_wrist_fit<1>(C, H, hook) : fbp_wrist_fit<0>(C, H, hook);
            tp = load_tips(H);
        }
        TS(1);
        float a = 0.0f;
        if (live) a = hand_x_mean(qconj(W), tp.h0, tp.t);   // the gripper needs only W (:142-158 / :165-175)
        TS(2);
        lds_wait(&sflag[1 + side]);   // the arm waited for R10 first: both are visible (release / acquire chain)
        TS(3);
        if (live) {
            const float4 t = sfit[lane], c = schain[side][lane];
            const Q R10{t.x, t.y, t.z, t.w}, chain{c.x, c.y, c.z, c.w};
            float *brow = body_rot ? body_rot + f * 236 : nullptr;
            const int D0 = side ? 27 : 18;
            if (PRECISE) {
                const float sc = clamp_lohi(a / C.orig - 0.5f, 0.0f, 0.5f) / 0.5f;
                E.row[D0] = sc * 0.044f;
                E.row[D0 + 1] = sc * -0.044f;
            } else {
                const bool closed = a / C.orig < 0.7f;
                E.row[D0] = closed ? 0.0f : 0.044f;
                E.row[D0 + 1] = closed ? 0.0f : -0.044f;
            }
            const Q loc = qmul_norm(qconj(qmul_norm(R10, chain)), W);
            if (side) emit_euler_xyz<25>(E, loc);
            else emit_euler_xyz<16>(E, loc);
            if (brow) {   // body_global_rotation rows (:116, :172-173), as solve_fbp_side
                st4(brow + 4 * (side ? 39 : 14), W);
                if (!side)
                    for (int j = 0; j < 59; ++j)
                        if (j != 14 && j != 39) st4(brow + 4 * j, j == 10 ? R10 : qident());
            }
            TS(4);
            E.finalize(side ? 11 : 4, 3);
        }
    }
    TS(5);
    __syncthreads();
    TS(6);
    const int64_t nrows = (B - f0) < kLatFrames ? (B - f0) : kLatFrames;
    const int nvals = (int)nrows * 30;
    float *dst = dof + f0 * 30;
    auto at = [&](int i) {
        const int rr = i / 30;
        return sdof[rr * kDofStride + (i - rr * 30)];
    };
    const int nvec = nvals >> 2;
    for (int v = threadIdx.x; v < nvec; v += 320) {
        const int i = v << 2;
        *reinterpret_cast<float4 *>(dst + i) = make_float4(at(i), at(i + 1), at(i + 2), at(i + 3));
    }
    for (int i = (nvec << 2) + threadIdx.x; i < nvals; i += 320) dst[i] = at(i);
    TS(7);
}

// ----------------------------------------------------------------------------
// ONE frame (B = 1: the teleop path -- k_frame_server and rtg_retarget_f32 at B = 1) on k_fbp_latency5's five
// waves, with the frame's independent sub-steps on separate LANES of a wave (they idle at B = 1 otherwise):
//   * each arm map (cal_shoulderPR / cal_elbowP_and_shoulderY): the pitch (yaw) angle on lane 0, the roll (elbow)
//     angle on lane 1 -- one radians_between + one quat_from_angle_axis instruction stream instead of two;
//   * the scipy Euler split of each wrist: its three atan2 on lanes 0-2, then one elementary quaternion per lane;
//   * the exp-map DOF read-out: one link per lane.
// Every value is computed by the same device functions on the same operands as in the batched kernels (the pitch
// angle as radians_between of the exact unit axes, which is radians_between_axes bit for bit), so the bits are the
// batched kernels' (test_frame_server_matches_batched, test_solver_batch_invariance).
// ----------------------------------------------------------------------------
RTG_DEV float rdl(float v, int l) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l)); }
RTG_DEV double rdl(double v, int l)
{
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// G frames per block, L = 64 / G lanes per frame: lane = frame-in-group * L + sub.  gb<G>(v, k): sub-lane k's v of
// this lane's frame (G == 1: v_readlane; else a shuffle inside the frame's L lanes).  Called with every lane active.
template <int G>
RTG_DEV float gb(float v, int k)
{
    if constexpr (G == 1) return rdl(v, k);
    else return __shfl(v, (int)((threadIdx.x & 63) & ~(64 / G - 1)) + k, 64);
}
template <int G>
RTG_DEV double gb(double v, int k)
{
    if constexpr (G == 1) return rdl(v, k);
    else return __shfl(v, (int)((threadIdx.x & 63) & ~(64 / G - 1)) + k, 64);
}
template <int G>
RTG_DEV Q gb(Q q, int k) { return Q{gb<G>(q.x, k), gb<G>(q.y, k), gb<G>(q.z, k), gb<G>(q.w, k)}; }
template <int G>
RTG_DEV int sub_lane() { return (int)(threadIdx.x & 63) & (64 / G - 1); }

// shoulder_pr (SHOULDER) / elbow_py of one frame: sub-lane 0 the first angle's quaternion, sub-lane 1 the second's
template <int G, bool SHOULDER>
RTG_DEV void arm_pair_lanes(V v1, ArmZero z0, Q parent, Q &first, Q &second)
{
    const int sub = sub_lane<G>();
    Q q = qident();
    if (sub < 2) {
        const V ex{1.f, 0.f, 0.f}, ey{0.f, 1.f, 0.f}, ez{0.f, 0.f, 1.f};
        const V pn = SHOULDER ? ey : ez;   // the plane of the first angle
        const V v1r = qrotate(qconj(parent), v1);
        const V v1p = proj_in_plane(v1r, pn);
        const bool l0 = sub == 0;
        const V a{l0 ? 1.f : v1p.x, l0 ? 0.f : v1p.y, l0 ? 0.f : v1p.z};
        const V b = l0 ? v1p : v1r;
        const V c = SHOULDER ? cross3(v1p, ey) : cross3(ez, v1p);
        const V n = l0 ? pn : c;
        const float ang = radians_between(a, b, n);
        const V ax = l0 ? pn : (SHOULDER ? ex : ey);
        q = qfrom_angle_unit_axis(ang - (l0 ? z0.th0 : z0.ph0), ax);
    }
    first = gb<G>(q, 0);
    second = gb<G>(q, 1);
}
// Emit::link with a run-time link index (lane-parallel writers)
RTG_DEV void link_rt(const Emit &E, int link, Q q)
{
    const int k = kHuDofAxis[link - 1];
    E.st[(link <= 18 ? link - 12 : link - 14) * E.sst] = make_float2(q.w, k == 0 ? q.x : (k == 1 ? q.y : q.z));
    if (E.lr) st4(E.lr + 4 * link, q);
}
template <int G, int L0>
RTG_DEV Q solve_arm_lanes(const Emit &E, V upper, V fore, ArmZero zs, ArmZero ze, Q parent, bool live)
{
    const bool w0 = live && sub_lane<G>() == 0;
    Q p, r, y, e;
    arm_pair_lanes<G, true>(upper, zs, parent, p, r);
    if (w0) { E.link<L0>(p); E.link<L0 + 1>(r); }
    arm_pair_lanes<G, false>(fore, ze, qmul(qmul(parent, p), r), y, e);
    if (w0) { E.link<L0 + 2>(y); E.link<L0 + 3>(e); }
    return qmul(qmul(qmul(p, r), y), e);
}
// emit_euler_xyz (quat_in_xyz_axis 'XYZ', scipy_as_euler's arithmetic) with the three atan2 on sub-lanes 0-2 and one
// elementary quaternion per sub-lane
template <int G, int L0>
RTG_DEV void emit_euler_xyz_lanes(const Emit &E, Q qf, bool live)
{
    const int sub = sub_lane<G>();
    // scipy_as_euler(q, 0, 1, 2, intrinsic): i = 2, j = 1, k = 0, not symmetric, sign = (2-1)(1-0)(0-2)/2 = -1
    double q[4] = {(double)qf.x, (double)qf.y, (double)qf.z, (double)qf.w};
    const double nrm = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    q[0] /= nrm; q[1] /= nrm; q[2] /= nrm; q[3] /= nrm;
    const int sign = -1;
    const double qi = q[2], qj = q[1], qk = q[0];
    const double a = q[3] - qj, b = qi + qk * sign, c = qj + q[3], d = qk * sign - qi;
    double at = 0.0;
    if (sub < 3) {
        const double Y = sub == 0 ? ::hypot(c, d) : (sub == 1 ? b : d);
        const double X = sub == 0 ? ::hypot(a, b) : (sub == 1 ? a : c);
        at = ::atan2(Y, X);
    }
    double ang[3];
    ang[1] = 2.0 * gb<G>(at, 0);
    const double half_sum = gb<G>(at, 1), half_diff = gb<G>(at, 2);
    int kase = 0;
    if (fabs(ang[1]) <= 1e-7) kase = 1;
    else if (fabs(ang[1] - M_PI) <= 1e-7) kase = 2;
    if (kase == 0) {
        ang[0] = half_sum - half_diff;
        ang[2] = half_sum + half_diff;
    } else {
        ang[0] = 0.0;
        ang[2] = kase == 1 ? 2.0 * half_sum : 2.0 * half_diff;
    }
    ang[2] *= sign;
    ang[1] -= M_PI / 2.0;
    { const double tt = ang[0]; ang[0] = ang[2]; ang[2] = tt; }
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        if (ang[t] < -M_PI) ang[t] += 2.0 * M_PI;
        else if (ang[t] > M_PI) ang[t] -= 2.0 * M_PI;
    }
    if (live && sub < 3) link_rt(E, L0 + sub, elementary_quat(sub, sub == 0 ? ang[0] : (sub == 1 ? ang[1] : ang[2])));
}
// Emit::finalize with one slot per sub-lane (slots s0 .. s0 + n - 1)
template <int G>
RTG_DEV void finalize_lanes(const Emit &E, int s0, int n, bool live)
{
    const int sub = sub_lane<G>();
    if (live && sub < n) {
        const int j = s0 + sub;
        const float2 v = E.st[j * E.sst];
        const ExpDof e = exp_dof_table_part(v.x, E.ang);
        float val = exp_dof_finish(e, v.y);
        if (__builtin_expect(e.exact, 0)) val = normalize_angle(2.0f * cr_acos(v.x)) * (v.y / e.sin_theta);
        E.row[j < 7 ? 11 + j : 13 + j] = val;
    }
}

// G frames (f0 .. f0 + nfr - 1) whose rows (body 63 | left hand 60 | right hand 60 floats) are in `rows`, G x 183
template <bool PRECISE, int G>
RTG_DEV void fbp_group_tile(const SolverConsts &C, const float *rows, int nfr, int64_t f0, float *__restrict__ dof,
                            float *__restrict__ local_rot, float *__restrict__ body_rot)
{
    static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "at least 4 lanes per frame");
    __shared__ float sdof[G * kDofStride];
    __shared__ float4 sfit[G], schain[2][G];
    __shared__ float2 sst[14 * G];
    __shared__ int sflag[3];   // R10 ready, left arm ready, right arm ready
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane / (64 / G), sub = sub_lane<G>();
    const bool live = g < nfr, w0 = live && sub == 0;
    const int64_t f = f0 + g;
    if (threadIdx.x < 3) sflag[threadIdx.x] = 0;
    __syncthreads();
    const Emit E{sdof + g * kDofStride, live && local_rot ? local_rot + f * 124 : nullptr, C.ang_tab, sst + g, G};
    const float *row = rows + g * 183;
    const FV<false> b{row};
    if (w == 0) {
        if (w0) {
            const Q q = fbp_torso(C, b);
            sfit[g] = make_float4(q.x, q.y, q.z, q.w);
        }
        lds_signal(&sflag[0]);
        if (w0) emit_fixed_links(E);
    } else if (w >= 3) {
        const int side = w - 3;
        const ArmPts ap = side ? load_arm<1>(b) : load_arm<0>(b);
        lds_wait(&sflag[0]);
        const float4 t = sfit[g];
        const Q R10{t.x, t.y, t.z, t.w};
        const V up = vsub(ap.el, ap.sh), fo = vsub(ap.wr, ap.el);
        const Q ch = side ? solve_arm_lanes<G, 21>(E, up, fo, C.rsh, C.rel, R10, live)
                          : solve_arm_lanes<G, 12>(E, up, fo, C.lsh, C.lel, R10, live);
        if (w0) schain[side][g] = make_float4(ch.x, ch.y, ch.z, ch.w);
        lds_signal(&sflag[1 + side]);
        finalize_lanes<G>(E, side ? 7 : 0, 4, live);
    } else {
        const int side = w - 1;
        const FV<false> H{row + (side ? 123 : 63)};
        Q W = qident();
        float a = 0.0f;
        if (w0) {
            W = side ? fbp_wrist_fit<1>(C, H) : fbp_wrist_fit<0>(C, H);
            const TipPts tp = load_tips(H);
            a = hand_x_mean(qconj(W), tp.h0, tp.t);   // the gripper needs only W (:142-158 / :165-175)
        }
        W = gb<G>(W, 0);
        lds_wait(&sflag[1 + side]);   // the arm waited for R10 first: both are visible (release / acquire chain)
        const float4 t = sfit[g], c = schain[side][g];
        const Q R10{t.x, t.y, t.z, t.w}, chain{c.x, c.y, c.z, c.w};
        if (w0) {
            const int D0 = side ? 27 : 18;
            if (PRECISE) {
                const float sc = clamp_lohi(a / C.orig - 0.5f, 0.0f, 0.5f) / 0.5f;
                E.row[D0] = sc * 0.044f;
                E.row[D0 + 1] = sc * -0.044f;
            } else {
                const bool closed = a / C.orig < 0.7f;
                E.row[D0] = closed ? 0.0f : 0.044f;
                E.row[D0 + 1] = closed ? 0.0f : -0.044f;
            }
            if (body_rot) {   // body_global_rotation rows (:116, :172-173), as solve_fbp_side
                float *brow = body_rot + f * 236;
                st4(brow + 4 * (side ? 39 : 14), W);
                if (!side)
                    for (int j = 0; j < 59; ++j)
                        if (j != 14 && j != 39) st4(brow + 4 * j, j == 10 ? R10 : qident());
            }
        }
        const Q loc = qmul_norm(qconj(qmul_norm(R10, chain)), W);
        if (side) emit_euler_xyz_lanes<G, 25>(E, loc, live);
        else emit_euler_xyz_lanes<G, 16>(E, loc, live);
        finalize_lanes<G>(E, side ? 11 : 4, 3, live);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nfr * 30; i += blockDim.x) {   // the group's contiguous DOF rows
        const int r = i / 30;
        dof[f0 * 30 + i] = sdof[r * kDofStride + (i - r * 30)];
    }
}
// The frames' rows cross into LDS once, all loads in flight together (one round trip even from host memory); SoA
// inputs are read component-major (consecutive threads, consecutive frames).
template <bool PRECISE, bool SOA, int G>
__global__ __launch_bounds__(320) void k_fbp_group(SolverConsts C, const float *__restrict__ in0,
                                                   const float *__restrict__ in1, const float *__restrict__ in2,
                                                   int64_t B, float *__restrict__ dof, float *__restrict__ local_rot,
                                                   float *__restrict__ body_rot)
{
    __shared__ float rows[G * 183 + 1];
    const int64_t f0 = (int64_t)blockIdx.x * G;
    const int nfr = (int)((B - f0) < G ? (B - f0) : G);
    for (int t = threadIdx.x; t < G * 183; t += blockDim.x) {
        const int g = SOA ? t % G : t / 183, e = SOA ? t / G : t % 183;
        float v = 0.0f;
        if (g < nfr) {
            const int64_t fg = f0 + g;
            if (SOA) v = e < 63 ? in0[e * B + fg] : (e < 123 ? in1[(e - 63) * B + fg] : in2[(e - 123) * B + fg]);
            else v = e < 63 ? in0[fg * 63 + e] : (e < 123 ? in1[fg * 60 + e - 63] : in2[fg * 60 + e - 123]);
        }
        rows[g * 183 + e] = v;
    }
    __syncthreads();
    fbp_group_tile<PRECISE, G>(C, rows, nfr, f0, dof, local_rot, body_rot);
}

template <bool PRECISE, bool SOA>
__global__ __launch_bounds__(320) void k_fbp_latency5(SolverConsts C, const float *__restrict__ in0,
                                                      const float *__restrict__ in1, const float *__restrict__ in2,
                                                      int64_t B, float *__restrict__ dof, float *__restrict__ local_rot,
                                                      float *__restrict__ body_rot)
{
    fbp_latency5_tile<PRECISE, SOA>(C, in0, in1, in2, B, (int64_t)blockIdx.x * kLatFrames, dof, local_rot, body_rot);
}

// ----------------------------------------------------------------------------
// Per-frame server (the teleop loop without a launch per frame; sim_full_body_teleop.py:109-119 calls the solver
// once per captured frame).  One resident workgroup of k_fbp_latency5's shape serves FULL_BODY_POS frames from
// host-mapped memory: the host writes a frame's rows (body | left hand | right hand, AoS) into `in` and then a new
// sequence number into ctl[0]; thread 0 sees it (system-scope acquire), the tile runs at B = 1 reading `in` and
// writing dof / local_rot / body_rot straight into host memory, every wave's stores are released at system scope,
// and thread 0 publishes the sequence number in ctl[1].  The loop ends on ctl[0] == RTG_SERVER_QUIT, or when no
// new frame arrives for idle_ticks (100 MHz wall clock) -- every wave reaches one of the two -- and sets ctl[2].
// ----------------------------------------------------------------------------
template <bool PRECISE>
__global__ __launch_bounds__(320) void k_frame_server(SolverConsts C, const float *in, float *dof, float *local_rot,
                                                      float *body_rot, uint32_t *ctl, uint64_t idle_ticks)
{
    __shared__ uint32_t scmd;
    __shared__ float sframe[184];
    uint32_t last = 0;
    if (threadIdx.x == 0) last = __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int frame = 0; frame < (1 << 30); ++frame) {
        if (threadIdx.x == 0) {
            const uint64_t t0 = wall_clock64();
            uint32_t db;
            for (;;) {
                db = __hip_atomic_load(ctl, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (db != last) break;
                if (wall_clock64() - t0 > idle_ticks) {
                    db = RTG_SERVER_QUIT;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            scmd = db;
        }
        __syncthreads();
        const uint32_t cmd = scmd;
        if (cmd == RTG_SERVER_QUIT) break;   // block-uniform
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // this wave's loads see the host's frame, not cached lines
        // the frame's 183 floats cross the host link ONCE, all in flight together, into LDS; the tile's dependent
        // loads (tips after the wrist fit, arm points after R10) then read LDS instead of host memory
        if (threadIdx.x < 183) sframe[threadIdx.x] = in[threadIdx.x];
        __syncthreads();
        if (RTG_SERVER_FRAME1) fbp_group_tile<PRECISE, 1>(C, sframe, 1, 0, dof, local_rot, body_rot);
        else fbp_latency5_tile<PRECISE, false>(C, sframe, sframe + 63, sframe + 123, 1, 0, dof, local_rot, body_rot);
        __syncthreads();   // every lane of every wave has issued its output stores (a convergent point) ...
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // ... so this wave's release covers all of them
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_store(ctl + 1, cmd, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            last = cmd;
        }
    }
    if (threadIdx.x == 0) __hip_atomic_store(ctl + 2, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Kernel choice.  The side-split kernel halves each wave's program and doubles the waves in flight.  Measured
// against the fused body (same box, same session): 1.6-1.9x at 4096 frames for every kind; at
// 262144 frames FULL_BODY_POS +4 %, FULL_BODY_ROT +15 %, UPPER_BODY and BODY_ROT within box-to-box noise
// (-6..+2 % and -3..+10 % across two boxes).  So every kind runs split; RTG_SOLVER_SIDES=0 builds the fused
// kernels for comparison.  Compile-time choices are `if constexpr`, so a TU instantiates only the kernels it can
// launch (rtg_solve_fbp_aos.hip / rtg_solve_fbp_soa.hip / rtg_solve_other.hip compile in parallel).
template <int KIND, bool PRECISE, bool SOA>
static void launch_kind(const SolverConsts &C, const float *in0, const float *in1, const float *in2,
                        const float *in3, int64_t B, float *dof, float *local_rot, float *body_rot, hipStream_t s)
{
    if constexpr (KIND == RTG_SOLVER_FULL_BODY_POS && RTG_FRAME1_LANES) {
        if (B == 1) {   // one frame on 64 lanes per frame
            hipLaunchKernelGGL((k_fbp_group<PRECISE, SOA, 1>), dim3(1), dim3(320), 0, s, C, in0, in1, in2, B, dof,
                               local_rot, body_rot);
            return;
        }
        if (B <= RTG_GROUP_MAX_B) {   // 16 frames per block, 4 lanes per frame
            hipLaunchKernelGGL((k_fbp_group<PRECISE, SOA, 16>), dim3(grid_for(B, 16)), dim3(320), 0, s, C, in0, in1,
                               in2, B, dof, local_rot, body_rot);
            return;
        }
    }
    if constexpr (KIND == RTG_SOLVER_FULL_BODY_POS && RTG_LATENCY_WAVES == 5) {
        if (B <= RTG_LATENCY_MAX_B) {
            hipLaunchKernelGGL((k_fbp_latency5<PRECISE, SOA>), dim3(grid_for(B, kLatFrames)), dim3(320), 0, s, C,
                               in0, in1, in2, B, dof, local_rot, body_rot);
            return;
        }
    } else if constexpr (KIND == RTG_SOLVER_FULL_BODY_POS) {
        if (B <= RTG_LATENCY_MAX_B) {
            hipLaunchKernelGGL((k_fbp_latency<PRECISE, SOA>), dim3(grid_for(B, kLatFrames)), dim3(192), 0, s, C, in0,
                               in1, in2, B, dof, local_rot, body_rot);
            return;
        }
    }
    if constexpr (!SOA && !RTG_SOLVER_SIDES)
        hipLaunchKernelGGL((k_retarget<KIND, PRECISE>), dim3(grid_for(B, kSolverBlock)), dim3(kSolverBlock), 0, s,
                           C, in0, in1, in2, in3, B, dof, local_rot, body_rot);
    else
        hipLaunchKernelGGL((k_solve_sides<KIND, PRECISE, SOA>), dim3(grid_for(B, kSideFrames)), dim3(256), 0, s, C,
                           in0, in1, in2, in3, B, dof, local_rot, body_rot);
}

// FULL_BODY_POS launches, one TU per input layout
hipError_t launch_fbp_aos(int precise, const SolverConsts &C, const float *in0, const float *in1, const float *in2,
                          int64_t B, float *dof, float *local_rot, float *body_rot, hipStream_t s);
hipError_t launch_fbp_soa(int precise, const SolverConsts &C, const float *in0, const float *in1, const float *in2,
                          int64_t B, float *dof, float *local_rot, float *body_rot, hipStream_t s);

}  // namespace rtg
