// rtg_kernels.hip -- CDNA4 (gfx950) kernels of the retargeting hot path.
//
// Work decomposition: one mocap frame per lane.  Frames are independent
// (SURVEY.md §0), every solver step is a short dependent chain of scalar-sized
// math, and a frame's working set (<= 32 input points) fits in VGPRs, so a
// lane solves its frame end-to-end with no cross-lane traffic.  Zero-pose-only
// terms are evaluated once per solver (k_solver_prep) and arrive as a by-value
// kernel argument (SGPR-resident).  The 30-float DOF row of each frame is
// staged through LDS so the block stores one contiguous, dwordx4-coalesced
// tile instead of 64 lanes writing 120-byte-strided rows.
#include "rtg_kernels.cuh"


namespace rtg {

// ----------------------------------------------------------------------------
// loads / stores
// ----------------------------------------------------------------------------
RTG_DEV V ld3(const float *__restrict__ p) { return V{p[0], p[1], p[2]}; }
RTG_DEV Q ld4(const float *__restrict__ p)
{
    const float4 v = *reinterpret_cast<const float4 *>(p);
    return Q{v.x, v.y, v.z, v.w};
}
RTG_DEV void st4(float *__restrict__ p, Q q) { *reinterpret_cast<float4 *>(p) = make_float4(q.x, q.y, q.z, q.w); }
RTG_DEV void st3(float *__restrict__ p, V v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }

// Launch-uniform tables (topology, schedule) read through the constant address
// space: the compiler cannot prove them unclobbered in a kernel that stores to
// global memory, so a plain load would be a vector load, and its s_waitcnt
// vmcnt would also drain every prefetch in flight.  These become s_load (lgkmcnt).
template <typename T>
RTG_DEV T ld_const(const T *p)
{
    return *(const __attribute__((address_space(4))) T *)p;
}
RTG_DEV V ld_const(const V *p) { return V{ld_const(&p->x), ld_const(&p->y), ld_const(&p->z)}; }
RTG_DEV Q ld_const(const Q *p) { return Q{ld_const(&p->x), ld_const(&p->y), ld_const(&p->z), ld_const(&p->w)}; }

// ----------------------------------------------------------------------------
// solver constants prep (1 thread): theta0 / phi0 of the four arm maps and the
// gripper denominator, computed with exactly the per-frame device math.
// ----------------------------------------------------------------------------
__global__ void k_solver_prep(SolverConsts *c)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    c->lsh = shoulder_zero(c->v0_lsh);
    c->rsh = shoulder_zero(c->v0_rsh);
    c->lel = elbow_zero(c->v0_lel);
    c->rel = elbow_zero(c->v0_rel);
    c->orig = mean5(c->grip_d[0], c->grip_d[1], c->grip_d[2], c->grip_d[3], c->grip_d[4]);
}

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
    RTG_DEV void finalize(int s0, int n) const
    {
#pragma unroll
        for (int j = 0; j < 14; ++j)
            if (j >= s0 && j < s0 + n) {
                const float2 v = st[j * sst];
                row[j < 7 ? 11 + j : 13 + j] = exp_dof_tab(v.x, v.y, ang);
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
#ifndef RTG_SIDES_REBALANCE
#define RTG_SIDES_REBALANCE 1   // FULL_BODY_POS side kernel: the right wave also runs the LEFT arm chain (it needs only
#endif                          // R10) while the left wave runs the left wrist fit -- 1.5 SVD-equivalents per wave
#ifndef RTG_SIDES_FIN_LEFT
#define RTG_SIDES_FIN_LEFT 7    // exp-map slots (of 14) the left wave reads out in the balanced kernel (7, 8, 9: within noise)
#endif
#ifndef RTG_SIDES_WAVES
#define RTG_SIDES_WAVES 1   // min waves per SIMD for the side kernel (1: the compiler picks; measured best)
#endif
#ifndef RTG_EXP_HOT_INPUTS
#define RTG_EXP_HOT_INPUTS 0
#endif
#ifndef RTG_SOLVER_SIDES
#define RTG_SOLVER_SIDES 1   // 0: always the fused one-lane-per-frame kernels (k_retarget), for comparison
#endif
#ifndef RTG_L2_PREFETCH
#define RTG_L2_PREFETCH 0    // 1: each side wave pulls the input rows it reads late into L2 at kernel start
#endif

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
#ifndef RTG_PRELOAD_ARM
#define RTG_PRELOAD_ARM 1    // (measured -4 %) 1: a side's arm points load at kernel start, with the torso / wrist-fit loads
#endif
#ifndef RTG_PRELOAD_TIPS
#define RTG_PRELOAD_TIPS 0   // 1: the gripper's hand points load with the wrist-fit points
#endif

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

template <int KIND, bool PRECISE, bool SOA>
__global__ __launch_bounds__(256, RTG_SIDES_WAVES) void k_solve_sides(SolverConsts C, const float *__restrict__ in0,
                                                     const float *__restrict__ in1, const float *__restrict__ in2,
                                                     const float *__restrict__ in3, int64_t B,
                                                     float *__restrict__ dof, float *__restrict__ local_rot,
                                                     float *__restrict__ body_rot)
{
    __shared__ float sdof[kSideFrames * kDofStride];
    __shared__ float4 storso[kSideFrames];   // the tile's torso fit, handed from the left wave to the right one
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
    __shared__ float4 sarm[RTG_SIDES_REBALANCE ? kSideFrames : 1];   // the left arm chain, right wave -> left wave
    if (KIND == RTG_SOLVER_FULL_BODY_POS && RTG_SIDES_REBALANCE) {
        // Balanced FULL_BODY_POS: left wave = torso fit, then the left wrist fit, then the left Euler split /
        // gripper; right wave = the right wrist fit, then BOTH arm chains (each needs only R10), then the right
        // Euler split / gripper.  Two barriers hand R10 (left -> right) and the left chain (right -> left) over LDS.
        const auto b = view(in0, 63);
        Q R10 = qident(), W = qident();
        ArmPts apL{}, apR{};
        if (live) {
            if (!side) {
                R10 = fbp_torso(C, b);
                storso[r] = make_float4(R10.x, R10.y, R10.z, R10.w);
            } else {
                apL = load_arm<0>(b);
                apR = load_arm<1>(b);
                W = fbp_wrist_fit<1>(C, view(in2, 60));
            }
        }
        __syncthreads();
        Q chain = qident();
        if (live) {
            if (side) {
                const float4 t = storso[r];
                R10 = Q{t.x, t.y, t.z, t.w};
                const Q cl = fbp_arm<0>(C, apL, R10, E);
                sarm[r] = make_float4(cl.x, cl.y, cl.z, cl.w);
                chain = fbp_arm<1>(C, apR, R10, E);
            } else {
                emit_fixed_links(E);
                W = fbp_wrist_fit<0>(C, view(in1, 60));
            }
        }
        __syncthreads();
        if (live) {
            float *brow = body_rot ? body_rot + f * 236 : nullptr;
            if (side) {
                fbp_side_after_arm<PRECISE, 1>(C, load_tips(view(in2, 60)), R10, chain, W, E, brow);
            } else {
                const float4 c = sarm[r];
                fbp_side_after_arm<PRECISE, 0>(C, load_tips(view(in1, 60)), R10, Q{c.x, c.y, c.z, c.w}, W, E, brow);
            }
        }
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
        // leaves the right wave the heavier side program (two arm chains), so the left wave takes more slots; every
        // slot was written before the last barrier, whichever wave wrote it.
        constexpr int NL = (KIND == RTG_SOLVER_FULL_BODY_POS && RTG_SIDES_REBALANCE) ? RTG_SIDES_FIN_LEFT : 7;
        E.finalize(side ? NL : 0, side ? 14 - NL : NL);
    }
    __syncthreads();
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
#ifndef RTG_LATENCY_MAX_B
#define RTG_LATENCY_MAX_B 49152   // batches up to this size use the latency kernel (swept: faster up to 49152, slower at 65536)
#endif
constexpr int kLatFrames = 64;
#ifndef RTG_EXP_TIMESTAMPS
#define RTG_EXP_TIMESTAMPS 0   // measurement knob: block 0's lane 0 of each wave records the 100 MHz wall clock at
#endif                         // each phase into body_rot (as u32 pairs) -- wrong body_rot, tools/latency_phases.py

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
#ifndef RTG_LATENCY_WAVES
#define RTG_LATENCY_WAVES 5   // 5: k_fbp_latency5 (arm chain concurrent with the wrist fits); 3: k_fbp_latency
#endif
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
        fbp_latency5_tile<PRECISE, false>(C, in, in + 63, in + 123, 1, 0, dof, local_rot, body_rot);
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

// ----------------------------------------------------------------------------
// forward kinematics -- one frame per lane, joints in topological (index) order.
// The parent's global rotation / position is reused from registers when the
// parent is the previous joint (chains), else re-read from the output rows this
// lane has just written (branch points; L2-resident).  Topology is uniform
// across the grid, so the loop body and all topology loads are scalar.
// ----------------------------------------------------------------------------
template <bool STATE>
RTG_DEV void fk_frame(const TopoView &T, const float *__restrict__ lr, const float *__restrict__ rt,
                      float *__restrict__ gr, float *__restrict__ gp)
{
    Q g = ld4(lr);            // root: global = local (not normalised) kinematics.py:27-29
    V t = ld3(rt);
    st4(gr, g);
    st3(gp, t);
    for (int j = 1; j < T.J; ++j) {
        const int p = T.parents[j];
        if (p != j - 1) {
            g = ld4(gr + 4 * p);
            t = ld3(gp + 3 * p);
        }
        Q lq = ld4(lr + 4 * j);
        if (STATE) lq = qmul_norm(T.tree_quat[j], lq);   // skeleton3d.py:412-418
        const V zl = T.local_t[j];
        const V rot = qrotate(g, zl);
        const Q ng = qmul_norm(g, lq);
        const V nt = V{rot.x + t.x, rot.y + t.y, rot.z + t.z};
        st4(gr + 4 * j, ng);
        st3(gp + 3 * j, nt);
        g = ng;
        t = nt;
    }
}

template <bool STATE>
__global__ __launch_bounds__(256) void k_fk(TopoView T, const float *__restrict__ local_rot,
                                            const float *__restrict__ root_t, int64_t B, float *__restrict__ g_rot,
                                            float *__restrict__ g_pos)
{
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= B) return;
    fk_frame<STATE>(T, local_rot + f * T.J * 4, root_t + f * 3, g_rot + f * T.J * 4, g_pos + f * T.J * 3);
}

template <bool STATE>
__global__ __launch_bounds__(256) void k_local_rotation(TopoView T, const float *__restrict__ g_rot, int64_t B,
                                                        float *__restrict__ local_rot)
{
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= B) return;
    const float *g = g_rot + f * T.J * 4;
    float *l = local_rot + f * T.J * 4;
    st4(l, ld4(g));
    for (int j = 1; j < T.J; ++j) {
        const int p = T.parents[j];
        Q q = qmul_norm(qconj(ld4(g + 4 * p)), ld4(g + 4 * j));
        if (STATE) q = qmul_norm(qnormalize(qconj(T.tree_quat[j])), q);   // skeleton3d.py:477-481
        st4(l + 4 * j, q);
    }
}

// ----------------------------------------------------------------------------
// Streaming FK (the production path).  One wave = one tile of 64 consecutive
// frames, walked in chunks of kFkChunk joints:
//   1. the chunk's local rotations -- kFkChunk*16 contiguous bytes per frame --
//      are copied into an LDS window with dwordx4 loads (8 lanes per frame
//      row: 128-byte segments);
//   2. each lane composes its own frame's joints in index order, keeping the
//      previous joint's global transform in registers; a parent that is not
//      j-1 comes from an LDS slot (fk_schedule);
//   3. the window -- global rotations written over the locals in place, and
//      positions -- goes back out as 128- / 96-byte row segments.
// LDS per wave: 9.2 KiB rotation window (row pitch 9 float4: ds_read_b128
// conflict-free) + 6.4 KiB position window (odd pitch 25) + 1.8 KiB per slot,
// ~19 KiB for every shipped skeleton, i.e. 8 waves per CU whatever J is.
// ----------------------------------------------------------------------------
#ifndef RTG_FK_CHUNK
#define RTG_FK_CHUNK 8
#endif
constexpr int kFkTile = 64;
constexpr int kFkChunk = RTG_FK_CHUNK;   // joints per LDS window (4 or 8)
static_assert(kFkChunk == 4 || kFkChunk == 8, "window of 4 or 8 joints");
constexpr int kRotPitch = 4 * (kFkChunk + 1);   // floats per frame row (LDS)
constexpr int kPosPitch = 3 * kFkChunk + 1;

#ifndef RTG_FK_POS_REGS
#define RTG_FK_POS_REGS 1   // 1 (measured +3-4 %, bit-exact): positions held in registers and staged through the rotation window after it is
                            //    stored (no separate position window: 12.8 instead of 19.2 KiB per wave)
#endif
constexpr int kPosWin = RTG_FK_POS_REGS ? 0 : kFkTile * kPosPitch;   // floats of the separate position window

// Branch-parent slots: the first RTG_FK_REG_SLOTS live in registers (a slot is private to its lane, and its
// index is launch-uniform, so the choice is a scalar branch), the rest in LDS.  Every shipped skeleton needs <= 2
// slots, so their tiles use only the 9.2 KiB rotation window: 17 waves per CU instead of 12, and the 4096 tiles of
// a 262144-frame batch fit the 256 CUs in one round.
#ifndef RTG_FK_MIN_WAVES
#define RTG_FK_MIN_WAVES 0   // >0: min waves per SIMD asked of the streaming FK kernels (4: <= 128 VGPRs, 16 waves/CU)
#endif
#if RTG_FK_MIN_WAVES > 0
#define RTG_FK_WAVES __attribute__((amdgpu_waves_per_eu(RTG_FK_MIN_WAVES, 8)))
#else
#define RTG_FK_WAVES
#endif
#ifndef RTG_FK_ALIGNED_STORE
#define RTG_FK_ALIGNED_STORE 0   // 1: FK output rows leave as whole 64-byte sectors (chunk_store_aligned; measured 11-15 % slower); 0: per-window rows
#endif
#ifndef RTG_FK_REG_SLOTS
#define RTG_FK_REG_SLOTS (RTG_FK_ALIGNED_STORE ? 2 : 0)   // aligned stores need 8 KiB of carry LDS: slots move to VGPRs
#endif
#ifndef RTG_FK_NT_STORE
#define RTG_FK_NT_STORE 0   // 1: FK output rows leave with non-temporal stores (written once, never re-read here)
#endif
#ifndef RTG_DOF_FK_POS_REGS
#define RTG_DOF_FK_POS_REGS 1   // k_dof_fk positions staged through the rotation window (as RTG_FK_POS_REGS; measured +7-9 %)
#endif
constexpr int kCarryFloats = RTG_FK_ALIGNED_STORE ? 2 * kFkTile * 16 : 0;   // rotation + position carries
static inline size_t lds_slot_floats(int nslots)
{
    return nslots > RTG_FK_REG_SLOTS ? (size_t)(nslots - RTG_FK_REG_SLOTS) * 7 * kFkTile : 0;
}
static inline size_t fk_stream_lds_bytes(int nslots)
{
    return sizeof(float) * ((size_t)kFkTile * kRotPitch + (size_t)kPosWin + kCarryFloats + lds_slot_floats(nslots));
}
constexpr int kDofPosWin = RTG_DOF_FK_POS_REGS ? 0 : kFkTile * kPosPitch;
static inline size_t dof_fk_lds_bytes(int nslots)
{
    return sizeof(float) * ((size_t)kFkTile * kRotPitch + (size_t)kDofPosWin + kCarryFloats + lds_slot_floats(nslots));
}

// A streaming tile is one wave, so ordering its LDS traffic needs no block
// barrier: a wave's LDS instructions execute in issue order, and the
// wavefront-scope fence + wave_barrier only stop the compiler from moving
// memory operations across this point.  (__syncthreads would also make the
// compiler drain every outstanding global store, s_waitcnt vmcnt(0), per chunk.)
RTG_DEV void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Chunk [c0, c0+nC) of rows f0.. (nfr frames, J joints of W floats per row).
// Lane v of iteration `it` handles (frame (it*64+v) / kFkChunk, joint % kFkChunk):
// 8 lanes cover one frame's contiguous segment.
// eight named registers (an indexed array of them is left in scratch by the compiler)
struct ChunkRegs {
    Q v0, v1, v2, v3, v4, v5, v6, v7;
};
#define RTG_REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
RTG_DEV void chunk_load(ChunkRegs &r, const float *__restrict__ g, int64_t f0, int nfr, int J, int c0, int nC)
{
    // unconditional loads (lanes past the tile re-read the tile's first element)
    // keep the prefetch registers fully defined across the chunk loop
#define RTG_LD(I)                                                                          \
    if ((I) < kFkChunk) {                                                                  \
        const int v = (I) * kFkTile + (int)threadIdx.x;                                    \
        const int fr = v / kFkChunk, k = v % kFkChunk;                                     \
        const int64_t e = (fr < nfr && k < nC) ? (f0 + fr) * J + c0 + k : f0 * J;         \
        r.v##I = ld4(g + e * 4);                                                           \
    }
    RTG_REP8(RTG_LD)
#undef RTG_LD
}
RTG_DEV void chunk_to_lds(const ChunkRegs &r, float *lds, int nfr, int nC)
{
    const bool full = nfr == kFkTile && nC == kFkChunk;   // unpredicated: the writes issue back to back
#define RTG_ST(I)                                                                          \
    if ((I) < kFkChunk) {                                                                  \
        const int v = (I) * kFkTile + (int)threadIdx.x;                                    \
        const int fr = v / kFkChunk, k = v % kFkChunk;                                     \
        if (full || (fr < nfr && k < nC)) st4(lds + fr * kRotPitch + k * 4, r.v##I);       \
    }
    RTG_REP8(RTG_ST)
#undef RTG_ST
}
template <int W>
RTG_DEV void chunk_store(float *__restrict__ g, const float *lds, int pitch, int64_t f0, int nfr, int J, int c0, int nC)
{
    auto one = [&](int it) {
        const int v = it * kFkTile + (int)threadIdx.x;
        const int fr = v / kFkChunk, k = v % kFkChunk;
        float *gp = g + ((f0 + fr) * J + c0 + k) * W;
        const float *lp = lds + fr * pitch + k * W;
        if (W == 4) {
            if (RTG_FK_NT_STORE) {
                typedef float f4v __attribute__((ext_vector_type(4)));
                const f4v v = *reinterpret_cast<const f4v *>(lp);
                __builtin_nontemporal_store(v, reinterpret_cast<f4v *>(gp));
            } else {
                *reinterpret_cast<float4 *>(gp) = *reinterpret_cast<const float4 *>(lp);
            }
        } else {
#pragma unroll
            for (int c = 0; c < W; ++c) {
                if (RTG_FK_NT_STORE) __builtin_nontemporal_store(lp[c], gp + c);
                else gp[c] = lp[c];
            }
        }
    };
    if (nfr == kFkTile && nC == kFkChunk) {   // full window: unpredicated, LDS reads batch ahead of the stores
#pragma unroll
        for (int it = 0; it < kFkChunk; ++it) one(it);
    } else {
#pragma unroll
        for (int it = 0; it < kFkChunk; ++it) {
            const int v = it * kFkTile + (int)threadIdx.x;
            if (v / kFkChunk < nfr && v % kFkChunk < nC) one(it);
        }
    }
}

// Sector-aligned streaming store of one window (RTG_FK_ALIGNED_STORE).  A window's piece of a frame's output row is
// 96 or 128 bytes at a 16-byte-aligned, not 64-byte-aligned, offset (the row stride is J x 12 / 16 bytes), so the
// per-window store left two partly written 64-byte sectors per frame and window -- measured as 1.43x the
// algorithmic WRITE_SIZE on Hu FK.  Here only whole sectors are written (4 lanes x float4); the floats of a
// frame's last, incomplete sector wait in LDS (`carry`, 16 floats per frame) and go out with the next window.  Only
// the frame's first and last sector (shared with the neighbouring frames' rows) are written per dword.
// Tile-relative float x of frame fr lies in [fr S, fr S + S), S = W J; this window holds [a, b) = [fr S + W c0,
// fr S + W (c0 + nC)) at win[fr * pitch + (x - a)]; the carry holds [a - 16, a) at carry[fr * 16 + (x - a + 16)].
// Every store stays inside rows fr < nfr of this tile.
RTG_DEV int floor16(int x) { return x & ~15; }
RTG_DEV int ceil16(int x) { return (x + 15) & ~15; }
template <int W>
RTG_DEV void chunk_store_aligned(float *__restrict__ g, const float *win, int pitch, float *carry, int64_t f0, int nfr,
                                 int J, int c0, int nC)
{
    const int S = W * J;
    float *__restrict__ gt = g + f0 * S;   // 64 frames from a 64-frame boundary: 64-byte aligned
    const bool first = c0 == 0, last = c0 + nC == J;
    auto at = [&](int fr, int a, int x) { return x < a ? carry[fr * 16 + (x - a + 16)] : win[fr * pitch + (x - a)]; };
    // whole sectors: at most two per frame and window (W nC <= 32 floats plus a carry of <= 15)
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int v = it * kFkTile + (int)threadIdx.x;
        const int fr = v >> 3, q = (v >> 2) & 1, part = v & 3;
        if (fr < nfr) {
            const int A = fr * S, a = A + W * c0, b = a + W * nC;
            const int s0 = first ? ceil16(A) : floor16(a), s1 = last ? floor16(A + S) : floor16(b);
            const int x = s0 + 16 * q + 4 * part;
            if (s0 + 16 * q + 16 <= s1)
                *reinterpret_cast<float4 *>(gt + x) = make_float4(at(fr, a, x), at(fr, a, x + 1), at(fr, a, x + 2),
                                                                  at(fr, a, x + 3));
        }
    }
    const int fr = threadIdx.x;
    const int A = fr * S, a = A + W * c0, b = a + W * nC, E = A + S;
    if (fr < nfr && (first || last)) {   // the row's first and last sector, shared with the neighbouring rows
        const int h1 = ceil16(A) < E ? ceil16(A) : E;
        if (first)
            for (int x = A; x < h1; ++x) gt[x] = at(fr, a, x);
        if (last) {
            int t0 = floor16(E);
            const int lo = first ? h1 : floor16(a);
            t0 = t0 > lo ? t0 : lo;
            for (int x = t0; x < E; ++x) gt[x] = at(fr, a, x);
        }
    }
    wave_sync();   // every lane has read the old carry
    if (fr < nfr && !last)
        for (int x = floor16(b); x < b; ++x) carry[fr * 16 + (x - b + 16)] = win[fr * pitch + (x - a)];
}

// slot s < RTG_FK_REG_SLOTS: registers (named members: an indexed array would be left in scratch); else LDS
// [s - RTG_FK_REG_SLOTS][7][64].  s is launch-uniform (SGPR), so the selection is a scalar branch.
struct Slots {
    float *lds;
    Q q0, q1;
    V t0, t1;
};
RTG_DEV void slot_put(Slots &S, int s, Q q, V t)
{
    if (RTG_FK_REG_SLOTS > 0 && s == 0) { S.q0 = q; S.t0 = t; return; }
    if (RTG_FK_REG_SLOTS > 1 && s == 1) { S.q1 = q; S.t1 = t; return; }
    float *p = S.lds + (s - RTG_FK_REG_SLOTS) * 7 * kFkTile + threadIdx.x;
    p[0] = q.x; p[kFkTile] = q.y; p[2 * kFkTile] = q.z; p[3 * kFkTile] = q.w;
    p[4 * kFkTile] = t.x; p[5 * kFkTile] = t.y; p[6 * kFkTile] = t.z;
}
RTG_DEV void slot_get(const Slots &S, int s, Q &q, V &t)
{
    if (RTG_FK_REG_SLOTS > 0 && s == 0) { q = S.q0; t = S.t0; return; }
    if (RTG_FK_REG_SLOTS > 1 && s == 1) { q = S.q1; t = S.t1; return; }
    const float *p = S.lds + (s - RTG_FK_REG_SLOTS) * 7 * kFkTile + threadIdx.x;
    q = Q{p[0], p[kFkTile], p[2 * kFkTile], p[3 * kFkTile]};
    t = V{p[4 * kFkTile], p[5 * kFkTile], p[6 * kFkTile]};
}
static_assert(RTG_FK_REG_SLOTS >= 0 && RTG_FK_REG_SLOTS <= 2, "0..2 register slots");

template <bool STATE>
RTG_DEV void fk_stream_tile(const TopoView &T, const float *__restrict__ local_rot, const float *__restrict__ root_t,
                            int64_t B, int64_t f0, float *__restrict__ g_rot, float *__restrict__ g_pos, float *lds)
{
    const int J = T.J;
    const int nfr = (int)((B - f0) < kFkTile ? (B - f0) : kFkTile);
    float *rot = lds;                                   // [64][kRotPitch]
    float *pos = lds + kFkTile * kRotPitch;             // [64][kPosPitch] (RTG_FK_POS_REGS: none)
    float *carry = pos + kPosWin;                       // [2][64][16] (RTG_FK_ALIGNED_STORE)
    Slots slots{carry + kCarryFloats, qident(), qident(), V{0.0f, 0.0f, 0.0f}, V{0.0f, 0.0f, 0.0f}};
    const int lane = threadIdx.x;
    const bool active = lane < nfr;
    Q g = qident();
    V t = V{0.0f, 0.0f, 0.0f};
    V pk[kFkChunk];   // RTG_FK_POS_REGS: the window's positions (constant indices: registers)
    const V root = ld3(root_t + (f0 + (active ? lane : 0)) * 3);   // before the prefetches (vmcnt order)
    ChunkRegs next;
    chunk_load(next, local_rot, f0, nfr, J, 0, J < kFkChunk ? J : kFkChunk);
    for (int c0 = 0; c0 < J; c0 += kFkChunk) {
        const int nC = (J - c0) < kFkChunk ? (J - c0) : kFkChunk;
        chunk_to_lds(next, rot, nfr, nC);
        wave_sync();
        if (c0 + kFkChunk < J)   // prefetch the next window while this one is composed
            chunk_load(next, local_rot, f0, nfr, J, c0 + kFkChunk,
                       (J - c0 - kFkChunk) < kFkChunk ? (J - c0 - kFkChunk) : kFkChunk);
        if (active) {
            float *R = rot + lane * kRotPitch;
            float *P = pos + lane * kPosPitch;
            // unrolled: the window's LDS reads and the topology's scalar loads are
            // issued together at the chunk head instead of once per chained joint
#pragma unroll
            for (int k = 0; k < kFkChunk; ++k) {
                if (k >= nC) break;
                const int j = c0 + k;
                const int32_t sc = ld_const(T.sched + j);
                Q lq = Q{R[4 * k], R[4 * k + 1], R[4 * k + 2], R[4 * k + 3]};
                Q ng;
                V nt;
                if (j == 0) {   // root: global = local, unnormalised (kinematics.py:27-29)
                    ng = lq;
                    nt = root;
                } else {
                    if ((sc & 0xFF) != kNoSlot) slot_get(slots, sc & 0xFF, g, t);
                    if (STATE) lq = qmul_norm(ld_const(T.tree_quat + j), lq);   // skeleton3d.py:412-418
                    const V rv = qrotate(g, ld_const(T.local_t + j));
                    ng = qmul_norm(g, lq);
                    nt = V{rv.x + t.x, rv.y + t.y, rv.z + t.z};
                }
                R[4 * k] = ng.x; R[4 * k + 1] = ng.y; R[4 * k + 2] = ng.z; R[4 * k + 3] = ng.w;
                if (RTG_FK_POS_REGS) pk[k] = nt;
                else { P[3 * k] = nt.x; P[3 * k + 1] = nt.y; P[3 * k + 2] = nt.z; }
                if (((sc >> 8) & 0xFF) != kNoSlot) slot_put(slots, (sc >> 8) & 0xFF, ng, nt);
                g = ng;
                t = nt;
            }
        }
        wave_sync();
        if (RTG_FK_ALIGNED_STORE) chunk_store_aligned<4>(g_rot, rot, kRotPitch, carry, f0, nfr, J, c0, nC);
        else chunk_store<4>(g_rot, rot, kRotPitch, f0, nfr, J, c0, nC);
        if (RTG_FK_POS_REGS) {   // the rotation rows are out: reuse the window for the positions
            wave_sync();
            if (active) {
                float *P = rot + lane * kRotPitch;
#pragma unroll
                for (int k = 0; k < kFkChunk; ++k)
                    if (k < nC) { P[3 * k] = pk[k].x; P[3 * k + 1] = pk[k].y; P[3 * k + 2] = pk[k].z; }
            }
            wave_sync();
            if (RTG_FK_ALIGNED_STORE)
                chunk_store_aligned<3>(g_pos, rot, kRotPitch, carry + kFkTile * 16, f0, nfr, J, c0, nC);
            else chunk_store<3>(g_pos, rot, kRotPitch, f0, nfr, J, c0, nC);
        } else {
            chunk_store<3>(g_pos, pos, kPosPitch, f0, nfr, J, c0, nC);
        }
        wave_sync();
    }
}

template <bool STATE>
__global__ __launch_bounds__(kFkTile) RTG_FK_WAVES void k_fk_stream(TopoView T, const float *__restrict__ local_rot,
                                                       const float *__restrict__ root_t, int64_t B,
                                                       float *__restrict__ g_rot, float *__restrict__ g_pos)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    fk_stream_tile<STATE>(T, local_rot, root_t, B, (int64_t)blockIdx.x * kFkTile, g_rot, g_pos, fk_lds);
}

// inverse FK, streamed the same way: local[j] = normalise(conj(g[p]) * g[j]) (kinematics.py:41-63).
// The previous joint's global rotation stays in registers; branch parents come from slots.
template <bool STATE>
RTG_DEV void local_rotation_tile(const TopoView &T, const float *__restrict__ g_rot, int64_t B, int64_t f0,
                                 float *__restrict__ local_rot, float *fk_lds)
{
    const int J = T.J;
    const int nfr = (int)((B - f0) < kFkTile ? (B - f0) : kFkTile);
    float *win = fk_lds;                                 // [64][kRotPitch]
    float *carry = fk_lds + kFkTile * kRotPitch + kPosWin;
    Slots slots{carry + kCarryFloats, qident(), qident(), V{0.0f, 0.0f, 0.0f},
                V{0.0f, 0.0f, 0.0f}};   // the same LDS slot offset as fk_stream_tile
    const int lane = threadIdx.x;
    Q prev = qident();
    V unused = V{0.0f, 0.0f, 0.0f};
    ChunkRegs next;
    chunk_load(next, g_rot, f0, nfr, J, 0, J < kFkChunk ? J : kFkChunk);
    for (int c0 = 0; c0 < J; c0 += kFkChunk) {
        const int nC = (J - c0) < kFkChunk ? (J - c0) : kFkChunk;
        chunk_to_lds(next, win, nfr, nC);
        wave_sync();
        if (c0 + kFkChunk < J)
            chunk_load(next, g_rot, f0, nfr, J, c0 + kFkChunk,
                       (J - c0 - kFkChunk) < kFkChunk ? (J - c0 - kFkChunk) : kFkChunk);
        if (lane < nfr) {
            float *W = win + lane * kRotPitch;
#pragma unroll
            for (int k = 0; k < kFkChunk; ++k) {
                if (k >= nC) break;
                const int j = c0 + k;
                const int32_t sc = ld_const(T.sched + j);
                const Q gj = Q{W[4 * k], W[4 * k + 1], W[4 * k + 2], W[4 * k + 3]};
                Q q = gj;   // root copied (kinematics.py:49)
                if (j > 0) {
                    Q gp = prev;
                    if ((sc & 0xFF) != kNoSlot) slot_get(slots, sc & 0xFF, gp, unused);
                    q = qmul_norm(qconj(gp), gj);
                    if (STATE) q = qmul_norm(qnormalize(qconj(ld_const(T.tree_quat + j))), q);   // skeleton3d.py:470-478
                }
                if (((sc >> 8) & 0xFF) != kNoSlot) slot_put(slots, (sc >> 8) & 0xFF, gj, unused);
                W[4 * k] = q.x; W[4 * k + 1] = q.y; W[4 * k + 2] = q.z; W[4 * k + 3] = q.w;
                prev = gj;
            }
        }
        wave_sync();
        if (RTG_FK_ALIGNED_STORE) chunk_store_aligned<4>(local_rot, win, kRotPitch, carry, f0, nfr, J, c0, nC);
        else chunk_store<4>(local_rot, win, kRotPitch, f0, nfr, J, c0, nC);
        wave_sync();
    }
}

template <bool STATE>
__global__ __launch_bounds__(kFkTile) RTG_FK_WAVES void k_local_rotation_stream(TopoView T, const float *__restrict__ g_rot,
                                                                   int64_t B, float *__restrict__ local_rot)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    local_rotation_tile<STATE>(T, g_rot, B, (int64_t)blockIdx.x * kFkTile, local_rot, fk_lds);
}

// Mixed-target kinematics (BASELINE config 5): every 64-frame tile of every segment is one wave; a segment is FK
// (op 0) or inverse FK (op 1), so FK and inverse FK of several skeletons share one launch.
__global__ __launch_bounds__(kFkTile) RTG_FK_WAVES void k_fk_multi_stream(FkMultiArgs A)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    int s = 0;
#pragma unroll
    for (int i = 1; i < RTG_MAX_SEGMENTS; ++i)
        if (i < A.n && (int64_t)blockIdx.x >= A.block_start[i]) s = i;
    const FkSeg &S = A.seg[s];
    const int64_t f0 = ((int64_t)blockIdx.x - A.block_start[s]) * kFkTile;
    if (S.op == 0) fk_stream_tile<false>(S.T, S.local_rot, S.root_t, S.B, f0, S.g_rot, S.g_pos, fk_lds);
    else local_rotation_tile<false>(S.T, S.local_rot, S.B, f0, S.g_rot, fk_lds);
}

// Joint-angle FK (HuForwardModel.forward_kinematics, hu_forward_model.py:17-33): the streaming tile of
// k_fk_stream, but joint j's local rotation is built in-lane from its DOF --
// quat_from_angle_axis(a', e_axis) with a' = (clamp(a) - a) + a when clipping -- so no (B,J,4) local-rotation
// tensor ever exists in HBM.  Each lane's next window of 8 angles is prefetched during the current window.
struct DofRegs {
    float a0, a1, a2, a3, a4, a5, a6, a7;
};
RTG_DEV void dof_load(DofRegs &r, const float *__restrict__ row, int J, int c0)
{
    // angles of joints c0..c0+7 are dof[c0-1 .. c0+6]; indices are clamped into the row (unused ones are dropped)
    auto at = [&](int k) {
        int i = c0 + k - 1;
        i = i < 0 ? 0 : (i > J - 2 ? J - 2 : i);
        return row[i];
    };
    r.a0 = at(0); r.a1 = at(1); r.a2 = at(2); r.a3 = at(3); r.a4 = at(4); r.a5 = at(5); r.a6 = at(6); r.a7 = at(7);
}
RTG_DEV float dof_get(const DofRegs &r, int k)
{
    return k == 0 ? r.a0 : k == 1 ? r.a1 : k == 2 ? r.a2 : k == 3 ? r.a3 : k == 4 ? r.a4 : k == 5 ? r.a5
                                                                                           : k == 6 ? r.a6 : r.a7;
}

template <bool CLIP>
__global__ __launch_bounds__(kFkTile) RTG_FK_WAVES void k_dof_fk(TopoView T, DofView D, const float *__restrict__ dof,
                                                    const float *__restrict__ root_rot,
                                                    const float *__restrict__ root_t, int64_t B,
                                                    float *__restrict__ g_rot, float *__restrict__ g_pos)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    const int J = T.J;
    const int64_t f0 = (int64_t)blockIdx.x * kFkTile;
    const int nfr = (int)((B - f0) < kFkTile ? (B - f0) : kFkTile);
    float *rot = fk_lds;
    float *pos = fk_lds + kFkTile * kRotPitch;   // [64][kPosPitch] (RTG_DOF_FK_POS_REGS: none)
    float *carry = pos + kDofPosWin;
    Slots slots{carry + kCarryFloats, qident(), qident(), V{0.0f, 0.0f, 0.0f}, V{0.0f, 0.0f, 0.0f}};
    V pk[kFkChunk];   // RTG_DOF_FK_POS_REGS: the window's positions
    const int lane = threadIdx.x;
    const bool active = lane < nfr;
    const int64_t f = f0 + (active ? lane : 0);
    const float *drow = dof + f * (J - 1);
    const Q rroot = ld4(root_rot + f * 4);
    const V troot = ld3(root_t + f * 3);
    DofRegs cur, next;
    if (J > 1) dof_load(next, drow, J, 0);
    Q g = qident();
    V t = V{0.0f, 0.0f, 0.0f};
    for (int c0 = 0; c0 < J; c0 += kFkChunk) {
        const int nC = (J - c0) < kFkChunk ? (J - c0) : kFkChunk;
        cur = next;
        if (c0 + kFkChunk < J) dof_load(next, drow, J, c0 + kFkChunk);
        if (active) {
            float *R = rot + lane * kRotPitch;
            float *P = pos + lane * kPosPitch;
#pragma unroll
            for (int k = 0; k < kFkChunk; ++k) {
                if (k >= nC) break;
                const int j = c0 + k;
                const int32_t sc = ld_const(T.sched + j);
                Q ng;
                V nt;
                if (j == 0) {   // root: global = local = the root rotation, unnormalised (:24, kinematics.py:27-29)
                    ng = rroot;
                    nt = troot;
                } else {
                    float a = dof_get(cur, k);
                    if (CLIP) {   // torch.clamp (min then max; NaN passes), then the straight-through sum
                        const float lo = ld_const(D.lower + (j - 1)), hi = ld_const(D.upper + (j - 1));
                        float c = a < lo ? lo : a;
                        c = c > hi ? hi : c;
                        a = (c - a) + a;
                    }
                    const int ax = ld_const(D.axis + (j - 1));
                    const Q lq = qfrom_angle_axis(a, V{ax == 0 ? 1.0f : 0.0f, ax == 1 ? 1.0f : 0.0f,
                                                       ax == 2 ? 1.0f : 0.0f});
                    if ((sc & 0xFF) != kNoSlot) slot_get(slots, sc & 0xFF, g, t);
                    const V rv = qrotate(g, ld_const(T.local_t + j));
                    ng = qmul_norm(g, lq);
                    nt = V{rv.x + t.x, rv.y + t.y, rv.z + t.z};
                }
                R[4 * k] = ng.x; R[4 * k + 1] = ng.y; R[4 * k + 2] = ng.z; R[4 * k + 3] = ng.w;
                if (RTG_DOF_FK_POS_REGS) pk[k] = nt;
                else { P[3 * k] = nt.x; P[3 * k + 1] = nt.y; P[3 * k + 2] = nt.z; }
                if (((sc >> 8) & 0xFF) != kNoSlot) slot_put(slots, (sc >> 8) & 0xFF, ng, nt);
                g = ng;
                t = nt;
            }
        }
        wave_sync();
        if (RTG_FK_ALIGNED_STORE) chunk_store_aligned<4>(g_rot, rot, kRotPitch, carry, f0, nfr, J, c0, nC);
        else chunk_store<4>(g_rot, rot, kRotPitch, f0, nfr, J, c0, nC);
        if (RTG_DOF_FK_POS_REGS) {   // the rotation rows are out: reuse the window for the positions
            wave_sync();
            if (active) {
                float *P = rot + lane * kRotPitch;
#pragma unroll
                for (int k = 0; k < kFkChunk; ++k)
                    if (k < nC) { P[3 * k] = pk[k].x; P[3 * k + 1] = pk[k].y; P[3 * k + 2] = pk[k].z; }
            }
            wave_sync();
            if (RTG_FK_ALIGNED_STORE)
                chunk_store_aligned<3>(g_pos, rot, kRotPitch, carry + kFkTile * 16, f0, nfr, J, c0, nC);
            else chunk_store<3>(g_pos, rot, kRotPitch, f0, nfr, J, c0, nC);
        } else {
            chunk_store<3>(g_pos, pos, kPosPitch, f0, nfr, J, c0, nC);
        }
        wave_sync();
    }
}

// ----------------------------------------------------------------------------
// retarget/main.py motion-level prep, one frame per lane.
// ----------------------------------------------------------------------------
struct Dir3 {
    float x, y, z;
    int32_t on;
};

// Retarget.rescale_motion_to_standard_size (main.py:37-47) after coord_transform(dir) (:170).  A bone's parent
// end is the parent's RESCALED position: re-read from this lane's own output row (program order).
__global__ __launch_bounds__(256) void k_rescale_motion(TopoView T, const float *__restrict__ motion, int64_t B,
                                                        Dir3 dir, float *__restrict__ out)
{
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= B) return;
    const int J = T.J;
    const float *m = motion + f * J * 3;
    float *o = out + f * J * 3;
    auto mp = [&](int j) {
        const V v = ld3(m + 3 * j);
        return dir.on ? V{v.x * dir.x, v.y * dir.y, v.z * dir.z} : v;
    };
    for (int j = 0; j < J; ++j) {
        const int p = ld_const(T.parents + j);
        const V mj = mp(j);
        if (p < 0) {
            st3(o + 3 * j, mj);
            continue;
        }
        const V d = vsub(mj, mp(p));
        const float scale = lnorm3(d) / lnorm3(ld_const(T.local_t + j));
        const V q = vdiv(d, scale);
        const V op = ld3(o + 3 * p);
        st3(o + 3 * j, V{op.x + q.x, op.y + q.y, op.z + q.z});
    }
}

// torch.max over a batch of norms: every norm is >= 0 or NaN, so the float bits order as ints once NaN is
// pinned to the largest pattern.  Wave-reduced, then one atomic per wave.
RTG_DEV int32_t max_key(float v) { return v != v ? 0x7fffffff : __float_as_int(v); }
RTG_DEV int32_t wave_max(int32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int32_t w = __shfl_xor(v, o, 64);
        v = w > v ? w : v;
    }
    return v;
}
RTG_DEV bool batch_small(const float *ws, int i)   // (max norm) <= 1e-6, false for NaN
{
    const int32_t k = reinterpret_cast<const int32_t *>(ws)[i];
    return k != 0x7fffffff && __int_as_float(k) <= 1e-6f;
}

// quat_between_two_vecs (transform3d.py:8-21) for one pair; `ident`: the batch-level branch of :11-12
RTG_DEV Q quat_between(V v1, V v2, bool ident)
{
    if (ident) return qident();
    v1 = vdiv(v1, lnorm3(v1));
    v2 = vdiv(v2, lnorm3(v2));
    const V c = cross3(v1, v2);
    return qnormalize(Q{c.x, c.y, c.z, 1.0f + dot3(v1, v2)});   // torch.sum(v1*v2): left fold (measured)
}

__global__ __launch_bounds__(256) void k_qbtv_norm_max(const float *__restrict__ v1, const float *__restrict__ v2,
                                                       int64_t n, float *ws)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int32_t a = 0, b = 0;
    if (i < n) {
        a = max_key(lnorm3(ld3(v1 + 3 * i)));   // torch.norm(dim=-1): the fma form (measured)
        b = max_key(lnorm3(ld3(v2 + 3 * i)));
    }
    a = wave_max(a);
    b = wave_max(b);
    if ((threadIdx.x & 63) == 0) {
        atomicMax(reinterpret_cast<int32_t *>(ws), a);
        atomicMax(reinterpret_cast<int32_t *>(ws) + 1, b);
    }
}

__global__ __launch_bounds__(256) void k_quat_between(const float *__restrict__ v1, const float *__restrict__ v2,
                                                      int64_t n, const float *ws, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const bool ident = batch_small(ws, 0) || batch_small(ws, 1);
    st4(out + 4 * i, quat_between(ld3(v1 + 3 * i), ld3(v2 + 3 * i), ident));
}

// _rebuild_with_vtrdyn_zero_pose (main.py:116-165): pass 1, per child joint j the batch max of |m_j - m_p|
__global__ __launch_bounds__(256) void k_rebuild_norm_max(TopoView T, const float *__restrict__ motion, int64_t B,
                                                          float *ws)
{
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int J = T.J;
    const float *m = motion + (f < B ? f : 0) * J * 3;
    for (int j = 1; j < J; ++j) {
        const int p = ld_const(T.parents + j);
        if (p == 0 || p == 10) continue;
        int32_t k = f < B ? max_key(lnorm3(vsub(ld3(m + 3 * j), ld3(m + 3 * p)))) : 0;
        k = wave_max(k);
        if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<int32_t *>(ws) + j, k);
    }
}

// pass 2: rows 0 and 10 from the Kabsch fits (:126-136); every other row r takes quat_between_two_vecs of its
// LAST child c (the loop :144-152 overwrites row r once per child, in index order), or stays identity; then
// SkeletonState.from_rotation_and_root_translation normalises every row (skeleton3d.py:610).
__global__ __launch_bounds__(256) void k_rebuild_vtrdyn(TopoView T, const float *__restrict__ motion, int64_t B,
                                                        const float *ws, float *__restrict__ g_rot,
                                                        float *__restrict__ root_t)
{
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= B) return;
    const int J = T.J;
    const float *m = motion + f * J * 3;
    float *gr = g_rot + f * J * 4;
    auto zl = [&](int j) { return ld_const(T.local_t + j); };
    const V m0 = ld3(m), m10 = ld3(m + 30);
    {
        const V Z[3] = {zl(4), zl(1), zl(7)};
        const V M[3] = {vsub(ld3(m + 12), m0), vsub(ld3(m + 3), m0), vsub(ld3(m + 21), m0)};
        st4(gr, qnormalize(cal_joint_quat<3>(Z, M)));
    }
    {
        const V Z[3] = {zl(17), zl(13), zl(11)};
        const V M[3] = {vsub(ld3(m + 51), m10), vsub(ld3(m + 39), m10), vsub(ld3(m + 33), m10)};
        st4(gr + 40, qnormalize(cal_joint_quat<3>(Z, M)));
    }
    for (int r = 1; r < J; ++r) {
        if (r == 10) continue;
        int c = -1;   // uniform scalar search: last child of r
        for (int k = r + 1; k < J; ++k)
            if (ld_const(T.parents + k) == r) c = k;
        Q q = qident();
        if (c > 0)   // batch condition: max |vec1| = |zl_c| (one vector repeated), max |vec2| from pass 1
            q = quat_between(zl(c), vsub(ld3(m + 3 * c), ld3(m + 3 * r)), lnorm3(zl(c)) <= 1e-6f || batch_small(ws, c));
        st4(gr + 4 * r, qnormalize(q));
    }
    st3(root_t + f * 3, m0);
}

// ----------------------------------------------------------------------------
// VTRDyn ingest: sim_full_body_teleop.py:109 (body 23 -> 21), :111-112 (hand order), :92 (skip all-zero frames)
// ----------------------------------------------------------------------------
__constant__ int8_t c_body23_to_21[21] = {0, 1, 2, 3, 5, 6, 7, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22};
__constant__ int8_t c_hand_order[20] = {0, 4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 12, 13, 14, 15, 1, 2, 3};

// element (frame f, point j, component c) of a (B, P, C) batch in the given layout (rtg.h rtg_layout)
RTG_DEV int64_t lay_idx(bool soa, int64_t f, int j, int c, int P, int C, int64_t B)
{
    return soa ? ((int64_t)(j * C + c)) * B + f : f * (P * C) + C * j + c;
}

__global__ __launch_bounds__(256) void k_ingest_vtrdyn(const float *__restrict__ bp, const float *__restrict__ lhp,
                                                       const float *__restrict__ rhp, int64_t B,
                                                       float *__restrict__ body, float *__restrict__ lh,
                                                       float *__restrict__ rh, uint8_t *__restrict__ valid, bool soa)
{
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= B) return;
    const float *b = bp + f * 69;
    bool close = true;   // np.allclose(body_pos, 0): |x| <= 1e-8 everywhere (a NaN is never close)
    for (int i = 0; i < 69; ++i) close = close && (fabsf(b[i]) <= 1e-8f);
    valid[f] = close ? 0 : 1;
    if (!soa) {
        for (int j = 0; j < 21; ++j) st3(body + f * 63 + 3 * j, ld3(b + 3 * c_body23_to_21[j]));
        for (int j = 0; j < 20; ++j) {
            st3(lh + f * 60 + 3 * j, ld3(lhp + f * 60 + 3 * c_hand_order[j]));
            st3(rh + f * 60 + 3 * j, ld3(rhp + f * 60 + 3 * c_hand_order[j]));
        }
        return;
    }
    for (int j = 0; j < 21; ++j)   // SoA planes: each store instruction writes 256 contiguous bytes per wave
        for (int c = 0; c < 3; ++c) body[lay_idx(true, f, j, c, 21, 3, B)] = b[3 * c_body23_to_21[j] + c];
    for (int j = 0; j < 20; ++j)
        for (int c = 0; c < 3; ++c) {
            lh[lay_idx(true, f, j, c, 20, 3, B)] = lhp[f * 60 + 3 * c_hand_order[j] + c];
            rh[lay_idx(true, f, j, c, 20, 3, B)] = rhp[f * 60 + 3 * c_hand_order[j] + c];
        }
}

int32_t fk_schedule(const int32_t *parents, int32_t J, int32_t *sched)
{
    // last non-consecutive child of every branch parent
    int32_t *last = new int32_t[J];
    int32_t *slot_of = new int32_t[J];
    for (int j = 0; j < J; ++j) last[j] = slot_of[j] = -1;
    for (int k = 1; k < J; ++k)
        if (parents[k] != k - 1) last[parents[k]] = k;
    uint32_t used = 0;   // bitmask of live slots (the schedule is only used when nslots <= kMaxFkSlots)
    int32_t nslots = 0, overflow = 0;
    for (int j = 0; j < J; ++j) {
        int32_t ld = kNoSlot, sv = kNoSlot;
        const int p = j > 0 ? parents[j] : -1;
        if (j > 0 && p != j - 1) {
            ld = slot_of[p];
            if (last[p] == j && ld >= 0 && ld < 32) used &= ~(1u << ld);   // free after this read
        }
        if (last[j] >= 0) {
            int s = 0;
            while (s < 32 && (used >> s) & 1u) ++s;
            if (s >= 32) { overflow = 1; s = 31; }
            used |= 1u << s;
            slot_of[j] = s;
            sv = s;
            nslots = s + 1 > nslots ? s + 1 : nslots;
        }
        sched[j] = (ld & 0xFF) | ((sv & 0xFF) << 8);
    }
    delete[] last;
    delete[] slot_of;
    return overflow ? 1 << 30 : nslots;
}

__global__ __launch_bounds__(256) void k_fk_multi(FkMultiArgs A)
{
    int s = 0;
#pragma unroll
    for (int i = 1; i < RTG_MAX_SEGMENTS; ++i)
        if (i < A.n && (int64_t)blockIdx.x >= A.block_start[i]) s = i;
    const FkSeg &S = A.seg[s];
    const int64_t f = ((int64_t)blockIdx.x - A.block_start[s]) * blockDim.x + threadIdx.x;
    if (f >= S.B) return;
    if (S.op == 0) {
        fk_frame<false>(S.T, S.local_rot + f * S.T.J * 4, S.root_t + f * 3, S.g_rot + f * S.T.J * 4,
                        S.g_pos + f * S.T.J * 3);
        return;
    }
    const float *g = S.local_rot + f * S.T.J * 4;   // inverse FK, kinematics.py:41-63
    float *l = S.g_rot + f * S.T.J * 4;
    st4(l, ld4(g));
    for (int j = 1; j < S.T.J; ++j) st4(l + 4 * j, qmul_norm(qconj(ld4(g + 4 * S.T.parents[j])), ld4(g + 4 * j)));
}

// ----------------------------------------------------------------------------
// elementwise primitives
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_quat_op(int op, const float *__restrict__ a, const float *__restrict__ b,
                                                 const float *__restrict__ c, int64_t n, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    switch (op) {
    case RTG_OP_QUAT_MUL: st4(out + 4 * i, qmul(ld4(a + 4 * i), ld4(b + 4 * i))); break;
    case RTG_OP_QUAT_MUL_NORM: st4(out + 4 * i, qmul_norm(ld4(a + 4 * i), ld4(b + 4 * i))); break;
    case RTG_OP_QUAT_NORMALIZE: st4(out + 4 * i, qnormalize(ld4(a + 4 * i))); break;
    case RTG_OP_QUAT_ROTATE: st3(out + 3 * i, qrotate(ld4(a + 4 * i), ld3(b + 3 * i))); break;
    case RTG_OP_QUAT_INVERSE: st4(out + 4 * i, qconj(ld4(a + 4 * i))); break;
    case RTG_OP_QUAT_FROM_ANGLE_AXIS: st4(out + 4 * i, qfrom_angle_axis(a[i], ld3(b + 3 * i))); break;
    case RTG_OP_QUAT_FROM_ROTMAT: {
        float m[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) m[k] = a[9 * i + k];
        st4(out + 4 * i, qfrom_rotmat(m));
        break;
    }
    case RTG_OP_QUAT_TO_EXP_MAP: st3(out + 3 * i, qexp_map(ld4(a + 4 * i))); break;
    case RTG_OP_RADIANS_BETWEEN: out[i] = radians_between(ld3(a + 3 * i), ld3(b + 3 * i), ld3(c + 3 * i)); break;
    case RTG_OP_PROJ_IN_PLANE: st3(out + 3 * i, proj_in_plane(ld3(a + 3 * i), ld3(b + 3 * i))); break;
    case RTG_OP_QUAT_TO_DOF_POS: {
        const float *q = a + i * 124 + 4;   // local_rot[1:]
#pragma unroll
        for (int k = 0; k < 30; ++k) out[i * 30 + k] = qexp_component(ld4(q + 4 * k), hu_dof_axis(k));
        break;
    }
    case RTG_OP_SHOULDER_PR: {
        Q p, r;
        const V v0 = ld3(b + 3 * i);
        shoulder_pr(ld3(a + 3 * i), shoulder_zero(v0), ld4(c + 4 * i), p, r);
        st4(out + 8 * i, p);
        st4(out + 8 * i + 4, r);
        break;
    }
    case RTG_OP_ELBOW_PY: {
        Q y, e;
        const V v0 = ld3(b + 3 * i);
        elbow_py(ld3(a + 3 * i), elbow_zero(v0), ld4(c + 4 * i), y, e);
        st4(out + 8 * i, y);
        st4(out + 8 * i + 4, e);
        break;
    }
    case RTG_OP_QUAT_TO_ANGLE_AXIS: st4(out + 4 * i, qangle_axis(ld4(a + 4 * i))); break;
    case RTG_OP_NORMALIZE_ANGLE: out[i] = normalize_angle(a[i]); break;
    case RTG_OP_QUAT_ABS: out[i] = qabs(ld4(a + 4 * i)); break;
    case RTG_OP_QUAT_UNIT: st4(out + 4 * i, qunit(ld4(a + 4 * i))); break;
    case RTG_OP_QUAT_ANGLE_AXIS: st4(out + 4 * i, qangle_axis_abs(ld4(a + 4 * i))); break;
    default: break;
    }
}

template <int N>
__global__ __launch_bounds__(256) void k_cal_joint_quat(const float *__restrict__ Z, const float *__restrict__ M,
                                                        int64_t n, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    V z[N], m[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        z[j] = ld3(Z + (i * N + j) * 3);
        m[j] = ld3(M + (i * N + j) * 3);
    }
    st4(out + 4 * i, cal_joint_quat<N>(z, m));
}

__global__ __launch_bounds__(256) void k_quat_in_xyz_axis(const float *__restrict__ q, int s0, int s1, int s2,
                                                          int extrinsic, int64_t n, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Q e[3];
    quat_in_xyz_axis(ld4(q + 4 * i), s0, s1, s2, extrinsic != 0, e);
#pragma unroll
    for (int t = 0; t < 3; ++t) st4(out + (i * 3 + t) * 4, e[t]);
}

// ----------------------------------------------------------------------------
// motion velocities: thread per (sequence, frame, channel), channel fastest
// (coalesced over the J*C channels of a frame).
// ----------------------------------------------------------------------------
// np.gradient along frames (edge_order 1, unit spacing) then / dt, all float32
__global__ __launch_bounds__(256) void k_gradient_dt(const float *__restrict__ p, int64_t nseq, int64_t L, int64_t S,
                                                     float dt, float *__restrict__ v)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nseq * L * S) return;
    const int64_t s = i % S, t = (i / S) % L, base = i - s - t * S;
    float g;
    if (L == 1) g = 0.0f;   // numpy raises for < 2 frames; rtg_* rejects L < 2 before launch
    else if (t == 0) g = (p[base + S + s] - p[base + s]) / 1.0f;
    else if (t == L - 1) g = (p[base + t * S + s] - p[base + (t - 1) * S + s]) / 1.0f;
    else g = (p[base + (t + 1) * S + s] - p[base + (t - 1) * S + s]) / 2.0f;
    v[i] = g / dt;
}

// quat_mul_norm(r[t+1], quat_inverse(r[t])) -> quat_angle_axis -> axis * angle / dt (last frame: identity -> 0)
__global__ __launch_bounds__(256) void k_angular_raw(const float *__restrict__ r, int64_t nseq, int64_t L, int64_t J,
                                                     float dt, float *__restrict__ v)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nseq * L * J) return;
    const int64_t t = (i / J) % L;
    Q d = qident();
    if (t < L - 1) d = qmul_norm(ld4(r + 4 * (i + J)), qconj(ld4(r + 4 * i)));
    const Q aa = qangle_axis_abs(d);
    v[3 * i + 0] = (aa.y * aa.x) / dt;
    v[3 * i + 1] = (aa.z * aa.x) / dt;
    v[3 * i + 2] = (aa.w * aa.x) / dt;
}

// scipy.ndimage.gaussian_filter1d(mode='nearest') along frames: symmetric correlate1d,
// float64 accumulation from the outermost tap pair inwards, rounded to float32 once
__global__ __launch_bounds__(256) void k_gauss_nearest(const float *__restrict__ v, int64_t nseq, int64_t L, int64_t S,
                                                       GaussTaps taps, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nseq * L * S) return;
    const int64_t s = i % S, t = (i / S) % L, base = i - s - t * S;
    const int R = taps.radius;
    auto at = [&](int64_t tt) { tt = tt < 0 ? 0 : (tt > L - 1 ? L - 1 : tt); return (double)v[base + tt * S + s]; };
    double acc = at(t) * taps.w[R];
    for (int jj = -R; jj < 0; ++jj) acc += (at(t + jj) + at(t - jj)) * taps.w[R + jj];
    out[i] = (float)acc;
}

hipError_t launch_linear_velocity(const float *p, int64_t nseq, int64_t L, int64_t S, float dt, const GaussTaps *taps,
                                  float *tmp, float *out, hipStream_t s)
{
    const int64_t n = nseq * L * S;
    const unsigned g = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_gradient_dt, dim3(g), dim3(256), 0, s, p, nseq, L, S, dt, taps ? tmp : out);
    if (taps) hipLaunchKernelGGL(k_gauss_nearest, dim3(g), dim3(256), 0, s, tmp, nseq, L, S, *taps, out);
    return hipGetLastError();
}

hipError_t launch_angular_velocity(const float *r, int64_t nseq, int64_t L, int64_t J, float dt,
                                   const GaussTaps *taps, float *tmp, float *out, hipStream_t s)
{
    const int64_t n = nseq * L * J;
    hipLaunchKernelGGL(k_angular_raw, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, r, nseq, L, J, dt,
                       taps ? tmp : out);
    if (taps)
        hipLaunchKernelGGL(k_gauss_nearest, dim3((unsigned)((3 * n + 255) / 256)), dim3(256), 0, s, tmp, nseq, L,
                           3 * J, *taps, out);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------
// synthetic mocap on the device (bench / large-size tests)
// counter-based hash RNG: frame f, draw k -> uniform in (0,1)
// ----------------------------------------------------------------------------
RTG_DEV uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
RTG_DEV float urand(uint64_t seed, uint64_t f, uint32_t k)
{
    const uint64_t h = mix64(seed * 0x9e3779b97f4a7c15ull ^ mix64(f * 0x100000001b3ull + k));
    return ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
}
RTG_DEV float nrand(uint64_t seed, uint64_t f, uint32_t k)   // Box-Muller
{
    const float u1 = urand(seed, f, k), u2 = urand(seed, f, k + 0x8000u);
    return sqrtf(-2.0f * logf(u1)) * cosf(6.28318530718f * u2);
}
RTG_DEV Q axis_angle_f(V ax, float ang)
{
    const float n = sqrtf(ax.x * ax.x + ax.y * ax.y + ax.z * ax.z);
    const float s = sinf(0.5f * ang) / n, c = cosf(0.5f * ang);
    return Q{ax.x * s, ax.y * s, ax.z * s, c};
}
RTG_DEV Q fast_qmul(Q a, Q b)
{
    return Q{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
             a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
RTG_DEV V fast_rot(Q q, V v)
{
    const V u{q.x, q.y, q.z};
    const V t{2.0f * (u.y * v.z - u.z * v.y), 2.0f * (u.z * v.x - u.x * v.z), 2.0f * (u.x * v.y - u.y * v.x)};
    return V{v.x + q.w * t.x + (u.y * t.z - u.z * t.y), v.y + q.w * t.y + (u.z * t.x - u.x * t.z),
             v.z + q.w * t.z + (u.x * t.y - u.y * t.x)};
}

// joint group of VTRDYN_FULL (retarget/robot_config/VTRDYN_FULL.py:9-69): 0 root, 1 spine/arm, 2 leg, 3 finger
RTG_DEV int full_group(int j)
{
    if (j == 0) return 0;
    if (j <= 6) return 2;
    if ((j >= 15 && j <= 33) || j >= 40) return 3;
    return 1;
}

__constant__ int kFullToBody[21] = {0, 4, 5, 6, 1, 2, 3, 7, 8, 9, 10, 34, 35, 36, 37, 38, 39, 11, 12, 13, 14};

__global__ __launch_bounds__(64) void k_synth_full_body(TopoView T, uint64_t seed, int64_t off, int64_t B,
                                                        float *__restrict__ body, float *__restrict__ lh,
                                                        float *__restrict__ rh, float *__restrict__ body_rot, bool soa)
{
    __shared__ float sp[64][59 * 3 + 1];
    __shared__ float sq[64][59 * 4];
    const int64_t f = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (f >= B) return;
    const uint64_t fr = (uint64_t)(off + f);
    float *P = sp[threadIdx.x];
    float *G = sq[threadIdx.x];
    for (int j = 0; j < T.J; ++j) {
        const int grp = full_group(j);
        const uint32_t k = 16u * (uint32_t)j;
        Q lq;
        if (grp == 0) {
            lq = axis_angle_f(V{0.f, 0.f, 1.f}, (urand(seed, fr, k) * 2.0f - 1.0f) * 3.14159265f);
        } else if (grp == 3) {
            const bool yax = urand(seed, fr, k + 1) < 0.5f;
            lq = axis_angle_f(yax ? V{0.f, 1.f, 0.f} : V{0.f, 0.f, 1.f}, 1.2f * urand(seed, fr, k + 2));
        } else {
            const V ax{nrand(seed, fr, k + 3), nrand(seed, fr, k + 4), nrand(seed, fr, k + 5)};
            lq = axis_angle_f(ax, (grp == 1 ? 1.0f : 0.5f) * urand(seed, fr, k + 6));
        }
        Q g;
        V t;
        const int p = T.parents[j];
        if (p < 0) {
            g = lq;
            t = V{0.1f * nrand(seed, fr, 2000), 0.1f * nrand(seed, fr, 2001), 0.1f * nrand(seed, fr, 2002)};
        } else {
            const Q gp{G[4 * p], G[4 * p + 1], G[4 * p + 2], G[4 * p + 3]};
            const V r = fast_rot(gp, T.local_t[j]);
            g = fast_qmul(gp, lq);
            t = V{r.x + P[3 * p], r.y + P[3 * p + 1], r.z + P[3 * p + 2]};
        }
        G[4 * j] = g.x; G[4 * j + 1] = g.y; G[4 * j + 2] = g.z; G[4 * j + 3] = g.w;
        P[3 * j] = t.x; P[3 * j + 1] = t.y; P[3 * j + 2] = t.z;
    }
    auto jit = [&](int j, int c) { return P[3 * j + c] + 0.002f * nrand(seed, fr, 3000u + 3u * j + c); };
    for (int i = 0; i < 21; ++i) {
        const int j = kFullToBody[i];
#pragma unroll
        for (int c = 0; c < 3; ++c) body[lay_idx(soa, f, i, c, 21, 3, B)] = jit(j, c);
        if (body_rot) {
            float n = sqrtf(G[4 * j] * G[4 * j] + G[4 * j + 1] * G[4 * j + 1] + G[4 * j + 2] * G[4 * j + 2] +
                            G[4 * j + 3] * G[4 * j + 3]);
            if (G[4 * j + 3] < 0.0f) n = -n;
#pragma unroll
            for (int c = 0; c < 4; ++c) body_rot[lay_idx(soa, f, i, c, 21, 4, B)] = G[4 * j + c] / n;
        }
    }
    for (int i = 0; i < 20; ++i) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            lh[lay_idx(soa, f, i, c, 20, 3, B)] = jit(14 + i, c);
            rh[lay_idx(soa, f, i, c, 20, 3, B)] = jit(39 + i, c);
        }
    }
}

// ----------------------------------------------------------------------------
// launchers (host side, called from rtg_api.cpp)
// ----------------------------------------------------------------------------
static inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

hipError_t launch_solver_prep(SolverConsts *dev_consts, hipStream_t s)
{
    hipLaunchKernelGGL(k_solver_prep, dim3(1), dim3(64), 0, s, dev_consts);
    return hipGetLastError();
}

// exp-map angle table (rtg_math.cuh, qexp_component_tab): one word of codes per thread, each code
// from the exact path it replaces.
__global__ __launch_bounds__(256) void k_build_ang_tab(uint32_t *tab)
{
    const uint32_t wd = blockIdx.x * 256u + threadIdx.x;
    if (wd >= kAngTabWords) return;
    tab[wd] = ang_tab_build_word(wd);
}

hipError_t launch_build_ang_tab(uint32_t *tab, hipStream_t s)
{
    hipLaunchKernelGGL(k_build_ang_tab, dim3((kAngTabWords + 255u) / 256u), dim3(256), 0, s, tab);
    return hipGetLastError();
}

// Kernel choice.  The side-split kernel halves each wave's program and doubles the waves in flight.  Measured
// against the fused body (same box, same session): 1.6-1.9x at 4096 frames for every kind; at
// 262144 frames FULL_BODY_POS +4 %, FULL_BODY_ROT +15 %, UPPER_BODY and BODY_ROT within box-to-box noise
// (-6..+2 % and -3..+10 % across two boxes).  So every kind runs split; RTG_SOLVER_SIDES=0 builds the fused
// kernels for comparison.
template <int KIND, bool PRECISE>
static void launch_kind(const SolverConsts &C, const float *in0, const float *in1, const float *in2,
                        const float *in3, int64_t B, int layout, float *dof, float *local_rot, float *body_rot,
                        hipStream_t s)
{
    if (KIND == RTG_SOLVER_FULL_BODY_POS && B <= RTG_LATENCY_MAX_B && RTG_LATENCY_WAVES == 5) {
        if (layout == RTG_LAYOUT_SOA)
            hipLaunchKernelGGL((k_fbp_latency5<PRECISE, true>), dim3(grid_for(B, kLatFrames)), dim3(320), 0, s, C,
                               in0, in1, in2, B, dof, local_rot, body_rot);
        else
            hipLaunchKernelGGL((k_fbp_latency5<PRECISE, false>), dim3(grid_for(B, kLatFrames)), dim3(320), 0, s, C,
                               in0, in1, in2, B, dof, local_rot, body_rot);
    } else if (KIND == RTG_SOLVER_FULL_BODY_POS && B <= RTG_LATENCY_MAX_B) {
        if (layout == RTG_LAYOUT_SOA)
            hipLaunchKernelGGL((k_fbp_latency<PRECISE, true>), dim3(grid_for(B, kLatFrames)), dim3(192), 0, s, C, in0,
                               in1, in2, B, dof, local_rot, body_rot);
        else
            hipLaunchKernelGGL((k_fbp_latency<PRECISE, false>), dim3(grid_for(B, kLatFrames)), dim3(192), 0, s, C, in0,
                               in1, in2, B, dof, local_rot, body_rot);
    } else if (layout == RTG_LAYOUT_SOA)
        hipLaunchKernelGGL((k_solve_sides<KIND, PRECISE, true>), dim3(grid_for(B, kSideFrames)), dim3(256), 0, s, C,
                           in0, in1, in2, in3, B, dof, local_rot, body_rot);
    else if (!RTG_SOLVER_SIDES)
        hipLaunchKernelGGL((k_retarget<KIND, PRECISE>), dim3(grid_for(B, kSolverBlock)), dim3(kSolverBlock), 0, s,
                           C, in0, in1, in2, in3, B, dof, local_rot, body_rot);
    else
        hipLaunchKernelGGL((k_solve_sides<KIND, PRECISE, false>), dim3(grid_for(B, kSideFrames)), dim3(256), 0, s, C,
                           in0, in1, in2, in3, B, dof, local_rot, body_rot);
}

hipError_t launch_frame_server(int precise, const SolverConsts &C, const float *in, float *dof, float *local_rot,
                               float *body_rot, uint32_t *ctl, uint64_t idle_ticks, hipStream_t s)
{
    if (precise)
        hipLaunchKernelGGL((k_frame_server<true>), dim3(1), dim3(320), 0, s, C, in, dof, local_rot, body_rot, ctl,
                           idle_ticks);
    else
        hipLaunchKernelGGL((k_frame_server<false>), dim3(1), dim3(320), 0, s, C, in, dof, local_rot, body_rot, ctl,
                           idle_ticks);
    return hipGetLastError();
}

hipError_t launch_retarget(int kind, int precise, const SolverConsts &C, const float *in0, const float *in1,
                           const float *in2, const float *in3, int64_t B, int layout, float *dof, float *local_rot,
                           float *body_rot, hipStream_t s)
{
    switch (kind) {
    case RTG_SOLVER_FULL_BODY_POS:
        if (precise) launch_kind<RTG_SOLVER_FULL_BODY_POS, true>(C, in0, in1, in2, in3, B, layout, dof, local_rot, body_rot, s);
        else launch_kind<RTG_SOLVER_FULL_BODY_POS, false>(C, in0, in1, in2, in3, B, layout, dof, local_rot, body_rot, s);
        break;
    case RTG_SOLVER_UPPER_BODY:
        launch_kind<RTG_SOLVER_UPPER_BODY, false>(C, in0, in1, in2, in3, B, layout, dof, local_rot, body_rot, s);
        break;
    case RTG_SOLVER_FULL_BODY_ROT:
        launch_kind<RTG_SOLVER_FULL_BODY_ROT, false>(C, in0, in1, in2, in3, B, layout, dof, local_rot, body_rot, s);
        break;
    default:
        launch_kind<RTG_SOLVER_BODY_ROT, false>(C, in0, in1, in2, in3, B, layout, dof, local_rot, body_rot, s);
        break;
    }
    return hipGetLastError();
}

hipError_t launch_fk(const TopoView &T, bool state, const float *lr, const float *rt, int64_t B, float *gr, float *gp,
                     hipStream_t s)
{
    if (T.nslots <= kMaxFkSlots) {
        const dim3 g(grid_for(B, kFkTile)), b(kFkTile);
        const size_t lds = fk_stream_lds_bytes(T.nslots);
        if (state) hipLaunchKernelGGL(k_fk_stream<true>, g, b, lds, s, T, lr, rt, B, gr, gp);
        else hipLaunchKernelGGL(k_fk_stream<false>, g, b, lds, s, T, lr, rt, B, gr, gp);
    } else if (state) {   // pathological branching (> kMaxFkSlots live branch parents): lane-walk kernel
        hipLaunchKernelGGL(k_fk<true>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, lr, rt, B, gr, gp);
    } else {
        hipLaunchKernelGGL(k_fk<false>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, lr, rt, B, gr, gp);
    }
    return hipGetLastError();
}

hipError_t launch_local_rotation(const TopoView &T, bool state, const float *g, int64_t B, float *l, hipStream_t s)
{
    if (T.nslots <= kMaxFkSlots) {
        const dim3 gd(grid_for(B, kFkTile)), b(kFkTile);
        const size_t lds = fk_stream_lds_bytes(T.nslots);
        if (state) hipLaunchKernelGGL(k_local_rotation_stream<true>, gd, b, lds, s, T, g, B, l);
        else hipLaunchKernelGGL(k_local_rotation_stream<false>, gd, b, lds, s, T, g, B, l);
    } else if (state) {
        hipLaunchKernelGGL(k_local_rotation<true>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, g, B, l);
    } else {
        hipLaunchKernelGGL(k_local_rotation<false>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, g, B, l);
    }
    return hipGetLastError();
}

hipError_t launch_fk_multi(FkMultiArgs &A, hipStream_t s)
{
    int maxS = 0;
    for (int i = 0; i < A.n; ++i) maxS = A.seg[i].T.nslots > maxS ? A.seg[i].T.nslots : maxS;
    const bool stream = maxS <= kMaxFkSlots;
    const int per = stream ? kFkTile : 256;
    int64_t blocks = 0;
    for (int i = 0; i < A.n; ++i) {
        A.block_start[i] = blocks;
        blocks += grid_for(A.seg[i].B, per);
    }
    for (int i = A.n; i < RTG_MAX_SEGMENTS; ++i) A.block_start[i] = blocks;
    if (blocks == 0) return hipSuccess;
    if (stream)
        hipLaunchKernelGGL(k_fk_multi_stream, dim3((unsigned)blocks), dim3(kFkTile), fk_stream_lds_bytes(maxS), s, A);
    else
        hipLaunchKernelGGL(k_fk_multi, dim3((unsigned)blocks), dim3(256), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_dof_fk(const TopoView &T, const DofView &D, bool clip, const float *dof, const float *root_rot,
                         const float *root_t, int64_t B, float *gr, float *gp, hipStream_t s)
{
    if (T.nslots > kMaxFkSlots) return hipErrorInvalidValue;   // rejected at rtg_dof_model_create
    const dim3 g(grid_for(B, kFkTile)), b(kFkTile);
    const size_t lds = dof_fk_lds_bytes(T.nslots);
    if (clip) hipLaunchKernelGGL(k_dof_fk<true>, g, b, lds, s, T, D, dof, root_rot, root_t, B, gr, gp);
    else hipLaunchKernelGGL(k_dof_fk<false>, g, b, lds, s, T, D, dof, root_rot, root_t, B, gr, gp);
    return hipGetLastError();
}

hipError_t launch_rescale_motion(const TopoView &T, const float *motion, int64_t B, const float *dir, float *out,
                                 hipStream_t s)
{
    const Dir3 d = dir ? Dir3{dir[0], dir[1], dir[2], 1} : Dir3{1.0f, 1.0f, 1.0f, 0};
    hipLaunchKernelGGL(k_rescale_motion, dim3(grid_for(B, 256)), dim3(256), 0, s, T, motion, B, d, out);
    return hipGetLastError();
}

hipError_t launch_quat_between(const float *v1, const float *v2, int64_t n, float *out, float *ws, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(ws, 0, 2 * sizeof(float), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_qbtv_norm_max, dim3(grid_for(n, 256)), dim3(256), 0, s, v1, v2, n, ws);
    hipLaunchKernelGGL(k_quat_between, dim3(grid_for(n, 256)), dim3(256), 0, s, v1, v2, n, ws, out);
    return hipGetLastError();
}

hipError_t launch_rebuild_vtrdyn(const TopoView &T, const float *motion, int64_t B, float *g_rot, float *root_t,
                                 float *ws, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(ws, 0, T.J * sizeof(float), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_rebuild_norm_max, dim3(grid_for(B, 256)), dim3(256), 0, s, T, motion, B, ws);
    hipLaunchKernelGGL(k_rebuild_vtrdyn, dim3(grid_for(B, 256)), dim3(256), 0, s, T, motion, B, ws, g_rot, root_t);
    return hipGetLastError();
}

hipError_t launch_ingest_vtrdyn(const float *bp, const float *lhp, const float *rhp, int64_t B, int layout,
                                float *body, float *lh, float *rh, uint8_t *valid, hipStream_t s)
{
    hipLaunchKernelGGL(k_ingest_vtrdyn, dim3(grid_for(B, 256)), dim3(256), 0, s, bp, lhp, rhp, B, body, lh, rh, valid,
                       layout == RTG_LAYOUT_SOA);
    return hipGetLastError();
}

hipError_t launch_quat_op(int op, const float *a, const float *b, const float *c, int64_t n, float *out,
                          hipStream_t s)
{
    hipLaunchKernelGGL(k_quat_op, dim3(grid_for(n, 256)), dim3(256), 0, s, op, a, b, c, n, out);
    return hipGetLastError();
}

hipError_t launch_cal_joint_quat(const float *Z, const float *M, int npts, int64_t n, float *out, hipStream_t s)
{
    const dim3 g(grid_for(n, 256)), b(256);
    switch (npts) {
    case 1: hipLaunchKernelGGL(k_cal_joint_quat<1>, g, b, 0, s, Z, M, n, out); break;
    case 2: hipLaunchKernelGGL(k_cal_joint_quat<2>, g, b, 0, s, Z, M, n, out); break;
    case 3: hipLaunchKernelGGL(k_cal_joint_quat<3>, g, b, 0, s, Z, M, n, out); break;
    case 4: hipLaunchKernelGGL(k_cal_joint_quat<4>, g, b, 0, s, Z, M, n, out); break;
    case 5: hipLaunchKernelGGL(k_cal_joint_quat<5>, g, b, 0, s, Z, M, n, out); break;
    case 6: hipLaunchKernelGGL(k_cal_joint_quat<6>, g, b, 0, s, Z, M, n, out); break;
    case 7: hipLaunchKernelGGL(k_cal_joint_quat<7>, g, b, 0, s, Z, M, n, out); break;
    default: hipLaunchKernelGGL(k_cal_joint_quat<8>, g, b, 0, s, Z, M, n, out); break;
    }
    return hipGetLastError();
}

hipError_t launch_quat_in_xyz_axis(const float *q, int s0, int s1, int s2, int extrinsic, int64_t n, float *out,
                                   hipStream_t s)
{
    hipLaunchKernelGGL(k_quat_in_xyz_axis, dim3(grid_for(n, 256)), dim3(256), 0, s, q, s0, s1, s2, extrinsic, n, out);
    return hipGetLastError();
}

hipError_t launch_synth_full_body(const TopoView &T, uint64_t seed, int64_t off, int64_t B, float *body, float *lh,
                                  float *rh, float *body_rot, int layout, hipStream_t s)
{
    hipLaunchKernelGGL(k_synth_full_body, dim3(grid_for(B, 64)), dim3(64), 0, s, T, seed, off, B, body, lh, rh,
                       body_rot,
                       layout == RTG_LAYOUT_SOA);
    return hipGetLastError();
}

}  // namespace rtg
