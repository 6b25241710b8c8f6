// rtg_solver.cuh -- the retarget solver bodies and kernel templates (included by rtg_solve_*.hip, which
// instantiate disjoint subsets so the heavy kernels compile in parallel).
//
// Work decomposition: one mocap frame per lane.  Frames are independent
// (SURVEY.md §0), every solver step is a short dependent chain of scalar-sized
// math, and a frame's working set (<= 32 input points) fits in VGPRs, so a
// lane solves its frame with no cross-lane traffic; the frame program is split
// between the two (or, for small batches, five) waves of a tile.  Zero-pose-only
// terms are evaluated once per solver (k_solver_prep) and arrive as a by-value
// kernel argument (SGPR-resident).  The 30-float DOF row of each frame is
// staged through LDS so a tile leaves as contiguous dwordx4 stores instead of
// 64 lanes writing 120-byte-strided rows.
//
// Kernels (launch_kind picks by batch size):
//   B == 1                    k_fbp_frame1    one frame, its independent sub-steps on separate lanes (teleop)
//   B <= RTG_QUAD_MAX_B       k_fbp_quad      five waves per 16-frame tile, a frame's sub-steps on a lane quad
//   B <= RTG_LATENCY_MAX_B    k_fbp_latency5  five waves per 64-frame tile (latency-bound batches)
//   larger                    k_solve_sides   two waves per 64-frame tile (throughput; the bench headline)
// and k_frame_server, the resident per-frame server on k_fbp_frame1's tile.
#pragma once
#include "rtg_device.cuh"

namespace rtg {

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
    // k_solve_sides FULL_BODY_POS (round 6): the wave's LDS block of table words, [slot][lane] (stride 64, the same
    // slots as st).  link() starts the load of its read-out's table word straight into it (global_load_lds: no VGPR,
    // asynchronous), so the word is there long before the read-out; finalize reads it from LDS after a vmcnt wait.
    // nullptr: finalize loads the words itself.
    uint32_t *wd = nullptr;
    // links 12..18 and 21..27 (DOFs 11..17, 20..26) -> stash slots 0..13
    template <int LINK>
    static constexpr int slot() { return LINK <= 18 ? LINK - 12 : LINK - 14; }
    RTG_DEV void load_word(int s, float w) const
    {
#if !RTG_EXP_NO_TABLE
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(ang + ang_tab_word_of(w)),
                                         (__attribute__((address_space(3))) void *)(wd + s * 64), 4, 0, 0);
#endif
    }
    template <int LINK>
    RTG_DEV void link(Q q) const
    {
        constexpr int k = hu_dof_axis(LINK - 1);
        st[slot<LINK>() * sst] = make_float2(q.w, k == 0 ? q.x : (k == 1 ? q.y : q.z));
        if (wd) load_word(slot<LINK>(), q.w);
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
        if (wd) wait_words();
#pragma unroll
        for (int j = 0; j < 14; ++j)
            if (j >= s0 && j < s0 + n) {
                const float2 v = st[j * sst];
                const ExpDof e = wd ? exp_dof_word_part(v.x, wd[j * 64 + (threadIdx.x & 63)]) : exp_dof_table_part(v.x, ang);
                exact |= (uint32_t)e.exact << j;
                row[j < 7 ? 11 + j : 13 + j] = exp_dof_finish(e, v.y);
            }
        if (__builtin_expect(exact != 0u, 0)) {
#pragma unroll 1
            for (int j = s0; j < s0 + n; ++j)
                if ((exact >> j) & 1u) {
                    const float2 v = st[j * sst];
                    row[j < 7 ? 11 + j : 13 + j] = exp_dof_exact(v.x, v.y);
                }
        }
    }
    // this wave's table-word loads into LDS have landed (vmcnt 0; expcnt / lgkmcnt not waited on)
    static RTG_DEV void wait_words() { __builtin_amdgcn_s_waitcnt(0x0F70); }
};

RTG_DEV void emit_fixed_links(const Emit &E, bool write_lr = true)
{
#pragma unroll
    for (int k = 0; k < 11; ++k) E.row[k] = 0.0f;
    E.row[29] = 0.0f;
    if (E.lr && write_lr) {
#pragma unroll
        for (int j = 0; j < 12; ++j) st4(E.lr + 4 * j, qident());
        st4(E.lr + 4 * 19, qident());
        st4(E.lr + 4 * 20, qident());
        st4(E.lr + 4 * 28, qident());
        st4(E.lr + 4 * 29, qident());
        st4(E.lr + 4 * 30, qident());
    }
}

// ----------------------------------------------------------------------------
// Frames the reference raises on (rtg.h rtg_frame_error).  Each wave collects the steps of its share of the frame
// program that would raise, as bits in the reference's own order of those steps (full_body_pos_retargeter.py:68,
// :138, :145, :161, :167); the wave that stores the tile combines both sides' bits and, on the rare flagged frame,
// replaces every output of the row by NaN -- the reference returns nothing for it -- with the first raise's code in
// dof[0]'s payload.
// ----------------------------------------------------------------------------
enum : uint32_t {
    kStTorsoSvd = 1,      // torso cal_joint_quat: torch.linalg.svd of a NaN matrix      (RuntimeError)
    kStLeftSvd = 2,       // left wrist cal_joint_quat                                    (RuntimeError)
    kStLeftEuler = 4,     // left quat_in_xyz_axis: zero-norm / NaN quaternion            (ValueError)
    kStRightSvd = 8,      // right wrist cal_joint_quat                                   (RuntimeError)
    kStRightEuler = 16,   // right quat_in_xyz_axis                                       (ValueError)
};
RTG_DEV uint32_t frame_error_code(uint32_t bits)
{
    const uint32_t first = bits & (0u - bits);
    return (first & (kStTorsoSvd | kStLeftSvd | kStRightSvd)) ? RTG_FRAME_SVD_NONFINITE : RTG_FRAME_ZERO_NORM_QUAT;
}
// the row of a frame with status bits != 0: dof (LDS row), local_rot and body_rot rows (global, may be null)
RTG_DEV void poison_frame(float *drow, float *__restrict__ lr, float *__restrict__ br, uint32_t bits)
{
    const float qn = __builtin_bit_cast(float, RTG_FRAME_NAN);
    drow[0] = __builtin_bit_cast(float, RTG_FRAME_NAN | frame_error_code(bits));
#pragma unroll
    for (int k = 1; k < 30; ++k) drow[k] = qn;
    const Q qq{qn, qn, qn, qn};
    if (lr)
        for (int j = 0; j < 31; ++j) st4(lr + 4 * j, qq);
    if (br)
        for (int j = 0; j < 59; ++j) st4(br + 4 * j, qq);
}

// the device error word of the solver (SolverConsts::err, host-mapped), set from any lane
RTG_DEV void report_device_error(uint32_t *err, uint32_t code)
{
    if (err) __hip_atomic_fetch_or(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one arm: shoulder pitch/roll then shoulder yaw / elbow pitch (full_body_pos_retargeter.py:75-93);
// returns quat_mul_four of the four link rotations (the wrist parent chain, :128-136)
// (round 6: on arm_pair_n, the two angles of each map in one instruction stream with shared rare-case branches; the
// same values as shoulder_pr / elbow_py)
template <int L0, typename Tab = NoTab>
RTG_DEV Q solve_arm(const Emit &E, V upper, V fore, ArmZero zs, ArmZero ze, Q parent, Tab tab = Tab{})
{
    Q p, r, y, e;
    {
        const V v[1] = {upper};
        const ArmZero z[1] = {zs};
        const Q par[1] = {parent};
        Q a[1], b[1];
        arm_pair_n<true, 1>(v, z, par, a, b, tab);
        p = a[0];
        r = b[0];
    }
    E.link<L0>(p);
    E.link<L0 + 1>(r);
    {
        const V v[1] = {fore};
        const ArmZero z[1] = {ze};
        const Q par[1] = {qmul(qmul(parent, p), r)};
        Q a[1], b[1];
        arm_pair_n<false, 1>(v, z, par, a, b, tab);
        y = a[0];
        e = b[0];
    }
    E.link<L0 + 2>(y);
    E.link<L0 + 3>(e);
    return qmul(qmul(qmul(p, r), y), e);
}

// Emit::link with a run-time link index (lane-parallel writers; a wave without early table words, Emit::wd null)
RTG_DEV void link_rt(const Emit &E, int link, Q q)
{
    const int k = kHuDofAxis[link - 1];
    E.st[(link <= 18 ? link - 12 : link - 14) * E.sst] = make_float2(q.w, k == 0 ? q.x : (k == 1 ? q.y : q.z));
    if (E.lr) st4(E.lr + 4 * link, q);
}
// solve_arm / emit_euler_xyz with a run-time first link: two waves of a side pair run one copy of the code
template <typename Tab = NoTab>
RTG_DEV Q solve_arm_rt(const Emit &E, int L0, V upper, V fore, ArmZero zs, ArmZero ze, Q parent, Tab tab = Tab{})
{
    Q p, r, y, e;
    {
        const V v[1] = {upper};
        const ArmZero z[1] = {zs};
        const Q par[1] = {parent};
        Q a[1], b[1];
        arm_pair_n<true, 1>(v, z, par, a, b, tab);
        p = a[0];
        r = b[0];
    }
    link_rt(E, L0, p);
    link_rt(E, L0 + 1, r);
    {
        const V v[1] = {fore};
        const ArmZero z[1] = {ze};
        const Q par[1] = {qmul(qmul(parent, p), r)};
        Q a[1], b[1];
        arm_pair_n<false, 1>(v, z, par, a, b, tab);
        y = a[0];
        e = b[0];
    }
    link_rt(E, L0 + 2, y);
    link_rt(E, L0 + 3, e);
    return qmul(qmul(qmul(p, r), y), e);
}
RTG_DEV bool emit_euler_xyz_rt(const Emit &E, int L0, Q local)
{
    Q eul[3];
    const bool refused = quat_in_xyz_intrinsic(local, eul);
    link_rt(E, L0, eul[0]);
    link_rt(E, L0 + 1, eul[1]);
    link_rt(E, L0 + 2, eul[2]);
    return refused;
}
// quat_in_xyz_axis(q, 'XYZ') -> links L0..L0+2; true where scipy refuses q (transform3d.py:53)
template <int L0>
RTG_DEV bool emit_euler_xyz(const Emit &E, Q local)
{
    Q eul[3];
    const bool refused = quat_in_xyz_intrinsic(local, eul);
    E.link<L0>(eul[0]);
    E.link<L0 + 1>(eul[1]);
    E.link<L0 + 2>(eul[2]);
    return refused;
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
    RTG_DEV float e(int64_t i) const
    {
        if (RTG_IN_NT_LOAD) return __builtin_nontemporal_load(p + i);   // A/B knob: streaming input planes
        return p[i];
    }
    RTG_DEV V p3(int j) const { return V{e((3 * j) * s), e((3 * j + 1) * s), e((3 * j + 2) * s)}; }
    RTG_DEV Q q4(int j) const { return Q{e((4 * j) * s), e((4 * j + 1) * s), e((4 * j + 2) * s), e((4 * j + 3) * s)}; }
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

constexpr int kDofStride = 31;   // LDS row pitch (dwords): odd -> conflict-free ds_write_b32

// Cooperative store of `nrows` DOF rows staged in LDS at pitch kDofStride into the contiguous dst rows, by
// `nthr` threads (this one is `t`).  dst is 16-byte aligned (a tile starts at a multiple of 64 frames), so
// the rows leave as dwordx4 stores (full-line writes).
RTG_DEV void store_dof_rows(float *__restrict__ dst, const float *src, int64_t nrows, int t, int nthr)
{
    const int nvals = (int)nrows * 30;
    auto at = [&](int i) {
        const int rr = i / 30;
        return src[rr * kDofStride + (i - rr * 30)];
    };
    const int nvec = nvals >> 2;
    typedef float f4v __attribute__((ext_vector_type(4)));
    for (int v = t; v < nvec; v += nthr) {
        const int i = v << 2;
        const f4v q = {at(i), at(i + 1), at(i + 2), at(i + 3)};
        if (RTG_DOF_NT_STORE) __builtin_nontemporal_store(q, reinterpret_cast<f4v *>(dst + i));   // A/B knob
        else *reinterpret_cast<f4v *>(dst + i) = q;
    }
    for (int i = (nvec << 2) + t; i < nvals; i += nthr) dst[i] = at(i);
}

// ----------------------------------------------------------------------------
// Every solver kind, two waves per frame tile.  After the torso fit (or, for the rotation solvers, from the
// start) the two sides are independent (full_body_pos_retargeter.py:70-175, retarget_solver.py:72-99,
// full_body_retargeter.py:60-177, body_retargeter.py:48-81), so waves 2k and 2k+1 of a block take the left
// and the right side of the same 64 frames.  The side is wave-uniform: its constants stay scalar, the branch
// never diverges, and each wave runs about half the frame program -- twice the waves in flight, about half the
// per-frame latency, the same arithmetic per value.
// ----------------------------------------------------------------------------
constexpr int kSideTiles = RTG_SIDES_TILES;        // 64-frame tiles per block (two waves each)
constexpr int kSideThreads = 128 * kSideTiles;
constexpr int kSideFrames = 64 * kSideTiles;       // frames per block

// torso fit R10 (full_body_pos_retargeter.py:69-70 / retarget_solver.py:49-50)
template <typename View, typename Hook = NoHook, typename Tab = NoTab>
RTG_DEV Q fbp_torso(const SolverConsts &C, const View &b, bool &svd_nan, const Hook &hook = Hook{}, Tab tab = Tab{})
{
    const V b10 = b.p3(10);
    const V Mt[3] = {vsub(b.p3(17), b10), vsub(b.p3(13), b10), vsub(b.p3(11), b10)};
    return cal_joint_quat<3>(C.Zt, Mt, svd_nan, hook, tab);
}
RTG_DEV Q upper_pt_sign(V v) { return Q{v.x * -1.0f, v.y * -1.0f, v.z * 1.0f, 0.0f}; }   // coord_transform :41
template <typename View>
RTG_DEV Q upper_torso(const SolverConsts &C, const View &x, bool &svd_nan)
{
    auto pt = [&](int j) {
        const Q q = upper_pt_sign(x.p3(j));
        return V{q.x, q.y, q.z};
    };
    const V s10 = pt(10);
    const V Mt[3] = {vsub(pt(17), s10), vsub(pt(13), s10), vsub(pt(11), s10)};
    return cal_joint_quat<3>(C.Zt, Mt, svd_nan);
}
// wrist fit W (full_body_pos_retargeter.py:137-140 left, :160-163 right)
template <int SIDE, typename View, typename Hook = NoHook, typename Tab = NoTab>
RTG_DEV Q fbp_wrist_fit(const SolverConsts &C, const View &H, bool &svd_nan, const Hook &hook = Hook{}, Tab tab = Tab{})
{
    const V h0 = H.p3(0);
    const V M[5] = {vsub(H.p3(2), h0), vsub(H.p3(6), h0), vsub(H.p3(10), h0), vsub(H.p3(14), h0), vsub(H.p3(17), h0)};
    return cal_joint_quat<5>(SIDE ? C.Zr : C.Zl, M, svd_nan, hook, tab);
}
// fbp_wrist_fit with a run-time side (the B = 1 kernel: both wrist waves run ONE copy of the fit's code, not two
// template instances -- the I-cache then holds one; RTG_FRAME1_SHARED_CODE).  Z is C.Zl or C.Zr itself: the same bits.
template <typename View, typename Hook = NoHook, typename Tab = NoTab>
RTG_DEV Q fbp_wrist_fit_rt(const SolverConsts &C, const View &H, int side, bool &svd_nan, const Hook &hook = Hook{},
                           Tab tab = Tab{})
{
    const V h0 = H.p3(0);
    const V M[5] = {vsub(H.p3(2), h0), vsub(H.p3(6), h0), vsub(H.p3(10), h0), vsub(H.p3(14), h0), vsub(H.p3(17), h0)};
    V Z[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) Z[k] = side ? C.Zr[k] : C.Zl[k];
    return cal_joint_quat<5>(Z, M, svd_nan, hook, tab);
}
// A side's body points (shoulder, elbow, wrist), loaded at kernel start with the torso / wrist-fit loads of the
// same rows (measured -4 %: DESIGN.md §5), and its hand points for the gripper (0 and the tips 4,8,12,16,19).
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
// Both arms' chains at once (round 6): solve_arm for the left and the right arm on the N-way leaf math, so the two
// independent chains interleave in one instruction stream (the same values: arm_pair_n).  Returns the chains.
template <typename Tab = NoTab>
RTG_DEV void fbp_arms2(const SolverConsts &C, const ArmPts &apL, const ArmPts &apR, Q R10, const Emit &E, Q &chL,
                       Q &chR, Tab tab = Tab{})
{
    const V up[2] = {vsub(apL.el, apL.sh), vsub(apR.el, apR.sh)};
    const V fo[2] = {vsub(apL.wr, apL.el), vsub(apR.wr, apR.el)};
    const ArmZero zs[2] = {C.lsh, C.rsh}, ze[2] = {C.lel, C.rel};
    const Q par[2] = {R10, R10};
    Q p[2], r[2], y[2], e[2];
    arm_pair_n<true, 2>(up, zs, par, p, r, tab);
    E.link<12>(p[0]);
    E.link<13>(r[0]);
    E.link<21>(p[1]);
    E.link<22>(r[1]);
    const Q par2[2] = {qmul(qmul(R10, p[0]), r[0]), qmul(qmul(R10, p[1]), r[1])};
    arm_pair_n<false, 2>(fo, ze, par2, y, e, tab);
    E.link<14>(y[0]);
    E.link<15>(e[0]);
    E.link<23>(y[1]);
    E.link<24>(e[1]);
    chL = qmul(qmul(qmul(p[0], r[0]), y[0]), e[0]);
    chR = qmul(qmul(qmul(p[1], r[1]), y[1]), e[1]);
}
// the gripper DOFs of one side from its x-spread a (full_body_pos_retargeter.py:199-215)
template <bool PRECISE>
RTG_DEV void fbp_gripper(const SolverConsts &C, float a, float *row_d0)
{
    if (PRECISE) {
        const float sc = clamp_lohi(a / C.orig - 0.5f, 0.0f, 0.5f) / 0.5f;
        row_d0[0] = sc * 0.044f;
        row_d0[1] = sc * -0.044f;
    } else {
        const bool closed = a / C.orig < 0.7f;
        row_d0[0] = closed ? 0.0f : 0.044f;
        row_d0[1] = closed ? 0.0f : -0.044f;
    }
}
// body_global_rotation rows (:116, :172-173) of one side: the left side also writes row 10 and the identities
template <int SIDE>
RTG_DEV void fbp_body_rows(float *__restrict__ brow, Q R10, Q W, bool const_rows = true)
{
    st4(brow + 4 * (SIDE ? 39 : 14), W);
    if (!SIDE) {
        if (const_rows) {
            for (int j = 0; j < 59; ++j)
                if (j != 14 && j != 39) st4(brow + 4 * j, j == 10 ? R10 : qident());
        } else {
            st4(brow + 4 * 10, R10);
        }
    }
}
// the Euler split of the wrist (:128-136), the gripper (:142-158 / :165-175) and the body_rot rows; true where
// scipy refuses the wrist's local quaternion
template <bool PRECISE, int SIDE, typename Tab = NoTab>
RTG_DEV bool fbp_side_after_arm(const SolverConsts &C, const TipPts &tp, Q R10, Q chain, Q W, const Emit &E,
                                float *__restrict__ brow, Tab tab = Tab{})
{
    constexpr int E0 = SIDE ? 25 : 16, D0 = SIDE ? 27 : 18;
    const bool refused = emit_euler_xyz<E0>(E, qnormalize_t(qmul(qconj(qnormalize_t(qmul(R10, chain), tab)), W), tab));
    fbp_gripper<PRECISE>(C, hand_x_mean(qconj(W), tp.h0, tp.t), E.row + D0);
    if (brow) fbp_body_rows<SIDE>(brow, R10, W);
    return refused;
}

// HuUpperBodyFromMocapRetarget (retarget_solver.py:40-99), one side: one arm given the torso fit; wrists untouched
template <int SIDE, typename View, typename Tab = NoTab>
RTG_DEV void solve_upper_side(const SolverConsts &C, const View &x, Q R10, const Emit &E, Tab tab = Tab{})
{
    auto pt = [&](int j) {   // coord_transform(dir=[-1,-1,1]) :41
        const Q q = upper_pt_sign(x.p3(j));
        return V{q.x, q.y, q.z};
    };
    constexpr int L0 = SIDE ? 21 : 12, E0 = SIDE ? 25 : 16, D0 = SIDE ? 27 : 18;
    constexpr int SH = SIDE ? 14 : 18, EL = SIDE ? 15 : 19, WR = SIDE ? 16 : 20;
    const V sel = pt(EL);
    solve_arm<L0>(E, vsub(sel, pt(SH)), vsub(pt(WR), sel), SIDE ? C.rsh : C.lsh, SIDE ? C.rel : C.lel, R10, tab);
    E.identity<E0>(); E.identity<E0 + 1>(); E.identity<E0 + 2>();
    E.row[D0] = 0.0f; E.row[D0 + 1] = 0.0f;
}

// VtrdynFullBodyRetargeter (full_body_retargeter.py:19-177), one side; true where scipy refuses (:121 / :138)
template <int SIDE, typename View, typename Tab = NoTab>
RTG_DEV bool solve_full_body_rot_side(const SolverConsts &C, const View &q, const View &b, const View &H,
                                      const Emit &E, Tab tab = Tab{})
{
    constexpr int L0 = SIDE ? 21 : 12, E0 = SIDE ? 25 : 16, D0 = SIDE ? 27 : 18;
    constexpr int SH = SIDE ? 14 : 18, EL = SIDE ? 15 : 19, WR = SIDE ? 16 : 20, PAR = SIDE ? 13 : 17;
    const Q par = q.q4(PAR);
    const V bel = b.p3(EL);
    const Q chain = solve_arm<L0>(E, vsub(bel, b.p3(SH)), vsub(b.p3(WR), bel), SIDE ? C.rsh : C.lsh,
                                  SIDE ? C.rel : C.lel, par, tab);
    const Q w = q.q4(WR);
    const bool refused = emit_euler_xyz<E0>(E, qnormalize_t(qmul(qconj(qnormalize_t(qmul(par, chain), tab)), w), tab));
    constexpr int tips[5] = {3, 7, 11, 15, 19};   // :145-177 rotates by the wrist quaternion itself
    const bool closed = hand_x_mean(w, H, tips) / C.orig < 0.7f;
    E.row[D0] = closed ? 0.0f : 0.044f;
    E.row[D0 + 1] = closed ? 0.0f : -0.044f;
    return refused;
}

// Mocap2HuBodyRetargeter (body_retargeter.py:34-81), one side; true where scipy refuses either split (:42-55)
template <int SIDE, typename View, typename Tab = NoTab>
RTG_DEV bool solve_body_rot_side(const SolverConsts &C, const View &g, const Emit &E, Tab tab = Tab{})
{
    auto local = [&](int j, int p) { return qnormalize_t(qmul(qconj(g.q4(p)), g.q4(j)), tab); };
    constexpr int SH = SIDE ? 14 : 18, EL = SIDE ? 15 : 19, D0 = SIDE ? 27 : 18;
    Q s3[3], e3[3];
    bool refused = quat_in_xyz_axis(local(SH, C.par[SIDE ? 1 : 0]), 1, 0, 2, false, s3);   // 'YXZ'
    refused |= quat_in_xyz_axis(local(EL, C.par[SIDE ? 3 : 2]), 2, 1, 0, false, e3);       // 'ZYX'
    if (SIDE) {
        E.link<21>(s3[0]); E.link<22>(s3[1]); E.link<23>(qnormalize_t(qmul(e3[0], s3[2]), tab));
        E.link<24>(e3[1]); E.link<25>(e3[2]);
        E.identity<26>(); E.identity<27>();
    } else {
        E.link<12>(s3[0]); E.link<13>(s3[1]); E.link<14>(qnormalize_t(qmul(e3[0], s3[2]), tab));
        E.link<15>(e3[1]); E.link<16>(e3[2]);
        E.identity<17>(); E.identity<18>();
    }
    E.row[D0] = 0.0f; E.row[D0 + 1] = 0.0f;
    return refused;
}

// ----------------------------------------------------------------------------
// Wave-to-wave hand-over through LDS flags.  A release is per lane, but the hand-over is per wave: every lane
// fences its own LDS writes (release, workgroup scope), then -- after a convergent ballot, where the whole wave has
// rejoined (the compiler once ran the idle lanes' path first and raised the flag before the live lanes' writes) --
// one lane raises the flag.  The waiting wave spins on an acquire load in every lane.
// ----------------------------------------------------------------------------
RTG_DEV void lds_signal(int *flag)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    const uint64_t joined = __builtin_amdgcn_ballot_w64(true);
    if (joined != 0 && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(joined))
        __hip_atomic_store(flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Every wave of a workgroup is resident together and a producer never waits on its consumer, so the flag always
// arrives; the iteration cap (~0.1 s at s_sleep 1) is a bound every wave reaches even if that were ever broken.
// Giving up is reported in the solver's error word (rtg.h RTG_DEVERR_HANDOVER_TIMEOUT), never silently.
RTG_DEV void lds_wait(int *flag, uint32_t *err)
{
    for (int it = 0; it < (1 << 22); ++it) {
        if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) return;
        __builtin_amdgcn_s_sleep(1);
    }
    if ((threadIdx.x & 63) == 0) report_device_error(err, RTG_DEVERR_HANDOVER_TIMEOUT);
}

template <int KIND, bool PRECISE, bool SOA>
__global__ __launch_bounds__(kSideThreads, RTG_SIDES_WAVES) void k_solve_sides(SolverConsts C, const float *__restrict__ in0,
                                                     const float *__restrict__ in1, const float *__restrict__ in2,
                                                     const float *__restrict__ in3, int64_t B,
                                                     float *__restrict__ dof, float *__restrict__ local_rot,
                                                     float *__restrict__ body_rot)
{
    __shared__ float sdof[kSideFrames * kDofStride];
    __shared__ float4 storso[kSideFrames];   // FULL_BODY_POS: R10 left -> right wave, then the left chain right -> left
    __shared__ float2 sst[kSideTiles * 14 * 64];   // exp-map stash, [tile][slot][lane]
    __shared__ uint8_t sstat[2][kSideFrames];   // each side's frame-status bits (kSt*)
    const int w = threadIdx.x >> 6, side = w & 1, lane = threadIdx.x & 63;
    const int r = (w >> 1) * 64 + lane;   // tile row
    const int64_t f0 = (int64_t)blockIdx.x * kSideFrames, f = f0 + r;
    const bool live = f < B;
    float *const lrow = live && local_rot ? local_rot + f * 124 : nullptr;
#if RTG_SIDES_EARLY_WORDS
    __shared__ uint32_t swd[kSideTiles * 14 * 64];   // FULL_BODY_POS: the read-outs' table words, [tile][slot][lane]
    // AoS only: SoA 99.5-102.8 vs 99.9-100.9 us without, AoS 110.1-111.2 vs 110.7-113.4 (profiles/r06/early_words/)
    uint32_t *const wds = KIND == RTG_SOLVER_FULL_BODY_POS && !SOA ? swd + (w >> 1) * 14 * 64 : nullptr;
#else
    uint32_t *const wds = nullptr;
#endif
    const Emit E{sdof + r * kDofStride, lrow, C.ang_tab, sst + (w >> 1) * 14 * 64 + lane, 64, wds};
#if RTG_EXP_HOT_INPUTS   // measurement knob (tools/build_variants.sh): every tile reads the first block's rows
    const int64_t fi = f & (kSideFrames - 1);
#else
    const int64_t fi = f;
#endif
    auto view = [&](const float *base, int row_floats) { return frame_view<SOA>(base, fi, row_floats, B); };
#if RTG_EXP_TIMESTAMPS
    // measurement knob: lane 0 of each wave of every 8th block records the 100 MHz wall clock at the phase
    // boundaries into the body_rot buffer (tools/side_phases.py): 16 slots per wave, 2 * kSideTiles waves per block
    float *const tsb = body_rot;
    body_rot = nullptr;
    auto TS = [&](int k) {
        if (tsb && (blockIdx.x & 7) == 0 && lane == 0) {
            const uint64_t t = wall_clock64();
            uint32_t *o = reinterpret_cast<uint32_t *>(tsb) + 2 * (((blockIdx.x >> 3) * (2 * kSideTiles) + w) * 16 + k);
            o[0] = (uint32_t)t;
            o[1] = (uint32_t)(t >> 32);
        }
    };
#else
    auto TS = [](int) {};
#endif
    uint32_t st = 0;   // this wave's status bits for its frame (the side kernel keeps per-step flags: lane masks)
    bool fit1_nan = false, fit2_nan = false, euler_refused = false;
    if constexpr (KIND == RTG_SOLVER_FULL_BODY_POS) {
        // Balanced FULL_BODY_POS: left wave = torso fit, then the left wrist fit, then the left Euler split /
        // gripper; right wave = the right wrist fit, then BOTH arm chains (each needs only R10), then the right
        // Euler split / gripper -- 1.5 SVD-equivalents per wave.  Two per-tile LDS flags hand R10 (left -> right)
        // and the left chain (right -> left) over, so each wave waits only for what it reads; a third counts the
        // waves out, and the second one to finish stores the tile's DOF rows while the first exits.
        __shared__ int sflag[kSideTiles][4];   // per tile: [0] R10 ready, [1] left chain ready, [2] waves done, [3] right chain ready
        if (threadIdx.x < 4 * kSideTiles) (&sflag[0][0])[threadIdx.x] = 0;
        // the near-unit normalisation table (rtg_math.cuh), per site: 1 the fits' quaternions, 2 the arm maps'
        // angle-axis quaternions, 4 the Euler split's products (RTG_SIDES_UNIT_TAB for SoA, _AOS for AoS)
        constexpr int kTab = SOA ? RTG_SIDES_UNIT_TAB : RTG_SIDES_UNIT_TAB_AOS;
        __shared__ UnitEnt sut[2 * kUnitTabK + 1];
        if constexpr (kTab != 0) unit_tab_fill(sut, (int)threadIdx.x);
        const auto tabF = TabSel<(kTab & 1) != 0>::get(sut);
        const auto tabA = TabSel<(kTab & 2) != 0>::get(sut);
        const auto tabE = TabSel<(kTab & 4) != 0>::get(sut);
        __syncthreads();
        int *const fl = sflag[w >> 1];
        auto hook1 = [&](int k) { if (k < 2) TS(1 + k); };    // 1: first fit's A formed (its points loaded), 2: its SVD + R done
        auto hook2 = [&](int k) { if (k < 2) TS(10 + k); };   // 10 / 11: the same for the left wave's second fit
        TS(0);
        const auto b = view(in0, 63);
        Q R10 = qident(), W = qident();
        ArmPts apL{}, apR{};
        // AoS (RTG_AOS_PRELOAD_TIPS): the gripper's hand points load with the wrist fit's, while the hand row's lines
        // are in the L2 -- loaded after the arm chains they come back from the MALL or HBM (AoS fetch 1.57x the rows)
        constexpr bool kPreTips = RTG_AOS_PRELOAD_TIPS && !SOA;
        TipPts tpre{};
        // RTG_SIDES_SHARED_FIT: each wave's first fit (left: torso, right: right wrist) forms its A, then both run ONE
        // inlined copy of the SVD's code (the same operations on the same A as cal_joint_quat)
        constexpr bool kSharedFit = RTG_SIDES_SHARED_FIT >= (SOA ? 1 : 2);
        if (live) {
            if constexpr (kSharedFit) {
                float A[9];
                if (!side) {
                    const V b10 = b.p3(10);
                    const V Mt[3] = {vsub(b.p3(17), b10), vsub(b.p3(13), b10), vsub(b.p3(11), b10)};
                    fit1_nan = form_joint_A<3>(C.Zt, Mt, A);
                } else {
                    apL = load_arm<0>(b);
                    apR = load_arm<1>(b);
                    const auto H = view(in2, 60);
                    if (kPreTips) tpre = load_tips(H);
                    const V h0 = H.p3(0);
                    const V M[5] = {vsub(H.p3(2), h0), vsub(H.p3(6), h0), vsub(H.p3(10), h0), vsub(H.p3(14), h0),
                                    vsub(H.p3(17), h0)};
                    fit1_nan = form_joint_A<5>(C.Zr, M, A);
                }
                const Q q = joint_quat_of_A(A, hook1, tabF);
                if (!side) {
                    R10 = q;
                    storso[r] = make_float4(R10.x, R10.y, R10.z, R10.w);
                } else {
                    W = q;
                }
            } else {
                bool nan = false;
                if (!side) {
                    R10 = fbp_torso(C, b, nan, hook1, tabF);
                    storso[r] = make_float4(R10.x, R10.y, R10.z, R10.w);
                    fit1_nan = nan;
                } else {
                    apL = load_arm<0>(b);
                    apR = load_arm<1>(b);
                    if (kPreTips) tpre = load_tips(view(in2, 60));
                    W = fbp_wrist_fit<1>(C, view(in2, 60), nan, hook1, tabF);
                    fit1_nan = nan;
                }
            }
        }
        TS(3);
        if (!side) {
            // R10 of this tile is in storso.  RTG_EXP_SKIP_SIGNAL (measurement knob): block 0's first tile never
            // raises it, so its right wave times out -- the error-word report is tested on that build
            if (!(RTG_EXP_SKIP_SIGNAL && blockIdx.x == 0 && w == 0)) lds_signal(&fl[0]);
        } else {
            lds_wait(&fl[0], C.err);
        }
        TS(4);
        Q chain = qident();
        if (side) {
#if RTG_SIDES_ARMS2
            // both arm chains in one instruction stream (fbp_arms2), then both hand-overs
            if (live) {
                const float4 t = storso[r];   // read R10 before the same lane overwrites the slot with the chain
                R10 = Q{t.x, t.y, t.z, t.w};
                Q cl;
                fbp_arms2(C, apL, apR, R10, E, cl, chain, tabA);
                storso[r] = make_float4(cl.x, cl.y, cl.z, cl.w);
            }
            if (wds) Emit::wait_words();   // the left chain's table words (slots 0-3) have landed in LDS
            lds_signal(&fl[1]);   // the left chain and its exp-map slots 0-3 are in LDS
            if (RTG_SIDES_SPLIT_READOUT) lds_signal(&fl[3]);   // the right chain's exp-map slots 7-10 are in LDS
#else
            if (live) {
                const float4 t = storso[r];   // read R10 before the same lane overwrites the slot with the chain
                R10 = Q{t.x, t.y, t.z, t.w};
                const Q cl = fbp_arm<0>(C, apL, R10, E);
                storso[r] = make_float4(cl.x, cl.y, cl.z, cl.w);
            }
            lds_signal(&fl[1]);   // the left chain and its exp-map slots 0-3 are in LDS
            if (live) chain = fbp_arm<1>(C, apR, R10, E);
            if (RTG_SIDES_SPLIT_READOUT) lds_signal(&fl[3]);   // the right chain's exp-map slots 7-10 are in LDS
#endif
        } else if (live) {
            emit_fixed_links(E);
            bool nan = false;
            if (kPreTips) tpre = load_tips(view(in1, 60));
            W = fbp_wrist_fit<0>(C, view(in1, 60), nan, hook2, tabF);
            fit2_nan = nan;
        }
        TS(5);
        if (!side) lds_wait(&fl[1], C.err);
        TS(6);
        if (live) {
            float *brow = body_rot ? body_rot + f * 236 : nullptr;
            const TipPts tp = kPreTips ? tpre : load_tips(view(side ? in2 : in1, 60));
            if (side) {
                euler_refused = fbp_side_after_arm<PRECISE, 1>(C, tp, R10, chain, W, E, brow, tabE);
            } else {
                const float4 c = storso[r];
                euler_refused = fbp_side_after_arm<PRECISE, 0>(C, tp, R10, Q{c.x, c.y, c.z, c.w}, W, E, brow, tabE);
            }
        }
        TS(7);
        // exp-map read-out: the left wave reads slots 0-6 (the left chain's 0-3, written by the right wave before
        // the flag, and its own wrist's 4-6), the right wave 7-13 (all its own).  RTG_SIDES_SPLIT_READOUT: the left
        // wave (the shorter program) also reads the right chain's slots 7-10, after the right wave's flag for them
        if (RTG_SIDES_SPLIT_READOUT) {
            if (side) {
                if (live) E.finalize(11, 3);
            } else {
                if (live) E.finalize(0, 7);
                lds_wait(&fl[3], C.err);
                if (live) E.finalize(7, 4);
            }
        } else if (live) {
            E.finalize(side ? 7 : 0, 7);
        }
        st = side ? ((fit1_nan ? kStRightSvd : 0u) | (euler_refused ? kStRightEuler : 0u))
                  : ((fit1_nan ? kStTorsoSvd : 0u) | (fit2_nan ? kStLeftSvd : 0u) | (euler_refused ? kStLeftEuler : 0u));
        sstat[side][r] = (uint8_t)st;
        TS(8);
        // The tile's two waves meet at an LDS counter instead of the block barrier: the first to arrive exits (its
        // VGPRs free for the next block, whose LDS already fits beside this one's), the second stores the tile's
        // rows.  Release by every lane before the counter, acquire by every lane of the storing wave after it: the
        // first wave's sdof / sstat writes are visible to the second wave's reads below.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        const uint64_t joined = __builtin_amdgcn_ballot_w64(true);
        const int first = __builtin_ctzll(joined);
        int prev = 0;
        if (lane == first) prev = __hip_atomic_fetch_add(&fl[2], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_readlane(prev, first) == 0) {
            TS(9);
            TS(12);
            return;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        TS(9);
        const int64_t t0 = f0 + (w >> 1) * 64;
        const int64_t nrows = (B - t0) < 64 ? (B - t0) : 64;
        if (nrows <= 0) return;
        float *const tile = sdof + (w >> 1) * 64 * kDofStride;
        const uint32_t bits = live ? (uint32_t)(sstat[0][r] | sstat[1][r]) : 0u;
        if (__builtin_amdgcn_ballot_w64(bits != 0u)) {   // rare: a frame the reference raises on
            if (bits) {
                const int64_t fr = t0 + lane;
                poison_frame(tile + lane * kDofStride, local_rot ? local_rot + fr * 124 : nullptr,
                             body_rot ? body_rot + fr * 236 : nullptr, bits);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // the patched rows before the cross-lane reads
        }
        store_dof_rows(dof + t0 * 30, tile, nrows, lane, 64);   // (f0 + 64 t) * 120 bytes: 16-byte aligned
        TS(12);
        return;
    } else {
        TS(0);
        if constexpr (KIND == RTG_SOLVER_UPPER_BODY) {
            // The torso fit is shared by both sides: the left wave fits it, then one block barrier hands R10 over
            // LDS (nothing for the right wave to overlap with it here).
            const auto b = view(in0, 63);   // mocap points (B, 21, 3)
            Q R10 = qident();
            // the near-unit normalisation table for the arm maps (RTG_UPPER_UNIT_TAB), filled by the right waves while
            // the left ones fit the torso
            __shared__ UnitEnt sut[2 * kUnitTabK + 1];
            if (RTG_UPPER_UNIT_TAB && side) unit_tab_fill(sut, lane);
            const auto tab = TabSel<RTG_UPPER_UNIT_TAB != 0>::get(sut);
            if (live && !side) {
                bool nan = false;
                R10 = upper_torso(C, b, nan);
                storso[r] = make_float4(R10.x, R10.y, R10.z, R10.w);
                st |= nan ? kStTorsoSvd : 0u;
            }
            __syncthreads();
            if (live) {
                if (side) {
                    const float4 t = storso[r];
                    R10 = Q{t.x, t.y, t.z, t.w};
                    solve_upper_side<1>(C, b, R10, E, tab);
                } else {
                    emit_fixed_links(E);
                    solve_upper_side<0>(C, b, R10, E, tab);
                }
            }
        } else {
            // the near-unit normalisation table (RTG_ROT_UNIT_TAB, FULL_BODY_ROT: 56.5-57.0 -> 53.9-54.8 us; BODY_ROT
            // measured 2 % slower with it, off): one copy per wave, filled by ALL its lanes (live or not: a batch's last
            // tile has idle lanes) and read by the wave itself (its LDS operations execute in order; the fences keep
            // the compiler from reordering them)
            constexpr bool kRotTab = RTG_ROT_UNIT_TAB && KIND == RTG_SOLVER_FULL_BODY_ROT;
            __shared__ UnitEnt sutw[2 * kSideTiles][2 * kUnitTabK + 1];
            if (kRotTab) {
                unit_tab_fill(sutw[w], lane);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            const auto tab = TabSel<kRotTab>::get(sutw[w]);
            if (live) {
                if (!side) emit_fixed_links(E);
                bool refused;
                if constexpr (KIND == RTG_SOLVER_FULL_BODY_ROT) {
                    refused = side ? solve_full_body_rot_side<1>(C, view(in0, 84), view(in1, 63), view(in3, 60), E, tab)
                                   : solve_full_body_rot_side<0>(C, view(in0, 84), view(in1, 63), view(in2, 60), E, tab);
                } else {
                    refused = side ? solve_body_rot_side<1>(C, view(in0, 84), E, tab)
                                   : solve_body_rot_side<0>(C, view(in0, 84), E, tab);
                }
                st |= refused ? (side ? kStRightEuler : kStLeftEuler) : 0u;
            }
        }
        if (live) E.finalize(side ? 7 : 0, 7);   // each wave reads out its own side's slots
        sstat[side][r] = (uint8_t)st;
        TS(8);
        __syncthreads();
        TS(9);
        const uint32_t bits = (live && !side) ? (uint32_t)(sstat[0][r] | sstat[1][r]) : 0u;
        if (__syncthreads_or(bits != 0u)) {   // rare: a frame the reference raises on (one writer per row)
            if (bits) poison_frame(E.row, lrow, nullptr, bits);
            __syncthreads();
        }
        const int64_t nrows = (B - f0) < kSideFrames ? (B - f0) : kSideFrames;
        store_dof_rows(dof + f0 * 30, sdof, nrows, threadIdx.x, kSideThreads);
        TS(12);
    }
}

// ----------------------------------------------------------------------------
// FULL_BODY_POS for small batches (the teleop / config-2 latency path): five waves per 64-frame tile.  The arm
// chain (shoulder_pr / elbow_py, full_body_pos_retargeter.py:75-93) needs only the torso fit R10, not the wrist
// fit, so it runs on its own wave as soon as R10 is in LDS -- concurrently with the (longer) wrist SVDs -- instead
// of after all three fits (measured phase split, tools/latency_phases.py: torso fit 6-8 us, wrist fits 9-13 us,
// arm 5-7 us, Euler 3-4 us).
//   wave 0      torso fit -> R10 -> fixed links
//   wave 1, 2   left / right wrist fit -> gripper; then (arm chain ready) Euler split, body_rot rows, exp-maps
//   wave 3, 4   left / right arm points; (R10 ready) arm chain -> LDS; the arm links' exp-maps
// Every value is computed by the same device function from the same operands as in k_solve_sides: the same bits
// (test_solver_batch_invariance covers both sizes).
// ----------------------------------------------------------------------------
constexpr int kLatFrames = 64;

// one 64-frame tile (frames f0..) by the 320 threads of a workgroup
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
    __shared__ uint8_t sstat[3][kLatFrames];   // status bits of the torso wave and the two wrist waves
    __shared__ UnitEnt sut[2 * kUnitTabK + 1];   // the near-unit normalisation table (RTG_LAT_UNIT_TAB)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t f = f0 + lane;
    const bool live = f < B;
    if (threadIdx.x < 3) sflag[threadIdx.x] = 0;
    if (RTG_LAT_UNIT_TAB) unit_tab_fill(sut, (int)threadIdx.x - 256);   // wave 4 (the arm wave with the least to do)
    const auto tabF = TabSel<(RTG_LAT_UNIT_TAB & 1) != 0>::get(sut);
    const auto tab = TabSel<(RTG_LAT_UNIT_TAB & 6) != 0>::get(sut);
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
    auto hook = [&](int k) { if (k < 2) TS(8 + k); };
    TS(0);
    float *const lrow = live && local_rot ? local_rot + f * 124 : nullptr;
    const Emit E{sdof + lane * kDofStride, lrow, C.ang_tab, sst + lane, kLatFrames};
    auto view = [&](const float *base, int row_floats) { return frame_view<SOA>(base, f, row_floats, B); };
    const auto b = view(in0, 63);
    bool fit_nan = false, euler_refused = false;   // this wave's raise points (lane masks, not a VGPR)
    // RTG_LAT5_SHARED_CODE: the three fits form their A per wave and run ONE inlined copy of the SVD; the two waves
    // of each side pair run one copy of their code (run-time side); the same operations on the same operands
    constexpr bool kShared = RTG_LAT5_SHARED_CODE != 0;
    Q fitq = qident();
    if (kShared && w < 3 && live) {
        float A[9];
        if (w == 0) {
            const V b10 = b.p3(10);
            const V Mt[3] = {vsub(b.p3(17), b10), vsub(b.p3(13), b10), vsub(b.p3(11), b10)};
            fit_nan = form_joint_A<3>(C.Zt, Mt, A);
        } else {
            const auto H = view(w == 2 ? in2 : in1, 60);
            const V h0 = H.p3(0);
            const V M[5] = {vsub(H.p3(2), h0), vsub(H.p3(6), h0), vsub(H.p3(10), h0), vsub(H.p3(14), h0),
                            vsub(H.p3(17), h0)};
            V Z[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) Z[k] = w == 2 ? C.Zr[k] : C.Zl[k];
            fit_nan = form_joint_A<5>(Z, M, A);
        }
        fitq = joint_quat_of_A(A, hook, tabF);
    }
    if (w == 0) {
        if (live) {
            bool nan = false;
            const Q q = kShared ? fitq : fbp_torso(C, b, nan, hook, tabF);
            sfit[lane] = make_float4(q.x, q.y, q.z, q.w);
            if (!kShared) fit_nan = nan;
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
        lds_wait(&sflag[0], C.err);
        TS(2);
        if (live) {
            const float4 t = sfit[lane];
            const Q R10{t.x, t.y, t.z, t.w};
            const V up = vsub(ap.el, ap.sh), fo = vsub(ap.wr, ap.el);
            const Q ch = kShared ? solve_arm_rt(E, side ? 21 : 12, up, fo, side ? C.rsh : C.lsh, side ? C.rel : C.lel, R10, tab)
                         : side ? solve_arm<21>(E, up, fo, C.rsh, C.rel, R10, tab)
                                : solve_arm<12>(E, up, fo, C.lsh, C.lel, R10, tab);
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
            if (kShared) {
                W = fitq;
            } else {
                bool nan = false;
                W = side ? fbp_wrist_fit<1>(C, H, nan, hook, tabF) : fbp_wrist_fit<0>(C, H, nan, hook, tabF);
                fit_nan = nan;
            }
            tp = load_tips(H);
        }
        TS(1);
        float a = 0.0f;
        if (live) a = hand_x_mean(qconj(W), tp.h0, tp.t);   // the gripper needs only W (:142-158 / :165-175)
        TS(2);
        lds_wait(&sflag[1 + side], C.err);   // the arm waited for R10 first: both are visible (release / acquire chain)
        TS(3);
        if (live) {
            const float4 t = sfit[lane], c = schain[side][lane];
            const Q R10{t.x, t.y, t.z, t.w}, chain{c.x, c.y, c.z, c.w};
            float *brow = body_rot ? body_rot + f * 236 : nullptr;
            fbp_gripper<PRECISE>(C, a, E.row + (side ? 27 : 18));
            const Q loc = qnormalize_t(qmul(qconj(qnormalize_t(qmul(R10, chain), tab)), W), tab);
            euler_refused = kShared ? emit_euler_xyz_rt(E, side ? 25 : 16, loc)
                                    : side ? emit_euler_xyz<25>(E, loc) : emit_euler_xyz<16>(E, loc);
            if (brow) {
                if (side) fbp_body_rows<1>(brow, R10, W);
                else fbp_body_rows<0>(brow, R10, W);
            }
            TS(4);
            E.finalize(side ? 11 : 4, 3);
        }
    }
    if (w < 3) {
        const uint32_t svd_bit = w == 0 ? kStTorsoSvd : (w == 1 ? kStLeftSvd : kStRightSvd);
        sstat[w][lane] = (uint8_t)((fit_nan ? svd_bit : 0u) | (euler_refused ? (w == 1 ? kStLeftEuler : kStRightEuler) : 0u));
    }
    TS(5);
    __syncthreads();
    TS(6);
    const uint32_t bits = (w == 0 && live) ? (uint32_t)(sstat[0][lane] | sstat[1][lane] | sstat[2][lane]) : 0u;
    if (__syncthreads_or(bits != 0u)) {   // rare: a frame the reference raises on
        if (bits) poison_frame(E.row, local_rot ? local_rot + f * 124 : nullptr, body_rot ? body_rot + f * 236 : nullptr, bits);
        __syncthreads();
    }
    const int64_t nrows = (B - f0) < kLatFrames ? (B - f0) : kLatFrames;
    store_dof_rows(dof + f0 * 30, sdof, nrows, threadIdx.x, 320);   // f0 * 30 floats: 16-byte aligned
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
// ONE frame (B = 1: the teleop path -- k_frame_server and rtg_retarget_f32 at B = 1) on k_fbp_latency5's five
// waves, with the frame's independent sub-steps on separate LANES of a wave (they idle at B = 1 otherwise):
//   * each arm map (cal_shoulderPR / cal_elbowP_and_shoulderY): the pitch (yaw) angle on lane 0, the roll (elbow)
//     angle on lane 1 -- one radians_between + one quat_from_angle_axis instruction stream instead of two;
//   * the scipy Euler split of each wrist: its three atan2 on lanes 0-2, then one elementary quaternion per lane;
//   * the exp-map DOF read-out: one link per lane.
// Every value is computed by the same device functions on the same operands as in the batched kernels (the pitch
// angle as radians_between of the exact unit axes, which is radians_between_axes bit for bit), so the bits are the
// batched kernels' (test_frame_server_matches_batched, test_solver_batch_invariance).  Partial results cross
// lanes by v_readlane.
// ----------------------------------------------------------------------------
RTG_DEV float rdl(float v, int l) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l)); }
RTG_DEV double rdl(double v, int l)
{
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
RTG_DEV Q rdl(Q q, int k) { return Q{rdl(q.x, k), rdl(q.y, k), rdl(q.z, k), rdl(q.w, k)}; }
// Broadcast of sub-lane K within this lane's group of G lanes: G = 64, the wave (v_readlane: k_fbp_frame1, one frame
// per block); G = 4, a quad (DPP quad_perm, one VALU op: k_fbp_quad, one frame per quad).  Called where every lane of
// the group is active (DPP reads an inactive source lane as 0).
template <int G, int K>
RTG_DEV float gbc(float v)
{
    static_assert(G == 64 || G == 4, "group of 64 or 4 lanes");
    if constexpr (G == 64) return rdl(v, K);
    else return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), K * 0x55, 0xF, 0xF, false));
}
template <int G, int K>
RTG_DEV double gbc(double v)
{
    if constexpr (G == 64) return rdl(v, K);
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_bit_cast(uint32_t, gbc<G, K>(__builtin_bit_cast(float, (uint32_t)u)));
    const uint32_t hi = __builtin_bit_cast(uint32_t, gbc<G, K>(__builtin_bit_cast(float, (uint32_t)(u >> 32))));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <int G, int K>
RTG_DEV Q gbc(Q q) { return Q{gbc<G, K>(q.x), gbc<G, K>(q.y), gbc<G, K>(q.z), gbc<G, K>(q.w)}; }
template <int G>
RTG_DEV int sublane() { return (int)(threadIdx.x & (G - 1)); }

// shoulder_pr (SHOULDER) / elbow_py of the frame: sub-lane 0 the first angle's quaternion, sub-lane 1 the second's
template <bool SHOULDER, int G = 64, typename Hook = NoHook, typename Tab = NoTab>
RTG_DEV void arm_pair_lanes(V v1, ArmZero z0, Q parent, Q &first, Q &second, const Hook &hook = Hook{}, Tab tab = Tab{})
{
    const int sub = sublane<G>();
    Q q = qident();
    if (sub < 2) {
        const V ex{1.f, 0.f, 0.f}, ey{0.f, 1.f, 0.f}, ez{0.f, 0.f, 1.f};
        const V pn = SHOULDER ? ey : ez;   // the plane of the first angle
        const V v1r = qrotate(qconj(parent), v1);
        hook(0);
        const V v1p = proj_in_plane(v1r, pn);
        hook(1);
        const bool l0 = sub == 0;
        const V a{l0 ? 1.f : v1p.x, l0 ? 0.f : v1p.y, l0 ? 0.f : v1p.z};
        const V b = l0 ? v1p : v1r;
        const V c = SHOULDER ? cross3(v1p, ey) : cross3(ez, v1p);
        const V n = l0 ? pn : c;
        const float ang = radians_between(a, b, n);
        hook(2);
        const V ax = l0 ? pn : (SHOULDER ? ex : ey);
        q = qfrom_angle_unit_axis_t(ang - (l0 ? z0.th0 : z0.ph0), ax, tab);
        hook(3);
    }
    first = gbc<G, 0>(q);
    second = gbc<G, 1>(q);
}
template <int L0, int G = 64, typename Hook = NoHook, typename Tab = NoTab>
RTG_DEV Q solve_arm_lanes(const Emit &E, V upper, V fore, ArmZero zs, ArmZero ze, Q parent, const Hook &hook = Hook{},
                          Tab tab = Tab{})
{
    const bool w0 = sublane<G>() == 0;
    Q p, r, y, e;
    arm_pair_lanes<true, G>(upper, zs, parent, p, r, [&](int k) { hook(k); }, tab);
    if (w0) { E.link<L0>(p); E.link<L0 + 1>(r); }
    arm_pair_lanes<false, G>(fore, ze, qmul(qmul(parent, p), r), y, e, [&](int k) { hook(4 + k); }, tab);
    if (w0) { E.link<L0 + 2>(y); E.link<L0 + 3>(e); }
    return qmul(qmul(qmul(p, r), y), e);
}
// solve_arm_lanes with a run-time first link (both arm waves of the B = 1 kernel run one copy; link_rt writes what
// Emit::link writes when the wave has no early table words, as there)
template <int G = 64, typename Hook = NoHook, typename Tab = NoTab>
RTG_DEV Q solve_arm_lanes_rt(const Emit &E, int L0, V upper, V fore, ArmZero zs, ArmZero ze, Q parent,
                             const Hook &hook = Hook{}, Tab tab = Tab{})
{
    const bool w0 = sublane<G>() == 0;
    Q p, r, y, e;
    arm_pair_lanes<true, G>(upper, zs, parent, p, r, [&](int k) { hook(k); }, tab);
    if (w0) { link_rt(E, L0, p); link_rt(E, L0 + 1, r); }
    arm_pair_lanes<false, G>(fore, ze, qmul(qmul(parent, p), r), y, e, [&](int k) { hook(4 + k); }, tab);
    if (w0) { link_rt(E, L0 + 2, y); link_rt(E, L0 + 3, e); }
    return qmul(qmul(qmul(p, r), y), e);
}
// emit_euler_xyz (quat_in_xyz_axis 'XYZ', scipy_as_euler's arithmetic) with the three atan2 on sub-lanes 0-2 and one
// elementary quaternion per sub-lane; every lane of the group holds the same qf, so every lane returns the same
// refusal flag
template <int G = 64>
RTG_DEV bool emit_euler_xyz_lanes_rt(const Emit &E, int L0, Q qf)
{
    const int sub = sublane<G>();
    {   // round 5: the atan2-free split (quat_in_xyz_fast, same values) on every lane -- qf is the same on all lanes
        // of the group, so the branch is uniform in it; where it declines, the lane-parallel scipy restatement runs
        Q eul[3];
        if (quat_in_xyz_fast(qf, eul)) {   // implies |q| > 0: scipy does not refuse it
            // per-component selects (an indexed eul[sub] went through scratch memory)
            const bool s0 = sub == 0, s1 = sub == 1;
            const Q e{s0 ? eul[0].x : (s1 ? eul[1].x : eul[2].x), s0 ? eul[0].y : (s1 ? eul[1].y : eul[2].y),
                      s0 ? eul[0].z : (s1 ? eul[1].z : eul[2].z), s0 ? eul[0].w : (s1 ? eul[1].w : eul[2].w)};
            if (sub < 3) link_rt(E, L0 + sub, e);
            return false;
        }
    }
    // scipy_as_euler(q, 0, 1, 2, intrinsic): i = 2, j = 1, k = 0, not symmetric, sign = (2-1)(1-0)(0-2)/2 = -1
    double q[4] = {(double)qf.x, (double)qf.y, (double)qf.z, (double)qf.w};
    const double nrm = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const bool refused = !(nrm > 0.0);
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
    ang[1] = 2.0 * gbc<G, 0>(at);
    const double half_sum = gbc<G, 1>(at), half_diff = gbc<G, 2>(at);
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
    if (sub < 3) link_rt(E, L0 + sub, elementary_quat(sub, sub == 0 ? ang[0] : (sub == 1 ? ang[1] : ang[2])));
    return refused;
}
template <int L0, int G = 64>
RTG_DEV bool emit_euler_xyz_lanes(const Emit &E, Q qf)
{
    return emit_euler_xyz_lanes_rt<G>(E, L0, qf);
}
// Emit::finalize with one slot per sub-lane (slots s0 .. s0 + n - 1, n <= G)
template <int G = 64>
RTG_DEV void finalize_lanes(const Emit &E, int s0, int n)
{
    const int sub = sublane<G>();
    if (sub < n) {
        const int j = s0 + sub;
        const float2 v = E.st[j * E.sst];
        const ExpDof e = exp_dof_table_part(v.x, E.ang);
        float val = exp_dof_finish(e, v.y);
        if (__builtin_expect(e.exact, 0)) val = normalize_angle(2.0f * cr_acos(v.x)) * (v.y / e.sin_theta);
        E.row[j < 7 ? 11 + j : 13 + j] = val;
    }
}

// The frame whose rows (body 63 | left hand 60 | right hand 60 floats) are in `rows` (LDS); dof / local_rot /
// body_rot point at the frame's output rows
// const_rows false (the frame server, once its output buffers hold them): the rows that are the same for every
// frame -- the 17 fixed links of local_rot and the 56 identity rows of body_rot -- are not rewritten; they are still
// in the server's own pinned output rows from an earlier frame.  Returns the frame's status bits (block-uniform).
// tab: the near-unit normalisation table, filled and made visible by the caller (or NoTab)
template <bool PRECISE, typename Tab = NoTab, typename TabF = NoTab>
RTG_DEV uint32_t fbp_frame1_tile(const SolverConsts &C, const float *rows, float *__restrict__ dof,
                                 float *__restrict__ local_rot, float *__restrict__ body_rot, bool const_rows = true,
                                 Tab tab = Tab{}, TabF tabF = TabF{})
{
    __shared__ float sdof[kDofStride];
    __shared__ float4 sfit, schain[2];
    __shared__ float2 sst[14];
    __shared__ int sflag[3];       // R10 ready, left arm ready, right arm ready
    __shared__ uint32_t sstat[3];  // status bits of the torso wave and the two wrist waves
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool w0 = lane == 0;
#if RTG_EXP_TIMESTAMPS
    // measurement knob: lane 0 of each wave records the 100 MHz wall clock at its stage boundaries into body_rot
    // (16 u32 pairs per wave; tools/latency_phases.py frame1): 0 start; fits (waves 0-2): 1 A formed, 2 SGEBD2 done,
    // 3 SBDSQR done, 4 rotation done; wave 0: 5 R10 signalled; waves 1 / 2: 5 gripper done, 6 arm chain received,
    // 7 Euler split done, 8 read-out done; waves 3 / 4: 1 points loaded, 6 R10 received, 8-11 the shoulder pair (parent
    // rotated, projected, angle, quaternion), 12 the elbow pair's quaternion, 7 arm chain done, 13 read-out done; every
    // wave: 14 at the final barrier, 15 past it
    float *const tsb = body_rot;
    body_rot = nullptr;
    auto TS = [&](int k) {
        if (tsb && lane == 0) {
            const uint64_t t = wall_clock64();
            reinterpret_cast<uint32_t *>(tsb)[2 * (16 * w + k)] = (uint32_t)t;
            reinterpret_cast<uint32_t *>(tsb)[2 * (16 * w + k) + 1] = (uint32_t)(t >> 32);
        }
    };
#else
    auto TS = [](int) {};
#endif
    auto hook = [&](int k) { TS(k == 0 ? 1 : (k == 10 ? 2 : (k == 11 ? 3 : 4))); };
    TS(0);
    if (threadIdx.x < 3) sflag[threadIdx.x] = 0;
    __syncthreads();
    const Emit E{sdof, local_rot, C.ang_tab, sst, 1};
    const FV<false> b{rows};
    uint32_t st = 0;
#if RTG_FRAME1_SHARED_CODE >= 3
    // the three fits (torso on wave 0, the wrists on waves 1 / 2) form their A per wave and then run ONE inlined copy of
    // the SVD's code (the same operations on the same A as cal_joint_quat)
    Q fitq = qident();
    bool fit_nan = false;
    if (w < 3 && w0) {
        float A[9];
        if (w == 0) {
            const V b10 = b.p3(10);
            const V Mt[3] = {vsub(b.p3(17), b10), vsub(b.p3(13), b10), vsub(b.p3(11), b10)};
            fit_nan = form_joint_A<3>(C.Zt, Mt, A);
        } else {
            const FV<false> H{rows + (w == 2 ? 123 : 63)};
            const V h0 = H.p3(0);
            const V M[5] = {vsub(H.p3(2), h0), vsub(H.p3(6), h0), vsub(H.p3(10), h0), vsub(H.p3(14), h0),
                            vsub(H.p3(17), h0)};
            V Z[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) Z[k] = w == 2 ? C.Zr[k] : C.Zl[k];
            fit_nan = form_joint_A<5>(Z, M, A);
        }
        fitq = joint_quat_of_A(A, hook, tabF);
    }
#endif
    if (w == 0) {
        if (w0) {
#if RTG_FRAME1_SHARED_CODE >= 3
            const Q q = fitq;
            const bool nan = fit_nan;
#else
            bool nan = false;
            const Q q = fbp_torso(C, b, nan, hook, tabF);
#endif
            sfit = make_float4(q.x, q.y, q.z, q.w);
            st = nan ? kStTorsoSvd : 0u;
        }
        lds_signal(&sflag[0]);
        TS(5);
        if (w0) emit_fixed_links(E, const_rows);
    } else if (w >= 3) {
        const int side = w - 3;
        const ArmPts ap = side ? load_arm<1>(b) : load_arm<0>(b);
        TS(1);
        lds_wait(&sflag[0], C.err);
        TS(6);
        const float4 t = sfit;
        const Q R10{t.x, t.y, t.z, t.w};
        const V up = vsub(ap.el, ap.sh), fo = vsub(ap.wr, ap.el);
        auto ahook = [&](int k) {   // arm stages: 8 + (0 rotated, 1 projected, 2 angle, 3 quaternion); 12 the elbow's quaternion
            if (k < 4) TS(8 + k);
            else if (k == 7) TS(12);
        };
#if RTG_FRAME1_SHARED_CODE
        const Q ch = solve_arm_lanes_rt(E, side ? 21 : 12, up, fo, side ? C.rsh : C.lsh, side ? C.rel : C.lel, R10, ahook,
                                        tab);
#else
        const Q ch = side ? solve_arm_lanes<21>(E, up, fo, C.rsh, C.rel, R10, ahook, tab)
                          : solve_arm_lanes<12>(E, up, fo, C.lsh, C.lel, R10, ahook, tab);
#endif
        if (w0) schain[side] = make_float4(ch.x, ch.y, ch.z, ch.w);
        lds_signal(&sflag[1 + side]);
        TS(7);
        finalize_lanes(E, side ? 7 : 0, 4);
        TS(13);
    } else {
        const int side = w - 1;
        const FV<false> H{rows + (side ? 123 : 63)};
        Q W = qident();
        float a = 0.0f;
        if (w0) {
            bool nan = false;
#if RTG_FRAME1_SHARED_CODE >= 3
            W = fitq;
            nan = fit_nan;
#elif RTG_FRAME1_SHARED_CODE
            W = fbp_wrist_fit_rt(C, H, side, nan, hook, tabF);
#else
            W = side ? fbp_wrist_fit<1>(C, H, nan, hook, tabF) : fbp_wrist_fit<0>(C, H, nan, hook, tabF);
#endif
            st = nan ? (side ? kStRightSvd : kStLeftSvd) : 0u;
            const TipPts tp = load_tips(H);
            a = hand_x_mean(qconj(W), tp.h0, tp.t);   // the gripper needs only W (:142-158 / :165-175)
        }
        W = gbc<64, 0>(W);
        TS(5);
        lds_wait(&sflag[1 + side], C.err);   // the arm waited for R10 first: both are visible (release / acquire chain)
        TS(6);
        const float4 t = sfit, c = schain[side];
        const Q R10{t.x, t.y, t.z, t.w}, chain{c.x, c.y, c.z, c.w};
        if (w0) {
            fbp_gripper<PRECISE>(C, a, E.row + (side ? 27 : 18));
            if (body_rot) {
                if (side) fbp_body_rows<1>(body_rot, R10, W);
                else fbp_body_rows<0>(body_rot, R10, W, const_rows);
            }
        }
        const Q loc = qnormalize_t(qmul(qconj(qnormalize_t(qmul(R10, chain), tab)), W), tab);
#if RTG_FRAME1_SHARED_CODE
        const bool refused = emit_euler_xyz_lanes_rt(E, side ? 25 : 16, loc);
#else
        const bool refused = side ? emit_euler_xyz_lanes<25>(E, loc) : emit_euler_xyz_lanes<16>(E, loc);
#endif
        st |= refused ? (side ? kStRightEuler : kStLeftEuler) : 0u;
        TS(7);
        finalize_lanes(E, side ? 11 : 4, 3);
        TS(8);
    }
    if (w < 3 && w0) sstat[w] = st;
    TS(14);
    __syncthreads();
    TS(15);
    const uint32_t bits = sstat[0] | sstat[1] | sstat[2];   // block-uniform
    if (bits) {   // rare: the reference raises on this frame
        if (threadIdx.x == 0) poison_frame(sdof, local_rot, body_rot, bits);
        __syncthreads();
    }
    if (threadIdx.x < 30) dof[threadIdx.x] = sdof[threadIdx.x];
    return bits;
}
// The frame's 183 input floats cross into LDS once, all loads in flight together (one round trip even from host
// memory).  At B = 1 the SoA planes (P, C, 1) are the AoS rows, so one kernel serves both layouts.
template <bool PRECISE>
__global__ __launch_bounds__(320) void k_fbp_frame1(SolverConsts C, const float *__restrict__ in0,
                                                    const float *__restrict__ in1, const float *__restrict__ in2,
                                                    float *__restrict__ dof, float *__restrict__ local_rot,
                                                    float *__restrict__ body_rot)
{
    __shared__ float rows[184];
    __shared__ UnitEnt sut[2 * kUnitTabK + 1];   // the near-unit normalisation table (RTG_FRAME1_UNIT_TAB)
    if (threadIdx.x < 183) {
        const int e = threadIdx.x;
        rows[e] = e < 63 ? in0[e] : (e < 123 ? in1[e - 63] : in2[e - 123]);
    }
    if (RTG_FRAME1_UNIT_TAB) unit_tab_fill(sut, (int)threadIdx.x - 256);   // wave 4, while the rows are in flight
    __syncthreads();
    fbp_frame1_tile<PRECISE>(C, rows, dof, local_rot, body_rot, true, TabSel<(RTG_FRAME1_UNIT_TAB & 6) != 0>::get(sut),
                             TabSel<(RTG_FRAME1_UNIT_TAB & 1) != 0>::get(sut));
}

// ----------------------------------------------------------------------------
// FULL_BODY_POS for small batches (round 5, config 2): k_fbp_frame1's lane-parallel frame program on 16 frames per
// block, one frame per QUAD of lanes.  k_fbp_latency5 puts 64 frames in a block, so B = 4096 fills 64 of the 256
// CUs and each frame's chain runs its sub-steps one after another; here the same 4096 frames are 256 blocks (every
// CU), and inside a frame the sub-steps that k_fbp_frame1 spreads over lanes -- the arm maps' two angles, the three
// Euler elementary quaternions, up to four exp-map read-outs -- run on the quad's four lanes, their partial results
// crossing by DPP quad broadcasts.  The waves' roles are k_fbp_latency5's (0 torso fit, 1 / 2 wrist fits then the
// Euler split, 3 / 4 arm chains).  Every value comes from the same device functions on the same operands: the same
// bits (test_solver_batch_invariance, the GPU parity suite).
// ----------------------------------------------------------------------------
// FPB frames per block: 16 (one per lane quad) or 8 (the upper eight quads of each wave repeat the lower eight --
// same rows, same values, never stored): at one block per CU the eight-frame tile runs each SVD at the slowest of 8
// frames' sweep counts instead of 16 (measured 15.3 vs 16.4 us for B <= 2048; launch_fbp_small_kind)
template <bool PRECISE, bool SOA, int FPB>
__global__ __launch_bounds__(320) void k_fbp_quad(SolverConsts C, const float *__restrict__ in0,
                                                  const float *__restrict__ in1, const float *__restrict__ in2,
                                                  int64_t B, float *__restrict__ dof, float *__restrict__ local_rot,
                                                  float *__restrict__ body_rot)
{
    static_assert(FPB == 16 || FPB == 8, "k_fbp_quad: 8 or 16 frames per block");
    constexpr int kQuadFrames = FPB, kQuadLog2 = FPB == 16 ? 4 : 3;
    constexpr int RP = 184;                      // LDS row pitch of a frame: body 63 | left hand 60 | right hand 60
    __shared__ float rows[kQuadFrames * RP];
    __shared__ float sdof[kQuadFrames * kDofStride];
    __shared__ float4 sfit[kQuadFrames], schain[2][kQuadFrames];
    __shared__ float2 sst[kQuadFrames * 14];
    __shared__ int sflag[3];                     // R10 ready, left arm ready, right arm ready
    __shared__ uint8_t sstat[3][kQuadFrames];    // status bits of the torso wave and the two wrist waves
    __shared__ UnitEnt sut[2 * kUnitTabK + 1];   // the near-unit normalisation table (RTG_LAT_UNIT_TAB)
    const auto tabF = TabSel<(RTG_LAT_UNIT_TAB & 1) != 0>::get(sut);
    const auto tab = TabSel<(RTG_LAT_UNIT_TAB & 6) != 0>::get(sut);
    const int64_t f0 = (int64_t)blockIdx.x * kQuadFrames;
    const int nf = (int)((B - f0) < kQuadFrames ? (B - f0) : kQuadFrames);
    // the tile's rows into LDS, all loads in flight together; a frame slot past B repeats the last frame (every lane
    // runs the whole program -- the DPP broadcasts need the full quad -- and only live frames store)
    if (SOA) {
        for (int i = threadIdx.x; i < kQuadFrames * 183; i += 320) {
            const int q = i & (kQuadFrames - 1), e = i >> kQuadLog2;   // consecutive frames of one component
            const int64_t f = f0 + (q < nf ? q : nf - 1);
            rows[q * RP + e] = e < 63 ? in0[e * B + f] : (e < 123 ? in1[(e - 63) * B + f] : in2[(e - 123) * B + f]);
        }
    } else {
        for (int i = threadIdx.x; i < kQuadFrames * 183; i += 320) {
            const int q = i / 183, e = i - q * 183;
            const int64_t f = f0 + (q < nf ? q : nf - 1);
            rows[q * RP + e] = e < 63 ? in0[f * 63 + e] : (e < 123 ? in1[f * 60 + (e - 63)] : in2[f * 60 + (e - 123)]);
        }
    }
    if (threadIdx.x < 3) sflag[threadIdx.x] = 0;
    if (RTG_LAT_UNIT_TAB) unit_tab_fill(sut, (int)threadIdx.x - 256);   // wave 4, while the rows are in flight
    __syncthreads();
    // with 8 frames per block a wave's upper 8 quads repeat the lower 8 (same rows, same values, never stored)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, qq = lane >> 2, q = qq & (kQuadFrames - 1), sub = lane & 3;
    const int64_t f = f0 + q;
    const bool live = qq < nf;
    const Emit E{sdof + q * kDofStride, live && local_rot ? local_rot + f * 124 : nullptr, C.ang_tab, sst + q * 14, 1};
    const FV<false> b{rows + q * RP};
    uint32_t st = 0;
#if RTG_QUAD_SHARED_CODE >= 3
    // the three fits share one inlined copy of the SVD's code (k_fbp_frame1's level 3)
    Q fitq = qident();
    bool fit_nan = false;
    if (w < 3 && sub == 0) {
        float A[9];
        if (w == 0) {
            const V b10 = b.p3(10);
            const V Mt[3] = {vsub(b.p3(17), b10), vsub(b.p3(13), b10), vsub(b.p3(11), b10)};
            fit_nan = form_joint_A<3>(C.Zt, Mt, A);
        } else {
            const FV<false> H{rows + q * RP + (w == 2 ? 123 : 63)};
            const V h0 = H.p3(0);
            const V M[5] = {vsub(H.p3(2), h0), vsub(H.p3(6), h0), vsub(H.p3(10), h0), vsub(H.p3(14), h0),
                            vsub(H.p3(17), h0)};
            V Z[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) Z[k] = w == 2 ? C.Zr[k] : C.Zl[k];
            fit_nan = form_joint_A<5>(Z, M, A);
        }
        fitq = joint_quat_of_A(A, NoHook{}, tabF);
    }
#endif
    if (w == 0) {
        if (sub == 0) {
#if RTG_QUAD_SHARED_CODE >= 3
            const bool nan = fit_nan;
            const Q t = fitq;
#else
            bool nan = false;
            const Q t = fbp_torso(C, b, nan, NoHook{}, tabF);
#endif
            sfit[q] = make_float4(t.x, t.y, t.z, t.w);
            st = nan ? kStTorsoSvd : 0u;
        }
        lds_signal(&sflag[0]);
        if (sub == 0) emit_fixed_links(E);
    } else if (w >= 3) {
        const int side = w - 3;
        const ArmPts ap = side ? load_arm<1>(b) : load_arm<0>(b);
        lds_wait(&sflag[0], C.err);
        const float4 t = sfit[q];
        const Q R10{t.x, t.y, t.z, t.w};
        const V up = vsub(ap.el, ap.sh), fo = vsub(ap.wr, ap.el);
#if RTG_QUAD_SHARED_CODE
        const Q ch = solve_arm_lanes_rt<4>(E, side ? 21 : 12, up, fo, side ? C.rsh : C.lsh, side ? C.rel : C.lel, R10,
                                           NoHook{}, tab);
#else
        const Q ch = side ? solve_arm_lanes<21, 4>(E, up, fo, C.rsh, C.rel, R10, NoHook{}, tab)
                          : solve_arm_lanes<12, 4>(E, up, fo, C.lsh, C.lel, R10, NoHook{}, tab);
#endif
        if (sub == 0) schain[side][q] = make_float4(ch.x, ch.y, ch.z, ch.w);
        lds_signal(&sflag[1 + side]);
        finalize_lanes<4>(E, side ? 7 : 0, 4);
    } else {
        const int side = w - 1;
        const FV<false> H{rows + q * RP + (side ? 123 : 63)};
        Q W = qident();
        float a = 0.0f;
        if (sub == 0) {
            bool nan = false;
#if RTG_QUAD_SHARED_CODE >= 3
            W = fitq;
            nan = fit_nan;
#elif RTG_QUAD_SHARED_CODE
            W = fbp_wrist_fit_rt(C, H, side, nan, NoHook{}, tabF);
#else
            W = side ? fbp_wrist_fit<1>(C, H, nan, NoHook{}, tabF) : fbp_wrist_fit<0>(C, H, nan, NoHook{}, tabF);
#endif
            st = nan ? (side ? kStRightSvd : kStLeftSvd) : 0u;
            const TipPts tp = load_tips(H);
            a = hand_x_mean(qconj(W), tp.h0, tp.t);   // the gripper needs only W (:142-158 / :165-175)
        }
        W = gbc<4, 0>(W);
        lds_wait(&sflag[1 + side], C.err);   // the arm waited for R10 first: both are visible (release / acquire chain)
        const float4 t = sfit[q], c = schain[side][q];
        const Q R10{t.x, t.y, t.z, t.w}, chain{c.x, c.y, c.z, c.w};
        if (sub == 0) {
            fbp_gripper<PRECISE>(C, a, E.row + (side ? 27 : 18));
            if (body_rot && live) {
                float *const brow = body_rot + f * 236;
                if (side) fbp_body_rows<1>(brow, R10, W);
                else fbp_body_rows<0>(brow, R10, W);
            }
        }
        const Q loc = qnormalize_t(qmul(qconj(qnormalize_t(qmul(R10, chain), tab)), W), tab);
#if RTG_QUAD_SHARED_CODE
        const bool refused = emit_euler_xyz_lanes_rt<4>(E, side ? 25 : 16, loc);
#else
        const bool refused = side ? emit_euler_xyz_lanes<25, 4>(E, loc) : emit_euler_xyz_lanes<16, 4>(E, loc);
#endif
        st |= refused ? (side ? kStRightEuler : kStLeftEuler) : 0u;
        finalize_lanes<4>(E, side ? 11 : 4, 3);
    }
    if (w < 3 && sub == 0) sstat[w][q] = (uint8_t)st;
    __syncthreads();
    const uint32_t bits = (w == 0 && sub == 0 && live) ? (uint32_t)(sstat[0][q] | sstat[1][q] | sstat[2][q]) : 0u;
    if (__syncthreads_or(bits != 0u)) {   // rare: a frame the reference raises on
        if (bits) poison_frame(E.row, E.lr, body_rot ? body_rot + f * 236 : nullptr, bits);
        __syncthreads();
    }
    store_dof_rows(dof + f0 * 30, sdof, nf, threadIdx.x, 320);   // f0 * 30 floats: 16-byte aligned
}

// ----------------------------------------------------------------------------
// Per-frame server (the teleop loop without a launch per frame; sim_full_body_teleop.py:109-119 calls the solver
// once per captured frame).  One resident workgroup of k_fbp_frame1's shape serves FULL_BODY_POS frames from
// its inbox: the host writes a frame's rows (body | left hand | right hand, AoS) into `in` and then a new sequence
// number into in[RTG_SERVER_SEQ_WORD] (device memory through the BAR, or pinned host memory; rtg.h); thread 0 sees it
// (system-scope acquire), the tile runs reading `in` and writing
// dof / local_rot / body_rot straight into host memory, every wave's stores are released at system scope, and
// thread 0 publishes the sequence number in ctl[1].  The loop ends on the sequence word == RTG_SERVER_QUIT, or when no new
// frame arrives for idle_ticks (100 MHz wall clock) -- every wave reaches one of the two -- and sets ctl[2].
// Hand-over timeouts go to ctl[3] (the launch points C.err there).
// ----------------------------------------------------------------------------
template <bool PRECISE>
__global__ __launch_bounds__(320) void k_frame_server(SolverConsts C, const float *in, float *dof, float *local_rot,
                                                      float *body_rot, uint32_t *ctl, uint64_t idle_ticks)
{
    __shared__ uint32_t scmd;
    __shared__ float sframe[184];
    __shared__ UnitEnt sut[2 * kUnitTabK + 1];   // the near-unit normalisation table (RTG_FRAME1_UNIT_TAB), filled once
    if (RTG_FRAME1_UNIT_TAB) unit_tab_fill(sut, (int)threadIdx.x - 256);   // visible after the loop's first barrier
    uint32_t last = 0;
    bool const_ok = false;   // the output rows that never change are in place (written by an unpoisoned frame)
    if (threadIdx.x == 0) last = __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int frame = 0; frame < (1 << 30); ++frame) {
        if (threadIdx.x == 0) {
            const uint64_t t0 = wall_clock64();
            uint32_t db;
            for (;;) {
                db = __hip_atomic_load(reinterpret_cast<uint32_t *>(const_cast<float *>(in)) + RTG_SERVER_SEQ_WORD, __ATOMIC_ACQUIRE,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
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
        const uint32_t bits =
            fbp_frame1_tile<PRECISE>(C, sframe, dof, local_rot, body_rot, !const_ok,
                                     TabSel<(RTG_FRAME1_UNIT_TAB & 6) != 0>::get(sut), TabSel<(RTG_FRAME1_UNIT_TAB & 1) != 0>::get(sut));
        const_ok = bits == 0u;   // a poisoned frame overwrote every row with NaN: the next one rewrites them
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

// Kernel choice by batch size (measured crossovers).  Compile-time choices are `if constexpr`, so a
// TU instantiates only the kernels it can launch (rtg_solve_fbp_aos.hip / rtg_solve_fbp_soa.hip /
// rtg_solve_other.hip compile in parallel).
// FULL_BODY_POS at B <= RTG_LATENCY_MAX_B: k_fbp_frame1 / k_fbp_quad / k_fbp_latency5, instantiated in their own TU
// (rtg_solve_fbp_small.hip), which the Makefile compiles with the ILP-first scheduler: one or two waves per SIMD run
// these latency-bound chains, where interleaving independent work inside a wave pays (measured 2 % at B = 1 and
// 4096), unlike the throughput-bound side kernel (round 4: max-ilp raised it to 137 VGPRs, 3 waves/SIMD, slower)
hipError_t launch_fbp_small(int precise, bool soa, const SolverConsts &C, const float *in0, const float *in1,
                            const float *in2, int64_t B, float *dof, float *local_rot, float *body_rot, hipStream_t s);
template <bool PRECISE, bool SOA>
static void launch_fbp_small_kind(const SolverConsts &C, const float *in0, const float *in1, const float *in2,
                                  int64_t B, float *dof, float *local_rot, float *body_rot, hipStream_t s)
{
    if (B == 1) {
        hipLaunchKernelGGL((k_fbp_frame1<PRECISE>), dim3(1), dim3(320), 0, s, C, in0, in1, in2, dof, local_rot,
                           body_rot);
    } else if (B <= RTG_QUAD8_MAX_B) {
        hipLaunchKernelGGL((k_fbp_quad<PRECISE, SOA, 8>), dim3(grid_for(B, 8)), dim3(320), 0, s, C, in0, in1, in2, B,
                           dof, local_rot, body_rot);
    } else if (B <= RTG_QUAD_MAX_B) {
        hipLaunchKernelGGL((k_fbp_quad<PRECISE, SOA, 16>), dim3(grid_for(B, 16)), dim3(320), 0, s, C, in0, in1, in2, B,
                           dof, local_rot, body_rot);
    } else {
        hipLaunchKernelGGL((k_fbp_latency5<PRECISE, SOA>), dim3(grid_for(B, kLatFrames)), dim3(320), 0, s, C,
                           in0, in1, in2, B, dof, local_rot, body_rot);
    }
}
// Returns the launch's status.  launch_fbp_small reads (and so clears) the error state itself, so its result is passed
// up as it is; a caller must not read hipGetLastError() again after this (a failed small-batch launch was
// reported as RTG_OK).
template <int KIND, bool PRECISE, bool SOA>
static hipError_t launch_kind(const SolverConsts &C, const float *in0, const float *in1, const float *in2,
                              const float *in3, int64_t B, float *dof, float *local_rot, float *body_rot, hipStream_t s)
{
    if constexpr (KIND == RTG_SOLVER_FULL_BODY_POS) {
        if (B <= RTG_LATENCY_MAX_B) return launch_fbp_small(PRECISE, SOA, C, in0, in1, in2, B, dof, local_rot, body_rot, s);
    }
    hipLaunchKernelGGL((k_solve_sides<KIND, PRECISE, SOA>), dim3(grid_for(B, kSideFrames)), dim3(kSideThreads), 0, s, C, in0,
                       in1, in2, in3, B, dof, local_rot, body_rot);
    return hipGetLastError();
}

// FULL_BODY_POS launches, one TU per input layout
hipError_t launch_fbp_aos(int precise, const SolverConsts &C, const float *in0, const float *in1, const float *in2,
                          int64_t B, float *dof, float *local_rot, float *body_rot, hipStream_t s);
hipError_t launch_fbp_soa(int precise, const SolverConsts &C, const float *in0, const float *in1, const float *in2,
                          int64_t B, float *dof, float *local_rot, float *body_rot, hipStream_t s);

}  // namespace rtg
