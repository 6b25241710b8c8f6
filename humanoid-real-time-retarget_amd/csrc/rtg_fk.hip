// rtg_fk.hip -- forward / inverse kinematics kernels (kinematics.py:13-63, skeleton3d.py:402-484,
// hu_forward_model.py:17-33) and their launchers.  Every topology of J <= kGroupMaxJ joints (all shipped skeletons)
// runs the lane-group kernels below; larger trees fall back to the lane walks (one frame per thread).
#include "rtg_device.cuh"

#include <algorithm>
#include <type_traits>
#include <vector>

namespace rtg {

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


// HuForwardModel lane walk (J > kGroupMaxJ): joint j's local rotation from its DOF, then fk_frame's composition
template <bool CLIP>
__global__ __launch_bounds__(256) void k_dof_fk_walk(TopoView T, DofView D, const float *__restrict__ dof,
                                                     const float *__restrict__ root_rot,
                                                     const float *__restrict__ root_t, int64_t B,
                                                     float *__restrict__ g_rot, float *__restrict__ g_pos)
{
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= B) return;
    const int J = T.J;
    const float *drow = dof + f * (J - 1);
    float *gr = g_rot + f * J * 4, *gp = g_pos + f * J * 3;
    st4(gr, ld4(root_rot + f * 4));   // root: the root rotation, unnormalised (hu_forward_model.py:24)
    st3(gp, ld3(root_t + f * 3));
    for (int j = 1; j < T.J; ++j) {
        const int p = T.parents[j];
        float a = drow[j - 1];
        if (CLIP) {   // torch.clamp (min then max; NaN passes), then the straight-through sum
            float c = a < D.lower[j - 1] ? D.lower[j - 1] : a;
            c = c > D.upper[j - 1] ? D.upper[j - 1] : c;
            a = (c - a) + a;
        }
        const int ax = D.axis[j - 1];
        const Q lq = qfrom_angle_unit_axis(a, V{ax == 0 ? 1.0f : 0.0f, ax == 1 ? 1.0f : 0.0f, ax == 2 ? 1.0f : 0.0f});
        const Q g = ld4(gr + 4 * p);
        const V t = ld3(gp + 3 * p);
        const V rv = qrotate(g, T.local_t[j]);
        st4(gr + 4 * j, qmul_norm(g, lq));
        st3(gp + 3 * j, V{rv.x + t.x, rv.y + t.y, rv.z + t.z});
    }
}

// A lane-group tile is one wave, so ordering its LDS traffic needs no block
// barrier: a wave's LDS instructions execute in issue order, and the
// wavefront-scope fence + wave_barrier only stop the compiler from moving
// memory operations across this point.  (__syncthreads would also make the
// compiler drain every outstanding global store, s_waitcnt vmcnt(0), per step.)
RTG_DEV void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef float f4v __attribute__((ext_vector_type(4)));
// the lane-group tiles' output pieces (whole 1 KiB wave stores): non-temporal (RTG_FK_NT_OUT): never read back here,
// they would only evict the rows still to be read from the L2
RTG_DEV void st_out(f4v *p, f4v v)
{
    if (RTG_FK_NT_OUT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// the near-unit normalisation table (rtg_math.cuh) in the lane-group tiles' LDS, when any of them uses it
constexpr bool kUnitTab = RTG_FK_UNIT_TAB || RTG_DOF_UNIT_TAB;
constexpr size_t kUnitTabFloats = kUnitTab ? 4 * (2 * kUnitTabK + 1) : 0;
RTG_DEV Q qmul_norm_tab(Q a, Q b, const UnitEnt *tab)
{
    if (!RTG_FK_UNIT_TAB) return qmul_norm(a, b);
    return qnormalize_t(qmul(a, b), tab);
}

// ----------------------------------------------------------------------------
// Lane-group kinematics (round 6): a frame's joints spread over a GROUP of lanes, F frames per wave (F = 16: four
// lanes per frame for J <= 36; F = 8: eight lanes for J <= 64), so the tile's rows move as whole coalesced pieces.
// The windowed kernels above keep one frame per lane, and each of their load / store instructions touches 64 rows
// ~500 bytes apart (FETCH 1.75x, WRITE 1.22x the algorithmic bytes on Hu FK, round 4 PMC; a memory-pattern probe of
// those pieces alone tops out at 3.45 TB/s).  Here the F frames of a tile are F J consecutive 16-byte records: lane
// l of load k takes record 64 k + l, so every instruction reads or writes 1 KiB of consecutive bytes, each line of
// the rows is requested once, and the positions leave as consecutive dwordx4 pieces.  The records go through LDS:
//   1. every record of the tile is loaded (all loads in flight) and stored into the LDS image of the rows;
//   2. the joints are composed by a host-built list schedule (fk_group_schedule): at step s, sub-lane u of each
//      frame's group composes the joint the schedule names, reading its parent's global transform from the image and
//      writing its own over its local rotation -- a parent is always composed at an earlier step.  Each joint is
//      composed exactly as in kinematics.py:27-37 / fk_stream_tile (same device functions, same operands, same
//      order), so the bits are the same whatever the schedule; only which lane does it and when changes.  Hu: 31
//      joints in 10 steps (its depth + 1) on four lanes;
//   3. the global rotations and positions leave from the image, record-ordered (coalesced).
// LDS per wave: F J 28 bytes plus the schedule (Hu: 13.9 + 1.3 KiB).  Inverse FK (kinematics.py:41-63) has no chain:
// each record's parent is read from the image and its local rotation stored straight from the lane that loaded it.
// ----------------------------------------------------------------------------
template <int F>
struct Grp {
    static_assert(F == 16 || F == 8, "lane groups of 4 or 8 lanes");
    static constexpr int L = 64 / F;             // lanes per frame
    static constexpr int LOG_L = F == 16 ? 2 : 3;
    static constexpr int NR = F == 16 ? 9 : 8;   // records per lane: F J <= 64 NR (group_frames)
};
__host__ __device__ inline size_t pad16f(size_t nfloats) { return (nfloats + 3) & ~(size_t)3; }
// rot [F J] float4 | pos [F J 3] float | schedule [gsteps L] GEnt | extra floats (kernel-specific tables)
// ... | the near-unit table (kUnitTabFloats)
__host__ __device__ inline size_t group_core_floats(int J, int F, int steps)
{
    return (size_t)F * J * 4 + pad16f((size_t)F * J * 3) + (size_t)steps * (64 / F) * 8;
}
__host__ __device__ inline size_t group_lds_floats(int J, int F, int steps)
{
    return group_core_floats(J, F, steps) + kUnitTabFloats;
}

// the tile's schedule into LDS (float4 copies, in flight with the tile's own loads)
RTG_DEV void group_sched_fill(const TopoView &T, int L, GEnt *sch)
{
    const int n = T.gsteps * L * 2;
    const f4v *gs = reinterpret_cast<const f4v *>(T.gsched);
    f4v *d = reinterpret_cast<f4v *>(sch);
    for (int i = (int)threadIdx.x; i < n; i += 64) d[i] = gs[i];
}

// The schedule's steps over the tile image (rot: global rotations written over the local ones; pos: positions, the
// root's preset).  LQ(j, lq) gives joint j's local rotation from its image record (FK: the record itself, with the
// tree quaternion when STATE; DOF FK: built from the joint angle).
template <int F, typename LocalQ>
RTG_DEV void group_compose(const TopoView &T, f4v *rot, float *pos, const GEnt *sch, int nfr, const UnitEnt *utab,
                           const LocalQ &LQ)
{
    using G = Grp<F>;
    const int J = T.J, lane = (int)threadIdx.x;
    const int fr = lane >> G::LOG_L, sub = lane & (G::L - 1);
    const bool live = fr < nfr;
    const int base = fr * J;
    for (int s = 0; s < T.gsteps; ++s) {
        const GEnt e = sch[s * G::L + sub];
        const int j = e.code & 0xFF, p = (e.code >> 8) & 0xFF;
        if (live && j != 0xFF) {
            const f4v lv = rot[base + j];
            Q ng;
            V nt;
            if (j == 0) {   // root: global = local, unnormalised; position = the root translation (kinematics.py:27-29)
                ng = Q{lv.x, lv.y, lv.z, lv.w};
                nt = V{pos[3 * base], pos[3 * base + 1], pos[3 * base + 2]};
            } else {
                const Q lq = LQ(j, Q{lv.x, lv.y, lv.z, lv.w}, e, fr);
                const f4v gv = rot[base + p];
                const Q g{gv.x, gv.y, gv.z, gv.w};
                const float *tp = pos + 3 * (base + p);
                const V t{tp[0], tp[1], tp[2]};
                const V rv = qrotate(g, V{e.lx, e.ly, e.lz});
                ng = qmul_norm_tab(g, lq, utab);
                nt = V{rv.x + t.x, rv.y + t.y, rv.z + t.z};
            }
            rot[base + j] = f4v{ng.x, ng.y, ng.z, ng.w};
            float *op = pos + 3 * (base + j);
            op[0] = nt.x; op[1] = nt.y; op[2] = nt.z;
        }
        wave_sync();   // this step's records before the next step's parent reads (other lanes)
    }
}

// the tile image out: rotations record-ordered, positions as consecutive dwordx4 pieces (16-byte aligned rows; any
// other g_pos alignment stores dword by dword)
template <int F>
RTG_DEV void group_store(const f4v *rot, const float *pos, int nrec, float *__restrict__ g_rot, float *__restrict__ g_pos)
{
    using G = Grp<F>;
    const int lane = (int)threadIdx.x;
    f4v *dst = reinterpret_cast<f4v *>(g_rot);
    f4v o[G::NR];   // every LDS read first (unconditional), then the stores: no wait between two stores
#pragma unroll
    for (int k = 0; k < G::NR; ++k) {
        const int rec = k * 64 + lane;
        o[k] = rot[rec < nrec ? rec : 0];
    }
#pragma unroll
    for (int k = 0; k < G::NR; ++k) {
        const int rec = k * 64 + lane;
        if (rec < nrec) st_out(dst + rec, o[k]);
    }
    const int npos = 3 * nrec;
    if ((reinterpret_cast<uintptr_t>(g_pos) & 15u) == 0) {
        const int n4 = npos >> 2;
        f4v *pd = reinterpret_cast<f4v *>(g_pos);
        const f4v *ps = reinterpret_cast<const f4v *>(pos);
        for (int i = lane; i < n4; i += 64) st_out(pd + i, ps[i]);
        for (int i = 4 * n4 + lane; i < npos; i += 64) g_pos[i] = pos[i];
    } else {
        for (int i = lane; i < npos; i += 64) g_pos[i] = pos[i];
    }
}

// the tile's NR records per lane, all loads in flight (unconditional: a lane past the tile re-reads record 0, so no
// branch separates them), then -- after the caller's other loads -- into the LDS image
template <int F>
struct GroupRows {
    f4v v[Grp<F>::NR];
    RTG_DEV void load(const float *__restrict__ rows, int nrec)
    {
        const f4v *src = reinterpret_cast<const f4v *>(rows);
#pragma unroll
        for (int k = 0; k < Grp<F>::NR; ++k) {
            const int rec = k * 64 + (int)threadIdx.x;
            v[k] = src[rec < nrec ? rec : 0];
        }
    }
    RTG_DEV void to_lds(f4v *rot, int nrec) const
    {
#pragma unroll
        for (int k = 0; k < Grp<F>::NR; ++k) {
            const int rec = k * 64 + (int)threadIdx.x;
            if (rec < nrec) rot[rec] = v[k];
        }
    }
};

template <bool STATE, int F>
RTG_DEV void fk_group_tile(const TopoView &T, const float *__restrict__ local_rot, const float *__restrict__ root_t,
                           int64_t B, int64_t f0, float *__restrict__ g_rot, float *__restrict__ g_pos, float *lds)
{
    const int J = T.J, lane = (int)threadIdx.x;
    const int nfr = (int)((B - f0) < F ? (B - f0) : F);
    const int nrec = nfr * J;
    f4v *rot = reinterpret_cast<f4v *>(lds);
    float *pos = lds + 4 * F * J;
    GEnt *sch = reinterpret_cast<GEnt *>(pos + pad16f((size_t)3 * F * J));
    GroupRows<F> rows;
    rows.load(local_rot + f0 * J * 4, nrec);
    const float r = root_t[f0 * 3 + (lane < 3 * nfr ? lane : 0)];
    group_sched_fill(T, Grp<F>::L, sch);
    UnitEnt *utab = reinterpret_cast<UnitEnt *>(lds + group_core_floats(J, F, T.gsteps));
    if (RTG_FK_UNIT_TAB) unit_tab_fill(utab, (int)threadIdx.x);
    rows.to_lds(rot, nrec);
    if (lane < 3 * nfr) {
        const int fr = lane / 3;
        pos[3 * J * fr + (lane - 3 * fr)] = r;
    }
    wave_sync();
    group_compose<F>(T, rot, pos, sch, nfr, utab, [&](int, Q lq, const GEnt &e, int) {
        if (STATE) lq = qmul_norm_tab(Q{e.qx, e.qy, e.qz, e.qw}, lq, utab);   // skeleton3d.py:412-418
        return lq;
    });
    group_store<F>(rot, pos, nrec, g_rot + f0 * J * 4, g_pos + f0 * J * 3);
}

template <bool STATE, int F>
__global__ __launch_bounds__(64, 4) void k_fk_group(TopoView T, const float *__restrict__ local_rot,
                                                 const float *__restrict__ root_t, int64_t B, float *__restrict__ g_rot,
                                                 float *__restrict__ g_pos)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    fk_group_tile<STATE, F>(T, local_rot, root_t, B, (int64_t)blockIdx.x * F, g_rot, g_pos, fk_lds);
}

// inverse FK: LDS = the tile image | parents (J ints) | STATE: normalised conjugate tree quaternions (J float4)
constexpr int kLrotFrames = 8;   // frames per wave of the inverse tiles (any J <= kGroupMaxJ)
__host__ __device__ inline size_t lrot_core_floats(int J, int F) { return (size_t)F * J * 4 + pad16f((size_t)J) + (size_t)J * 4; }
__host__ __device__ inline size_t lrot_group_lds_floats(int J, int F) { return lrot_core_floats(J, F) + kUnitTabFloats; }
template <bool STATE, int F>
RTG_DEV void lrot_group_tile(const TopoView &T, const float *__restrict__ g_rot, int64_t B, int64_t f0,
                             float *__restrict__ local_rot, float *lds)
{
    using G = Grp<F>;
    const int J = T.J, lane = (int)threadIdx.x;
    const int nfr = (int)((B - f0) < F ? (B - f0) : F);
    const int nrec = nfr * J;
    f4v *rot = reinterpret_cast<f4v *>(lds);
    int *par = reinterpret_cast<int *>(lds + 4 * F * J);
    f4v *tqn = reinterpret_cast<f4v *>(lds + 4 * F * J + pad16f((size_t)J));
    const f4v *src = reinterpret_cast<const f4v *>(g_rot + f0 * J * 4);
    f4v v[G::NR];   // unconditional loads (a lane past the tile re-reads record 0): no branch between them
#pragma unroll
    for (int k = 0; k < G::NR; ++k) {
        const int rec = k * 64 + lane;
        v[k] = src[rec < nrec ? rec : 0];
    }
    UnitEnt *utab = reinterpret_cast<UnitEnt *>(lds + lrot_core_floats(J, F));
    if (RTG_FK_UNIT_TAB) unit_tab_fill(utab, (int)threadIdx.x);
    for (int j = lane; j < J; j += 64) {
        par[j] = ld_const(T.parents + j);
        if (STATE) {   // skeleton3d.py:470-478: quat_normalize(quat_conjugate(tree quat)), once per joint
            const Q c = qnormalize(qconj(ld_const(T.tree_quat + j)));
            tqn[j] = f4v{c.x, c.y, c.z, c.w};
        }
    }
#pragma unroll
    for (int k = 0; k < G::NR; ++k) {
        const int rec = k * 64 + lane;
        if (rec < nrec) rot[rec] = v[k];
    }
    wave_sync();
    const float rJ = 1.0f / (float)J;   // rec / J as ((rec + 1/2) / J) truncated: exact for rec < 2^12, J <= 64
    f4v *dst = reinterpret_cast<f4v *>(local_rot + f0 * J * 4);
#pragma unroll 3
    for (int k = 0; k < G::NR; ++k) {   // the records from the image: the loaded registers are free by now
        const int rec = k * 64 + lane;
        if (rec < nrec) {
            const int fr = (int)(((float)rec + 0.5f) * rJ), j = rec - fr * J;
            const f4v gv = rot[rec];
            const Q gj{gv.x, gv.y, gv.z, gv.w};
            Q q = gj;   // root copied (kinematics.py:49)
            if (j > 0) {
                const f4v pv = rot[fr * J + par[j]];
                q = qmul_norm_tab(qconj(Q{pv.x, pv.y, pv.z, pv.w}), gj, utab);
                if (STATE) {
                    const f4v c = tqn[j];
                    q = qmul_norm_tab(Q{c.x, c.y, c.z, c.w}, q, utab);
                }
            }
            st_out(dst + rec, f4v{q.x, q.y, q.z, q.w});
        }
    }
}

template <bool STATE, int F>
__global__ __launch_bounds__(64, 4) void k_lrot_group(TopoView T, const float *__restrict__ g_rot, int64_t B,
                                                   float *__restrict__ local_rot)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    lrot_group_tile<STATE, F>(T, g_rot, B, (int64_t)blockIdx.x * F, local_rot, fk_lds);
}

// HuForwardModel (hu_forward_model.py:17-33) on the lane groups.  The local rotations do not depend on the chain, so
// they are built first, all at once: each lane turns the DOFs it loaded (the tile's rows are nfr (J - 1) consecutive
// floats, NR loads per lane) into joint rotations -- quat_from_angle_axis of the clipped angle about the joint's unit
// axis -- and writes them into the tile image where FK's local rotations would be; then FK's compose runs as is.  (A
// first version built each joint's rotation inside its compose step: the f64 sincos sat on the chain's critical path
// and the kernel took 128 us against FK's 88, profiles/r06/fk/.)  LDS = the tile image | per-joint {axis, lower, upper}
// qfrom_angle_unit_axis(angle, e_ax) for N joints, element by element the same values: qnormalize's sign flip f
// (on cos), its |q|^2 in any component order (the zero components add +0 exactly), (n, 1/n) from the table, the two
// nonzero components' products by 1/n, and the zero components keep the sign of f sin (0 sin, times f, times 1/n > 0).
// A |q|^2 outside the table (NaN / inf angles) or a subnormal product: the scalar path, one rare-case branch per group.
template <int N>
RTG_DEV void joint_rot_n(const float (&angle)[N], const int (&ax)[N], const UnitEnt *tab, Q (&out)[N])
{
    double th[N];
#pragma unroll
    for (int i = 0; i < N; ++i) th[i] = (double)(angle[i] / 2.0f);
    SC t[N];
    cr_sincos_n<N>(th, t);
    bool ok[N], all = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const float f = 1.0f - 2.0f * (t[i].c < 0.0f ? 1.0f : 0.0f);
        const float s = f * t[i].s, c = f * t[i].c;
        const float n2 = s * s + c * c;
        uint32_t idx;
        const bool in = unit_tab_index(n2, idx);
        const double r = tab[idx].r;
        const double ps = (double)s * r, pc = (double)c * r;
        const float qs = (float)ps, z = __builtin_copysignf(0.0f, s);
        out[i] = Q{ax[i] == 0 ? qs : z, ax[i] == 1 ? qs : z, ax[i] == 2 ? qs : z, (float)pc};
        ok[i] = in & !((__builtin_fabs(ps) < 0x1p-126) & (ps != 0.0)) & !((__builtin_fabs(pc) < 0x1p-126) & (pc != 0.0));
        all &= ok[i];
    }
    if (__builtin_expect(!all, 0)) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (!ok[i])
                out[i] = qfrom_angle_unit_axis(angle[i], V{ax[i] == 0 ? 1.0f : 0.0f, ax[i] == 1 ? 1.0f : 0.0f,
                                                           ax[i] == 2 ? 1.0f : 0.0f});
    }
}
__host__ __device__ inline size_t dof_group_lds_floats(int J, int F, int steps)
{
    return group_lds_floats(J, F, steps) + (size_t)J * 4;
}
template <bool CLIP, int F>
__global__ __launch_bounds__(64, 4) void k_dof_fk_group(TopoView T, DofView D, const float *__restrict__ dof,
                                                     const float *__restrict__ root_rot,
                                                     const float *__restrict__ root_t, int64_t B,
                                                     float *__restrict__ g_rot, float *__restrict__ g_pos)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    using G = Grp<F>;
    const int J = T.J, lane = (int)threadIdx.x, nd = J - 1;
    const int64_t f0 = (int64_t)blockIdx.x * F;
    const int nfr = (int)((B - f0) < F ? (B - f0) : F);
    const int nrec = nfr * J;
    f4v *rot = reinterpret_cast<f4v *>(fk_lds);
    float *pos = fk_lds + 4 * F * J;
    GEnt *sch = reinterpret_cast<GEnt *>(pos + pad16f((size_t)3 * F * J));
    f4v *ntab = reinterpret_cast<f4v *>(fk_lds + group_lds_floats(J, F, T.gsteps));
    const float *drow = dof + f0 * nd;
    const int nang = nfr * nd;
    float a[G::NR];   // unconditional loads (a lane past the rows re-reads element 0)
#pragma unroll
    for (int k = 0; k < G::NR; ++k) {
        const int i = k * 64 + lane;
        a[k] = drow[i < nang ? i : 0];
    }
    const f4v rr = reinterpret_cast<const f4v *>(root_rot)[f0 + (lane < nfr ? lane : 0)];
    const float rt = root_t[f0 * 3 + (lane < 3 * nfr ? lane : 0)];
    group_sched_fill(T, G::L, sch);
    UnitEnt *utab = reinterpret_cast<UnitEnt *>(fk_lds + group_core_floats(J, F, T.gsteps));
    if (kUnitTab) unit_tab_fill(utab, (int)threadIdx.x);
    for (int j = 1 + lane; j < J; j += 64) {
        const int ax = ld_const(D.axis + (j - 1));
        ntab[j] = f4v{__int_as_float(ax), CLIP ? ld_const(D.lower + (j - 1)) : 0.0f,
                      CLIP ? ld_const(D.upper + (j - 1)) : 0.0f, 0.0f};
    }
    if (lane < nfr) rot[lane * J] = rr;   // root: global = the root rotation (hu_forward_model.py:24)
    if (lane < 3 * nfr) {
        const int fr = lane / 3;
        pos[3 * J * fr + (lane - 3 * fr)] = rt;
    }
    wave_sync();
    // angle i = (frame fr, joint i mod nd + 1): its rotation into record fr J + j (i / nd as ((i + 1/2) / nd)
    // truncated: exact for i < 2^12)
    const float rnd = 1.0f / (float)(nd > 0 ? nd : 1);
    // NW loads' rotations at a time on the N-way leaf math (one rare-case branch per group, the same bits); a lane
    // past the angles computes a dummy rotation (its j is still a joint) and does not store it
    auto rotations = [&](auto nw, int k0) {
        constexpr int NW = decltype(nw)::value;
        if (k0 * 64 >= nang) return;   // wave-uniform: no lane has an angle in this group
        float x[NW];
        int axi[NW], rec[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const int i = (k0 + w) * 64 + lane;
            const int fr = (int)(((float)i + 0.5f) * rnd), j = i - fr * nd + 1;
            const f4v t = ntab[j];
            x[w] = a[k0 + w];
            if (CLIP) {   // torch.clamp (min then max; NaN passes), then the straight-through sum
                float c = x[w] < t.y ? t.y : x[w];
                c = c > t.z ? t.z : c;
                x[w] = (c - x[w]) + x[w];
            }
            // the axis is an exact unit vector: quat_from_angle_axis's normalisation is the identity (round 5)
            axi[w] = __float_as_int(t.x);
            rec[w] = i < nang ? fr * J + j : -1;
        }
        Q q[NW];
#if RTG_DOF_UNIT_TAB
        joint_rot_n<NW>(x, axi, utab, q);
#else
        V axv[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w)
            axv[w] = V{axi[w] == 0 ? 1.0f : 0.0f, axi[w] == 1 ? 1.0f : 0.0f, axi[w] == 2 ? 1.0f : 0.0f};
        qfrom_angle_unit_axis_n<NW>(x, axv, q);
#endif
#pragma unroll
        for (int w = 0; w < NW; ++w)
            if (rec[w] >= 0) rot[rec[w]] = f4v{q[w].x, q[w].y, q[w].z, q[w].w};
    };
    constexpr int NW = RTG_DOF_NWAY, NFULL = G::NR - G::NR % NW;
#pragma unroll
    for (int k = 0; k < NFULL; k += NW) rotations(std::integral_constant<int, NW>{}, k);
#pragma unroll
    for (int k = NFULL; k < G::NR; ++k) rotations(std::integral_constant<int, 1>{}, k);
    wave_sync();
    group_compose<F>(T, rot, pos, sch, nfr, utab, [&](int, Q lq, const GEnt &, int) { return lq; });
    group_store<F>(rot, pos, nrec, g_rot + f0 * J * 4, g_pos + f0 * J * 3);
}

// Mixed-target kinematics on the lane groups (config 5): a block is one tile of one segment; the segment's F comes
// from its topology
__global__ __launch_bounds__(64, 4) void k_fk_multi_group(FkMultiArgs A)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    int s = 0;
#pragma unroll
    for (int i = 1; i < RTG_MAX_SEGMENTS; ++i)
        if (i < A.n && (int64_t)blockIdx.x >= A.block_start[i]) s = i;
    const FkSeg &S = A.seg[s];
    const int64_t t = (int64_t)blockIdx.x - A.block_start[s];
    if (S.op == 1) lrot_group_tile<false, kLrotFrames>(S.T, S.local_rot, S.B, t * kLrotFrames, S.g_rot, fk_lds);
    else if (S.T.gF == 16) fk_group_tile<false, 16>(S.T, S.local_rot, S.root_t, S.B, t * 16, S.g_rot, S.g_pos, fk_lds);
    else fk_group_tile<false, 8>(S.T, S.local_rot, S.root_t, S.B, t * 8, S.g_rot, S.g_pos, fk_lds);
}

// Host: the lane-group list schedule.  Joints become ready once their parent's step is past; each step takes up to L
// ready joints, longest remaining chain (height) first, ties by index -- for a tree that is the critical-path bound
// (depth + 1 steps) whenever L covers the widest level the chains keep busy (Hu on 4 lanes: 10 steps for 31 joints).
// The bits do not depend on it (group_compose).  Returns the step count, or -1 if it would exceed max_steps.
int32_t fk_group_schedule(const int32_t *parents, const V *local_t, const Q *tree_quat, int32_t J, int32_t F,
                          GEnt *out, int32_t max_steps)
{
    const int L = 64 / F;
    std::vector<int> h(J, 1), done(J, -1);
    for (int j = J - 1; j > 0; --j) h[parents[j]] = std::max(h[parents[j]], h[j] + 1);
    int steps = 0, placed = 0;
    std::vector<int> ready;
    while (placed < J) {
        if (steps >= max_steps) return -1;
        ready.clear();
        for (int j = 0; j < J; ++j)
            if (done[j] < 0 && (j == 0 || (done[parents[j]] >= 0 && done[parents[j]] < steps))) ready.push_back(j);
        std::stable_sort(ready.begin(), ready.end(), [&](int a, int b) { return h[a] > h[b]; });
        for (int u = 0; u < L; ++u) {
            GEnt &e = out[steps * L + u];
            e = GEnt{0.f, 0.f, 0.f, 0xFFFF, 0.f, 0.f, 0.f, 1.f};
            if (u < (int)ready.size()) {
                const int j = ready[u];
                done[j] = steps;
                ++placed;
                e = GEnt{local_t[j].x, local_t[j].y, local_t[j].z, j | ((j ? parents[j] : 0xFF) << 8),
                         tree_quat[j].x, tree_quat[j].y, tree_quat[j].z, tree_quat[j].w};
            }
        }
        ++steps;
    }
    return steps;
}

hipError_t launch_fk(const TopoView &T, bool state, const float *lr, const float *rt, int64_t B, float *gr, float *gp,
                     hipStream_t s)
{
    if (T.gsched) {
        const int F = T.gF;
        const size_t lds = sizeof(float) * group_lds_floats(T.J, F, T.gsteps);
        const dim3 g(grid_for(B, F)), b(64);
        if (F == 16) {
            if (state) hipLaunchKernelGGL((k_fk_group<true, 16>), g, b, lds, s, T, lr, rt, B, gr, gp);
            else hipLaunchKernelGGL((k_fk_group<false, 16>), g, b, lds, s, T, lr, rt, B, gr, gp);
        } else {
            if (state) hipLaunchKernelGGL((k_fk_group<true, 8>), g, b, lds, s, T, lr, rt, B, gr, gp);
            else hipLaunchKernelGGL((k_fk_group<false, 8>), g, b, lds, s, T, lr, rt, B, gr, gp);
        }
    } else if (state) {   // J > kGroupMaxJ: lane walk
        hipLaunchKernelGGL(k_fk<true>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, lr, rt, B, gr, gp);
    } else {
        hipLaunchKernelGGL(k_fk<false>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, lr, rt, B, gr, gp);
    }
    return hipGetLastError();
}

hipError_t launch_local_rotation(const TopoView &T, bool state, const float *g, int64_t B, float *l, hipStream_t s)
{
    if (T.gsched) {   // 8 frames per wave whatever J: no chain here, so the smallest tile -- the most waves per CU --
                      // wins (Hu: 41.4 vs 46.8 us at 16 frames, profiles/r06/fk/)
        const size_t lds = sizeof(float) * lrot_group_lds_floats(T.J, kLrotFrames);
        const dim3 gd(grid_for(B, kLrotFrames)), b(64);
        if (state) hipLaunchKernelGGL((k_lrot_group<true, kLrotFrames>), gd, b, lds, s, T, g, B, l);
        else hipLaunchKernelGGL((k_lrot_group<false, kLrotFrames>), gd, b, lds, s, T, g, B, l);
    } else if (state) {   // J > kGroupMaxJ: lane walk
        hipLaunchKernelGGL(k_local_rotation<true>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, g, B, l);
    } else {
        hipLaunchKernelGGL(k_local_rotation<false>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, g, B, l);
    }
    return hipGetLastError();
}

hipError_t launch_fk_multi(FkMultiArgs &A, hipStream_t s)
{
    bool group = true;
    for (int i = 0; i < A.n; ++i) group = group && A.seg[i].T.gsched != nullptr;
    // every segment on the lane groups: one block per F-frame tile of its segment; else every segment's lane walk
    int64_t blocks = 0;
    size_t lds = 0;
    for (int i = 0; i < A.n; ++i) {
        const TopoView &T = A.seg[i].T;
        A.block_start[i] = blocks;
        blocks += grid_for(A.seg[i].B, group ? (A.seg[i].op == 0 ? T.gF : kLrotFrames) : 256);
        if (group) {
            const size_t need =
                A.seg[i].op == 0 ? group_lds_floats(T.J, T.gF, T.gsteps) : lrot_group_lds_floats(T.J, kLrotFrames);
            lds = need > lds ? need : lds;
        }
    }
    for (int i = A.n; i < RTG_MAX_SEGMENTS; ++i) A.block_start[i] = blocks;
    if (blocks == 0) return hipSuccess;
    if (group) hipLaunchKernelGGL(k_fk_multi_group, dim3((unsigned)blocks), dim3(64), sizeof(float) * lds, s, A);
    else hipLaunchKernelGGL(k_fk_multi, dim3((unsigned)blocks), dim3(256), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_dof_fk(const TopoView &T, const DofView &D, bool clip, const float *dof, const float *root_rot,
                         const float *root_t, int64_t B, float *gr, float *gp, hipStream_t s)
{
    if (T.gsched) {
        const int F = T.gF;
        const size_t lds = sizeof(float) * dof_group_lds_floats(T.J, F, T.gsteps);
        const dim3 g(grid_for(B, F)), b(64);
        if (F == 16) {
            if (clip) hipLaunchKernelGGL((k_dof_fk_group<true, 16>), g, b, lds, s, T, D, dof, root_rot, root_t, B, gr, gp);
            else hipLaunchKernelGGL((k_dof_fk_group<false, 16>), g, b, lds, s, T, D, dof, root_rot, root_t, B, gr, gp);
        } else {
            if (clip) hipLaunchKernelGGL((k_dof_fk_group<true, 8>), g, b, lds, s, T, D, dof, root_rot, root_t, B, gr, gp);
            else hipLaunchKernelGGL((k_dof_fk_group<false, 8>), g, b, lds, s, T, D, dof, root_rot, root_t, B, gr, gp);
        }
    } else if (clip) {   // J > kGroupMaxJ: lane walk
        hipLaunchKernelGGL(k_dof_fk_walk<true>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, D, dof, root_rot, root_t, B,
                           gr, gp);
    } else {
        hipLaunchKernelGGL(k_dof_fk_walk<false>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, D, dof, root_rot, root_t, B,
                           gr, gp);
    }
    return hipGetLastError();
}

}  // namespace rtg
