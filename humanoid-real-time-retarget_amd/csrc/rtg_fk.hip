// rtg_fk.hip -- forward / inverse kinematics kernels (kinematics.py:13-63, skeleton3d.py:402-484,
// hu_forward_model.py:17-33) and their launchers.
#include "rtg_device.cuh"

#include <algorithm>
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
constexpr int kFkTile = 64;
constexpr int kFkChunk = 8;                     // joints per LDS window
constexpr int kRotPitch = 4 * (kFkChunk + 1);   // floats per frame row (LDS)

// POS16 (the mixed launch, config 5): positions collect in a 16-joint LDS window and leave every second window as
// 192-byte row pieces (measured 151 -> 130 us there; +3 % slower for plain FK, which keeps them in registers)
constexpr int kPos16Pitch = 3 * 16 + 1;
template <bool POS16>
constexpr int pos_win() { return POS16 ? kFkTile * kPos16Pitch : 0; }

// Branch-parent slots live in LDS: [slot][7][64] (q x y z w, t x y z per lane).  Every shipped skeleton needs <= 2.
__host__ __device__ inline size_t lds_slot_floats(int nslots) { return (size_t)nslots * 7 * kFkTile; }
static inline size_t fk_stream_lds_bytes(int nslots, bool pos16 = false)
{
    const size_t pw = pos16 ? pos_win<true>() : pos_win<false>();
    return sizeof(float) * ((size_t)kFkTile * kRotPitch + pw + lds_slot_floats(nslots));
}
static inline size_t dof_fk_lds_bytes(int nslots)
{
    return sizeof(float) * ((size_t)kFkTile * kRotPitch + lds_slot_floats(nslots));
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
typedef float f4v __attribute__((ext_vector_type(4)));
RTG_DEV void out_st4(float *gp, const float *lp) { *reinterpret_cast<f4v *>(gp) = *reinterpret_cast<const f4v *>(lp); }
RTG_DEV void out_st1(float *gp, float v) { *gp = v; }
template <int W>
RTG_DEV void chunk_store(float *__restrict__ g, const float *lds, int pitch, int64_t f0, int nfr, int J, int c0, int nC)
{
    auto one = [&](int it) {
        const int v = it * kFkTile + (int)threadIdx.x;
        const int fr = v / kFkChunk, k = v % kFkChunk;
        float *gp = g + ((f0 + fr) * J + c0 + k) * W;
        const float *lp = lds + fr * pitch + k * W;
        if (W == 4) {
            out_st4(gp, lp);
        } else {
#pragma unroll
            for (int c = 0; c < W; ++c) out_st1(gp + c, lp[c]);
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

// A window of JW joints (W floats each) of rows f0.. from LDS (row pitch `pitch`): JW lanes per frame piece.
template <int W, int JW>
RTG_DEV void chunk_store_n(float *__restrict__ g, const float *lds, int pitch, int64_t f0, int nfr, int J, int c0, int nC)
{
#pragma unroll
    for (int it = 0; it < JW; ++it) {
        const int v = it * kFkTile + (int)threadIdx.x;
        const int fr = v / JW, k = v % JW;
        if (fr < nfr && k < nC) {
            float *gp = g + ((f0 + fr) * J + c0 + k) * W;
            const float *lp = lds + fr * pitch + k * W;
#pragma unroll
            for (int c = 0; c < W; ++c) out_st1(gp + c, lp[c]);
        }
    }
}

struct Slots {
    float *lds;
};
RTG_DEV void slot_put(Slots &S, int s, Q q, V t)
{
    float *p = S.lds + s * 7 * kFkTile + threadIdx.x;
    p[0] = q.x; p[kFkTile] = q.y; p[2 * kFkTile] = q.z; p[3 * kFkTile] = q.w;
    p[4 * kFkTile] = t.x; p[5 * kFkTile] = t.y; p[6 * kFkTile] = t.z;
}
RTG_DEV void slot_get(const Slots &S, int s, Q &q, V &t)
{
    const float *p = S.lds + s * 7 * kFkTile + threadIdx.x;
    q = Q{p[0], p[kFkTile], p[2 * kFkTile], p[3 * kFkTile]};
    t = V{p[4 * kFkTile], p[5 * kFkTile], p[6 * kFkTile]};
}

template <bool STATE, bool POS16 = false>
RTG_DEV void fk_stream_tile(const TopoView &T, const float *__restrict__ local_rot, const float *__restrict__ root_t,
                            int64_t B, int64_t f0, float *__restrict__ g_rot, float *__restrict__ g_pos, float *lds)
{
    const int J = T.J;
    const int nfr = (int)((B - f0) < kFkTile ? (B - f0) : kFkTile);
    float *rot = lds;                                   // [64][kRotPitch]
    float *pos = lds + kFkTile * kRotPitch;             // [64][kPos16Pitch] (POS16), else none
    Slots slots{pos + pos_win<POS16>()};
    const int lane = threadIdx.x;
    const bool active = lane < nfr;
    Q g = qident();
    V t = V{0.0f, 0.0f, 0.0f};
    V pk[kFkChunk];   // the window's positions (constant indices: registers), staged through the window once the
                      // rotation rows are out (measured +3-4 % over a separate position window)
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
                if (RTG_EXP_FK_COPY) {   // measurement knob: the window goes straight back out (no chain)
                    ng = lq;
                    nt = V{lq.x, lq.y, lq.z};
                } else if (j == 0) {   // root: global = local, unnormalised (kinematics.py:27-29)
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
                if (POS16) {
                    float *P16 = pos + lane * kPos16Pitch + 3 * (k + (c0 & 8));
                    P16[0] = nt.x; P16[1] = nt.y; P16[2] = nt.z;
                } else {
                    pk[k] = nt;
                }
                if (!RTG_EXP_FK_COPY && ((sc >> 8) & 0xFF) != kNoSlot) slot_put(slots, (sc >> 8) & 0xFF, ng, nt);
                g = ng;
                t = nt;
            }
        }
        wave_sync();
        chunk_store<4>(g_rot, rot, kRotPitch, f0, nfr, J, c0, nC);
        if (RTG_EXP_FK_NOPOS) {   // measurement knob: no position rows
        } else if (POS16) {   // every second window (and the last): 16 joints' positions per frame piece
            if ((c0 & 8) || c0 + nC == J) {
                const int c16 = c0 & ~15;
                chunk_store_n<3, 16>(g_pos, pos, kPos16Pitch, f0, nfr, J, c16, c0 + nC - c16);
            }
        } else {   // the rotation rows are out: reuse the window for the positions
            wave_sync();
            if (active) {
                float *P = rot + lane * kRotPitch;
#pragma unroll
                for (int k = 0; k < kFkChunk; ++k)
                    if (k < nC) { P[3 * k] = pk[k].x; P[3 * k + 1] = pk[k].y; P[3 * k + 2] = pk[k].z; }
            }
            wave_sync();
            chunk_store<3>(g_pos, rot, kRotPitch, f0, nfr, J, c0, nC);
        }
        wave_sync();
    }
}

template <bool STATE>
__global__ __launch_bounds__(kFkTile) void k_fk_stream(TopoView T, const float *__restrict__ local_rot,
                                                       const float *__restrict__ root_t, int64_t B,
                                                       float *__restrict__ g_rot, float *__restrict__ g_pos)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    fk_stream_tile<STATE>(T, local_rot, root_t, B, (int64_t)blockIdx.x * kFkTile, g_rot, g_pos, fk_lds);
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
__global__ __launch_bounds__(kFkTile) void k_dof_fk(TopoView T, DofView D, const float *__restrict__ dof,
                                                    const float *__restrict__ root_rot,
                                                    const float *__restrict__ root_t, int64_t B,
                                                    float *__restrict__ g_rot, float *__restrict__ g_pos)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    const int J = T.J;
    const int64_t f0 = (int64_t)blockIdx.x * kFkTile;
    const int nfr = (int)((B - f0) < kFkTile ? (B - f0) : kFkTile);
    float *rot = fk_lds;
    Slots slots{fk_lds + kFkTile * kRotPitch};
    V pk[kFkChunk];   // the window's positions, staged through the window after its rotation rows (measured +7-9 %)
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
                    // the axis is an exact unit vector: its normalisation is the identity (sqrt(1) = 1, 0 and 1
                    // divided by 1), so the unit-axis form gives quat_from_angle_axis's bits without it (round 5)
                    const Q lq = qfrom_angle_unit_axis(a, V{ax == 0 ? 1.0f : 0.0f, ax == 1 ? 1.0f : 0.0f,
                                                            ax == 2 ? 1.0f : 0.0f});
                    if ((sc & 0xFF) != kNoSlot) slot_get(slots, sc & 0xFF, g, t);
                    const V rv = qrotate(g, ld_const(T.local_t + j));
                    ng = qmul_norm(g, lq);
                    nt = V{rv.x + t.x, rv.y + t.y, rv.z + t.z};
                }
                R[4 * k] = ng.x; R[4 * k + 1] = ng.y; R[4 * k + 2] = ng.z; R[4 * k + 3] = ng.w;
                pk[k] = nt;
                if (((sc >> 8) & 0xFF) != kNoSlot) slot_put(slots, (sc >> 8) & 0xFF, ng, nt);
                g = ng;
                t = nt;
            }
        }
        wave_sync();
        chunk_store<4>(g_rot, rot, kRotPitch, f0, nfr, J, c0, nC);
        wave_sync();   // the rotation rows are out: reuse the window for the positions
        if (active) {
            float *P = rot + lane * kRotPitch;
#pragma unroll
            for (int k = 0; k < kFkChunk; ++k)
                if (k < nC) { P[3 * k] = pk[k].x; P[3 * k + 1] = pk[k].y; P[3 * k + 2] = pk[k].z; }
        }
        wave_sync();
        chunk_store<3>(g_pos, rot, kRotPitch, f0, nfr, J, c0, nC);
        wave_sync();
    }
}

// ----------------------------------------------------------------------------
// Inverse FK, line-synchronous (k_local_rotation_line; the inverse segments of k_fk_multi_stream).  A 64-frame tile's rows are 64 J records of 16 B, i.e. 8 J whole
// 128-byte lines, and a frame's row starts (f J) mod 8 records into a line.  The windowed kernels above move, per
// frame, joints [8k, 8k+8): a 128-B piece at 16-B alignment that straddles two lines, so every line is requested by
// two windows ~15 us apart and the second request misses L2 (FETCH 1.75x the input on Hu FK).  Here, at step m,
// every lane moves the records of ITS OWN m-th line instead: the pieces are whole lines (8 lanes x 16 B), each line
// of the rows is requested once (a line two frames share, once by each for its own records), and the position
// piece of rotation line L is bytes [96 L, 96 L + 96) of the position rows (32-B aligned).  The price: a lane's
// joint index at a step differs across lanes, so the topology (local_t, schedule, tree quaternion) is read from an
// LDS table instead of scalar registers, and J joints take ceil((J + 8 - gcd(J, 8)) / 8) steps of 8 (Hu: 5 x 8
// for 31).  Per lane the joints are still composed in index order with the same operations, so the bits are the
// windowed kernel's.  Measured (tools/fk_pattern_probe.hip, Hu, B = 262144): the bare copy pattern takes 104 us
// against 115 us for the windows; inverse FK 75.7 vs 82.7 us with the windows, bit-exact.  Forward FK in this form
// was SLOWER (123 vs 120 us; the mixed launch 147 vs 132 us): its heavier chain pays for the extra step slots and
// the per-lane topology reads, so forward FK keeps the windows above (git history has the line form).
// ----------------------------------------------------------------------------
RTG_DEV int line_steps(int J)
{
    const int g = (J & 7) == 0 ? 8 : (J & 3) == 0 ? 4 : (J & 1) == 0 ? 2 : 1;   // gcd(J, 8)
    return (J + 8 - g + 7) >> 3;
}
// LDS topology table: per joint {local_t.x, .y, .z, sched bits} and its tree quaternion
static inline size_t line_topo_floats(int J) { return (size_t)J * 8; }
static inline size_t fk_line_lds_bytes(int J, int nslots)
{
    return sizeof(float) * ((size_t)kFkTile * kRotPitch + lds_slot_floats(nslots) + line_topo_floats(J));
}
RTG_DEV void line_topo_fill(const TopoView &T, float *topo)
{
    for (int j = threadIdx.x; j < T.J; j += kFkTile) {
        const V lt = ld_const(T.local_t + j);
        const Q tq = ld_const(T.tree_quat + j);
        st4(topo + 8 * j, Q{lt.x, lt.y, lt.z, __int_as_float(ld_const(T.sched + j))});
        st4(topo + 8 * j + 4, tq);
    }
}
// piece (it, lane) of step m: frame fr's sub-th record of its m-th line, ok when that record is the frame's own
struct LinePiece {
    int fr, sub, g;
    bool ok;
};
RTG_DEV LinePiece line_piece(int it, int m, int J, int nfr)
{
    const int v = it * kFkTile + (int)threadIdx.x, fr = v >> 3, sub = v & 7;
    const int g = 8 * (((fr * J) >> 3) + m) + sub;
    return LinePiece{fr, sub, g, fr < nfr && g >= fr * J && g < fr * J + J};
}
RTG_DEV void line_load(ChunkRegs &r, const float *__restrict__ rows, int m, int J, int nfr)
{
#define RTG_LLD(I)                                                                         \
    {                                                                                      \
        const LinePiece P = line_piece(I, m, J, nfr);                                      \
        r.v##I = ld4(rows + 4 * (P.ok ? P.g : 0));                                         \
    }
    RTG_REP8(RTG_LLD)
#undef RTG_LLD
}
RTG_DEV void line_to_lds(const ChunkRegs &r, float *win, int m, int J, int nfr)
{
#define RTG_LST(I)                                                                         \
    {                                                                                      \
        const LinePiece P = line_piece(I, m, J, nfr);                                      \
        st4(win + P.fr * kRotPitch + P.sub * 4, r.v##I);                                   \
    }
    RTG_REP8(RTG_LST)
#undef RTG_LST
}
template <int W>
RTG_DEV void line_store(float *__restrict__ rows, const float *win, int m, int J, int nfr)
{
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const LinePiece P = line_piece(it, m, J, nfr);
        if (P.ok) {
            float *gp = rows + (int64_t)W * P.g;
            const float *lp = win + P.fr * kRotPitch + P.sub * W;
            if (W == 4) {
                out_st4(gp, lp);
            } else {
#pragma unroll
                for (int c = 0; c < W; ++c) gp[c] = lp[c];
            }
        }
    }
}
// a branch parent's transform from its slot, for lanes whose schedule names one (per-lane slot index)
RTG_DEV void slot_get_lane(const Slots &S, int nslots, int32_t sc, Q &q, V &t)
{
    const int si = sc & 0xFF;
    if (nslots > 0) {
        Q sq;
        V st;
        slot_get(S, si != kNoSlot ? si : 0, sq, st);
        if (si != kNoSlot) {
            q = sq;
            t = st;
        }
    }
}

template <bool STATE>
RTG_DEV void lrot_line_tile(const TopoView &T, const float *__restrict__ g_rot, int64_t B, int64_t f0,
                            float *__restrict__ local_rot, float *lds)
{
    const int J = T.J;
    const int nfr = (int)((B - f0) < kFkTile ? (B - f0) : kFkTile);
    float *win = lds;
    Slots slots{lds + kFkTile * kRotPitch};
    float *topo = slots.lds + lds_slot_floats(T.nslots);
    const int lane = threadIdx.x;
    const bool active = lane < nfr;
    const int64_t r0 = f0 * J;
    const float *in = g_rot + 4 * r0;
    float *out = local_rot + 4 * r0;
    Q prev = qident();
    line_topo_fill(T, topo);
    ChunkRegs next;
    line_load(next, in, 0, J, nfr);
    const int M = line_steps(J);
    for (int m = 0; m < M; ++m) {
        line_to_lds(next, win, m, J, nfr);
        wave_sync();
        if (m + 1 < M) line_load(next, in, m + 1, J, nfr);
        const int b = 8 * (((lane * J) >> 3) + m) - lane * J;
        float *W = win + lane * kRotPitch;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int j = b + k;
            const bool ok = active && j >= 0 && j < J;
            const int jj = j < 0 ? 0 : (j >= J ? J - 1 : j);
            const float *tp = topo + 8 * jj;
            const int32_t sc = __float_as_int(tp[3]);
            const Q gj = Q{W[4 * k], W[4 * k + 1], W[4 * k + 2], W[4 * k + 3]};
            Q q = gj;   // root copied (kinematics.py:49)
            if (j > 0) {
                Q gp = prev;
                V unused = V{0.0f, 0.0f, 0.0f};
                slot_get_lane(slots, T.nslots, sc, gp, unused);
                q = qmul_norm(qconj(gp), gj);
                if (STATE) q = qmul_norm(qnormalize(qconj(Q{tp[4], tp[5], tp[6], tp[7]})), q);   // skeleton3d.py:470-478
            }
            if (ok && ((sc >> 8) & 0xFF) != kNoSlot) slot_put(slots, (sc >> 8) & 0xFF, gj, V{0.0f, 0.0f, 0.0f});
            W[4 * k] = q.x; W[4 * k + 1] = q.y; W[4 * k + 2] = q.z; W[4 * k + 3] = q.w;
            if (ok) prev = gj;
        }
        wave_sync();
        line_store<4>(out, win, m, J, nfr);
        wave_sync();
    }
}

template <bool STATE>
__global__ __launch_bounds__(kFkTile) void k_local_rotation_line(TopoView T, const float *__restrict__ g_rot,
                                                                 int64_t B, float *__restrict__ local_rot)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    lrot_line_tile<STATE>(T, g_rot, B, (int64_t)blockIdx.x * kFkTile, local_rot, fk_lds);
}
// Mixed-target kinematics (BASELINE config 5): every 64-frame tile of every segment is one wave; a segment is FK
// (op 0) or inverse FK (op 1), so FK and inverse FK of several skeletons share one launch.
__global__ __launch_bounds__(kFkTile) void k_fk_multi_stream(FkMultiArgs A)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    int s = 0;
#pragma unroll
    for (int i = 1; i < RTG_MAX_SEGMENTS; ++i)
        if (i < A.n && (int64_t)blockIdx.x >= A.block_start[i]) s = i;
    const FkSeg &S = A.seg[s];
    const int64_t f0 = ((int64_t)blockIdx.x - A.block_start[s]) * kFkTile;
    if (S.op == 0) fk_stream_tile<false, true>(S.T, S.local_rot, S.root_t, S.B, f0, S.g_rot, S.g_pos, fk_lds);
    else lrot_line_tile<false>(S.T, S.local_rot, S.B, f0, S.g_rot, fk_lds);
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
__host__ __device__ inline size_t group_lds_floats(int J, int F, int steps)
{
    return (size_t)F * J * 4 + pad16f((size_t)F * J * 3) + (size_t)steps * (64 / F) * 8;
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
RTG_DEV void group_compose(const TopoView &T, f4v *rot, float *pos, const GEnt *sch, int nfr, const LocalQ &LQ)
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
                ng = qmul_norm(g, lq);
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
        if (rec < nrec) dst[rec] = o[k];
    }
    const int npos = 3 * nrec;
    if ((reinterpret_cast<uintptr_t>(g_pos) & 15u) == 0) {
        const int n4 = npos >> 2;
        f4v *pd = reinterpret_cast<f4v *>(g_pos);
        const f4v *ps = reinterpret_cast<const f4v *>(pos);
        for (int i = lane; i < n4; i += 64) pd[i] = ps[i];
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
    rows.to_lds(rot, nrec);
    if (lane < 3 * nfr) {
        const int fr = lane / 3;
        pos[3 * J * fr + (lane - 3 * fr)] = r;
    }
    wave_sync();
    group_compose<F>(T, rot, pos, sch, nfr, [&](int, Q lq, const GEnt &e, int) {
        if (STATE) lq = qmul_norm(Q{e.qx, e.qy, e.qz, e.qw}, lq);   // skeleton3d.py:412-418
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
static inline size_t lrot_group_lds_floats(int J, int F) { return (size_t)F * J * 4 + pad16f((size_t)J) + (size_t)J * 4; }
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
                q = qmul_norm(qconj(Q{pv.x, pv.y, pv.z, pv.w}), gj);
                if (STATE) {
                    const f4v c = tqn[j];
                    q = qmul_norm(Q{c.x, c.y, c.z, c.w}, q);
                }
            }
            dst[rec] = f4v{q.x, q.y, q.z, q.w};
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

// HuForwardModel (hu_forward_model.py:17-33) on the lane groups: LDS = the tile image (root rotation at joint 0) |
// the tile's DOF rows (F (J - 1) floats) | per-joint {axis, lower, upper}
static inline size_t dof_group_lds_floats(int J, int F, int steps)
{
    return group_lds_floats(J, F, steps) + pad16f((size_t)F * (J - 1)) + (size_t)J * 4;
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
    float *ang = fk_lds + group_lds_floats(J, F, T.gsteps);
    f4v *ntab = reinterpret_cast<f4v *>(ang + pad16f((size_t)F * nd));
    // the tile's DOF rows are nfr * nd consecutive floats: NR dword loads per lane, all in flight
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
    for (int j = 1 + lane; j < J; j += 64) {
        const int ax = ld_const(D.axis + (j - 1));
        ntab[j] = f4v{__int_as_float(ax), CLIP ? ld_const(D.lower + (j - 1)) : 0.0f,
                      CLIP ? ld_const(D.upper + (j - 1)) : 0.0f, 0.0f};
    }
#pragma unroll
    for (int k = 0; k < G::NR; ++k) {
        const int i = k * 64 + lane;
        if (i < nang) ang[i] = a[k];
    }
    if (lane < nfr) rot[lane * J] = rr;   // root: global = the root rotation (hu_forward_model.py:24)
    if (lane < 3 * nfr) {
        const int fr = lane / 3;
        pos[3 * J * fr + (lane - 3 * fr)] = rt;
    }
    wave_sync();
    group_compose<F>(T, rot, pos, sch, nfr, [&](int j, Q, const GEnt &, int fr) {
        const f4v t = ntab[j];
        float x = ang[fr * nd + (j - 1)];
        if (CLIP) {   // torch.clamp (min then max; NaN passes), then the straight-through sum
            float c = x < t.y ? t.y : x;
            c = c > t.z ? t.z : c;
            x = (c - x) + x;
        }
        const int ax = __float_as_int(t.x);
        // the axis is an exact unit vector: quat_from_angle_axis's normalisation is the identity (round 5)
        return qfrom_angle_unit_axis(x, V{ax == 0 ? 1.0f : 0.0f, ax == 1 ? 1.0f : 0.0f, ax == 2 ? 1.0f : 0.0f});
    });
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
    if (S.T.gF == 16) {
        if (S.op == 0) fk_group_tile<false, 16>(S.T, S.local_rot, S.root_t, S.B, t * 16, S.g_rot, S.g_pos, fk_lds);
        else lrot_group_tile<false, 16>(S.T, S.local_rot, S.B, t * 16, S.g_rot, fk_lds);
    } else {
        if (S.op == 0) fk_group_tile<false, 8>(S.T, S.local_rot, S.root_t, S.B, t * 8, S.g_rot, S.g_pos, fk_lds);
        else lrot_group_tile<false, 8>(S.T, S.local_rot, S.B, t * 8, S.g_rot, fk_lds);
    }
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
    if (RTG_FK_GROUP && T.gsched) {
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
    } else if (T.nslots <= kMaxFkSlots) {
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
    if (RTG_FK_GROUP && T.gsched) {
        const int F = T.gF;
        const size_t lds = sizeof(float) * lrot_group_lds_floats(T.J, F);
        const dim3 gd(grid_for(B, F)), b(64);
        if (F == 16) {
            if (state) hipLaunchKernelGGL((k_lrot_group<true, 16>), gd, b, lds, s, T, g, B, l);
            else hipLaunchKernelGGL((k_lrot_group<false, 16>), gd, b, lds, s, T, g, B, l);
        } else {
            if (state) hipLaunchKernelGGL((k_lrot_group<true, 8>), gd, b, lds, s, T, g, B, l);
            else hipLaunchKernelGGL((k_lrot_group<false, 8>), gd, b, lds, s, T, g, B, l);
        }
    } else if (T.nslots <= kMaxFkSlots) {
        const dim3 gd(grid_for(B, kFkTile)), b(kFkTile);
        const size_t lds = fk_line_lds_bytes(T.J, T.nslots);
        if (state) hipLaunchKernelGGL(k_local_rotation_line<true>, gd, b, lds, s, T, g, B, l);
        else hipLaunchKernelGGL(k_local_rotation_line<false>, gd, b, lds, s, T, g, B, l);
    } else if (state) {
        hipLaunchKernelGGL(k_local_rotation<true>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, g, B, l);
    } else {
        hipLaunchKernelGGL(k_local_rotation<false>, dim3(grid_for(B, 256)), dim3(256), 0, s, T, g, B, l);
    }
    return hipGetLastError();
}

hipError_t launch_fk_multi(FkMultiArgs &A, hipStream_t s)
{
    bool group = RTG_FK_GROUP != 0;
    for (int i = 0; i < A.n; ++i) group = group && A.seg[i].T.gsched != nullptr;
    if (group) {   // every segment on the lane groups: one block per F-frame tile of its segment
        int64_t blocks = 0;
        size_t lds = 0;
        for (int i = 0; i < A.n; ++i) {
            const TopoView &T = A.seg[i].T;
            A.block_start[i] = blocks;
            blocks += grid_for(A.seg[i].B, T.gF);
            const size_t need = A.seg[i].op == 0 ? group_lds_floats(T.J, T.gF, T.gsteps) : lrot_group_lds_floats(T.J, T.gF);
            lds = need > lds ? need : lds;
        }
        for (int i = A.n; i < RTG_MAX_SEGMENTS; ++i) A.block_start[i] = blocks;
        if (blocks == 0) return hipSuccess;
        hipLaunchKernelGGL(k_fk_multi_group, dim3((unsigned)blocks), dim3(64), sizeof(float) * lds, s, A);
        return hipGetLastError();
    }
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
    int maxJ = 0;
    for (int i = 0; i < A.n; ++i) maxJ = A.seg[i].T.J > maxJ ? A.seg[i].T.J : maxJ;
    if (stream) {   // FK segments use the windows (16-joint position window), inverse segments the line tile
        const size_t lf = fk_stream_lds_bytes(maxS, true), ll = fk_line_lds_bytes(maxJ, maxS);
        hipLaunchKernelGGL(k_fk_multi_stream, dim3((unsigned)blocks), dim3(kFkTile), lf > ll ? lf : ll, s, A);
    }
    else
        hipLaunchKernelGGL(k_fk_multi, dim3((unsigned)blocks), dim3(256), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_dof_fk(const TopoView &T, const DofView &D, bool clip, const float *dof, const float *root_rot,
                         const float *root_t, int64_t B, float *gr, float *gp, hipStream_t s)
{
    if (RTG_FK_GROUP && T.gsched) {
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
        return hipGetLastError();
    }
    if (T.nslots > kMaxFkSlots) return hipErrorInvalidValue;   // rejected at rtg_dof_model_create
    const dim3 g(grid_for(B, kFkTile)), b(kFkTile);
    const size_t lds = dof_fk_lds_bytes(T.nslots);
    if (clip) hipLaunchKernelGGL(k_dof_fk<true>, g, b, lds, s, T, D, dof, root_rot, root_t, B, gr, gp);
    else hipLaunchKernelGGL(k_dof_fk<false>, g, b, lds, s, T, D, dof, root_rot, root_t, B, gr, gp);
    return hipGetLastError();
}

}  // namespace rtg
