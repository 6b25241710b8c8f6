// rtg_fk.hip -- forward / inverse kinematics kernels (kinematics.py:13-63, skeleton3d.py:402-484,
// hu_forward_model.py:17-33) and their launchers.
#include "rtg_device.cuh"

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
constexpr int kFkChunk = RTG_FK_CHUNK;   // joints per LDS window (4 or 8)
static_assert(kFkChunk == 4 || kFkChunk == 8, "window of 4 or 8 joints");
constexpr int kRotPitch = 4 * (kFkChunk + 1);   // floats per frame row (LDS)
constexpr int kPosPitch = 3 * kFkChunk + 1;

// RTG_FK_POS_WIN16: positions collect in a 16-joint LDS window and leave every second window as 192-byte row pieces
constexpr int kPos16Pitch = 3 * 16 + 1;
static_assert(kFkChunk == 8 || !(RTG_FK_POS_WIN16 || RTG_FK_MULTI_POS16), "the 16-joint position window pairs 8-joint windows");
template <bool POS16>
constexpr int pos_win() { return POS16 ? kFkTile * kPos16Pitch : (RTG_FK_POS_REGS ? 0 : kFkTile * kPosPitch); }

// Branch-parent slots: the first RTG_FK_REG_SLOTS live in registers (a slot is private to its lane, and its
// index is launch-uniform, so the choice is a scalar branch), the rest in LDS.  Every shipped skeleton needs <= 2
// slots, so their tiles use only the 9.2 KiB rotation window: 17 waves per CU instead of 12, and the 4096 tiles of
// a 262144-frame batch fit the 256 CUs in one round.
#if RTG_FK_MIN_WAVES > 0
#define RTG_FK_WAVES __attribute__((amdgpu_waves_per_eu(RTG_FK_MIN_WAVES, 8)))
#else
#define RTG_FK_WAVES
#endif
constexpr int kCarryFloats = RTG_FK_ALIGNED_STORE ? 2 * kFkTile * 16 : 0;   // rotation + position carries
static inline size_t lds_slot_floats(int nslots)
{
    return nslots > RTG_FK_REG_SLOTS ? (size_t)(nslots - RTG_FK_REG_SLOTS) * 7 * kFkTile : 0;
}
static inline size_t fk_stream_lds_bytes(int nslots, bool pos16 = RTG_FK_POS_WIN16)   // (+ RTG_FK_LDS_PAD: an occupancy experiment)
{
    const size_t pw = pos16 ? pos_win<true>() : pos_win<false>();
    return sizeof(float) * ((size_t)kFkTile * kRotPitch + pw + kCarryFloats + lds_slot_floats(nslots)) +
           RTG_FK_LDS_PAD;
}
constexpr int kDofPosWin = RTG_DOF_FK_POS_REGS ? 0 : kFkTile * kPosPitch;
static inline size_t dof_fk_lds_bytes(int nslots)
{
    return sizeof(float) * ((size_t)kFkTile * kRotPitch + (size_t)kDofPosWin + kCarryFloats + lds_slot_floats(nslots)) +
           RTG_FK_LDS_PAD;
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
            for (int c = 0; c < W; ++c) gp[c] = lp[c];
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

template <bool STATE, bool POS16 = RTG_FK_POS_WIN16>
RTG_DEV void fk_stream_tile(const TopoView &T, const float *__restrict__ local_rot, const float *__restrict__ root_t,
                            int64_t B, int64_t f0, float *__restrict__ g_rot, float *__restrict__ g_pos, float *lds)
{
    const int J = T.J;
    const int nfr = (int)((B - f0) < kFkTile ? (B - f0) : kFkTile);
    float *rot = lds;                                   // [64][kRotPitch]
    float *pos = lds + kFkTile * kRotPitch;             // [64][kPosPitch] (RTG_FK_POS_REGS: none)
    float *carry = pos + pos_win<POS16>();              // [2][64][16] (RTG_FK_ALIGNED_STORE)
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
                } else if (RTG_FK_POS_REGS) pk[k] = nt;
                else { P[3 * k] = nt.x; P[3 * k + 1] = nt.y; P[3 * k + 2] = nt.z; }
                if (!RTG_EXP_FK_COPY && ((sc >> 8) & 0xFF) != kNoSlot) slot_put(slots, (sc >> 8) & 0xFF, ng, nt);
                g = ng;
                t = nt;
            }
        }
        wave_sync();
        if (RTG_FK_ALIGNED_STORE) chunk_store_aligned<4>(g_rot, rot, kRotPitch, carry, f0, nfr, J, c0, nC);
        else chunk_store<4>(g_rot, rot, kRotPitch, f0, nfr, J, c0, nC);
        if (RTG_EXP_FK_NOPOS) {   // measurement knob: no position rows
        } else if (POS16) {   // every second window (and the last): 16 joints' positions per frame piece
            if ((c0 & 8) || c0 + nC == J) {
                const int c16 = c0 & ~15;
                chunk_store_n<3, 16>(g_pos, pos, kPos16Pitch, f0, nfr, J, c16, c0 + nC - c16);
            }
        } else if (RTG_FK_POS_REGS) {   // the rotation rows are out: reuse the window for the positions
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
template <bool STATE, bool POS16 = RTG_FK_POS_WIN16>
RTG_DEV void local_rotation_tile(const TopoView &T, const float *__restrict__ g_rot, int64_t B, int64_t f0,
                                 float *__restrict__ local_rot, float *fk_lds)
{
    const int J = T.J;
    const int nfr = (int)((B - f0) < kFkTile ? (B - f0) : kFkTile);
    float *win = fk_lds;                                 // [64][kRotPitch]
    float *carry = fk_lds + kFkTile * kRotPitch + pos_win<POS16>();
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
    if (S.op == 0) fk_stream_tile<false, RTG_FK_MULTI_POS16>(S.T, S.local_rot, S.root_t, S.B, f0, S.g_rot, S.g_pos, fk_lds);
    else local_rotation_tile<false, RTG_FK_MULTI_POS16>(S.T, S.local_rot, S.B, f0, S.g_rot, fk_lds);
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
// Row-staged FK, one quaternion component per lane (the production path).
//
// The windowed streaming kernels above move their bytes at ~3 TB/s whatever they compute (a build that skips the
// chain and copies each window straight out, RTG_EXP_FK_COPY, is only 4 % faster): every frame's row leaves in 96- and
// 128-byte pieces at 16-byte (not line) alignment, one window at a time, and lines left partly read or written
// between windows are fetched again (PMC: FETCH 1.75x, WRITE 1.22x the algorithmic bytes).  Here a wave owns a tile
// of kQuadFrames consecutive frames whose input rows and output rows are each ONE contiguous span of global memory:
//   1. the tile's input rows land in LDS as one contiguous image (16-byte LDS-DMA, 1 KiB per wave-instruction);
//   2. the tile is composed joint by joint in the image, in place (global rotations over the locals), positions into a
//      second image -- a branch parent is read back from the images, so no parent slots;
//   3. the images leave as contiguous 1 KiB wave-stores: every line is written whole, by one instruction.
// The composition runs with FOUR lanes per frame, lane 4f + c holding component c (x, y, z, w) of frame f's
// quaternions: a Hamilton product is one instruction stream in which each lane folds its own component's four
// products in the reference's order (rtg_math.cuh qmul), its operands fetched across the quad by DPP quad_perm; the
// normalisation's sum of squares is the same left fold in every lane of the quad.  So all 64 lanes are busy with 16
// frames, a wave's dependent chain is a quarter of a one-lane-per-frame chain, and the images of a 16-frame tile
// (J x 28 bytes per frame) leave ~11 waves per CU -- where the one-lane-per-frame row kernel (36 frames per wave,
// 28 lanes idle, 5 waves per CU) was slower than the streaming one.  Every value is the scalar
// device functions' own arithmetic: bit-identical (test_gpu_parity FK / inverse-FK / mixed tests).
// ----------------------------------------------------------------------------
constexpr int kQuadFrames = 16;   // frames per tile = 64 lanes / 4 components

// nbytes (a multiple of 4) from global src to LDS dst, both 16-byte aligned: 16-byte LDS-DMA (1 KiB per
// wave-instruction, lane-linear), then the last 0-3 dwords by 4-byte LDS-DMA -- nothing past src + nbytes is read
RTG_DEV void rows_load(const float *__restrict__ src, float *dst, int nbytes)
{
    const int lane = threadIdx.x & 63;
    const int n16 = nbytes & ~15;
    for (int o = 0; o < n16; o += 1024)
        if (o + 16 * lane < n16)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + (o >> 2) + 4 * lane),
                                             (__attribute__((address_space(3))) void *)(dst + (o >> 2)), 16, 0, 0);
    if (n16 < nbytes && lane < ((nbytes - n16) >> 2))
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + (n16 >> 2) + lane),
                                         (__attribute__((address_space(3))) void *)(dst + (n16 >> 2)), 4, 0, 0);
}
RTG_DEV void rows_load_wait()   // this wave's LDS-DMA has landed (the wave reads only what it loaded itself)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// n bytes (multiple of 4) from LDS src to global dst (16-byte aligned): whole 1 KiB wave-stores, then the dword tail
RTG_DEV void rows_store(float *__restrict__ dst, const float *src, int nbytes)
{
    const int lane = threadIdx.x & 63;
    const int n16 = nbytes & ~15;
    int o = 0;
    for (; o + 4096 <= n16; o += 4096) {   // four wave-stores per step: the LDS reads issue together
        float4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const float4 *>(src + ((o + 1024 * k) >> 2) + 4 * lane);
#pragma unroll
        for (int k = 0; k < 4; ++k) *reinterpret_cast<float4 *>(dst + ((o + 1024 * k) >> 2) + 4 * lane) = v[k];
    }
    for (; o < n16; o += 1024)
        if (o + 16 * lane < n16)
            *reinterpret_cast<float4 *>(dst + (o >> 2) + 4 * lane) = *reinterpret_cast<const float4 *>(src + (o >> 2) + 4 * lane);
    for (int i = (n16 >> 2) + lane; i < (nbytes >> 2); i += 64) dst[i] = src[i];
}
RTG_DEV void lds_reads_done()   // every LDS read this wave issued has returned (before an LDS-DMA overwrites it)
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// ---- component-per-lane quaternion algebra: lane c of a quad holds component c (0 x, 1 y, 2 z, 3 w)
template <int P0, int P1, int P2, int P3>
RTG_DEV float qperm(float v)   // the quad's lane P<c> value, in lane c (DPP quad_perm)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v),
                                                              P0 | (P1 << 2) | (P2 << 4) | (P3 << 6), 0xF, 0xF, false));
}
RTG_DEV float xorf(float v, uint32_t m) { return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, v) ^ m); }
struct QLane {
    int c;           // this lane's component
    uint32_t wneg;   // sign bit in the w lane: its 2nd and 3rd products are subtracted (a - b == a + (-b), exactly)
    uint32_t conj;   // sign bit in the x, y, z lanes (qconj)
};
RTG_DEV QLane qlane()
{
    const int c = threadIdx.x & 3;
    return QLane{c, c == 3 ? 0x80000000u : 0u, c < 3 ? 0x80000000u : 0u};
}
RTG_DEV float qsel(const QLane &L, Q q) { return L.c == 0 ? q.x : (L.c == 1 ? q.y : (L.c == 2 ? q.z : q.w)); }
// qmul (rotation3d.py:14-27): component c = ((t1 +- t2) +- t3) - t4, each product rounded, in the scalar order:
//   x: ((aw bx + ax bw) + ay bz) - az by      y: ((aw by + ay bw) + az bx) - ax bz
//   z: ((aw bz + az bw) + ax by) - ay bx      w: ((aw bw - ax bx) - ay by) - az bz
RTG_DEV float qmul_l(const QLane &L, float a, float b)
{
    const float t1 = qperm<3, 3, 3, 3>(a) * b;
    const float t2 = xorf(qperm<0, 1, 2, 0>(a), L.wneg) * qperm<3, 3, 3, 0>(b);
    const float t3 = xorf(qperm<1, 2, 0, 1>(a), L.wneg) * qperm<2, 0, 1, 1>(b);
    const float t4 = qperm<2, 0, 1, 2>(a) * qperm<1, 2, 0, 2>(b);
    return ((t1 + t2) + t3) - t4;
}
// qnormalize (quat_unit(quat_pos(q)), rotation3d.py:30-56): w >= 0, then / max(|q|, 1e-9) -- the sum of squares is
// the same left fold in every lane of the quad, and a lane's quotient is mulr's (equal to mulr_k's, rtg_math.cuh)
RTG_DEV float qnormalize_l(float q)
{
    const float f = 1.0f - 2.0f * (qperm<3, 3, 3, 3>(q) < 0.0f ? 1.0f : 0.0f);
    q = f * q;
    const float q0 = qperm<0, 0, 0, 0>(q), q1 = qperm<1, 1, 1, 1>(q), q2 = qperm<2, 2, 2, 2>(q), q3 = qperm<3, 3, 3, 3>(q);
    const Rcp r = sqrt_clamp_rcp(((q0 * q0 + q1 * q1) + q2 * q2) + q3 * q3, 1e-9f).r;
    return mulr(q, r);
}
RTG_DEV float qmul_norm_l(const QLane &L, float a, float b) { return qnormalize_l(qmul_l(L, a, b)); }
// qrotate (rotation3d.py:205-211): imag((q (v, 0)) conj(q)); lanes 0-2 hold x, y, z
RTG_DEV float qrotate_l(const QLane &L, float q, V v)
{
    const float vb = L.c == 0 ? v.x : (L.c == 1 ? v.y : (L.c == 2 ? v.z : 0.0f));
    return qmul_l(L, qmul_l(L, q, vb), xorf(q, L.conj));
}

// FK of a tile (nfr frames valid; the quads of the others compute on whatever the image holds and store nothing
// that leaves LDS) whose input rows are in the rotation image (kinematics.py:13-39; STATE: skeleton3d.py:402-430):
// global rotations over the locals in place, translations into the position image.  rootc: this lane's component
// of its frame's root translation (lanes 0-2).
template <bool STATE>
RTG_DEV void fk_quad_compute(const TopoView &T, float rootc, float *rot, float *pos)
{
    const int J = T.J;
    const QLane L = qlane();
    const int fr = (threadIdx.x & 63) >> 2;
    float *R = rot + fr * J * 4 + L.c;
    float *P = pos + fr * J * 3 + (L.c < 3 ? L.c : 2);
    float g = R[0];   // root: global = local, unnormalised (kinematics.py:27-29)
    float t = rootc;
    if (L.c < 3) P[0] = t;
    float next = J > 1 ? R[4] : g;   // joint j+1's input is read while joint j composes
    for (int j = 1; j < J; ++j) {
        float lq = next;
        if (j + 1 < J) next = R[4 * (j + 1)];
        const int p = ld_const(T.parents + j);
        if (p != j - 1) {   // a branch parent: read back from the images (launch-uniform branch)
            g = R[4 * p];
            t = P[3 * p];
        }
        if (STATE) lq = qmul_norm_l(L, qsel(L, ld_const(T.tree_quat + j)), lq);   // skeleton3d.py:412-418
        const float rv = qrotate_l(L, g, ld_const(T.local_t + j));
        g = qmul_norm_l(L, g, lq);
        t = rv + t;
        R[4 * j] = g;
        if (L.c < 3) P[3 * j] = t;
    }
}

// inverse FK of a tile in the image (kinematics.py:41-63; STATE: skeleton3d.py:468-484).  Joints run from the last
// to the first, in place: joint j needs g[p] (p < j, not yet overwritten) and g[j].
template <bool STATE>
RTG_DEV void local_quad_compute(const TopoView &T, float *img)
{
    const int J = T.J;
    const QLane L = qlane();
    float *W = img + ((threadIdx.x & 63) >> 2) * J * 4 + L.c;
    for (int j = J - 1; j > 0; --j) {   // the root row is copied as it is (kinematics.py:49)
        const int p = ld_const(T.parents + j);
        float q = qmul_norm_l(L, xorf(W[4 * p], L.conj), W[4 * j]);
        if (STATE) {   // skeleton3d.py:470-478
            const float tq = qnormalize_l(xorf(qsel(L, ld_const(T.tree_quat + j)), L.conj));
            q = qmul_norm_l(L, tq, q);
        }
        W[4 * j] = q;
    }
}

// Tiles of every segment (FK or inverse FK) in one persistent launch.  The rotation image sits at the start of the
// wave's LDS, the position image at pos_off floats (past the largest rotation image, so a next tile of another
// segment never overlaps it).  Each wave walks tiles blockIdx.x, + gridDim.x, ...: it stores tile t's rotation
// image, then issues tile t+1's input DMA into that image (the image's LDS reads are done), then stores t's
// positions -- the next input is in flight while the stores leave.
template <bool STATE>
__global__ __launch_bounds__(64) void k_kin_quad(FkMultiArgs A, int32_t pos_off, int64_t ntiles)
{
    extern __shared__ __attribute__((aligned(16))) float fk_lds[];
    const int lane = threadIdx.x & 63;
    float *img = fk_lds, *pos = fk_lds + pos_off;
    struct Tile {
        int s, nfr;
        int64_t f0;
    };
    auto decode = [&](int64_t t) {
        int s = 0;
#pragma unroll
        for (int i = 1; i < RTG_MAX_SEGMENTS; ++i)
            if (i < A.n && t >= A.block_start[i]) s = i;
        const int64_t f0 = (t - A.block_start[s]) * kQuadFrames, left = A.seg[s].B - f0;
        return Tile{s, (int)(left < kQuadFrames ? left : kQuadFrames), f0};
    };
    auto issue = [&](const Tile &k, float &rootc) {   // the tile's input rows -> the image; the root translations
        const FkSeg &S = A.seg[k.s];
        rows_load(S.local_rot + k.f0 * S.T.J * 4, img, k.nfr * S.T.J * 16);
        const int fr = lane >> 2, c = lane & 3;
        if (S.op == 0 && fr < k.nfr && c < 3) rootc = S.root_t[(k.f0 + fr) * 3 + c];
    };
    int64_t t = blockIdx.x;
    if (t >= ntiles) return;
    Tile k = decode(t);
    float root = 0.0f;
    issue(k, root);
    for (;;) {
        rows_load_wait();
        const FkSeg &S = A.seg[k.s];
        const int J = S.T.J;
        const int64_t tn = t + gridDim.x;
        const bool more = tn < ntiles;
        const Tile kn = more ? decode(tn) : k;
        float rootn = 0.0f;
        if (S.op == 0) fk_quad_compute<STATE>(S.T, root, img, pos);
        else local_quad_compute<STATE>(S.T, img);
        wave_sync();
        rows_store(S.g_rot + k.f0 * J * 4, img, k.nfr * J * 16);
        lds_reads_done();
        wave_sync();
        if (more) issue(kn, rootn);
        if (S.op == 0) rows_store(S.g_pos + k.f0 * J * 3, pos, k.nfr * J * 12);
        if (!more) break;
        wave_sync();
        t = tn;
        k = kn;
        root = rootn;
    }
}

static inline bool al16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

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

// The quad kernel needs 16-byte aligned rows (LDS-DMA and dwordx4 stores)
static bool quad_ok(const FkMultiArgs &A)
{
    if (!RTG_FK_QUAD) return false;
    for (int i = 0; i < A.n; ++i) {
        const FkSeg &S = A.seg[i];
        if (!al16(S.local_rot) || !al16(S.g_rot) || (S.op == 0 && !al16(S.g_pos))) return false;
    }
    return true;
}
// Launch k_kin_quad over A's segments: tile starts, image offsets, a persistent grid of what fits the device.
static hipError_t launch_quad(FkMultiArgs &A, bool state, hipStream_t s)
{
    int64_t tiles = 0;
    int rot = 4, pos = 0;   // floats of the largest rotation / position image
    for (int i = 0; i < A.n; ++i) {
        const int J = A.seg[i].T.J;
        A.block_start[i] = tiles;
        tiles += grid_for(A.seg[i].B, kQuadFrames);
        rot = kQuadFrames * J * 4 > rot ? kQuadFrames * J * 4 : rot;
        if (A.seg[i].op == 0) pos = kQuadFrames * J * 3 > pos ? kQuadFrames * J * 3 : pos;
    }
    for (int i = A.n; i < RTG_MAX_SEGMENTS; ++i) A.block_start[i] = tiles;
    if (tiles == 0) return hipSuccess;
    const size_t lds = sizeof(float) * (size_t)(rot + pos);
    const void *fn = state ? (const void *)k_kin_quad<true> : (const void *)k_kin_quad<false>;
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, lds);
    if (e != hipSuccess) return e;
    const int64_t slots = (int64_t)(per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 1);
    const unsigned grid = (unsigned)(tiles < slots ? tiles : slots);
    if (state) hipLaunchKernelGGL(k_kin_quad<true>, dim3(grid), dim3(64), lds, s, A, rot, tiles);
    else hipLaunchKernelGGL(k_kin_quad<false>, dim3(grid), dim3(64), lds, s, A, rot, tiles);
    return hipGetLastError();
}
static FkMultiArgs one_segment(const TopoView &T, int op, const float *in, const float *rt, int64_t B, float *out,
                               float *pos)
{
    FkMultiArgs A{};
    A.seg[0] = FkSeg{T, in, rt, out, pos, B, op};
    A.n = 1;
    return A;
}

hipError_t launch_fk(const TopoView &T, bool state, const float *lr, const float *rt, int64_t B, float *gr, float *gp,
                     hipStream_t s)
{
    FkMultiArgs A = one_segment(T, 0, lr, rt, B, gr, gp);
    if (quad_ok(A)) return launch_quad(A, state, s);
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
    FkMultiArgs A = one_segment(T, 1, g, nullptr, B, l, nullptr);
    if (quad_ok(A)) return launch_quad(A, state, s);
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
    if (quad_ok(A)) return launch_quad(A, false, s);
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
        hipLaunchKernelGGL(k_fk_multi_stream, dim3((unsigned)blocks), dim3(kFkTile), fk_stream_lds_bytes(maxS, RTG_FK_MULTI_POS16), s, A);
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

}  // namespace rtg
