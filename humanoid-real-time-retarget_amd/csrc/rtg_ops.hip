// rtg_ops.hip -- motion prep, ingest, elementwise primitives, Kabsch / Euler ops, velocities, synthetic
// frames, and the build-configuration record.
#include "rtg_device.cuh"

namespace rtg {

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

// VTRDyn ingest (sim_full_body_teleop.py:92,109-112: body 23 -> 21 points, hands reordered, the "frame carries data"
// flag): one 256-thread block per tile of TILE frames.  Each input's tile rows are ONE contiguous span (TILE x 69 / 60 /
// 60 floats); every thread issues all its loads of the three spans before it stores any into LDS (a load-then-store
// loop leaves the tile latency-bound), and the outputs leave coalesced too -- AoS rows (the tile's TILE x 63 / 60
// floats are again one span) or SoA planes (TILE consecutive frames per plane).  LDS rows are padded to an odd
// stride so the SoA pass (lanes on consecutive frames) reads distinct banks.  Round 3 moved each frame on one
// thread: 12-byte pieces 276 / 240 bytes apart per lane, 64 lines per wave instruction (1.3 TB/s).
// frames per block, measured at B = 262144 (profiles/r04/aux/ingest_tiles.log): AoS out 64 / 32 / 16 frames 89 / 82 /
// 80 us; SoA out 128 / 64 / 32 / 16 frames 200 / 111 / 90 / 104 us (smaller tiles: more blocks per CU; SoA below
// 32 frames writes half lines per plane)
constexpr int kIngAosTile = 16, kIngSoaTile = 32;
constexpr int kIngBodyS = 69, kIngHandS = 61;   // LDS row strides (floats)
template <int TILE, int R, int RS, int O>
RTG_DEV void ingest_rows_out(const float *srow, float *__restrict__ out, const int8_t *map, int64_t f0, int nfr,
                             int64_t B, bool soa)
{
    if (!soa) {
        const int n = nfr * O;
        float *dst = out + f0 * O;
        for (int e = threadIdx.x; e < n; e += 256) {
            const int fr = e / O, k = e - fr * O, j = k / 3, c = k - 3 * j;
            dst[e] = srow[fr * RS + 3 * map[j] + c];
        }
    } else {
        for (int e = threadIdx.x; e < O * TILE; e += 256) {
            const int plane = e / TILE, fr = e - plane * TILE, j = plane / 3, c = plane - 3 * j;
            if (fr < nfr) out[(int64_t)plane * B + f0 + fr] = srow[fr * RS + 3 * map[j] + c];
        }
    }
}
// the tile's span of R-float rows (n floats) into registers: element tid + 256 k
template <int TILE, int R>
RTG_DEV void ingest_load(const float *src, int n, float (&v)[(TILE * R + 255) / 256])
{
#pragma unroll
    for (int k = 0; k < (TILE * R + 255) / 256; ++k) {
        const int e = (int)threadIdx.x + 256 * k;
        v[k] = e < n ? src[e] : 0.0f;
    }
}
template <int TILE, int R, int RS>
RTG_DEV void ingest_to_lds(const float (&v)[(TILE * R + 255) / 256], int n, float *srow)
{
#pragma unroll
    for (int k = 0; k < (TILE * R + 255) / 256; ++k) {
        const int e = (int)threadIdx.x + 256 * k;
        if (e < n) srow[(e / R) * RS + e % R] = v[k];
    }
}
template <int TILE>
__global__ __launch_bounds__(256) void k_ingest_vtrdyn(const float *__restrict__ bp, const float *__restrict__ lhp,
                                                       const float *__restrict__ rhp, int64_t B,
                                                       float *__restrict__ body, float *__restrict__ lh,
                                                       float *__restrict__ rh, uint8_t *__restrict__ valid, bool soa)
{
    __shared__ float sbody[TILE * kIngBodyS], slh[TILE * kIngHandS], srh[TILE * kIngHandS];
    __shared__ int sdata[TILE];   // the frame carries data: not np.allclose(body_pos, 0)
    const int64_t f0 = (int64_t)blockIdx.x * TILE;
    const int nfr = (int)((B - f0) < TILE ? (B - f0) : TILE);
    const int tid = threadIdx.x;
    float vb[(TILE * 69 + 255) / 256], vl[(TILE * 60 + 255) / 256], vr[(TILE * 60 + 255) / 256];
    ingest_load<TILE, 69>(bp + f0 * 69, nfr * 69, vb);
    ingest_load<TILE, 60>(lhp + f0 * 60, nfr * 60, vl);
    ingest_load<TILE, 60>(rhp + f0 * 60, nfr * 60, vr);
    for (int e = tid; e < TILE; e += 256) sdata[e] = 0;
    __syncthreads();
    // the flag over all 69 body values (|x| <= 1e-8 everywhere; a NaN is never close): every writer stores 1
#pragma unroll
    for (int k = 0; k < (TILE * 69 + 255) / 256; ++k) {
        const int e = tid + 256 * k;
        if (e < nfr * 69 && !(fabsf(vb[k]) <= 1e-8f)) sdata[e / 69] = 1;
    }
    ingest_to_lds<TILE, 69, kIngBodyS>(vb, nfr * 69, sbody);
    ingest_to_lds<TILE, 60, kIngHandS>(vl, nfr * 60, slh);
    ingest_to_lds<TILE, 60, kIngHandS>(vr, nfr * 60, srh);
    __syncthreads();
    ingest_rows_out<TILE, 69, kIngBodyS, 63>(sbody, body, c_body23_to_21, f0, nfr, B, soa);
    ingest_rows_out<TILE, 60, kIngHandS, 60>(slh, lh, c_hand_order, f0, nfr, B, soa);
    ingest_rows_out<TILE, 60, kIngHandS, 60>(srh, rh, c_hand_order, f0, nfr, B, soa);
    for (int e = tid; e < nfr; e += 256) valid[f0 + e] = sdata[e] ? 1 : 0;
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
    case RTG_OP_EXP_MAP_TO_ANGLE_AXIS: st4(out + 4 * i, exp_map_angle_axis(ld3(a + 3 * i))); break;
    case RTG_OP_EXP_MAP_TO_QUAT: {
        const Q aa = exp_map_angle_axis(ld3(a + 3 * i));
        st4(out + 4 * i, qfrom_angle_axis(aa.x, V{aa.y, aa.z, aa.w}));
        break;
    }
    case RTG_OP_QUAT_SLERP: st4(out + 4 * i, qslerp(ld4(a + 4 * i), ld4(b + 4 * i), c[i])); break;
    case RTG_OP_QUAT_FROM_XYZ: {
        const V v = ld3(a + 3 * i);
        st4(out + 4 * i, Q{v.x, v.y, v.z, 1.0f - lnorm3(v)});
        break;
    }
    case RTG_OP_ROT_MATRIX_DET: {
        float m[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) m[k] = a[9 * i + k];
        out[i] = rotmat_det(m);
        break;
    }
    case RTG_OP_ROT_MATRIX_FROM_QUAT: {
        float m[9];
        rotmat_from_quat(ld4(a + 4 * i), m);
#pragma unroll
        for (int k = 0; k < 9; ++k) out[9 * i + k] = m[k];
        break;
    }
    case RTG_OP_ROTATION_ALONG_X:
    case RTG_OP_ROTATION_ALONG_Y:
    case RTG_OP_ROTATION_ALONG_Z: out[i] = axis_angle_of(ld4(a + 4 * i), op - RTG_OP_ROTATION_ALONG_X); break;
    case RTG_OP_PROJECT_QUAT_X:
    case RTG_OP_PROJECT_QUAT_Y:
    case RTG_OP_PROJECT_QUAT_Z: {
        const int ax = op - RTG_OP_PROJECT_QUAT_X;
        st4(out + 4 * i, axis_half_quat(ax, axis_angle_of(ld4(a + 4 * i), ax)));
        break;
    }
    case RTG_OP_PROJECT_QUAT_XY:
    case RTG_OP_PROJECT_QUAT_XZ: {
        const Q q = ld4(a + 4 * i);
        const int ax2 = op == RTG_OP_PROJECT_QUAT_XY ? 1 : 2;
        st4(out + 4 * i, qmul(axis_half_quat(0, axis_angle_of(q, 0)), axis_half_quat(ax2, axis_angle_of(q, ax2))));
        break;
    }
    default: break;
    }
}

// scipy Rotation.from_quat(q).as_euler(seq[, degrees]) in float64 (rotation3d.py:658-661 quat_to_eular)
__global__ __launch_bounds__(256) void k_quat_as_euler(const float *__restrict__ q, int s0, int s1, int s2,
                                                       int extrinsic, int degrees, int64_t n, double *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double ang[3];
    const bool refused = scipy_as_euler(ld4(q + 4 * i), s0, s1, s2, extrinsic != 0, ang);
    const double marked = __builtin_bit_cast(double, 0x7FF8000000000000ull | RTG_FRAME_ZERO_NORM_QUAT);
#pragma unroll
    for (int t = 0; t < 3; ++t) out[3 * i + t] = refused ? marked : (degrees ? ang[t] * (180.0 / M_PI) : ang[t]);   // np.rad2deg
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
    bool svd_nan;
    const Q q = cal_joint_quat<N>(z, m, svd_nan);
    const float marked = __builtin_bit_cast(float, RTG_FRAME_NAN | RTG_FRAME_SVD_NONFINITE);
    st4(out + 4 * i, svd_nan ? Q{marked, marked, marked, marked} : q);
}

__global__ __launch_bounds__(256) void k_quat_in_xyz_axis(const float *__restrict__ q, int s0, int s1, int s2,
                                                          int extrinsic, int64_t n, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Q e[3];
    const bool refused = quat_in_xyz_axis(ld4(q + 4 * i), s0, s1, s2, extrinsic != 0, e);
    const float marked = __builtin_bit_cast(float, RTG_FRAME_NAN | RTG_FRAME_ZERO_NORM_QUAT);
#pragma unroll
    for (int t = 0; t < 3; ++t) st4(out + (i * 3 + t) * 4, refused ? Q{marked, marked, marked, marked} : e[t]);
}

// ----------------------------------------------------------------------------
// motion velocities (skeleton3d.py:1126-1146).  The data are rows of C channels (one row per (sequence, frame),
// rows = nseq * L, the frame fastest within a sequence).  A 256-thread block covers 256 / Cp consecutive rows, Cp =
// C rounded up to a power of two, so a thread's (row, channel) is a shift and a mask, and its frame t = row % L is
// one 32-bit remainder per thread (round 3 divided the flat 64-bit index by C and L per thread: 64-bit division
// dominated the kernels).  Rows wider than 256 channels take one row per block and gridDim.y 256-channel slices.
// Launches cover at most 2^30 rows each (row0 offsets the chunks).
// ----------------------------------------------------------------------------
struct RowTile {
    int64_t row0;       // first row of this launch
    uint32_t rows;      // rows in this launch
    uint32_t L;         // frames per sequence
    int32_t C, cp_log2; // channels per row, log2(Cp)
};
RTG_DEV bool row_tile(const RowTile &rt, int64_t &row, int &ch, uint32_t &t)
{
    const uint32_t r = (blockIdx.x << (8 - rt.cp_log2)) + (threadIdx.x >> rt.cp_log2);
    ch = (int)(threadIdx.x & ((1u << rt.cp_log2) - 1u)) + (int)(blockIdx.y << 8);   // y: 256-channel slices
    if (r >= rt.rows || ch >= rt.C) return false;
    row = rt.row0 + r;
    t = (uint32_t)(row % (int64_t)rt.L);
    return true;
}
// np.gradient along frames (edge_order 1, unit spacing) then / dt, all float32
__global__ __launch_bounds__(256) void k_gradient_dt(const float *__restrict__ p, RowTile rt, float dt,
                                                     float *__restrict__ v)
{
    int64_t row;
    int ch;
    uint32_t t;
    if (!row_tile(rt, row, ch, t)) return;
    const int64_t S = rt.C, i = row * S + ch;
    const uint32_t L = rt.L;
    float g;
    if (L == 1) g = 0.0f;   // numpy raises for < 2 frames; rtg_* rejects L < 2 before launch
    else if (t == 0) g = (p[i + S] - p[i]) / 1.0f;
    else if (t == L - 1) g = (p[i] - p[i - S]) / 1.0f;
    else g = (p[i + S] - p[i - S]) / 2.0f;
    v[i] = g / dt;
}

// quat_mul_norm(r[t+1], quat_inverse(r[t])) -> quat_angle_axis -> axis * angle / dt (last frame: identity -> 0)
__global__ __launch_bounds__(256) void k_angular_raw(const float *__restrict__ r, RowTile rt, float dt,
                                                     float *__restrict__ v)
{
    int64_t row;
    int ch;
    uint32_t t;
    if (!row_tile(rt, row, ch, t)) return;
    const int64_t J = rt.C, i = row * J + ch;
    Q d = qident();
    if (t < rt.L - 1) d = qmul_norm(ld4(r + 4 * (i + J)), qconj(ld4(r + 4 * i)));
    const Q aa = qangle_axis_abs(d);
    v[3 * i + 0] = (aa.y * aa.x) / dt;
    v[3 * i + 1] = (aa.z * aa.x) / dt;
    v[3 * i + 2] = (aa.w * aa.x) / dt;
}

// scipy.ndimage.gaussian_filter1d(mode='nearest') along frames: symmetric correlate1d,
// float64 accumulation from the outermost tap pair inwards, rounded to float32 once
__global__ __launch_bounds__(256) void k_gauss_nearest(const float *__restrict__ v, RowTile rt, GaussTaps taps,
                                                       float *__restrict__ out)
{
    int64_t row;
    int ch;
    uint32_t t;
    if (!row_tile(rt, row, ch, t)) return;
    const int64_t S = rt.C, i = row * S + ch, base = i - (int64_t)t * S;
    const int R = taps.radius;
    const int64_t L = rt.L;
    auto at = [&](int64_t tt) { tt = tt < 0 ? 0 : (tt > L - 1 ? L - 1 : tt); return (double)v[base + tt * S]; };
    double acc = at(t) * taps.w[R];
    for (int jj = -R; jj < 0; ++jj) acc += (at((int64_t)t + jj) + at((int64_t)t - jj)) * taps.w[R + jj];
    out[i] = (float)acc;
}

// Smoothed velocities in one pass (the path the reference takes: SkeletonMotion always smooths).  A block owns
// frames [t0, t0 + T) of one sequence: it computes the raw velocity of frames [t0 - R, t0 + T + R) (clamped to
// the sequence, the 'nearest' edge) straight from the input rows into LDS, then the smoothed rows from LDS, so the
// intermediate never touches HBM and the input and output rows stream once each (the halo re-reads, 2R of T rows,
// hit L2).  Rows of a sequence are contiguous, so both passes walk contiguous memory with consecutive lanes.
// Arithmetic is the per-element kernels' above, operation for operation.
struct VelTile {
    int64_t seq0;       // first sequence of this launch
    uint32_t L, T;      // frames per sequence, frames per block
    uint32_t tiles;     // blocks per sequence
    uint32_t nblocks;   // blocks in this launch
    int32_t C, J;       // output channels per row; joints (angular) or input channels (linear)
    double rdt;         // RN(1 / (double)dt): the quotients by dt as mulr products (rtg_math.cuh), the same values
};
// (row, channel) of flat element e = row * C + ch, advanced by 256 elements per step without a division
struct RowWalk {
    uint32_t rr, ch, dq, dr;
    RTG_DEV RowWalk(uint32_t e0, uint32_t C) : rr(e0 / C), ch(e0 - (e0 / C) * C), dq(256u / C), dr(256u - (256u / C) * C) {}
    RTG_DEV void next(uint32_t C)
    {
        rr += dq;
        ch += dr;
        if (ch >= C) { ch -= C; ++rr; }
    }
};

// LDS row stride (floats) of one channel's raw values in a tile: T + 2R rows, odd so that lanes on consecutive
// channels hit distinct banks
__host__ __device__ inline uint32_t vel_lds_stride(uint32_t T, int R) { return (T + 2u * (uint32_t)R) | 1u; }

// W consecutive smoothed outputs of one channel from its raw values x[0 .. W + 2R) in LDS (x[k]: frame t - R + k,
// edges already replicated), the k_gauss_nearest sum operation for operation; each raw value is widened to double
// once for the W outputs that read it
template <int RC, int W>
RTG_DEV void gauss_rows(const float *x, const GaussTaps &taps, double (&acc)[W])
{
    constexpr int N = W + 2 * RC;
    double v[N];
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = (double)x[k];
#pragma unroll
    for (int r = 0; r < W; ++r) {
        double a = v[r + RC] * taps.w[RC];
#pragma unroll
        for (int jj = -RC; jj < 0; ++jj) a += (v[r + RC + jj] + v[r + RC - jj]) * taps.w[RC + jj];
        acc[r] = a;
    }
}
RTG_DEV double gauss_row_any(const float *x, const GaussTaps &taps)
{
    const int R = taps.radius;
    double a = (double)x[R] * taps.w[R];
    for (int jj = -R; jj < 0; ++jj) a += ((double)x[R + jj] + (double)x[R - jj]) * taps.w[R + jj];
    return a;
}

// Phase 1 computes the raw velocity of frames t0 - R .. t1 - 1 + R, each clamped into the sequence (the 'nearest'
// edge: a frame outside repeats the edge frame's raw value), into LDS channel-major; phase 2 runs the filter over
// LDS without a clamp.  RC >= 0: the filter radius as a constant (4 outputs per thread from a sliding window).
template <bool ANGULAR, int RC>
__global__ __launch_bounds__(256) void k_velocity_tile(const float *__restrict__ src, VelTile vt, float dt,
                                                       GaussTaps taps, float *__restrict__ out)
{
    extern __shared__ float sg[];   // [C][stride] raw values of frames t0 - R ..
    // XCD-aware order: the 8 XCDs take blocks round-robin, so give each XCD a contiguous run of tiles (their
    // halo rows are then in that XCD's L2)
    uint32_t b = blockIdx.x;
    if ((vt.nblocks & 7u) == 0u) b = (b & 7u) * (vt.nblocks >> 3) + (b >> 3);
    const uint32_t tile = b % vt.tiles;
    const int64_t seq = vt.seq0 + b / vt.tiles;
    const int R = RC >= 0 ? RC : taps.radius;
    const int C = vt.C;
    const int L = (int)vt.L;
    const uint32_t NS = vel_lds_stride(vt.T, R);
    const int t0 = (int)(tile * vt.T);
    const int t1 = min(t0 + (int)vt.T, L);
    const uint32_t nx = (uint32_t)(t1 - t0 + 2 * R);   // raw rows this tile reads
    // every thread issues the loads of NB elements before it uses any (latency, not bandwidth, bounds a
    // load-then-use loop at this occupancy)
    if (!ANGULAR) {
        // Round 5: a thread owns a run of SEG rows of one channel and loads the run's SEG + 2 raw values (frames
        // x0 - 1 .. x0 + SEG) all at once -- 64 lanes on consecutive channels read one row's 256 contiguous bytes
        // per instruction -- then takes the SEG gradients from its own registers (round 4: two global loads per
        // gradient, 8 gradients at a time, four memory round trips per tile).  Runs that reach a sequence end take
        // the clamped, one-sided per-element form.
        constexpr int SEG = RTG_VEL_SEG;
        const float *p = src + seq * L * C;
        const uint32_t nseg = (nx + SEG - 1) / SEG;
        const uint32_t items = nseg * (uint32_t)C;
        for (uint32_t it = threadIdx.x; it < items; it += 256u) {
            const uint32_t sgi = it / (uint32_t)C, ch = it - sgi * (uint32_t)C;
            const int r0 = (int)sgi * SEG, x0 = t0 - R + r0;
            const int nr = min(SEG, (int)nx - r0);
            float *dst = sg + ch * NS + r0;
            if (x0 >= 1 && x0 + nr <= L - 1) {   // every frame of the run and its neighbours inside the sequence
                const float *q = p + (int64_t)(x0 - 1) * C + ch;
                float raw[SEG + 2];
#pragma unroll
                for (int k = 0; k < SEG + 2; ++k) raw[k] = k < nr + 2 ? q[(int64_t)k * C] : 0.0f;
                // np.gradient inside the sequence: (p[t+1] - p[t-1]) / 2 (x / 2 == x * 0.5, correctly rounded)
#if RTG_VEL_IEEE_DIV   // A/B knob (same values): one IEEE division per gradient
#pragma unroll
                for (int j = 0; j < SEG; ++j)
                    if (j < nr) dst[j] = ((raw[j + 2] - raw[j]) * 0.5f) / dt;
#else
                // the SEG quotients by dt through the shared reciprocal (mulr_k: one rare-case branch per run)
                float g[SEG], v[SEG];
#pragma unroll
                for (int j = 0; j < SEG; ++j) g[j] = (raw[j + 2] - raw[j]) * 0.5f;
                mulr_k<SEG>(g, Rcp{vt.rdt, dt}, v);
#pragma unroll
                for (int j = 0; j < SEG; ++j)
                    if (j < nr) dst[j] = v[j];
#endif
            } else {
                for (int j = 0; j < nr; ++j) {
                    const int x = x0 + j;
                    const int t = x < 0 ? 0 : (x > L - 1 ? L - 1 : x);
                    const int64_t i = (int64_t)t * C + ch;
                    // one-sided differences / 1 at the ends
                    const int64_t ih = t == L - 1 ? i : i + C, il = t == 0 ? i : i - C;
                    const float hf = (t == 0 || t == L - 1) ? 1.0f : 0.5f;
                    dst[j] = ((p[ih] - p[il]) * hf) / dt;
                }
            }
        }
    } else {
        // measured: NB 2 > 4 > 8 (78 VGPRs, 6 waves/SIMD at 2); round 5's per-thread runs of 6 joint rows (the linear
        // branch's form) 128-132 vs 124-125 us (86 VGPRs, 5 waves/SIMD; profiles/r05/aux/)
        constexpr int NB = RTG_VEL_ANG_NB;
        const int J = vt.J;
        const float *r = src + seq * L * J * 4;
        const uint32_t n = nx * (uint32_t)J;
        RowWalk w(threadIdx.x, (uint32_t)J);
        // batches of NB elements: loads, then arithmetic (the next batch's loads issued before this batch's arithmetic
        // measured slower, 119-121 vs 116 us, profiles/r05/aux/angpipe_*)
        Q qa[NB], qb[NB];
        bool last[NB];
        uint32_t at[NB];
        auto fetch = [&](uint32_t e0) {
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                const uint32_t e = e0 + 256u * k;
                const int x = t0 - R + (int)w.rr;
                const int t = x < 0 ? 0 : (x > L - 1 ? L - 1 : x);
                const int64_t i = (int64_t)t * J + w.ch;
                last[k] = t >= L - 1;
                at[k] = 3u * w.ch * NS + w.rr;
                if (e < n && !last[k]) { qa[k] = ld4(r + 4 * (i + J)); qb[k] = ld4(r + 4 * i); }
                w.next((uint32_t)J);
            }
        };
        if (threadIdx.x < n) fetch(threadIdx.x);
#if RTG_VEL_UNIT_TAB && RTG_VEL_ANG_NWAY && !RTG_VEL_IEEE_DIV
        // the near-unit normalisation table (rtg_math.cuh) for the quaternion products, filled while the first loads fly
        __shared__ UnitEnt utab[2 * kUnitTabK + 1];
        unit_tab_fill(utab, (int)threadIdx.x);
        __syncthreads();
#endif
        for (uint32_t e0 = threadIdx.x; e0 < n; e0 += 256 * NB) {
            Q ca[NB], cb[NB];
            bool cl[NB];
            uint32_t cat[NB];
#pragma unroll
            for (int k = 0; k < NB; ++k) { ca[k] = qa[k]; cb[k] = qb[k]; cl[k] = last[k]; cat[k] = at[k]; }
#if RTG_VEL_ANG_NWAY && !RTG_VEL_IEEE_DIV
            // round 6: the NB elements on the N-way leaf math (one rare-case branch per step for all of them, so
            // their instruction streams interleave); every element's value as below.  Elements past the rows and
            // last frames compute on whatever they hold and are replaced / not stored.
            {
                Q prod[NB], dn[NB], d[NB];
#pragma unroll
                for (int k = 0; k < NB; ++k) prod[k] = qmul(ca[k], qconj(cb[k]));
#if RTG_VEL_UNIT_TAB
                qnormalize_tab_n<NB>(prod, utab, dn);
#else
                qnormalize_n<NB>(prod, dn);
#endif
                float c[NB], s3[NB];
                V xyz[NB];
#pragma unroll
                for (int k = 0; k < NB; ++k) {   // quat_angle_axis (rotation3d.py:230-240), qangle_axis_abs
                    d[k] = cl[k] ? qident() : dn[k];
                    c[k] = clamp_lohi(2.0f * (d[k].w * d[k].w) - 1.0f, -1.0f, 1.0f);
                    s3[k] = (d[k].x * d[k].x + d[k].y * d[k].y) + d[k].z * d[k].z;
                    xyz[k] = V{d[k].x, d[k].y, d[k].z};
                }
                float ang[NB];
                cr_acos_n<NB>(c, ang);
                NormRcp nr[NB], rdt[NB];
                sqrt_clamp_rcp_n<NB>(s3, 1e-9f, nr);
                V ax[NB], prod3[NB], av[NB];
                mulr_v_n<NB>(xyz, nr, ax);
#pragma unroll
                for (int k = 0; k < NB; ++k) {
                    prod3[k] = V{ax[k].x * ang[k], ax[k].y * ang[k], ax[k].z * ang[k]};
                    rdt[k] = NormRcp{dt, Rcp{vt.rdt, dt}};
                }
                mulr_v_n<NB>(prod3, rdt, av);
#pragma unroll
                for (int k = 0; k < NB; ++k)
                    if (e0 + 256u * k < n) {
                        sg[cat[k]] = av[k].x;
                        sg[cat[k] + NS] = av[k].y;
                        sg[cat[k] + 2 * NS] = av[k].z;
                    }
            }
#else
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                if (e0 + 256u * k >= n) continue;
                Q d = qident();
                if (!cl[k]) d = qmul_norm(ca[k], qconj(cb[k]));
                const Q aa = qangle_axis_abs(d);
#if RTG_VEL_IEEE_DIV
                sg[cat[k]] = (aa.y * aa.x) / dt;
                sg[cat[k] + NS] = (aa.z * aa.x) / dt;
                sg[cat[k] + 2 * NS] = (aa.w * aa.x) / dt;
#else
                const V av = mulr_v(V{aa.y * aa.x, aa.z * aa.x, aa.w * aa.x}, Rcp{vt.rdt, dt});
                sg[cat[k]] = av.x;
                sg[cat[k] + NS] = av.y;
                sg[cat[k] + 2 * NS] = av.z;
#endif
            }
#endif
            if (e0 + 256 * NB < n) fetch(e0 + 256 * NB);
        }
    }
    __syncthreads();
    float *o = out + (seq * L + t0) * C;
    const uint32_t rows = (uint32_t)(t1 - t0);
    if constexpr (RC >= 0) {
        constexpr int W = RTG_VEL_W;   // outputs per thread (each raw value widened to double once for W of them)
        const uint32_t n = ((rows + W - 1) / W) * (uint32_t)C;   // (row group, channel) items
        RowWalk w(threadIdx.x, (uint32_t)C);
        for (uint32_t e = threadIdx.x; e < n; e += 256) {
            const uint32_t r0 = w.rr * W;
            double acc[W];
            gauss_rows<RC, W>(sg + w.ch * NS + r0, taps, acc);
#pragma unroll
            for (int r = 0; r < W; ++r)
                if (r0 + r < rows) {
                    o[(int64_t)(r0 + r) * C + w.ch] = (float)acc[r];
                }
            w.next((uint32_t)C);
        }
    } else {
        const uint32_t n = rows * (uint32_t)C;
        RowWalk w(threadIdx.x, (uint32_t)C);
        for (uint32_t e = threadIdx.x; e < n; e += 256) {
            o[e] = (float)gauss_row_any(sg + w.ch * NS + w.rr, taps);
            w.next((uint32_t)C);
        }
    }
}

// frames per block for the one-pass kernel: 64 while the raw rows fit 48 KB of LDS, fewer for wide rows; 0 when even
// 16 frames do not fit (the two-pass kernels then run)
static uint32_t vel_tile_frames(int64_t C, int R)
{
    // measured at 64 x 4096 x 31 (profiles/r04/aux/vel_tiles.log): 64 / 32 / 16 frames linear 79 / 90 / 108 us,
    // angular 125 / 140 / 169 us (the halo's share grows faster than the extra blocks per CU help)
    // (128-frame tiles in 64 KB: linear 72 vs 56 us, angular 117 vs 113 us, profiles/r06/aux/vel128_*)
    for (uint32_t T = 64; T >= 16; T /= 2)
        if ((int64_t)vel_lds_stride(T, R) * C * 4 <= 48 * 1024) return T;
    return 0;
}

template <bool ANGULAR>
static hipError_t launch_velocity_tile(const float *src, int64_t nseq, int64_t L, int64_t J, int64_t C, uint32_t T,
                                       float dt, const GaussTaps &taps, float *out, hipStream_t s)
{
    const uint32_t tiles = (uint32_t)((L + T - 1) / T);
    const int64_t per = ((int64_t)1 << 30) / tiles;   // sequences per launch
    size_t lds = (size_t)vel_lds_stride(T, taps.radius) * C * sizeof(float);
    if (RTG_VEL_LDS_MIN > 0 && lds < (size_t)RTG_VEL_LDS_MIN) lds = RTG_VEL_LDS_MIN;   // measurement knob: fewer blocks/CU
    for (int64_t q0 = 0; q0 < nseq; q0 += per) {
        const int64_t nq = nseq - q0 < per ? nseq - q0 : per;
        const VelTile vt{q0, (uint32_t)L, T, tiles, (uint32_t)(nq * tiles), (int32_t)C, (int32_t)J, 1.0 / (double)dt};
        if (taps.radius == 8)   // sigma 2, truncate 4: the reference's filter
            hipLaunchKernelGGL((k_velocity_tile<ANGULAR, 8>), dim3(vt.nblocks), dim3(256), lds, s, src, vt, dt, taps, out);
        else
            hipLaunchKernelGGL((k_velocity_tile<ANGULAR, -1>), dim3(vt.nblocks), dim3(256), lds, s, src, vt, dt, taps,
                               out);
    }
    return hipGetLastError();
}

// the launches of one kernel over all rows, in chunks of <= 2^30 rows
template <typename F>
static hipError_t over_rows(int64_t nrows, int64_t L, int64_t C, F launch)
{
    int cl = 0;
    while (cl < 8 && (1 << cl) < C) ++cl;
    const unsigned slices = (unsigned)((C + 255) / 256);
    const int64_t chunk = (int64_t)1 << 30;
    for (int64_t r0 = 0; r0 < nrows; r0 += chunk) {
        const int64_t n = nrows - r0 < chunk ? nrows - r0 : chunk;
        const RowTile rt{r0, (uint32_t)n, (uint32_t)L, (int32_t)C, cl};
        const int64_t rpb = (int64_t)256 >> cl;
        launch(rt, dim3((unsigned)((n + rpb - 1) / rpb), slices > 0 ? slices : 1u));
    }
    return hipGetLastError();
}

hipError_t launch_linear_velocity(const float *p, int64_t nseq, int64_t L, int64_t S, float dt, const GaussTaps *taps,
                                  float *tmp, float *out, hipStream_t s)
{
    if (nseq == 0) return hipSuccess;
    const uint32_t T = taps && L < (1 << 30) ? vel_tile_frames(S, taps->radius) : 0;
    if (T) return launch_velocity_tile<false>(p, nseq, L, S, S, T, dt, *taps, out, s);
    float *g = taps ? tmp : out;
    hipError_t e = over_rows(nseq * L, L, S, [&](const RowTile &rt, dim3 grid) {
        hipLaunchKernelGGL(k_gradient_dt, grid, dim3(256), 0, s, p, rt, dt, g);
    });
    if (e != hipSuccess || !taps) return e;
    return over_rows(nseq * L, L, S, [&](const RowTile &rt, dim3 grid) {
        hipLaunchKernelGGL(k_gauss_nearest, grid, dim3(256), 0, s, tmp, rt, *taps, out);
    });
}

hipError_t launch_angular_velocity(const float *r, int64_t nseq, int64_t L, int64_t J, float dt,
                                   const GaussTaps *taps, float *tmp, float *out, hipStream_t s)
{
    if (nseq == 0) return hipSuccess;
    const uint32_t T = taps && L < (1 << 30) ? vel_tile_frames(3 * J, taps->radius) : 0;
    if (T) return launch_velocity_tile<true>(r, nseq, L, J, 3 * J, T, dt, *taps, out, s);
    float *raw = taps ? tmp : out;
    hipError_t e = over_rows(nseq * L, L, J, [&](const RowTile &rt, dim3 grid) {
        hipLaunchKernelGGL(k_angular_raw, grid, dim3(256), 0, s, r, rt, dt, raw);
    });
    if (e != hipSuccess || !taps) return e;
    return over_rows(nseq * L, L, 3 * J, [&](const RowTile &rt, dim3 grid) {
        hipLaunchKernelGGL(k_gauss_nearest, grid, dim3(256), 0, s, tmp, rt, *taps, out);
    });
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
    if (layout == RTG_LAYOUT_SOA)
        hipLaunchKernelGGL(k_ingest_vtrdyn<kIngSoaTile>, dim3(grid_for(B, kIngSoaTile)), dim3(256), 0, s, bp,
                           lhp, rhp, B, body, lh, rh, valid, true);
    else
        hipLaunchKernelGGL(k_ingest_vtrdyn<kIngAosTile>, dim3(grid_for(B, kIngAosTile)), dim3(256), 0, s, bp,
                           lhp, rhp, B, body, lh, rh, valid, false);
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

hipError_t launch_quat_as_euler(const float *q, int s0, int s1, int s2, int extrinsic, int degrees, int64_t n,
                               double *out, hipStream_t s)
{
    hipLaunchKernelGGL(k_quat_as_euler, dim3(grid_for(n, 256)), dim3(256), 0, s, q, s0, s1, s2, extrinsic, degrees, n,
                       out);
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

// ----------------------------------------------------------------------------
// box probe (rtg.h rtg_box_probe): what this GPU delivers right now, so a throughput number from one box can be
// set against another's.  k_probe_valu keeps every SIMD busy with independent f32 FMA chains; one lane of
// every 64th workgroup reads the shader-cycle counter and the 100 MHz wall clock around its own loop, so
// cycles / wall time is the shader clock under load.  k_probe_copy streams a buffer (16 B per lane per
// access, a grid-stride loop) into another: HBM copy bandwidth.
// ----------------------------------------------------------------------------
constexpr int kProbeIters = 4096;
__global__ __launch_bounds__(256) void k_probe_valu(float seed, float *__restrict__ sink, uint64_t *__restrict__ clk)
{
    float a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = seed + (float)(threadIdx.x + k);
    const bool rec = (blockIdx.x & 63) == 0 && threadIdx.x == 0;
    uint64_t c0 = 0, w0 = 0;
    if (rec) {
        c0 = clock64();
        w0 = wall_clock64();
    }
    for (int i = 0; i < kProbeIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = __builtin_fmaf(a[k], 0.999999f, 1e-7f);
    }
    if (rec) {
        const uint64_t c1 = clock64(), w1 = wall_clock64();
        clk[2 * (blockIdx.x >> 6)] = c1 - c0;
        clk[2 * (blockIdx.x >> 6) + 1] = w1 - w0;
    }
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k];
    if (s == 12345.678f) sink[threadIdx.x] = s;   // never true; keeps the chains alive
}
__global__ __launch_bounds__(256) void k_probe_copy(const float4 *__restrict__ src, float4 *__restrict__ dst,
                                                    int64_t n)
{
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

hipError_t launch_probe_valu(int nblocks, float *sink, uint64_t *clk, hipStream_t s)
{
    hipLaunchKernelGGL(k_probe_valu, dim3(nblocks), dim3(256), 0, s, 1.0f, sink, clk);
    return hipGetLastError();
}
hipError_t launch_probe_copy(const float *src, float *dst, int64_t nfloat4, hipStream_t s)
{
    hipLaunchKernelGGL(k_probe_copy, dim3(256 * 32), dim3(256), 0, s, reinterpret_cast<const float4 *>(src),
                       reinterpret_cast<float4 *>(dst), nfloat4);
    return hipGetLastError();
}
int probe_valu_iters() { return kProbeIters; }

}  // namespace rtg

// ----------------------------------------------------------------------------
// build configuration (rtg.h rtg_build_info): every RTG_* knob as compiled into this library
// ----------------------------------------------------------------------------
#if RTG_EXP_STUB_SVD + RTG_EXP_NO_TABLE + RTG_EXP_HOT_INPUTS + RTG_EXP_MULR_NOBRANCH + RTG_EXP_NO_RARE + \
    RTG_EXP_TIMESTAMPS + RTG_EXP_SKIP_SIGNAL == 0
#define RTG_WRONG_ANSWER_KNOBS 0
#else
#define RTG_WRONG_ANSWER_KNOBS 1
#endif
#define RTG_STR2(x) #x
#define RTG_STR(x) RTG_STR2(x)
#define RTG_KNOB(k) "\"" #k "\":\"" RTG_STR(k) "\","   // values as written (some are expressions)
extern "C" const char *rtg_build_info(void)
{
    return "{\"abi\":" RTG_STR(RTG_ABI_VERSION) ",\"arch\":\"gfx950\",\"knobs\":{"
        RTG_KNOB(RTG_DOF_NWAY) RTG_KNOB(RTG_DOF_UNIT_TAB) RTG_KNOB(RTG_FK_UNIT_TAB) RTG_KNOB(RTG_UNIT_TAB_K) RTG_KNOB(RTG_SIDES_SHARED_FIT) RTG_KNOB(RTG_UPPER_UNIT_TAB) RTG_KNOB(RTG_ROT_UNIT_TAB) RTG_KNOB(RTG_SIDES_UNIT_TAB) RTG_KNOB(RTG_SIDES_UNIT_TAB_AOS) RTG_KNOB(RTG_LAT_UNIT_TAB) RTG_KNOB(RTG_FRAME1_UNIT_TAB) RTG_KNOB(RTG_FRAME1_SHARED_CODE) RTG_KNOB(RTG_QUAD_SHARED_CODE) RTG_KNOB(RTG_LAT5_SHARED_CODE) RTG_KNOB(RTG_VEL_UNIT_TAB) RTG_KNOB(RTG_SIDES_WAVES) RTG_KNOB(RTG_SIDES_TILES) RTG_KNOB(RTG_SIDES_SPLIT_READOUT) RTG_KNOB(RTG_SIDES_ARMS2) RTG_KNOB(RTG_SIDES_EARLY_WORDS) RTG_KNOB(RTG_AOS_PRELOAD_TIPS) RTG_KNOB(RTG_QUAD8_MAX_B) RTG_KNOB(RTG_QUAD_MAX_B) RTG_KNOB(RTG_LATENCY_MAX_B)
        RTG_KNOB(RTG_EXP_TIMESTAMPS) RTG_KNOB(RTG_EXP_SKIP_SIGNAL) RTG_KNOB(RTG_EXP_STUB_SVD) RTG_KNOB(RTG_EXP_NO_TABLE) RTG_KNOB(RTG_EXP_MULR_NOBRANCH) RTG_KNOB(RTG_FK_F16_MAXJ) RTG_KNOB(RTG_FK_NT_OUT) RTG_KNOB(RTG_EXP_LARTG_RCP64) RTG_KNOB(RTG_EXP_SQRT64) RTG_KNOB(RTG_EXP_SQRT_CALL) RTG_KNOB(RTG_EXP_ACOS_LIBM) RTG_KNOB(RTG_EXP_EULER_SCIPY) RTG_KNOB(RTG_VEL_SEG) RTG_KNOB(RTG_VEL_LDS_MIN) RTG_KNOB(RTG_VEL_IEEE_DIV) RTG_KNOB(RTG_DOF_NT_STORE) RTG_KNOB(RTG_IN_NT_LOAD) RTG_KNOB(RTG_VEL_W) RTG_KNOB(RTG_VEL_ANG_NB) RTG_KNOB(RTG_VEL_ANG_NWAY) RTG_KNOB(RTG_EXP_NO_RARE)
        "\"RTG_EXP_HOT_INPUTS\":\"" RTG_STR(RTG_EXP_HOT_INPUTS) "\"},\"wrong_answer_knobs\":"
        RTG_STR(RTG_WRONG_ANSWER_KNOBS) "}";
}
