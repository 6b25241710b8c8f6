// rtg_api.cpp -- C ABI (include/rtg.h) over the gfx950 kernels.
//
// Host-side only: argument validation (mirroring the reference's assertions),
// handle lifetime, and stream-ordered launches.  Launch entry points never
// allocate, copy or synchronise, so callers may capture them into hipGraphs.
#include <immintrin.h>
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <new>
#include <vector>
#include <string>
#include <utility>

#include "rtg_kernels.cuh"

using namespace rtg;

struct rtg_topology_s {
    int32_t J = 0;
    int32_t *d_parents = nullptr;
    V *d_local_t = nullptr;
    Q *d_tree_quat = nullptr;
    GEnt *d_gsched = nullptr;   // lane-group FK schedule (J <= kGroupMaxJ), see fk_group_schedule
    int32_t gF = 0, gsteps = 0;
    TopoView view() const
    {
        return TopoView{d_parents, d_local_t, d_tree_quat, J, d_gsched, gF, gsteps};
    }
};

// HuForwardModel: the topology is borrowed (it must outlive the model); axis / limits are owned.
struct rtg_dof_model_s {
    rtg_topology_t topo = nullptr;
    int32_t *d_axis = nullptr;
    float *d_lower = nullptr;
    float *d_upper = nullptr;
    bool has_limits = false;
};

struct rtg_solver_s {
    int kind = 0;
    int precise = 0;
    SolverConsts consts{};
    uint32_t *d_ang_tab = nullptr;   // exp-map angle table (consts.ang_tab), device of creation
    uint32_t *h_err = nullptr;       // the device error word (consts.err is its device alias), pinned host memory
};

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_check(hipError_t e, const char *what)
{
    if (e == hipSuccess) return RTG_OK;
    return fail(e == hipErrorOutOfMemory ? RTG_ERR_OUT_OF_MEMORY : RTG_ERR_DEVICE, "%s: %s", what,
                hipGetErrorString(e));
}

#define RTG_TRY(expr, what)                          \
    do {                                             \
        int rc_ = hip_check((expr), (what));         \
        if (rc_ != RTG_OK) return rc_;               \
    } while (0)

inline hipStream_t as_stream(rtg_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
inline V v3(const float *p, int j) { return V{p[3 * j], p[3 * j + 1], p[3 * j + 2]}; }

int axis_of(char c, int *ax, int *lower)
{
    switch (c) {
    case 'x': *ax = 0; *lower = 1; return 1;
    case 'y': *ax = 1; *lower = 1; return 1;
    case 'z': *ax = 2; *lower = 1; return 1;
    case 'X': *ax = 0; *lower = 0; return 1;
    case 'Y': *ax = 1; *lower = 0; return 1;
    case 'Z': *ax = 2; *lower = 0; return 1;
    default: return 0;
    }
}

}  // namespace

extern "C" {

int rtg_abi_version(void) { return RTG_ABI_VERSION; }

const char *rtg_last_error(void) { return g_err.c_str(); }

int rtg_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// ---------------------------------------------------------------- topology
int rtg_topology_create(const int32_t *parents, const float *local_t, const float *tree_quat, int32_t J,
                        rtg_topology_t *out)
{
    if (!out) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_topology_create: out is NULL");
    *out = nullptr;
    if (!parents || !local_t) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_topology_create: NULL parents/local_t");
    if (J < 1 || J > 1024) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_topology_create: J=%d out of range", J);
    // parent-indexed tree in topological order (skeleton3d.py:87-88 asserts equal lengths;
    // the FK loop kinematics.py:27 requires parents before children)
    if (parents[0] != -1) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_topology_create: joint 0 must be the root");
    for (int j = 1; j < J; ++j)
        if (parents[j] < 0 || parents[j] >= j)
            return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_topology_create: parents[%d]=%d is not < %d", j, parents[j], j);
    rtg_topology_s *t = new (std::nothrow) rtg_topology_s();
    if (!t) return fail(RTG_ERR_OUT_OF_MEMORY, "rtg_topology_create: host allocation failed");
    t->J = J;
    Q *tq = new (std::nothrow) Q[J];
    if (!tq) {
        delete t;
        return fail(RTG_ERR_OUT_OF_MEMORY, "rtg_topology_create: host allocation failed");
    }
    for (int j = 0; j < J; ++j)
        tq[j] = tree_quat ? Q{tree_quat[4 * j], tree_quat[4 * j + 1], tree_quat[4 * j + 2], tree_quat[4 * j + 3]}
                          : Q{0.f, 0.f, 0.f, 1.f};
    int rc = hip_check(hipMalloc(&t->d_parents, sizeof(int32_t) * J), "hipMalloc(parents)");
    if (rc == RTG_OK) rc = hip_check(hipMalloc(&t->d_local_t, sizeof(V) * J), "hipMalloc(local_t)");
    if (rc == RTG_OK) rc = hip_check(hipMalloc(&t->d_tree_quat, sizeof(Q) * J), "hipMalloc(tree_quat)");
    if (rc == RTG_OK)
        rc = hip_check(hipMemcpy(t->d_parents, parents, sizeof(int32_t) * J, hipMemcpyHostToDevice), "hipMemcpy");
    if (rc == RTG_OK)
        rc = hip_check(hipMemcpy(t->d_local_t, local_t, sizeof(V) * J, hipMemcpyHostToDevice), "hipMemcpy");
    if (rc == RTG_OK) rc = hip_check(hipMemcpy(t->d_tree_quat, tq, sizeof(Q) * J, hipMemcpyHostToDevice), "hipMemcpy");
    // the lane-group schedule (rtg_fk.hip): J <= kGroupMaxJ, at most J steps
    const int gF = group_frames(J);
    if (rc == RTG_OK && gF > 0) {
        std::vector<V> lt(J);
        for (int j = 0; j < J; ++j) lt[j] = v3(local_t, j);
        std::vector<GEnt> gs((size_t)J * (64 / gF));
        const int steps = fk_group_schedule(parents, lt.data(), tq, J, gF, gs.data(), J);
        if (steps > 0) {
            rc = hip_check(hipMalloc(&t->d_gsched, sizeof(GEnt) * steps * (64 / gF)), "hipMalloc(group schedule)");
            if (rc == RTG_OK)
                rc = hip_check(hipMemcpy(t->d_gsched, gs.data(), sizeof(GEnt) * steps * (64 / gF), hipMemcpyHostToDevice),
                               "hipMemcpy");
            t->gF = gF;
            t->gsteps = steps;
        }
    }
    delete[] tq;
    if (rc != RTG_OK) {
        (void)hipFree(t->d_parents);
        (void)hipFree(t->d_local_t);
        (void)hipFree(t->d_tree_quat);
        (void)hipFree(t->d_gsched);
        delete t;
        return rc;
    }
    *out = t;
    return RTG_OK;
}

int rtg_topology_destroy(rtg_topology_t t)
{
    if (!t) return RTG_OK;
    (void)hipFree(t->d_parents);
    (void)hipFree(t->d_local_t);
    (void)hipFree(t->d_tree_quat);
    (void)hipFree(t->d_gsched);
    delete t;
    return RTG_OK;
}

int rtg_topology_num_joints(rtg_topology_t t) { return t ? t->J : -1; }

// ---------------------------------------------------------------- kinematics
static int check_fk(rtg_topology_t t, const void *a, const void *b, const void *c, const void *d, int64_t B,
                    const char *fn)
{
    if (!t) return fail(RTG_ERR_INVALID_ARGUMENT, "%s: NULL topology", fn);
    if (B < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "%s: negative batch %lld", fn, (long long)B);
    if (B > 0 && (!a || !b || !c || !d)) return fail(RTG_ERR_INVALID_ARGUMENT, "%s: NULL buffer", fn);
    return RTG_OK;
}

int rtg_fk_f32(rtg_topology_t t, const float *local_rot, const float *root_t, int64_t B, float *g_rot, float *g_pos,
               rtg_stream_t stream)
{
    int rc = check_fk(t, local_rot, root_t, g_rot, g_pos, B, "rtg_fk_f32");
    if (rc != RTG_OK || B == 0) return rc;
    RTG_TRY(launch_fk(t->view(), false, local_rot, root_t, B, g_rot, g_pos, as_stream(stream)), "k_fk");
    return RTG_OK;
}

int rtg_state_fk_f32(rtg_topology_t t, const float *local_rot, const float *root_t, int64_t B, float *g_rot,
                     float *g_pos, rtg_stream_t stream)
{
    int rc = check_fk(t, local_rot, root_t, g_rot, g_pos, B, "rtg_state_fk_f32");
    if (rc != RTG_OK || B == 0) return rc;
    RTG_TRY(launch_fk(t->view(), true, local_rot, root_t, B, g_rot, g_pos, as_stream(stream)), "k_fk<state>");
    return RTG_OK;
}

int rtg_local_rotation_f32(rtg_topology_t t, const float *g_rot, int64_t B, float *local_rot, rtg_stream_t stream)
{
    int rc = check_fk(t, g_rot, local_rot, g_rot, local_rot, B, "rtg_local_rotation_f32");
    if (rc != RTG_OK || B == 0) return rc;
    RTG_TRY(launch_local_rotation(t->view(), false, g_rot, B, local_rot, as_stream(stream)), "k_local_rotation");
    return RTG_OK;
}

int rtg_state_local_rotation_f32(rtg_topology_t t, const float *g_rot, int64_t B, float *local_rot,
                                 rtg_stream_t stream)
{
    int rc = check_fk(t, g_rot, local_rot, g_rot, local_rot, B, "rtg_state_local_rotation_f32");
    if (rc != RTG_OK || B == 0) return rc;
    RTG_TRY(launch_local_rotation(t->view(), true, g_rot, B, local_rot, as_stream(stream)), "k_local_rotation<state>");
    return RTG_OK;
}

int rtg_fk_multi_f32(const rtg_fk_segment *segs, int32_t n, rtg_stream_t stream)
{
    if (n < 0 || n > RTG_MAX_SEGMENTS)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_fk_multi_f32: %d segments (max %d)", n, RTG_MAX_SEGMENTS);
    if (n > 0 && !segs) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_fk_multi_f32: NULL segments");
    FkMultiArgs A{};
    A.n = n;
    for (int i = 0; i < n; ++i) {
        const rtg_fk_segment &s = segs[i];
        int rc = check_fk(s.topo, s.local_rot, s.root_t, s.g_rot, s.g_pos, s.B, "rtg_fk_multi_f32");
        if (rc != RTG_OK) return rc;
        A.seg[i] = FkSeg{s.topo->view(), s.local_rot, s.root_t, s.g_rot, s.g_pos, s.B, 0};
    }
    RTG_TRY(launch_fk_multi(A, as_stream(stream)), "k_fk_multi");
    return RTG_OK;
}

int rtg_kinematics_multi_f32(const rtg_fk_segment *fk, int32_t n_fk, const rtg_local_rotation_segment *inv,
                             int32_t n_inv, rtg_stream_t stream)
{
    if (n_fk < 0 || n_inv < 0 || n_fk + n_inv > RTG_MAX_SEGMENTS)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_kinematics_multi_f32: %d + %d segments (max %d in total)", n_fk,
                    n_inv, RTG_MAX_SEGMENTS);
    if ((n_fk > 0 && !fk) || (n_inv > 0 && !inv))
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_kinematics_multi_f32: NULL segments");
    FkMultiArgs A{};
    A.n = n_fk + n_inv;
    for (int i = 0; i < n_fk; ++i) {
        const rtg_fk_segment &s = fk[i];
        int rc = check_fk(s.topo, s.local_rot, s.root_t, s.g_rot, s.g_pos, s.B, "rtg_kinematics_multi_f32");
        if (rc != RTG_OK) return rc;
        A.seg[i] = FkSeg{s.topo->view(), s.local_rot, s.root_t, s.g_rot, s.g_pos, s.B, 0};
    }
    for (int i = 0; i < n_inv; ++i) {
        const rtg_local_rotation_segment &s = inv[i];
        int rc = check_fk(s.topo, s.g_rot, s.local_rot, s.g_rot, s.local_rot, s.B, "rtg_kinematics_multi_f32");
        if (rc != RTG_OK) return rc;
        A.seg[n_fk + i] = FkSeg{s.topo->view(), s.g_rot, nullptr, s.local_rot, nullptr, s.B, 1};
    }
    RTG_TRY(launch_fk_multi(A, as_stream(stream)), "k_fk_multi");
    return RTG_OK;
}

int rtg_local_rotation_multi_f32(const rtg_local_rotation_segment *segs, int32_t n, rtg_stream_t stream)
{
    return rtg_kinematics_multi_f32(nullptr, 0, segs, n, stream);
}

// ---------------------------------------------------------------- joint-angle forward model
int rtg_dof_model_create(rtg_topology_t topo, const int32_t *axis, const float *lower, const float *upper,
                         rtg_dof_model_t *out)
{
    if (!out) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_dof_model_create: out is NULL");
    *out = nullptr;
    if (!topo) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_dof_model_create: NULL topology");
    const int n = topo->J - 1;
    if (n > 0 && !axis) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_dof_model_create: NULL axis");
    for (int k = 0; k < n; ++k)
        if (axis[k] < 0 || axis[k] > 2)
            return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_dof_model_create: axis[%d]=%d is not 0, 1 or 2", k, axis[k]);
    if ((lower == nullptr) != (upper == nullptr))
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_dof_model_create: give both DOF limit arrays or neither");
    rtg_dof_model_s *m = new (std::nothrow) rtg_dof_model_s();
    if (!m) return fail(RTG_ERR_OUT_OF_MEMORY, "rtg_dof_model_create: host allocation failed");
    m->topo = topo;
    m->has_limits = lower != nullptr;
    const size_t na = sizeof(int32_t) * (n > 0 ? n : 1), nf = sizeof(float) * (n > 0 ? n : 1);
    int rc = hip_check(hipMalloc(&m->d_axis, na), "hipMalloc(axis)");
    if (rc == RTG_OK && n > 0) rc = hip_check(hipMemcpy(m->d_axis, axis, sizeof(int32_t) * n, hipMemcpyHostToDevice), "hipMemcpy");
    if (rc == RTG_OK && m->has_limits) {
        rc = hip_check(hipMalloc(&m->d_lower, nf), "hipMalloc(lower)");
        if (rc == RTG_OK) rc = hip_check(hipMalloc(&m->d_upper, nf), "hipMalloc(upper)");
        if (rc == RTG_OK && n > 0)
            rc = hip_check(hipMemcpy(m->d_lower, lower, sizeof(float) * n, hipMemcpyHostToDevice), "hipMemcpy");
        if (rc == RTG_OK && n > 0)
            rc = hip_check(hipMemcpy(m->d_upper, upper, sizeof(float) * n, hipMemcpyHostToDevice), "hipMemcpy");
    }
    if (rc != RTG_OK) {
        (void)hipFree(m->d_axis);
        (void)hipFree(m->d_lower);
        (void)hipFree(m->d_upper);
        delete m;
        return rc;
    }
    *out = m;
    return RTG_OK;
}

int rtg_dof_model_destroy(rtg_dof_model_t m)
{
    if (!m) return RTG_OK;
    (void)hipFree(m->d_axis);
    (void)hipFree(m->d_lower);
    (void)hipFree(m->d_upper);
    delete m;
    return RTG_OK;
}

int rtg_dof_fk_f32(rtg_dof_model_t m, const float *dof, const float *root_rot, const float *root_t, int64_t B,
                   int clip, float *g_rot, float *g_pos, rtg_stream_t stream)
{
    if (!m) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_dof_fk_f32: NULL model");
    if (B < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_dof_fk_f32: B=%lld < 0", (long long)B);
    if (clip && !m->has_limits)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_dof_fk_f32: clip_angles requested but the model has no DOF limits");
    if (B == 0) return RTG_OK;
    if ((m->topo->J > 1 && !dof) || !root_rot || !root_t || !g_rot || !g_pos)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_dof_fk_f32: NULL buffer");
    const DofView D{m->d_axis, m->d_lower, m->d_upper};
    RTG_TRY(launch_dof_fk(m->topo->view(), D, clip != 0, dof, root_rot, root_t, B, g_rot, g_pos, as_stream(stream)),
            "k_dof_fk");
    return RTG_OK;
}

// ---------------------------------------------------------------- VTRDyn ingest
int rtg_ingest_vtrdyn_f32(const float *bp, const float *lhp, const float *rhp, int64_t B, int layout, float *body,
                          float *lh, float *rh, uint8_t *valid, rtg_stream_t stream)
{
    if (B < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_ingest_vtrdyn_f32: B < 0");
    if (layout != RTG_LAYOUT_AOS && layout != RTG_LAYOUT_SOA)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_ingest_vtrdyn_f32: bad layout %d", layout);
    if (B == 0) return RTG_OK;
    if (!bp || !lhp || !rhp || !body || !lh || !rh || !valid)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_ingest_vtrdyn_f32: NULL buffer");
    RTG_TRY(launch_ingest_vtrdyn(bp, lhp, rhp, B, layout, body, lh, rh, valid, as_stream(stream)), "k_ingest_vtrdyn");
    return RTG_OK;
}

// ---------------------------------------------------------------- motion-level prep (retarget/main.py)
int rtg_rescale_motion_f32(rtg_topology_t topo, const float *motion, int64_t B, const float *dir, float *out,
                           rtg_stream_t stream)
{
    if (!topo) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_rescale_motion_f32: NULL topology");
    if (B < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_rescale_motion_f32: B < 0");
    if (B == 0) return RTG_OK;
    if (!motion || !out) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_rescale_motion_f32: NULL buffer");
    RTG_TRY(launch_rescale_motion(topo->view(), motion, B, dir, out, as_stream(stream)), "k_rescale_motion");
    return RTG_OK;
}

int rtg_quat_between_f32(const float *v1, const float *v2, int64_t n, float *out, float *ws, rtg_stream_t stream)
{
    if (n < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_between_f32: n < 0");
    if (n == 0) return RTG_OK;
    if (!v1 || !v2 || !out || !ws) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_between_f32: NULL buffer");
    RTG_TRY(launch_quat_between(v1, v2, n, out, ws, as_stream(stream)), "k_quat_between");
    return RTG_OK;
}

int rtg_rebuild_vtrdyn_f32(rtg_topology_t topo, const float *motion, int64_t B, float *g_rot, float *root_t,
                           float *ws, rtg_stream_t stream)
{
    if (!topo) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_rebuild_vtrdyn_f32: NULL topology");
    if (topo->J != 21)   // main.py:126-136 index the VTRDYN joints 0, 1, 4, 7, 10, 11, 13, 17
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_rebuild_vtrdyn_f32: expects the 21-joint VTRDYN zero pose, got %d",
                    topo->J);
    if (B < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_rebuild_vtrdyn_f32: B < 0");
    if (B == 0) return RTG_OK;
    if (!motion || !g_rot || !root_t || !ws) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_rebuild_vtrdyn_f32: NULL buffer");
    RTG_TRY(launch_rebuild_vtrdyn(topo->view(), motion, B, g_rot, root_t, ws, as_stream(stream)), "k_rebuild_vtrdyn");
    return RTG_OK;
}

// ---------------------------------------------------------------- solvers
int rtg_solver_create(int kind, const float *zl, const float *zg, const int32_t *parents, int32_t Js,
                      int precise_gripper, rtg_solver_t *out)
{
    if (!out) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_solver_create: out is NULL");
    *out = nullptr;
    if (!zl) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_solver_create: NULL zero-pose local translation");
    SolverConsts C{};
    switch (kind) {
    case RTG_SOLVER_FULL_BODY_POS: {
        if (Js != 59) return fail(RTG_ERR_INVALID_ARGUMENT, "FULL_BODY_POS expects the 59-joint VTRDYN_FULL zero pose, got %d", Js);
        if (!zg) return fail(RTG_ERR_INVALID_ARGUMENT, "FULL_BODY_POS needs the zero-pose global translation");
        // full_body_pos_retargeter.py:69, :139, :162, :78/:86/:99/:107, :184
        C.Zt[0] = v3(zl, 11); C.Zt[1] = v3(zl, 36); C.Zt[2] = v3(zl, 34);
        const int li[5] = {16, 20, 24, 28, 32}, ri[5] = {41, 45, 49, 53, 56}, gi[5] = {18, 22, 26, 30, 33};
        for (int t = 0; t < 5; ++t) {
            C.Zl[t] = v3(zl, li[t]);
            C.Zr[t] = v3(zl, ri[t]);
            C.grip_d[t] = zg[3 * gi[t]] - zg[3 * 14];
        }
        C.v0_lsh = v3(zl, 13); C.v0_lel = v3(zl, 14); C.v0_rsh = v3(zl, 38); C.v0_rel = v3(zl, 39);
        break;
    }
    case RTG_SOLVER_UPPER_BODY:
        if (Js != 21) return fail(RTG_ERR_INVALID_ARGUMENT, "UPPER_BODY expects the 21-joint VTRDYN zero pose, got %d", Js);
        // retarget_solver.py:49-86
        C.Zt[0] = v3(zl, 17); C.Zt[1] = v3(zl, 13); C.Zt[2] = v3(zl, 11);
        C.v0_lsh = v3(zl, 19); C.v0_lel = v3(zl, 20); C.v0_rsh = v3(zl, 15); C.v0_rel = v3(zl, 16);
        break;
    case RTG_SOLVER_FULL_BODY_ROT: {
        if (Js != 59) return fail(RTG_ERR_INVALID_ARGUMENT, "FULL_BODY_ROT expects the 59-joint VTRDYN_FULL zero pose, got %d", Js);
        // full_body_retargeter.py:64,72,85,93,152 (gripper uses LOCAL translations, joint 24)
        C.v0_lsh = v3(zl, 13); C.v0_lel = v3(zl, 14); C.v0_rsh = v3(zl, 38); C.v0_rel = v3(zl, 39);
        const int gi[5] = {18, 22, 26, 30, 33};
        for (int t = 0; t < 5; ++t) C.grip_d[t] = zl[3 * gi[t]] - zl[3 * 24];
        break;
    }
    case RTG_SOLVER_BODY_ROT:
        if (Js != 21) return fail(RTG_ERR_INVALID_ARGUMENT, "BODY_ROT expects the 21-joint VTRDYN zero pose, got %d", Js);
        if (!parents) return fail(RTG_ERR_INVALID_ARGUMENT, "BODY_ROT needs the source parent indices");
        C.par[0] = parents[18]; C.par[1] = parents[14]; C.par[2] = parents[19]; C.par[3] = parents[15];
        for (int i = 0; i < 4; ++i)
            if (C.par[i] < 0 || C.par[i] >= 21) return fail(RTG_ERR_INVALID_ARGUMENT, "BODY_ROT: bad parent index");
        break;
    default:
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_solver_create: unknown solver kind %d", kind);
    }
    SolverConsts *d = nullptr;
    RTG_TRY(hipMalloc(&d, sizeof(SolverConsts)), "hipMalloc(solver consts)");
    int rc = hip_check(hipMemcpy(d, &C, sizeof C, hipMemcpyHostToDevice), "hipMemcpy(consts)");
    if (rc == RTG_OK && kind != RTG_SOLVER_BODY_ROT) rc = hip_check(launch_solver_prep(d, nullptr), "k_solver_prep");
    if (rc == RTG_OK) rc = hip_check(hipMemcpy(&C, d, sizeof C, hipMemcpyDeviceToHost), "hipMemcpy(consts)");
    (void)hipFree(d);
    if (rc != RTG_OK) return rc;
    // exp-map angle table: built once per solver on the current device (6.7 MiB), read by every launch
    uint32_t *tab = nullptr;
    RTG_TRY(hipMalloc(&tab, kAngTabWords * sizeof(uint32_t)), "hipMalloc(exp-map angle table)");
    rc = hip_check(launch_build_ang_tab(tab, nullptr), "k_build_ang_tab");
    if (rc == RTG_OK) rc = hip_check(hipStreamSynchronize(nullptr), "k_build_ang_tab");
    if (rc != RTG_OK) {
        (void)hipFree(tab);
        return rc;
    }
    C.ang_tab = tab;
    // the error word: host-mapped, so the device's report is read on the next call without a HIP call
    uint32_t *h_err = nullptr;
    rc = hip_check(hipHostMalloc(reinterpret_cast<void **>(&h_err), sizeof(uint32_t), hipHostMallocMapped),
                   "hipHostMalloc(error word)");
    if (rc == RTG_OK) {
        *h_err = 0;
        rc = hip_check(hipHostGetDevicePointer(reinterpret_cast<void **>(&C.err), h_err, 0), "hipHostGetDevicePointer");
    }
    rtg_solver_s *s = rc == RTG_OK ? new (std::nothrow) rtg_solver_s() : nullptr;
    if (!s) {
        (void)hipFree(tab);
        if (h_err) (void)hipHostFree(h_err);
        return rc != RTG_OK ? rc : fail(RTG_ERR_OUT_OF_MEMORY, "rtg_solver_create: host allocation failed");
    }
    s->kind = kind;
    s->precise = precise_gripper ? 1 : 0;
    s->consts = C;
    s->d_ang_tab = tab;
    s->h_err = h_err;
    *out = s;
    return RTG_OK;
}

int rtg_solver_destroy(rtg_solver_t s)
{
    if (s) {
        (void)hipFree(s->d_ang_tab);
        if (s->h_err) (void)hipHostFree(s->h_err);
    }
    delete s;
    return RTG_OK;
}

// A device error a previous launch of this solver reported (rtg.h RTG_DEVERR_*): returned once, then cleared.
static int take_device_error(uint32_t *word, const char *fn)
{
    const uint32_t e = word ? __atomic_exchange_n(word, 0u, __ATOMIC_ACQ_REL) : 0u;
    if (e == 0) return RTG_OK;
    return fail(RTG_ERR_DEVICE, "%s: a previous launch reported device error 0x%x%s", fn, e,
                (e & RTG_DEVERR_HANDOVER_TIMEOUT) ? " (a wave hand-over timed out: that launch's outputs are not valid)"
                                                  : "");
}

int rtg_retarget_f32(rtg_solver_t s, const float *in0, const float *in1, const float *in2, const float *in3,
                     int64_t B, int layout, float *dof, float *local_rot, float *body_rot, rtg_stream_t stream)
{
    if (!s) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_retarget_f32: NULL solver");
    int rc = take_device_error(s->h_err, "rtg_retarget_f32");
    if (rc != RTG_OK) return rc;
    if (B < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_retarget_f32: negative batch");
    if (layout != RTG_LAYOUT_AOS && layout != RTG_LAYOUT_SOA)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_retarget_f32: bad layout %d", layout);
    if (B == 0) return RTG_OK;
    if (B > (int64_t)0x7fffffff * 256) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_retarget_f32: batch too large");
    if (!dof) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_retarget_f32: NULL dof");
    const int need = s->kind == RTG_SOLVER_FULL_BODY_ROT ? 4 : (s->kind == RTG_SOLVER_FULL_BODY_POS ? 3 : 1);
    const float *ins[4] = {in0, in1, in2, in3};
    for (int i = 0; i < 4; ++i) {
        if (i < need && !ins[i]) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_retarget_f32: input %d is NULL", i);
        if (i >= need && ins[i]) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_retarget_f32: input %d must be NULL", i);
    }
    if (body_rot && s->kind != RTG_SOLVER_FULL_BODY_POS)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_retarget_f32: body_rot is only produced by FULL_BODY_POS");
    RTG_TRY(launch_retarget(s->kind, s->precise, s->consts, in0, in1, in2, in3, B, layout, dof, local_rot, body_rot,
                            as_stream(stream)),
            "rtg_retarget_f32 launch");
    return RTG_OK;
}

int rtg_frame_server_launch(rtg_solver_t s, const float *in, float *dof, float *local_rot, float *body_rot,
                            uint32_t *ctl, uint32_t idle_ms, rtg_stream_t stream)
{
    if (!s) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_frame_server_launch: NULL solver");
    if (s->kind != RTG_SOLVER_FULL_BODY_POS)
        return fail(RTG_ERR_UNSUPPORTED, "rtg_frame_server_launch: only FULL_BODY_POS solvers are served per frame");
    if (!in || !dof || !ctl) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_frame_server_launch: NULL in / dof / ctl");
    if (idle_ms == 0 || idle_ms > 60000)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_frame_server_launch: idle_ms=%u (1..60000)", idle_ms);
    RTG_TRY(launch_frame_server(s->precise, s->consts, in, dof, local_rot, body_rot, ctl, (uint64_t)idle_ms * 100000u,
                                as_stream(stream)),
            "k_frame_server");
    return RTG_OK;
}

// The inbox's sequence word, stored after everything the host wrote before it and drained to the device: a device
// inbox (rtg_server_inbox_alloc) is mapped write-combining, so its stores sit in the CPU's write-combining buffers
// until a fence pushes them out (without one the device saw them 72 us - 7 ms late, tools/bar_probe.hip)
static void store_inbox_seq(float *in, uint32_t word)
{
    _mm_sfence();   // the frame's rows first (write-combined stores are not ordered by x86's TSO)
    __atomic_store_n(reinterpret_cast<uint32_t *>(in + RTG_SERVER_SEQ_WORD), word, __ATOMIC_RELEASE);
    _mm_sfence();   // ... and the word itself out now
}

int rtg_server_inbox_alloc(float **inbox)
{
    if (!inbox) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_server_inbox_alloc: NULL inbox");
    *inbox = nullptr;
    void *p = nullptr;
    const size_t bytes = RTG_SERVER_INBOX_FLOATS * sizeof(float);
    int rc = hip_check(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(inbox)");
    if (rc != RTG_OK) return rc;
    // the host reaches device memory at its own address only on a large-BAR device (MI355X: the whole HBM is in the
    // BAR; hipPointerGetAttributes reports no separate host pointer for it); otherwise the caller keeps a pinned inbox
    int dev = 0, large_bar = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, dev) != hipSuccess ||
        !large_bar) {
        (void)hipGetLastError();
        (void)hipFree(p);
        return fail(RTG_ERR_UNSUPPORTED, "rtg_server_inbox_alloc: not a large-BAR device (the host cannot store into its memory)");
    }
    // zeroed by the host itself, through the BAR (no device-wide synchronize: a server may be running elsewhere)
    std::memset(p, 0, bytes);
    _mm_sfence();
    *inbox = static_cast<float *>(p);
    return RTG_OK;
}

int rtg_server_inbox_free(float *inbox)
{
    if (!inbox) return RTG_OK;
    return hip_check(hipFree(inbox), "hipFree(inbox)");
}

int rtg_frame_server_signal(float *in, uint32_t word)
{
    if (!in) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_frame_server_signal: NULL inbox");
    store_inbox_seq(in, word);
    return RTG_OK;
}

int rtg_frame_server_post(uint32_t *ctl, uint32_t seq, float *in, const float *body, const float *left_hand,
                          const float *right_hand, const float *dof, const float *local_rot, const float *body_rot,
                          float *dof_dst, float *local_rot_dst, float *body_rot_dst, uint32_t timeout_us)
{
    if (!ctl || !in || !body || !left_hand || !right_hand || !dof)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_frame_server_post: NULL ctl / in / inputs / dof");
    if (seq == RTG_SERVER_QUIT) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_frame_server_post: seq is the quit value");
    if ((local_rot_dst && !local_rot) || (body_rot_dst && !body_rot))
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_frame_server_post: an output the server does not write");
    std::memcpy(in, body, 63 * sizeof(float));
    std::memcpy(in + 63, left_hand, 60 * sizeof(float));
    std::memcpy(in + 123, right_hand, 60 * sizeof(float));
    store_inbox_seq(in, seq);   // after the rows (the device acquires the word at system scope)
    struct timespec t0, t;
    bool timed = false;
    for (uint32_t spins = 1; __atomic_load_n(ctl + 1, __ATOMIC_ACQUIRE) != seq; ++spins) {
        if ((spins & 255u) != 0) continue;
        if (__atomic_load_n(ctl + 2, __ATOMIC_ACQUIRE) && __atomic_load_n(ctl + 1, __ATOMIC_ACQUIRE) != seq)
            return RTG_SERVER_ENDED;   // it ended on idle before it saw this frame
        clock_gettime(CLOCK_MONOTONIC, timed ? &t : &t0);
        if (!timed) { timed = true; continue; }
        const int64_t us = (int64_t)(t.tv_sec - t0.tv_sec) * 1000000 + (t.tv_nsec - t0.tv_nsec) / 1000;
        if (us > (int64_t)timeout_us) return fail(RTG_ERR_TIMEOUT, "rtg_frame_server_post: frame %u not served within %u us", seq, timeout_us);
    }
    if (dof_dst) std::memcpy(dof_dst, dof, 30 * sizeof(float));
    if (local_rot_dst) std::memcpy(local_rot_dst, local_rot, 124 * sizeof(float));
    if (body_rot_dst) std::memcpy(body_rot_dst, body_rot, 236 * sizeof(float));
    return take_device_error(ctl + 3, "rtg_frame_server_post");
}

// ---------------------------------------------------------------- primitives
int rtg_quat_op_f32(int op, const float *a, const float *b, const float *c, int64_t n, float *out,
                    rtg_stream_t stream)
{
    if (op < RTG_OP_QUAT_MUL || op > RTG_OP_PROJECT_QUAT_XZ) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_op_f32: bad op %d", op);
    if (n < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_op_f32: negative n");
    if (n == 0) return RTG_OK;
    const bool needs_b = op == RTG_OP_QUAT_MUL || op == RTG_OP_QUAT_MUL_NORM || op == RTG_OP_QUAT_ROTATE ||
                         op == RTG_OP_QUAT_FROM_ANGLE_AXIS || op == RTG_OP_RADIANS_BETWEEN ||
                         op == RTG_OP_PROJ_IN_PLANE || op == RTG_OP_SHOULDER_PR || op == RTG_OP_ELBOW_PY ||
                         op == RTG_OP_QUAT_SLERP;
    const bool needs_c = op == RTG_OP_RADIANS_BETWEEN || op == RTG_OP_SHOULDER_PR || op == RTG_OP_ELBOW_PY ||
                         op == RTG_OP_QUAT_SLERP;
    if (!a || !out || (needs_b && !b) || (needs_c && !c))
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_op_f32: NULL operand for op %d", op);
    RTG_TRY(launch_quat_op(op, a, b, c, n, out, as_stream(stream)), "k_quat_op");
    return RTG_OK;
}

int rtg_cal_joint_quat_f32(const float *Z, const float *M, int32_t npts, int64_t n, float *out, rtg_stream_t stream)
{
    if (npts < 1 || npts > 8) return fail(RTG_ERR_UNSUPPORTED, "rtg_cal_joint_quat_f32: npts=%d (1..8)", npts);
    if (n < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_cal_joint_quat_f32: negative n");
    if (n == 0) return RTG_OK;
    if (!Z || !M || !out) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_cal_joint_quat_f32: NULL buffer");
    RTG_TRY(launch_cal_joint_quat(Z, M, npts, n, out, as_stream(stream)), "k_cal_joint_quat");
    return RTG_OK;
}

int rtg_quat_in_xyz_axis_f32(const float *q, const char *seq, int64_t n, float *out, rtg_stream_t stream)
{
    if (!seq || std::strlen(seq) != 3) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_in_xyz_axis_f32: seq must have 3 axes");
    int ax[3], lower[3];
    for (int i = 0; i < 3; ++i)
        if (!axis_of(seq[i], &ax[i], &lower[i]))
            return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_in_xyz_axis_f32: bad axis '%c'", seq[i]);
    if (lower[0] != lower[1] || lower[1] != lower[2])
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_in_xyz_axis_f32: mixed intrinsic/extrinsic seq '%s'", seq);
    if (ax[0] == ax[1] || ax[1] == ax[2])
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_in_xyz_axis_f32: consecutive axes must differ ('%s')", seq);
    if (n < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_in_xyz_axis_f32: negative n");
    if (n == 0) return RTG_OK;
    if (!q || !out) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_in_xyz_axis_f32: NULL buffer");
    RTG_TRY(launch_quat_in_xyz_axis(q, ax[0], ax[1], ax[2], lower[0], n, out, as_stream(stream)), "k_quat_in_xyz_axis");
    return RTG_OK;
}

int rtg_quat_as_euler_f64(const float *q, const char *seq, int degrees, int64_t n, double *out, rtg_stream_t stream)
{
    if (!seq || std::strlen(seq) != 3) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_as_euler_f64: seq must have 3 axes");
    int ax[3], lower[3];
    for (int i = 0; i < 3; ++i)
        if (!axis_of(seq[i], &ax[i], &lower[i]))
            return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_as_euler_f64: bad axis '%c'", seq[i]);
    if (lower[0] != lower[1] || lower[1] != lower[2])
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_as_euler_f64: mixed intrinsic/extrinsic seq '%s'", seq);
    if (ax[0] == ax[1] || ax[1] == ax[2])
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_as_euler_f64: consecutive axes must differ ('%s')", seq);
    if (n < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_as_euler_f64: negative n");
    if (n == 0) return RTG_OK;
    if (!q || !out) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_quat_as_euler_f64: NULL buffer");
    RTG_TRY(launch_quat_as_euler(q, ax[0], ax[1], ax[2], lower[0], degrees != 0, n, out, as_stream(stream)),
            "k_quat_as_euler");
    return RTG_OK;
}

// ---------------------------------------------------------------- motion velocities
static int make_taps(const double *w, int32_t radius, GaussTaps *taps, const char *fn)
{
    if (!w) return RTG_OK;
    if (radius < 0 || radius > RTG_MAX_FILTER_RADIUS)
        return fail(RTG_ERR_UNSUPPORTED, "%s: filter radius %d (max %d)", fn, radius, RTG_MAX_FILTER_RADIUS);
    taps->radius = radius;
    for (int i = 0; i < 2 * radius + 1; ++i) taps->w[i] = w[i];
    return RTG_OK;
}

int rtg_linear_velocity_f32(const float *p, int64_t nseq, int64_t L, int64_t S, float dt, const double *w,
                            int32_t radius, float *tmp, float *out, rtg_stream_t stream)
{
    if (nseq < 0 || L < 0 || S < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_linear_velocity_f32: negative shape");
    if (nseq * L * S == 0) return RTG_OK;
    if (L < 2) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_linear_velocity_f32: np.gradient needs >= 2 frames");
    if (!p || !out || (w && !tmp)) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_linear_velocity_f32: NULL buffer");
    GaussTaps taps{};
    int rc = make_taps(w, radius, &taps, "rtg_linear_velocity_f32");
    if (rc != RTG_OK) return rc;
    RTG_TRY(launch_linear_velocity(p, nseq, L, S, dt, w ? &taps : nullptr, tmp, out, as_stream(stream)),
            "rtg_linear_velocity_f32 launch");
    return RTG_OK;
}

int rtg_angular_velocity_f32(const float *r, int64_t nseq, int64_t L, int64_t J, float dt, const double *w,
                             int32_t radius, float *tmp, float *out, rtg_stream_t stream)
{
    if (nseq < 0 || L < 0 || J < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_angular_velocity_f32: negative shape");
    if (nseq * L * J == 0) return RTG_OK;
    if (!r || !out || (w && !tmp)) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_angular_velocity_f32: NULL buffer");
    GaussTaps taps{};
    int rc = make_taps(w, radius, &taps, "rtg_angular_velocity_f32");
    if (rc != RTG_OK) return rc;
    RTG_TRY(launch_angular_velocity(r, nseq, L, J, dt, w ? &taps : nullptr, tmp, out, as_stream(stream)),
            "rtg_angular_velocity_f32 launch");
    return RTG_OK;
}

// ---------------------------------------------------------------- box probe
int rtg_box_probe(double *out, int32_t n_out, rtg_stream_t stream)
{
    if (!out || n_out < RTG_PROBE_FIELDS)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_box_probe: out needs %d doubles", RTG_PROBE_FIELDS);
    hipStream_t s = as_stream(stream);
    int dev = 0;
    hipDeviceProp_t prop{};
    RTG_TRY(hipGetDevice(&dev), "hipGetDevice");
    RTG_TRY(hipGetDeviceProperties(&prop, dev), "hipGetDeviceProperties");
    const int nblk = prop.multiProcessorCount * 8;   // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    const int nrec = (nblk + 63) / 64;
    const int64_t nf4 = (int64_t)1 << 26;             // 1 GiB per buffer: far beyond the 256 MiB Infinity Cache
    float *src = nullptr, *dst = nullptr;
    uint64_t *clk = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = hip_check(hipMalloc(&src, nf4 * 16), "hipMalloc(probe)");
    if (rc == RTG_OK) rc = hip_check(hipMalloc(&dst, nf4 * 16), "hipMalloc(probe)");
    if (rc == RTG_OK) rc = hip_check(hipMalloc(&clk, nrec * 2 * sizeof(uint64_t)), "hipMalloc(probe)");
    if (rc == RTG_OK) rc = hip_check(hipEventCreate(&e0), "hipEventCreate");
    if (rc == RTG_OK) rc = hip_check(hipEventCreate(&e1), "hipEventCreate");
    if (rc == RTG_OK) rc = hip_check(hipMemsetAsync(src, 0, nf4 * 16, s), "hipMemsetAsync");
    float best_valu = 1e30f, best_copy = 1e30f, ms = 0.0f;
    for (int rep = 0; rc == RTG_OK && rep < 4; ++rep) {   // rep 0 warms up; the best of the other three counts
        rc = hip_check(hipEventRecord(e0, s), "hipEventRecord");
        if (rc == RTG_OK) rc = hip_check(launch_probe_valu(nblk, dst, clk, s), "k_probe_valu");
        if (rc == RTG_OK) rc = hip_check(hipEventRecord(e1, s), "hipEventRecord");
        if (rc == RTG_OK) rc = hip_check(hipEventSynchronize(e1), "hipEventSynchronize");
        if (rc == RTG_OK) rc = hip_check(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
        if (rc == RTG_OK && rep > 0 && ms < best_valu) best_valu = ms;
        if (rc == RTG_OK) rc = hip_check(hipEventRecord(e0, s), "hipEventRecord");
        if (rc == RTG_OK) rc = hip_check(launch_probe_copy(src, dst, nf4, s), "k_probe_copy");
        if (rc == RTG_OK) rc = hip_check(hipEventRecord(e1, s), "hipEventRecord");
        if (rc == RTG_OK) rc = hip_check(hipEventSynchronize(e1), "hipEventSynchronize");
        if (rc == RTG_OK) rc = hip_check(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
        if (rc == RTG_OK && rep > 0 && ms < best_copy) best_copy = ms;
    }
    uint64_t h[2 * 64] = {};
    const int nr = nrec < 64 ? nrec : 64;
    if (rc == RTG_OK) rc = hip_check(hipMemcpy(h, clk, nr * 2 * sizeof(uint64_t), hipMemcpyDeviceToHost), "hipMemcpy");
    if (rc == RTG_OK) {
        double mhz[64];   // shader cycles per 100 MHz tick of each recording workgroup (the last rep), median
        int m = 0;
        for (int i = 0; i < nr; ++i)
            if (h[2 * i + 1] > 0) mhz[m++] = 100.0 * (double)h[2 * i] / (double)h[2 * i + 1];
        for (int i = 1; i < m; ++i)
            for (int j = i; j > 0 && mhz[j - 1] > mhz[j]; --j) std::swap(mhz[j - 1], mhz[j]);
        out[0] = m ? mhz[m / 2] : 0.0;
        out[1] = (double)nblk * 256 * probe_valu_iters() * 8 / (best_valu * 1e-3) / 1e12;
        out[2] = 2.0 * (double)nf4 * 16 / (best_copy * 1e-3) / 1e9;
        out[3] = best_valu;
        out[4] = best_copy;
        out[5] = prop.multiProcessorCount;
    }
    (void)hipFree(src);
    (void)hipFree(dst);
    (void)hipFree(clk);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return rc;
}

// ---------------------------------------------------------------- synthetic input
int rtg_synth_full_body_f32(rtg_topology_t t, uint64_t seed, int64_t off, int64_t B, int layout, float *body,
                            float *lh, float *rh, float *body_rot, rtg_stream_t stream)
{
    if (layout != RTG_LAYOUT_AOS && layout != RTG_LAYOUT_SOA)
        return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_synth_full_body_f32: bad layout %d", layout);
    if (!t || t->J != 59) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_synth_full_body_f32: needs the 59-joint VTRDYN_FULL topology");
    if (B < 0 || off < 0) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_synth_full_body_f32: negative batch/offset");
    if (B == 0) return RTG_OK;
    if (!body || !lh || !rh) return fail(RTG_ERR_INVALID_ARGUMENT, "rtg_synth_full_body_f32: NULL buffer");
    RTG_TRY(launch_synth_full_body(t->view(), seed, off, B, body, lh, rh, body_rot, layout, as_stream(stream)),
            "k_synth_full_body");
    return RTG_OK;
}

}  // extern "C"
