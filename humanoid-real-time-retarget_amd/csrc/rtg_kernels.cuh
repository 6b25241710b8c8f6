// rtg_kernels.cuh -- types shared by the kernels and the C-ABI layer.
#pragma once
#include "rtg_math.cuh"
#include "rtg.h"

namespace rtg {

// One (step, sub-lane) entry of the lane-group FK schedule (fk_group_schedule, rtg_fk.hip): at step s, sub-lane u of
// every frame's lane group composes joint `code & 0xFF` (0xFF: idle) from its parent `(code >> 8) & 0xFF`, with that
// joint's zero-pose local translation and tree quaternion alongside (two ds_read_b128 per step).
struct alignas(16) GEnt {
    float lx, ly, lz;
    int32_t code;
    float qx, qy, qz, qw;
};
constexpr int kGroupMaxJ = 64;   // the lane-group kernels serve J <= 64 (every shipped skeleton); larger: lane walks

// Device view of a topology (all pointers device memory, uniform per launch).
struct TopoView {
    const int32_t *parents;   // (J)   parents[j] < j, root -1
    const V *local_t;         // (J)   zero-pose local translation
    const Q *tree_quat;       // (J)   SkeletonTree pre-rotation
    int32_t J;
    const GEnt *gsched;       // (gsteps * 64 / gF) lane-group schedule, or nullptr (J > kGroupMaxJ: lane walks)
    int32_t gF;               // frames per wave of the lane-group kernels (16: J <= 36, 8: J <= 64)
    int32_t gsteps;           // steps of the lane-group schedule
};
// the lane-group frames per wave for J joints (0: J too large, the lane-walk kernels run); F J <= 64 * 9 records
inline int group_frames(int J) { return J <= RTG_FK_F16_MAXJ ? 16 : (J <= kGroupMaxJ ? 8 : 0); }
// fills `out` (steps x (64 / F) entries) and returns the step count
int32_t fk_group_schedule(const int32_t *parents, const V *local_t, const Q *tree_quat, int32_t J, int32_t F,
                          GEnt *out, int32_t max_steps);

// Per-solver constants, passed by value (kernel argument -> SGPRs).
struct SolverConsts {
    V Zt[3];          // torso Kabsch zero vectors
    V Zl[5], Zr[5];   // wrist Kabsch zero vectors
    V v0_lsh, v0_lel, v0_rsh, v0_rel;
    ArmZero lsh, lel, rsh, rel;   // theta0 / phi0, filled by k_solver_prep
    float grip_d[5];  // zero-pose x distances of the 5 finger tips to the wrist
    float orig;       // their mean (gripper denominator), filled by k_solver_prep
    int32_t par[4];   // BODY_ROT: parents of joints 18, 14, 19, 15
    const uint32_t *ang_tab;   // exp-map angle table (kAngTabWords words, device), owned by the solver handle
    uint32_t *err;             // host-mapped error word of the solver handle: a wave hand-over that timed out ORs
                               // RTG_DEVERR_HANDOVER_TIMEOUT in (rtg_retarget_f32 reports it on the next call)
};

// Joint-angle forward model (HuForwardModel): per-DOF axis and optional limits, device memory.
struct DofView {
    const int32_t *axis;   // (J-1) 0/1/2
    const float *lower;    // (J-1) or nullptr
    const float *upper;    // (J-1) or nullptr
};

struct FkSeg {
    TopoView T;
    const float *local_rot;   // op 1 (inverse FK): the global rotations in
    const float *root_t;      // op 1: unused
    float *g_rot;             // op 1: the local rotations out
    float *g_pos;             // op 1: unused
    int64_t B;
    int32_t op;               // 0: FK (kinematics.py:13-39), 1: inverse FK (kinematics.py:41-63)
};
struct FkMultiArgs {
    FkSeg seg[RTG_MAX_SEGMENTS];
    int64_t block_start[RTG_MAX_SEGMENTS];
    int32_t n;
};

hipError_t launch_solver_prep(SolverConsts *dev_consts, hipStream_t s);
hipError_t launch_build_ang_tab(uint32_t *tab, hipStream_t s);   // kAngTabWords words
hipError_t launch_frame_server(int precise, const SolverConsts &C, const float *in, float *dof, float *local_rot,
                               float *body_rot, uint32_t *ctl, uint64_t idle_ticks, hipStream_t s);
hipError_t launch_retarget(int kind, int precise, const SolverConsts &C, const float *in0, const float *in1,
                           const float *in2, const float *in3, int64_t B, int layout, float *dof, float *local_rot,
                           float *body_rot, hipStream_t s);
hipError_t launch_fk(const TopoView &T, bool state, const float *lr, const float *rt, int64_t B, float *gr, float *gp,
                     hipStream_t s);
hipError_t launch_local_rotation(const TopoView &T, bool state, const float *g, int64_t B, float *l, hipStream_t s);
hipError_t launch_fk_multi(FkMultiArgs &A, hipStream_t s);
hipError_t launch_dof_fk(const TopoView &T, const DofView &D, bool clip, const float *dof, const float *root_rot,
                         const float *root_t, int64_t B, float *gr, float *gp, hipStream_t s);
hipError_t launch_rescale_motion(const TopoView &T, const float *motion, int64_t B, const float *dir, float *out,
                                 hipStream_t s);
hipError_t launch_quat_between(const float *v1, const float *v2, int64_t n, float *out, float *ws, hipStream_t s);
hipError_t launch_rebuild_vtrdyn(const TopoView &T, const float *motion, int64_t B, float *g_rot, float *root_t,
                                 float *ws, hipStream_t s);
hipError_t launch_ingest_vtrdyn(const float *bp, const float *lhp, const float *rhp, int64_t B, int layout,
                                float *body, float *lh, float *rh, uint8_t *valid, hipStream_t s);
hipError_t launch_quat_op(int op, const float *a, const float *b, const float *c, int64_t n, float *out,
                          hipStream_t s);
hipError_t launch_cal_joint_quat(const float *Z, const float *M, int npts, int64_t n, float *out, hipStream_t s);
hipError_t launch_quat_as_euler(const float *q, int s0, int s1, int s2, int extrinsic, int degrees, int64_t n,
                               double *out, hipStream_t s);
hipError_t launch_quat_in_xyz_axis(const float *q, int s0, int s1, int s2, int extrinsic, int64_t n, float *out,
                                   hipStream_t s);
struct GaussTaps {
    double w[2 * RTG_MAX_FILTER_RADIUS + 1];
    int32_t radius;
};
hipError_t launch_linear_velocity(const float *p, int64_t nseq, int64_t L, int64_t S, float dt, const GaussTaps *taps,
                                  float *tmp, float *out, hipStream_t s);
hipError_t launch_angular_velocity(const float *r, int64_t nseq, int64_t L, int64_t J, float dt,
                                   const GaussTaps *taps, float *tmp, float *out, hipStream_t s);
hipError_t launch_synth_full_body(const TopoView &T, uint64_t seed, int64_t off, int64_t B, float *body, float *lh,
                                  float *rh, float *body_rot, int layout, hipStream_t s);
hipError_t launch_probe_valu(int nblocks, float *sink, uint64_t *clk, hipStream_t s);
hipError_t launch_probe_copy(const float *src, float *dst, int64_t nfloat4, hipStream_t s);
int probe_valu_iters();

}  // namespace rtg
