// rtg_solve_other.hip -- solver setup kernels (zero-pose constants, exp-map angle table), the UPPER_BODY /
// FULL_BODY_ROT / BODY_ROT kernels, and the rtg_retarget_f32 dispatch.
#include "rtg_solver.cuh"

namespace rtg {

// solver constants prep (1 thread): theta0 / phi0 of the four arm maps and the gripper denominator, computed with
// exactly the per-frame device math.
__global__ void k_solver_prep(SolverConsts *c)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    c->lsh = shoulder_zero(c->v0_lsh);
    c->rsh = shoulder_zero(c->v0_rsh);
    c->lel = elbow_zero(c->v0_lel);
    c->rel = elbow_zero(c->v0_rel);
    c->orig = mean5(c->grip_d[0], c->grip_d[1], c->grip_d[2], c->grip_d[3], c->grip_d[4]);
}

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

template <int KIND>
static hipError_t launch_other(const SolverConsts &C, const float *in0, const float *in1, const float *in2,
                               const float *in3, int64_t B, int layout, float *dof, float *local_rot, float *body_rot,
                               hipStream_t s)
{
    if (layout == RTG_LAYOUT_SOA) return launch_kind<KIND, false, true>(C, in0, in1, in2, in3, B, dof, local_rot, body_rot, s);
    return launch_kind<KIND, false, false>(C, in0, in1, in2, in3, B, dof, local_rot, body_rot, s);
}

hipError_t launch_retarget(int kind, int precise, const SolverConsts &C, const float *in0, const float *in1,
                           const float *in2, const float *in3, int64_t B, int layout, float *dof, float *local_rot,
                           float *body_rot, hipStream_t s)
{
    switch (kind) {
    case RTG_SOLVER_FULL_BODY_POS:
        return layout == RTG_LAYOUT_SOA ? launch_fbp_soa(precise, C, in0, in1, in2, B, dof, local_rot, body_rot, s)
                                        : launch_fbp_aos(precise, C, in0, in1, in2, B, dof, local_rot, body_rot, s);
    case RTG_SOLVER_UPPER_BODY:
        return launch_other<RTG_SOLVER_UPPER_BODY>(C, in0, in1, in2, in3, B, layout, dof, local_rot, body_rot, s);
    case RTG_SOLVER_FULL_BODY_ROT:
        return launch_other<RTG_SOLVER_FULL_BODY_ROT>(C, in0, in1, in2, in3, B, layout, dof, local_rot, body_rot, s);
    default:
        return launch_other<RTG_SOLVER_BODY_ROT>(C, in0, in1, in2, in3, B, layout, dof, local_rot, body_rot, s);
    }
}

}  // namespace rtg
