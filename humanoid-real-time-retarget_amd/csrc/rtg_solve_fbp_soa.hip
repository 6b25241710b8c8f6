// rtg_solve_fbp_soa.hip -- VtrdynFullBodyPosRetargeter kernels (SOA inputs): the side kernel (the small-batch
// kernels are in rtg_solve_fbp_small.hip).
#include "rtg_solver.cuh"

namespace rtg {

hipError_t launch_fbp_soa(int precise, const SolverConsts &C, const float *in0, const float *in1, const float *in2,
                          int64_t B, float *dof, float *local_rot, float *body_rot, hipStream_t s)
{
    return precise
               ? launch_kind<RTG_SOLVER_FULL_BODY_POS, true, true>(C, in0, in1, in2, nullptr, B, dof, local_rot, body_rot, s)
               : launch_kind<RTG_SOLVER_FULL_BODY_POS, false, true>(C, in0, in1, in2, nullptr, B, dof, local_rot, body_rot, s);
}

}  // namespace rtg
