// rtg_solve_fbp_aos.hip -- VtrdynFullBodyPosRetargeter kernels (AOS inputs): the side kernel, the
// small-batch latency kernel and the resident per-frame server.
#include "rtg_solver.cuh"

namespace rtg {

hipError_t launch_fbp_aos(int precise, const SolverConsts &C, const float *in0, const float *in1, const float *in2,
                          int64_t B, float *dof, float *local_rot, float *body_rot, hipStream_t s)
{
    if (precise)
        launch_kind<RTG_SOLVER_FULL_BODY_POS, true, false>(C, in0, in1, in2, nullptr, B, dof, local_rot, body_rot, s);
    else
        launch_kind<RTG_SOLVER_FULL_BODY_POS, false, false>(C, in0, in1, in2, nullptr, B, dof, local_rot, body_rot, s);
    return hipGetLastError();
}

hipError_t launch_frame_server(int precise, const SolverConsts &C0, const float *in, float *dof, float *local_rot,
                               float *body_rot, uint32_t *ctl, uint64_t idle_ticks, hipStream_t s)
{
    SolverConsts C = C0;
    C.err = ctl + 3;   // the server reports into its own control block (rtg.h rtg_frame_server_launch)
    if (precise)
        hipLaunchKernelGGL((k_frame_server<true>), dim3(1), dim3(320), 0, s, C, in, dof, local_rot, body_rot, ctl,
                           idle_ticks);
    else
        hipLaunchKernelGGL((k_frame_server<false>), dim3(1), dim3(320), 0, s, C, in, dof, local_rot, body_rot, ctl,
                           idle_ticks);
    return hipGetLastError();
}

}  // namespace rtg
