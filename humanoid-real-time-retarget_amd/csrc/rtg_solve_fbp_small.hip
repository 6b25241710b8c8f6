// rtg_solve_fbp_small.hip -- VtrdynFullBodyPosRetargeter at small batches (k_fbp_frame1, k_fbp_quad,
// k_fbp_latency5, both input layouts) and the resident per-frame server.  Compiled with the ILP-first scheduler
// (Makefile SMALL_FLAGS): these kernels run one or two waves per SIMD, so a wave's own instruction-level parallelism
// is what hides its latencies (launch_fbp_small in rtg_solver.cuh).
#include "rtg_solver.cuh"

namespace rtg {

hipError_t launch_fbp_small(int precise, bool soa, const SolverConsts &C, const float *in0, const float *in1,
                            const float *in2, int64_t B, float *dof, float *local_rot, float *body_rot, hipStream_t s)
{
    if (precise) {
        if (soa) launch_fbp_small_kind<true, true>(C, in0, in1, in2, B, dof, local_rot, body_rot, s);
        else launch_fbp_small_kind<true, false>(C, in0, in1, in2, B, dof, local_rot, body_rot, s);
    } else {
        if (soa) launch_fbp_small_kind<false, true>(C, in0, in1, in2, B, dof, local_rot, body_rot, s);
        else launch_fbp_small_kind<false, false>(C, in0, in1, in2, B, dof, local_rot, body_rot, s);
    }
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
