// _frame_post.cpp -- the teleop frame's host round trip (rtg_frame_server_post, include/rtg.h) as ONE Python call
// that takes the frame's three CPU tensors and returns the three result tensors (rtg/realtime.py FrameServer).
//
// Through ctypes the same frame costs ~6 us of Python on top of the C call (per-argument conversion, three
// torch.from_numpy wrappers, attribute reads for every input check); here the checks, the output allocation and
// the frame-mark read are C++.  The C ABI stays torch-free: this binding receives the address of
// rtg_frame_server_post from librtg_hip.so (ctypes) and calls it like any other client.  Host-only code: it never
// touches the GPU, and rtg/realtime.py keeps its ctypes path for a tree without this module.
#include <torch/extension.h>

#include <cstdint>
#include <cstring>
#include <tuple>

namespace {

using PostFn = int (*)(uint32_t *ctl, uint32_t seq, float *in, const float *body, const float *left_hand,
                       const float *right_hand, const float *dof, const float *local_rot, const float *body_rot,
                       float *dof_dst, float *local_rot_dst, float *body_rot_dst, uint32_t timeout_us);

constexpr uint32_t kFrameNan = 0x7FC00000u;   // rtg.h RTG_FRAME_NAN
constexpr int kServerEnded = 6;               // rtg.h RTG_SERVER_ENDED
constexpr int kNotHostF32 = -1;               // an input is not a contiguous CPU float32 tensor of its size

bool host_f32(const at::Tensor &t, int64_t n)
{
    return t.device().is_cpu() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n;
}

// (rc, frame error code, local_rot (31,4), dof (30,), body_rot (59,4) or None).  rc: rtg_status of the post, or
// kNotHostF32 before anything was posted (the caller converts the inputs and calls again).  A server that ended
// before taking the frame returns kServerEnded with the frame still posted: relaunch and call again with the same
// seq.  The frame error code is read off DOF 0 (rtg.h rtg_frame_error; 0: the reference returns a result).
std::tuple<int, int, at::Tensor, at::Tensor, c10::optional<at::Tensor>> post(
    int64_t fn, int64_t ctl, int64_t seq, int64_t in, const at::Tensor &body, const at::Tensor &lh, const at::Tensor &rh,
    int64_t dof_src, int64_t lr_src, int64_t br_src, int64_t timeout_us)
{
    if (!host_f32(body, 63) || !host_f32(lh, 60) || !host_f32(rh, 60))
        return {kNotHostF32, 0, at::Tensor(), at::Tensor(), c10::nullopt};
    const auto opt = at::TensorOptions().dtype(at::kFloat);
    at::Tensor lr = at::empty({31, 4}, opt), dof = at::empty({30}, opt);
    c10::optional<at::Tensor> br;
    if (br_src) br = at::empty({59, 4}, opt);
    float *const br_dst = br ? br->data_ptr<float>() : nullptr;
    int rc;
    {
        // the post spins until the frame is back (up to timeout_us when the server is late or relaunching): other
        // Python threads -- the teleop loop's mocap receiver -- run meanwhile, as they did under ctypes
        pybind11::gil_scoped_release nogil;
        rc = reinterpret_cast<PostFn>(fn)(
            reinterpret_cast<uint32_t *>(ctl), (uint32_t)seq, reinterpret_cast<float *>(in), body.data_ptr<float>(),
            lh.data_ptr<float>(), rh.data_ptr<float>(), reinterpret_cast<const float *>(dof_src),
            reinterpret_cast<const float *>(lr_src), reinterpret_cast<const float *>(br_src), dof.data_ptr<float>(),
            lr.data_ptr<float>(), br_dst, (uint32_t)timeout_us);
    }
    int code = 0;
    if (rc == 0) {
        uint32_t d0;
        std::memcpy(&d0, dof.data_ptr<float>(), 4);
        if ((d0 & ~0xFu) == kFrameNan) code = (int)(d0 & 0xFu);
    }
    return {rc, code, lr, dof, br};
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m)
{
    m.doc() = "rtg_frame_server_post with tensor arguments and results (the teleop frame's host round trip)";
    m.def("post", &post, "one frame through a running frame server");
    m.attr("SERVER_ENDED") = kServerEnded;
    m.attr("NOT_HOST_F32") = kNotHostF32;
}
