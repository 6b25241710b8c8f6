/*
 * rtg.h -- C ABI of the MI355X-native retargeting hot path (librtg_hip.so).
 *
 * The reference (shuoshuof/Humanoid-Real-Time-Retarget) has no native
 * boundary: its operator API is the set of Python classes / TorchScript
 * functions called in-process on CPU float32 tensors.  Each entry point below
 * replaces one of those (cited per function); the Python drop-in modules in
 * humanoid-real-time-retarget_amd/{retarget,robot_kinematics_model,poselib}
 * bind them with ctypes.
 *
 * Conventions
 *  - quaternions are [x, y, z, w] float32 (poselib/poselib/core/rotation3d.py:14-27);
 *  - every pointer argument is a caller-owned DEVICE pointer (hipMalloc / torch
 *    device tensor), C-contiguous, float32 unless stated; the library never
 *    frees caller memory and never allocates in a launch call;
 *  - launches are stream-ordered on `stream` (a hipStream_t; NULL = default
 *    stream) and thread-safe across distinct streams; nothing synchronises;
 *  - every call returns an rtg_status; on failure rtg_last_error() returns a
 *    thread-local message.  Argument errors mirror the reference's Python
 *    assertions (e.g. proj_in_plane's |n| > 1e-6, transform3d.py:70).
 */
#ifndef RTG_H
#define RTG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTG_ABI_VERSION 4   /* 4: the frame server's sequence word lives in its inbox (in[RTG_SERVER_SEQ_WORD]; ctl[0]
                                  reserved), the inbox may be device memory (rtg_server_inbox_alloc), rtg_frame_server_signal;
                               3: frames the reference raises on are marked (rtg_frame_error), the solver error word, ctl[3];
                               2: the input-layout argument of rtg_retarget_f32 / rtg_ingest_vtrdyn_f32 / rtg_synth_full_body_f32 */

typedef enum rtg_status {
    RTG_OK = 0,
    RTG_ERR_INVALID_ARGUMENT = 1,
    RTG_ERR_DEVICE = 2,          /* a HIP runtime call failed */
    RTG_ERR_OUT_OF_MEMORY = 3,
    RTG_ERR_UNSUPPORTED = 4,
    RTG_ERR_TIMEOUT = 5,         /* rtg_frame_server_post: the frame was not served in time */
    RTG_SERVER_ENDED = 6         /* rtg_frame_server_post: the server ended (idle) before it took the frame */
} rtg_status;

/* Frame-batch layout of solver inputs.  AOS: the reference's (B, P, C) rows (e.g. body
 * (B,21,3)), what sim_full_body_teleop.py:109-119 hands over.  SOA: component planes (P, C, B) -- element
 * (frame f, point j, component c) at [(j*C + c)*B + f] -- so a wavefront's load of one component of 64
 * consecutive frames is one 256-byte contiguous read.  The batched producers (ingest, synth) emit either. */
typedef enum rtg_layout { RTG_LAYOUT_AOS = 0, RTG_LAYOUT_SOA = 1 } rtg_layout;

typedef struct rtg_topology_s *rtg_topology_t;
typedef struct rtg_solver_s *rtg_solver_t;
typedef void *rtg_stream_t; /* hipStream_t */

/* Library / error handling. */
int rtg_abi_version(void);
const char *rtg_last_error(void);
/* Number of visible devices (0 when no GPU / driver). */
int rtg_device_count(void);
/* The compile-time configuration of this library as a JSON object: every RTG_* build knob and its value, and
 * "wrong_answer_knobs" = 1 when any measurement-only knob that changes results is on (RTG_EXP_STUB_SVD, _NO_TABLE,
 * _HOT_INPUTS, _FK_COPY, _FK_NOPOS, _MULR_NOBRANCH, _TIMESTAMPS, _SKIP_SIGNAL).  A product library has 0; the Python
 * binding refuses any other. */
const char *rtg_build_info(void);

/* ------------------------------------------------------------------------
 * Topology: a parent-indexed skeleton (SkeletonTree, skeleton3d.py:83-96;
 * RobotZeroPose, robot_kinematics_model/base_robot.py:24-58).
 * parents[J] (root = -1, parents[j] < j), local_t[J*3] zero-pose local
 * translation, tree_quat[J*4] the SkeletonTree pre-rotation (NULL = identity).
 * Host pointers; the data is copied to device memory owned by the handle.
 * ---------------------------------------------------------------------- */
int rtg_topology_create(const int32_t *parents, const float *local_t, const float *tree_quat, int32_t J,
                        rtg_topology_t *out);
int rtg_topology_destroy(rtg_topology_t topo);
int rtg_topology_num_joints(rtg_topology_t topo);

/* ------------------------------------------------------------------------
 * Kinematics
 * ---------------------------------------------------------------------- */
/* cal_forward_kinematics (robot_kinematics_model/kinematics.py:13-39).
 * local_rot (B,J,4), root_t (B,3) -> g_rot (B,J,4), g_pos (B,J,3). */
int rtg_fk_f32(rtg_topology_t topo, const float *local_rot, const float *root_t, int64_t B, float *g_rot,
               float *g_pos, rtg_stream_t stream);
/* cal_local_rotation (kinematics.py:41-63). g_rot (B,J,4) -> local_rot (B,J,4). */
int rtg_local_rotation_f32(rtg_topology_t topo, const float *g_rot, int64_t B, float *local_rot,
                           rtg_stream_t stream);
/* SkeletonState.global_transformation (poselib skeleton3d.py:402-425): FK with the
 * tree pre-rotation; local_rot must hold the state's (normalised) rotations. */
int rtg_state_fk_f32(rtg_topology_t topo, const float *local_rot, const float *root_t, int64_t B, float *g_rot,
                     float *g_pos, rtg_stream_t stream);
/* SkeletonState.local_rotation (skeleton3d.py:460-484): inverse FK incl. tree-quat fix-up. */
int rtg_state_local_rotation_f32(rtg_topology_t topo, const float *g_rot, int64_t B, float *local_rot,
                                 rtg_stream_t stream);

/* Mixed-target FK: up to RTG_MAX_SEGMENTS independent (topology, frame batch)
 * segments in ONE launch (BASELINE config 5). */
#define RTG_MAX_SEGMENTS 8
typedef struct rtg_fk_segment {
    rtg_topology_t topo;
    const float *local_rot; /* (B,J,4) */
    const float *root_t;    /* (B,3)   */
    float *g_rot;           /* (B,J,4) */
    float *g_pos;           /* (B,J,3) */
    int64_t B;
} rtg_fk_segment;
int rtg_fk_multi_f32(const rtg_fk_segment *segments, int32_t n_segments, rtg_stream_t stream);
/* Mixed-target inverse FK (cal_local_rotation, kinematics.py:41-63): up to RTG_MAX_SEGMENTS (topology, batch)
 * segments in one launch. */
typedef struct rtg_local_rotation_segment {
    rtg_topology_t topo;
    const float *g_rot;     /* (B,J,4) */
    float *local_rot;       /* (B,J,4) */
    int64_t B;
} rtg_local_rotation_segment;
int rtg_local_rotation_multi_f32(const rtg_local_rotation_segment *segments, int32_t n_segments, rtg_stream_t stream);
/* FK segments and inverse-FK segments together in ONE launch (BASELINE config 5: "FK plus inverse FK" on the
 * four robot_config skeletons); n_fk + n_inv <= RTG_MAX_SEGMENTS. */
int rtg_kinematics_multi_f32(const rtg_fk_segment *fk, int32_t n_fk, const rtg_local_rotation_segment *inv,
                             int32_t n_inv, rtg_stream_t stream);

/* ------------------------------------------------------------------------
 * Joint-angle forward model: HuForwardModel (robot_kinematics_model/
 * hu_forward_model.py:13-33).  A topology plus one rotation axis per DOF
 * (J-1 entries, 0=x 1=y 2=z: torch.eye(3)[Hu_DOF_AXIS], :16) and optional
 * DOF limits (J-1 each; both NULL = none).  Host pointers, copied.
 * ---------------------------------------------------------------------- */
typedef struct rtg_dof_model_s *rtg_dof_model_t;
int rtg_dof_model_create(rtg_topology_t topo, const int32_t *axis, const float *lower, const float *upper,
                         rtg_dof_model_t *out);
int rtg_dof_model_destroy(rtg_dof_model_t model);
/* forward_kinematics(motion_joint_angles (B,J-1), motion_root_translation (B,3),
 * motion_root_rotation (B,4), clip_angles) -> g_rot (B,J,4), g_pos (B,J,3).
 * clip != 0 applies a' = (clamp(a, lower, upper) - a) + a (:27-33) and needs limits.
 * local[j] = quat_from_angle_axis(a'[j-1], axis[j-1]) (:21-23), local[0] = root rotation (:24). */
int rtg_dof_fk_f32(rtg_dof_model_t model, const float *dof, const float *root_rot, const float *root_t, int64_t B,
                   int clip, float *g_rot, float *g_pos, rtg_stream_t stream);

/* ------------------------------------------------------------------------
 * VTRDyn ingest (sim_full_body_teleop.py:92, :109-112)
 * ---------------------------------------------------------------------- */
/* Raw broadcast frames body_pos (B,23,3), left/right_hand_pos (B,20,3) -> solver inputs body (B,21,3)
 * (23 -> 21 joint reindex), hands (B,20,3) (point reorder), and valid (B) uint8: 0 where every body value
 * is within 1e-8 of 0 (np.allclose(body_pos, 0): the teleop loop keeps the previous DOFs), else 1.
 * layout: of the outputs body / lh / rh (the raw inputs are the reference's rows). */
int rtg_ingest_vtrdyn_f32(const float *body_pos, const float *left_hand, const float *right_hand, int64_t B,
                          int layout, float *body, float *lh, float *rh, uint8_t *valid, rtg_stream_t stream);

/* ------------------------------------------------------------------------
 * Motion-level prep of the legacy motion path (retarget/main.py)
 * ---------------------------------------------------------------------- */
/* Retarget.rescale_motion_to_standard_size (main.py:37-47) after coord_transform(p, dir=dir) (:170;
 * transform3d.py:24-29).  motion (B,J,3) -> out (B,J,3): every bone scaled to its zero-pose length and hung
 * from the parent's rescaled position.  dir: 3 floats (host) or NULL. */
int rtg_rescale_motion_f32(rtg_topology_t topo, const float *motion, int64_t B, const float *dir, float *out,
                           rtg_stream_t stream);
/* quat_between_two_vecs (transform3d.py:8-21): v1, v2 (n,3) -> (n,4).  The identity branch is decided over the
 * whole batch (max norm <= 1e-6, :11-12), as the reference does.  workspace: 2 floats of device memory. */
int rtg_quat_between_f32(const float *v1, const float *v2, int64_t n, float *out, float *workspace,
                         rtg_stream_t stream);
/* RetargetHuV5fromMocap._rebuild_with_vtrdyn_zero_pose (main.py:116-165) up to the SkeletonState it builds
 * (rotations normalised, skeleton3d.py:610).  topo: the 21-joint VTRDYN zero pose; motion (B,21,3) rescaled
 * positions -> g_rot (B,21,4) global rotations, root_t (B,3).  workspace: J floats of device memory. */
int rtg_rebuild_vtrdyn_f32(rtg_topology_t topo, const float *motion, int64_t B, float *g_rot, float *root_t,
                           float *workspace, rtg_stream_t stream);

/* ------------------------------------------------------------------------
 * Retarget solvers (retarget/retarget_solver/__init__.py:9-14)
 * ---------------------------------------------------------------------- */
typedef enum rtg_solver_kind {
    /* VtrdynFullBodyPosRetargeter.retarget  full_body_pos_retargeter.py:25-217
     * in0 = body (B,21,3), in1 = left hand (B,20,3), in2 = right hand (B,20,3);
     * source zero pose = VTRDYN_FULL (59 joints). */
    RTG_SOLVER_FULL_BODY_POS = 0,
    /* HuUpperBodyFromMocapRetarget.retarget_from_global_translation  retarget_solver.py:40-99
     * in0 = raw VTRDyn positions (B,21,3); source zero pose = VTRDYN (21). */
    RTG_SOLVER_UPPER_BODY = 1,
    /* VtrdynFullBodyRetargeter.retarget  full_body_retargeter.py:19-177
     * in0 = body rotations (B,21,4), in1 = body positions (B,21,3),
     * in2 = left hand (B,20,3), in3 = right hand (B,20,3); source = VTRDYN_FULL (59). */
    RTG_SOLVER_FULL_BODY_ROT = 2,
    /* Mocap2HuBodyRetargeter.retarget_from_pose  body_retargeter.py:34-81
     * in0 = global rotations (B,21,4); source = VTRDYN (21). */
    RTG_SOLVER_BODY_ROT = 3
} rtg_solver_kind;

/* Create a solver.  src_zero_local_t / src_zero_global_t: the source
 * RobotZeroPose local / global translations (Js,3), src_parents (Js) -- host
 * pointers.  The target is always Hu v5 (31 links, 30 DOFs; Hu_v5.py:12-18).
 * Zero-pose-only terms of the joint maps (theta0 / phi0, Kabsch zero vectors,
 * gripper denominator) are evaluated once here, on the device.  The solver
 * also owns a 6.7 MiB exp-map angle table, built here on the current device
 * (synchronously); use the solver on that device only.  Replaces the
 * constructors at full_body_pos_retargeter.py:18, retarget_solver.py:28,
 * full_body_retargeter.py:16, body_retargeter.py:31. */
int rtg_solver_create(int kind, const float *src_zero_local_t, const float *src_zero_global_t,
                      const int32_t *src_parents, int32_t Js, int precise_gripper, rtg_solver_t *out);
int rtg_solver_destroy(rtg_solver_t solver);

/* Frames on which the reference raises.  The reference solves one frame per call and, on some degenerate
 * frames, raises instead of returning:
 *   RTG_FRAME_SVD_NONFINITE   cal_joint_quat's Kabsch matrix has a NaN entry: torch.linalg.svd raises
 *                             RuntimeError "linalg.svd: (Batch element 0): The algorithm failed to converge because
 *                             the input matrix contained non-finite values." (transform3d.py:40);
 *   RTG_FRAME_ZERO_NORM_QUAT  the quaternion handed to quat_in_xyz_axis is all zero or has a NaN: scipy raises
 *                             ValueError "Found zero norm quaternions in `quat`." (transform3d.py:53) -- e.g. a
 *                             zero-length arm segment, an upper arm along the shoulder plane's normal, a straight
 *                             elbow (radians_between_vecs of a zero projection is NaN, transform3d.py:77-100).
 * The code is the first raise in the reference's own order (torso fit, left wrist fit, left Euler split, right
 * wrist fit, right Euler split; full_body_pos_retargeter.py:68-167).  A batched launch marks such a frame instead
 * of raising: every dof of its row is NaN, and dof[f*30 + 0] -- exactly 0 for every other frame, the solvers never
 * write DOF 0 -- has the bit pattern RTG_FRAME_NAN | code; its local_rot / body_rot rows are RTG_FRAME_NAN. */
typedef enum rtg_frame_error {
    RTG_FRAME_OK = 0,
    RTG_FRAME_SVD_NONFINITE = 1,
    RTG_FRAME_ZERO_NORM_QUAT = 2
} rtg_frame_error;
#define RTG_FRAME_NAN 0x7FC00000u   /* quiet NaN; the low payload bits carry the rtg_frame_error code in dof[f*30] */

/* Errors a launch reports on the solver's NEXT call (launches never synchronise): the device ORs these into the
 * solver's host-mapped error word and rtg_retarget_f32 returns RTG_ERR_DEVICE with the word in rtg_last_error(),
 * then clears it.  A wave that waited ~0.1 s for its partner wave's hand-over flag gives up and sets
 * RTG_DEVERR_HANDOVER_TIMEOUT: that launch's outputs are not to be trusted. */
#define RTG_DEVERR_HANDOVER_TIMEOUT 0x1u

/* Batched retarget of B frames.  dof (B,30) required; local_rot (B,31,4) and
 * body_rot (B,59,4, FULL_BODY_POS only: the returned body_global_rotation) may
 * be NULL.  Unused in* must be NULL.  layout (rtg_layout) describes the inputs
 * only; the outputs are always (B, ...) rows.  Frames on which the reference
 * raises are marked as described at rtg_frame_error.  Replaces the per-frame
 * .retarget calls of sim_full_body_teleop.py:115-119 / sim_teleop_mujoco.py:104-108
 * / sim_teleop.py:102. */
int rtg_retarget_f32(rtg_solver_t solver, const float *in0, const float *in1, const float *in2,
                     const float *in3, int64_t B, int layout, float *dof, float *local_rot, float *body_rot,
                     rtg_stream_t stream);

/* Per-frame server for the teleop loop (sim_full_body_teleop.py:109-119 retargets one captured frame per
 * iteration through VtrdynFullBodyPosRetargeter.retarget, full_body_pos_retargeter.py:60-176): launches ONE
 * resident workgroup that serves FULL_BODY_POS frames without a launch per frame.
 *   in        the server's inbox, RTG_SERVER_INBOX_FLOATS floats: the frame in floats 0..182 -- body (21,3) | left
 *             hand (20,3) | right hand (20,3), rows as rtg_retarget_f32's AoS inputs -- and the frame sequence number
 *             (uint32) in float RTG_SERVER_SEQ_WORD, stored by the host after the frame's rows.  Either device memory
 *             from rtg_server_inbox_alloc (the host stores into it through the PCIe BAR: the faster hand-over) or
 *             device-accessible pinned host memory.
 *   dof (30), local_rot (31,4, may be NULL), body_rot (59,4, may be NULL): pinned host memory the server OWNS while it
 *             runs.  The dof row and the frame-dependent local_rot / body_rot rows are written per frame; the 73
 *             rows that never change (local_rot's fixed links, body_rot's identity rows) are written once per
 *             launch and again after a frame the reference raises on.  A client that clears or edits these
 *             buffers between frames must copy the rows out instead (rtg_frame_server_post does) or relaunch.
 *   ctl       4 x uint32, pinned host memory: [0] reserved (ABI <= 3: the sequence number);
 *             [1] the last sequence number served, written by the device after that frame's outputs;
 *             [2] set to 1 by the device when the server has ended;
 *             [3] the server's error word (RTG_DEVERR_*), set before [1] of the frame it concerns.
 *             Zero ctl[1..3] before the launch, and have the inbox's sequence word equal ctl[1] (both 0 at first).
 * Storing RTG_SERVER_QUIT as the sequence number (rtg_frame_server_signal) ends the server; so does idle_ms
 * (1..60000) without a new frame.  The stream is occupied until the server ends.  The values in the buffers after a
 * frame is served (ctl[1]) are bit-identical to rtg_retarget_f32's at B = 1. */
#define RTG_SERVER_QUIT 0xFFFFFFFFu
#define RTG_SERVER_INBOX_FLOATS 256
#define RTG_SERVER_SEQ_WORD 192
int rtg_frame_server_launch(rtg_solver_t solver, const float *in, float *dof, float *local_rot, float *body_rot,
                            uint32_t *ctl, uint32_t idle_ms, rtg_stream_t stream);

/* A frame-server inbox in device memory that the host can store into (hipExtMallocWithFlags, uncached; the CPU
 * reaches it through the PCIe BAR): RTG_SERVER_INBOX_FLOATS floats, zeroed.  Host stores into it are
 * write-combined: rtg_frame_server_post / rtg_frame_server_signal drain them (sfence) in order.  Free with
 * rtg_server_inbox_free.  A 184-float ping-pong through it takes 4.0 us against 4.8 us through pinned host memory
 * on MI355X (tools/bar_probe.hip). */
int rtg_server_inbox_alloc(float **inbox);
int rtg_server_inbox_free(float *inbox);

/* Stores `word` as the inbox's sequence number and drains it to the device (host only, no HIP call): RTG_SERVER_QUIT
 * ends a running server; after it has ended, store ctl[1] back before a relaunch. */
int rtg_frame_server_signal(float *in, uint32_t word);

/* One frame through a running rtg_frame_server_launch server, on the host alone (no HIP call): the whole per-frame
 * round trip of the teleop loop (sim_full_body_teleop.py:115-119) in one C call.  Copies the frame's rows into the
 * server's inbox `in` (body (21,3) | left hand (20,3) | right hand (20,3)), stores `seq` (!= the last one posted,
 * != RTG_SERVER_QUIT) as its sequence number after them, spins until the device publishes it in ctl[1], then copies
 * the pinned outputs the server writes (dof 30, local_rot 124, body_rot 236 floats) into the *_dst buffers that are
 * not NULL.  Returns RTG_OK; RTG_SERVER_ENDED if the server ended (idle_ms) before it took the frame -- relaunch it
 * and post the same seq again; RTG_ERR_TIMEOUT after timeout_us (the frame may still be served later);
 * RTG_ERR_DEVICE if the server set its error word (ctl[3]) while serving the frame (the outputs are copied anyway;
 * the word is cleared). */
int rtg_frame_server_post(uint32_t *ctl, uint32_t seq, float *in, const float *body, const float *left_hand,
                          const float *right_hand, const float *dof, const float *local_rot, const float *body_rot,
                          float *dof_dst, float *local_rot_dst, float *body_rot_dst, uint32_t timeout_us);

/* ------------------------------------------------------------------------
 * Elementwise primitives (poselib rotation3d.py, retarget transform3d.py)
 * ---------------------------------------------------------------------- */
typedef enum rtg_quat_op {
    RTG_OP_QUAT_MUL = 0,            /* a (n,4), b (n,4) -> (n,4)   rotation3d.py:14-27   */
    RTG_OP_QUAT_MUL_NORM = 1,       /* a, b -> (n,4)               :196-202             */
    RTG_OP_QUAT_NORMALIZE = 2,      /* a -> (n,4)                  :92-98               */
    RTG_OP_QUAT_ROTATE = 3,         /* q (n,4), v (n,3) -> (n,3)   :205-211             */
    RTG_OP_QUAT_INVERSE = 4,        /* a -> (n,4)                  :214-219             */
    RTG_OP_QUAT_FROM_ANGLE_AXIS = 5,/* angle (n), axis (n,3) -> (n,4)  :122-143         */
    RTG_OP_QUAT_FROM_ROTMAT = 6,    /* m (n,3,3) -> (n,4)          :146-193             */
    RTG_OP_QUAT_TO_EXP_MAP = 7,     /* q (n,4) -> (n,3)            :620-627             */
    RTG_OP_RADIANS_BETWEEN = 8,     /* v1 (n,3), v2 (n,3), c = n (n,3) -> (n)  transform3d.py:77-100 */
    RTG_OP_PROJ_IN_PLANE = 9,       /* v (n,3), n (n,3) -> (n,3)   transform3d.py:61-75 */
    RTG_OP_QUAT_TO_DOF_POS = 10,    /* local_rot (n,31,4) -> dof (n,30)  transform3d.py:176-183 (Hu) */
    RTG_OP_SHOULDER_PR = 11,        /* v1 (n,3), v0 (n,3), parent c (n,4) -> (n,2,4)  full_body_pos_retargeter.py:246-278 */
    RTG_OP_ELBOW_PY = 12,           /* v1, v0, parent -> (n,2,4)   full_body_pos_retargeter.py:220-243 */
    RTG_OP_QUAT_TO_ANGLE_AXIS = 13, /* q (n,4) -> (n,4) = [angle, axis xyz]  rotation3d.py:587-608 */
    RTG_OP_NORMALIZE_ANGLE = 14,    /* x (n) -> (n) atan2(sin x, cos x)      rotation3d.py:582-584 */
    RTG_OP_QUAT_ABS = 15,           /* q (n,4) -> (n) |q|                    rotation3d.py:41-47  */
    RTG_OP_QUAT_UNIT = 16,          /* q (n,4) -> q / max(|q|, 1e-9)         rotation3d.py:50-56  */
    RTG_OP_QUAT_ANGLE_AXIS = 17,    /* q (n,4) -> [acos(2w^2-1), xyz/|xyz|]  rotation3d.py:230-240 */
    /* the rest of the rotation3d / transform3d surface (off the solver path; same op-order contract) */
    RTG_OP_EXP_MAP_TO_ANGLE_AXIS = 18, /* e (n,3) -> (n,4) [angle, axis]      rotation3d.py:629-646 */
    RTG_OP_EXP_MAP_TO_QUAT = 19,    /* e (n,3) -> (n,4)      rotation3d.py:648-652 = transform3d.py:146-150 */
    RTG_OP_QUAT_SLERP = 20,         /* q0 a (n,4), q1 b (n,4), t c (n) -> (n,4)   transform3d.py:152-174 */
    RTG_OP_QUAT_FROM_XYZ = 21,      /* xyz (n,3) -> (n,4) [xyz, 1 - |xyz|], per row  rotation3d.py:101-108 */
    RTG_OP_ROT_MATRIX_DET = 22,     /* m (n,3,3) -> (n)                      rotation3d.py:338-350 */
    RTG_OP_ROT_MATRIX_FROM_QUAT = 23, /* q (n,4) -> (n,3,3)                  rotation3d.py:398-427 */
    RTG_OP_ROTATION_ALONG_X = 24,   /* q (n,4) -> (n) extract_rotation_along_axis(q, 0)  rotation3d.py:534-556 */
    RTG_OP_ROTATION_ALONG_Y = 25,   /* ... axis 1 */
    RTG_OP_ROTATION_ALONG_Z = 26,   /* ... axis 2 */
    RTG_OP_PROJECT_QUAT_X = 27,     /* q (n,4) -> (n,4)  project_quat_to_axis_x   rotation3d.py:479-486 */
    RTG_OP_PROJECT_QUAT_Y = 28,     /*                   project_quat_to_axis_y   :488-495 */
    RTG_OP_PROJECT_QUAT_Z = 29,     /*                   project_quat_to_axis_z   :497-504 */
    RTG_OP_PROJECT_QUAT_XY = 30,    /*                   project_quat_to_axis_xy  :506-517 */
    RTG_OP_PROJECT_QUAT_XZ = 31     /*                   project_quat_to_axis_xz  :519-530 */
} rtg_quat_op;
int rtg_quat_op_f32(int op, const float *a, const float *b, const float *c, int64_t n, float *out,
                    rtg_stream_t stream);

/* cal_joint_quat (transform3d.py:31-50): Kabsch fit of npts (1..8) point pairs.
 * Z (n,npts,3) zero-pose vectors, M (n,npts,3) motion vectors -> (n,4).  A fit whose Kabsch matrix has a NaN
 * entry (where torch.linalg.svd raises, rtg_frame_error) gets all four components = RTG_FRAME_NAN |
 * RTG_FRAME_SVD_NONFINITE. */
int rtg_cal_joint_quat_f32(const float *Z, const float *M, int32_t npts, int64_t n, float *out,
                           rtg_stream_t stream);

/* quat_in_xyz_axis (transform3d.py:52-59): scipy Euler split (float64) into three
 * single-axis quaternions.  seq: 3 chars of xyz/XYZ (upper = intrinsic). q (n,4) -> (n,3,4).  A quaternion scipy
 * refuses (zero norm or NaN, rtg_frame_error) gets all twelve outputs = RTG_FRAME_NAN | RTG_FRAME_ZERO_NORM_QUAT. */
int rtg_quat_in_xyz_axis_f32(const float *q, const char *seq, int64_t n, float *out, rtg_stream_t stream);
/* scipy Rotation.from_quat(q).as_euler(seq, degrees) in float64 (rotation3d.py:658-661 quat_to_eular uses
 * 'xyz', degrees=True; degrees multiply by 180/pi like np.rad2deg).  q (n,4) f32 -> out (n,3) f64.  A quaternion
 * scipy refuses gets the three f64 NaNs 0x7FF8000000000000 | RTG_FRAME_ZERO_NORM_QUAT. */
int rtg_quat_as_euler_f64(const float *q, const char *seq, int degrees, int64_t n, double *out, rtg_stream_t stream);

/* ------------------------------------------------------------------------
 * Motion velocities (SkeletonMotion.from_skeleton_state, poselib skeleton3d.py:1026-1049,
 * _compute_velocity :1126-1135, _compute_angular_velocity :1137-1146).
 * Time is the middle axis: nseq independent sequences of L frames of S channels.
 * weights: the 2*radius+1 Gaussian taps (scipy _gaussian_kernel1d, sigma=2 ->
 * radius 8, applied with mode='nearest' and float64 accumulation); NULL = no
 * smoothing.  tmp: caller-owned scratch of the output's size (required with
 * weights; the one-pass kernel, used while a 16-frame tile's raw rows fit
 * 48 KB of LDS, leaves it untouched; wider rows filter through it).
 * ---------------------------------------------------------------------- */
#define RTG_MAX_FILTER_RADIUS 16
/* p (nseq,L,S) -> out (nseq,L,S): np.gradient over frames / dt, then smoothing. */
int rtg_linear_velocity_f32(const float *p, int64_t nseq, int64_t L, int64_t S, float dt, const double *weights,
                            int32_t radius, float *tmp, float *out, rtg_stream_t stream);
/* r (nseq,L,J,4) global rotations -> out (nseq,L,J,3): axis*angle of
 * quat_mul_norm(r[t+1], conj(r[t])) / dt (last frame 0), then smoothing. */
int rtg_angular_velocity_f32(const float *r, int64_t nseq, int64_t L, int64_t J, float dt, const double *weights,
                             int32_t radius, float *tmp, float *out, rtg_stream_t stream);

/* ------------------------------------------------------------------------
 * Synthetic mocap (bench / tests): FK of the VTRDYN_FULL zero pose with random
 * rotations, generated on the device from a counter-based RNG.
 * topo must be the 59-joint VTRDYN_FULL topology.  Frame f uses stream
 * (seed, frame_offset + f).  Outputs body (B,21,3), lh (B,20,3), rh (B,20,3)
 * and optionally body_rot (B,21,4), in the given layout.
 * ---------------------------------------------------------------------- */
int rtg_synth_full_body_f32(rtg_topology_t topo, uint64_t seed, int64_t frame_offset, int64_t B, int layout,
                            float *body, float *lh, float *rh, float *body_rot, rtg_stream_t stream);

/* ------------------------------------------------------------------------
 * Box probe (diagnostics, no reference counterpart): what the current GPU delivers right now, so throughput
 * measured on one box can be set against another's.  Synchronous; allocates 2 GiB of scratch for its duration.
 * out (host, >= RTG_PROBE_FIELDS doubles):
 *   [0] shader clock under full VALU load, MHz (shader-cycle counter / 100 MHz wall clock, median workgroup)
 *   [1] f32 FMA issue rate, T lane-ops/s      [2] HBM copy bandwidth (read + write), GB/s
 *   [3] VALU kernel ms                        [4] copy kernel ms (1 GiB -> 1 GiB)     [5] compute units
 * ---------------------------------------------------------------------- */
#define RTG_PROBE_FIELDS 6
int rtg_box_probe(double *out, int32_t n_out, rtg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* RTG_H */
