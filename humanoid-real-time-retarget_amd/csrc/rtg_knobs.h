// rtg_knobs.h -- every compile-time knob of librtg_hip.so with its product default, in one place: each kernel
// TU sees the same values, and rtg_build_info() (rtg_ops.hip) reports them.  A knob here either selects a shipped
// path or builds a measurement variant (tools/build_variants.sh).  RTG_EXP_* are measurement-only, and those that
// change results (RTG_WRONG_ANSWER_KNOBS in rtg_ops.hip) make the Python binding refuse the library.  Variants
// measured and rejected are gone from the source; DESIGN.md keeps their numbers and git history their code.
#pragma once

// ---- used by rtg_solver.cuh
#ifndef RTG_SIDES_TILES
#define RTG_SIDES_TILES 2   // 64-frame tiles (two waves each) per k_solve_sides block
#endif
#ifndef RTG_SIDES_SPLIT_READOUT
#define RTG_SIDES_SPLIT_READOUT 0   // FULL_BODY_POS side kernel: the left wave also reads out the right chain's slots
                                    // (round 5: medians 101.8 / 103.3 vs 102.9 / 104.0 us SoA; off since round 6's
                                    // RTG_SIDES_ARMS2 shortened the right wave: 99.3 vs 100.6 us, profiles/r06/arms2/)
#endif
#ifndef RTG_SIDES_ARMS2
#define RTG_SIDES_ARMS2 1   // FULL_BODY_POS side kernel: both arm chains in one instruction stream (fbp_arms2)
#endif
#ifndef RTG_SIDES_EARLY_WORDS
#define RTG_SIDES_EARLY_WORDS 1   // FULL_BODY_POS side kernel, AoS inputs: each read-out's table word loaded into LDS
                                  // when its link is emitted (global_load_lds), not in the read-out's batch
#endif
#ifndef RTG_AOS_PRELOAD_TIPS
#define RTG_AOS_PRELOAD_TIPS 1   // AoS inputs: the gripper's hand points loaded with the wrist fit's (125 VGPRs, still
                                 // 4 waves/SIMD; AoS 111.2 vs 113.5 us, SoA unchanged, profiles/r06/arms2/)
#endif
#ifndef RTG_SIDES_WAVES
#define RTG_SIDES_WAVES 1   // min waves per SIMD for the side kernel (1: the compiler picks; measured best)
#endif
#ifndef RTG_QUAD8_MAX_B
#define RTG_QUAD8_MAX_B 2048   // 2 <= B <= this: k_fbp_quad with 8 frames per block (one block per CU up to 2048)
#endif
#ifndef RTG_QUAD_MAX_B
#define RTG_QUAD_MAX_B 4096   // 2 <= B <= this: k_fbp_quad (swept: 16.7 vs 17.2-17.7 us up to 4096, 19.8 vs 17.5 at 8192)
#endif
#ifndef RTG_LATENCY_MAX_B
#define RTG_LATENCY_MAX_B 49152   // 2 <= B <= this: k_fbp_latency5 (swept: faster up to 49152, slower at 65536)
#endif
#ifndef RTG_EXP_HOT_INPUTS
#define RTG_EXP_HOT_INPUTS 0   // measurement knob: every side-kernel tile reads the first block's rows (wrong answers)
#endif
#ifndef RTG_EXP_TIMESTAMPS
#define RTG_EXP_TIMESTAMPS 0   // measurement knob: lane 0 of each wave records the 100 MHz wall clock at each phase
#endif                         // into body_rot (as u32 pairs) -- wrong body_rot, tools/latency_phases.py / side_phases.py
#ifndef RTG_EXP_SKIP_SIGNAL
#define RTG_EXP_SKIP_SIGNAL 0   // measurement knob: block 0's first R10 hand-over is never raised, so its partner wave
#endif                          // times out (tests the RTG_DEVERR_HANDOVER_TIMEOUT report; wrong answers)
#ifndef RTG_VEL_SEG
#define RTG_VEL_SEG 10   // linear velocity tile: rows per thread run (10: 58.0 us vs 61.2 at 20 and 68.3 at 40, with RTG_VEL_W 8)
#endif
#ifndef RTG_VEL_LDS_MIN
#define RTG_VEL_LDS_MIN 0   // A/B knob: the velocity tile's LDS request raised to this many bytes (blocks per CU)
#endif
// ---- used by rtg_fk.hip
#ifndef RTG_FK_NT_OUT
#define RTG_FK_NT_OUT 1   // the lane-group kinematics' output rows stored non-temporal (whole 1 KiB wave stores;
                          // Hu FK 88 -> 80 us, mixed 112 -> 101 us, profiles/r06/fk/nt/)
#endif
#ifndef RTG_FK_F16_MAXJ
#define RTG_FK_F16_MAXJ 36   // lane-group kinematics: 16 frames per wave (4 lanes each) up to this J, else 8 (8 lanes)
#endif
// ---- used by rtg_math.cuh
#ifndef RTG_EXP_MULR_NOBRANCH
#define RTG_EXP_MULR_NOBRANCH 0   // measurement knob: mulr without its subnormal-quotient branch (wrong answers on rare inputs)
#endif
#ifndef RTG_EXP_NO_TABLE
#define RTG_EXP_NO_TABLE 0
#endif
#ifndef RTG_EXP_LARTG_RCP64
#define RTG_EXP_LARTG_RCP64 0   // A/B knob (same values): SLARTG / SLASV2 quotients by rcp64 + mulr_k<2> (round 4's form)
#endif
#ifndef RTG_EXP_SQRT64
#define RTG_EXP_SQRT64 0   // A/B knob (same values): cr_sqrt as round 4's v_sqrt_f64 + Newton
#endif
#ifndef RTG_EXP_SQRT_CALL
#define RTG_EXP_SQRT_CALL 0   // A/B knob (same values): cr_sqrt's x < 2^-96 / inf / NaN behind a call (round 5's first form)
#endif
#ifndef RTG_EXP_ACOS_LIBM
#define RTG_EXP_ACOS_LIBM 0   // A/B knob (same values): cr_acos as round 4's libm f64 acos
#endif
#ifndef RTG_EXP_EULER_SCIPY
#define RTG_EXP_EULER_SCIPY 0   // A/B knob (same values): the 'XYZ' split through the scipy restatement for every frame
#endif
#ifndef RTG_VEL_IEEE_DIV
#define RTG_VEL_IEEE_DIV 0   // A/B knob (same values): the velocity tiles' quotients by dt as IEEE divisions (round 4)
#endif
#ifndef RTG_DOF_NT_STORE
#define RTG_DOF_NT_STORE 1   // A/B knob (same values): the solvers' DOF rows (whole 128-B lines) as non-temporal stores
                             // (headline 101.3 vs 104.5 us SoA, 114.4 vs 117.7 AoS; profiles/r05/nt/)
#endif
#ifndef RTG_IN_NT_LOAD
#define RTG_IN_NT_LOAD 0   // A/B knob (same values): the solvers' SoA input planes loaded non-temporal
#endif
#ifndef RTG_VEL_W
#define RTG_VEL_W 8   // velocity tiles: consecutive smoothed outputs per thread (8 vs 4: linear 61.2 vs 65.1 us, angular 110.5 vs 113.1)
#endif
#ifndef RTG_VEL_ANG_NWAY
#define RTG_VEL_ANG_NWAY 1   // angular velocity tile: a batch's NB elements on the N-way leaf math (rtg_math.cuh)
#endif
#ifndef RTG_DOF_NWAY
#define RTG_DOF_NWAY 4   // HuForwardModel lane groups: joint rotations per N-way group (one rare-case branch each)
#endif
#ifndef RTG_UNIT_TAB_K
#define RTG_UNIT_TAB_K 16   // the near-unit normalisation table: the 2K + 1 f32 codes around 1.0f (32: no faster,
                            // profiles/r06/unit_tab/ab_k32*)
#endif
#ifndef RTG_SIDES_SHARED_FIT
#define RTG_SIDES_SHARED_FIT 1   // k_solve_sides FULL_BODY_POS: both waves' first fits run one inlined copy of the SVD
                                 // (134.6 -> 112.3 KB; SoA median 99.2 -> 97.9 us; AoS within noise and +1.4 % VALU, so
                                 // 1 = SoA only, 2 = AoS too; profiles/r06/shared_code/)
#endif
#ifndef RTG_UPPER_UNIT_TAB
#define RTG_UPPER_UNIT_TAB 1   // k_solve_sides UPPER_BODY: the arm maps normalise through the near-1.0f table
#endif
#ifndef RTG_ROT_UNIT_TAB
#define RTG_ROT_UNIT_TAB 1   // k_solve_sides FULL_BODY_ROT: the normalisations through the near-1.0f table
#endif
#ifndef RTG_SIDES_UNIT_TAB
#define RTG_SIDES_UNIT_TAB 7   // k_solve_sides FULL_BODY_POS, SoA: near-1.0f table normalisation at (1 fits | 2 arm maps | 4 Euler split)
#endif
#ifndef RTG_SIDES_UNIT_TAB_AOS
#define RTG_SIDES_UNIT_TAB_AOS 1   // the same for AoS: the fits only (the arm maps push it to 138-141 VGPRs, 3 waves/SIMD;
                                  // without the tip preload all sites fit in 120 but measured slower, profiles/r06/unit_tab/)
#endif
#ifndef RTG_FRAME1_SHARED_CODE
#define RTG_FRAME1_SHARED_CODE 3   // k_fbp_frame1 / k_frame_server: 1 the two wrist (arm) waves run one copy of their code
                                   // (120 -> 81 KB; B = 1 12.61-12.83 -> 12.32-12.42 us); 3 also the three fits one
                                   // INLINED SVD copy after a per-wave A (60 KB): 12.13-12.38 us.  (2, an out-of-line
                                   // shared SVD, measured slower -- 12.64-12.89 us, call overhead -- and was removed;
                                   // profiles/r06/shared_code/)
#endif
#ifndef RTG_QUAD_SHARED_CODE
#define RTG_QUAD_SHARED_CODE 3   // k_fbp_quad: the same code sharing, levels 1 / 3 (config 2: level 0 16.71-16.75, 1
                                 // 16.54-16.57, 3 16.32-16.35 us vs 16.48-16.50 for level 1 in its own A/B)
#endif
#ifndef RTG_LAT5_SHARED_CODE
#define RTG_LAT5_SHARED_CODE 0   // A/B knob (same values), k_fbp_latency5: the frame1 / quad code sharing; measured mixed
                                 // (24576-32768 frames +3 %, 49152 -2 %; profiles/r06/shared_code/latency5/), off
#endif
#ifndef RTG_FRAME1_UNIT_TAB
#define RTG_FRAME1_UNIT_TAB 6   // k_fbp_frame1 / k_frame_server (B = 1): the near-1.0f table at (1 fits | 6 arm maps + Euler
                                // split); 6: 12.65-12.80 vs 12.88-13.10 us (profiles/r06/unit_tab/latency/)
#endif
#ifndef RTG_LAT_UNIT_TAB
#define RTG_LAT_UNIT_TAB 0   // A/B knob (same values), k_fbp_quad / k_fbp_latency5: the near-1.0f table at (1 fits | 6 arm maps + Euler split);
                             // all sites: B = 1 12.7-13.0 vs 12.9-13.2 us, config 2 17.2 vs 16.8 us (slower), profiles/r06/unit_tab/
#endif
#ifndef RTG_FK_UNIT_TAB
#define RTG_FK_UNIT_TAB 1   // lane-group FK / inverse FK / HuForwardModel compose: qmul_norm through the near-1.0f table
#endif
#ifndef RTG_DOF_UNIT_TAB
#define RTG_DOF_UNIT_TAB 1   // HuForwardModel: joint rotations normalised through the near-1.0f (n, 1/n) table
#endif
#ifndef RTG_VEL_UNIT_TAB
#define RTG_VEL_UNIT_TAB 1   // angular velocity: the quaternion product's normalisation through the near-1.0f table
#endif
#ifndef RTG_VEL_ANG_NB
#define RTG_VEL_ANG_NB 2   // angular velocity tile: raw elements per thread per load batch (1-4 measured alike, ~110 us)
#endif
#ifndef RTG_EXP_NO_RARE
#define RTG_EXP_NO_RARE 0   // measurement knob, a bit mask: the rare-case branches of cr_sqrt (1) / cr_acos (2) /
#endif                      // cr_sincos (4) / mulr (8) / sqrt_clamp_rcp (16) removed (wrong answers on rare inputs)
#ifndef RTG_EXP_STUB_SVD
#define RTG_EXP_STUB_SVD 0   // measurement knob (tools/build_variants.sh): R = identity-ish, wrong answers
#endif
