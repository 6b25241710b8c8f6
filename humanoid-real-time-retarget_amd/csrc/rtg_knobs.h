// rtg_knobs.h -- every compile-time knob of librtg_hip.so with its product default, in one place: each kernel
// TU sees the same values, and rtg_build_info() (rtg_ops.hip) reports them.  A knob here either selects a shipped
// path or builds a measurement variant (tools/build_variants.sh).  RTG_EXP_* are measurement-only, and those that
// change results (RTG_WRONG_ANSWER_KNOBS in rtg_ops.hip) make the Python binding refuse the library.  Variants
// measured and rejected are gone from the source; DESIGN.md keeps their numbers and git history their code.
#pragma once

// ---- used by rtg_solver.cuh
#ifndef RTG_SIDES_WAVES
#define RTG_SIDES_WAVES 1   // min waves per SIMD for the side kernel (1: the compiler picks; measured best)
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
// ---- used by rtg_fk.hip
#ifndef RTG_FK_QUAD
#define RTG_FK_QUAD 1   // FK / inverse FK / mixed launches: k_kin_quad (row-staged tiles, four lanes per frame); 0: windowed streaming
#endif
#ifndef RTG_FK_LDS_PAD
#define RTG_FK_LDS_PAD 0   // extra LDS bytes per streaming-FK wave: fewer waves per CU (an L2-footprint experiment)
#endif
#ifndef RTG_FK_CHUNK
#define RTG_FK_CHUNK 8
#endif
#ifndef RTG_FK_POS_REGS
#define RTG_FK_POS_REGS 1   // 1 (measured +3-4 %, bit-exact): positions held in registers and staged through the rotation window after it is
                            //    stored (no separate position window: 12.8 instead of 19.2 KiB per wave)
#endif
#ifndef RTG_FK_POS_WIN16
#define RTG_FK_POS_WIN16 0   // 1: k_fk_stream positions via a 16-joint LDS window, stored every second window (Hu FK +3 %: off)
#endif
#ifndef RTG_FK_MULTI_POS16
#define RTG_FK_MULTI_POS16 1   // the mixed launch (config 5) with the 16-joint position window (measured: 151 -> 130 us, stable)
#endif
#ifndef RTG_FK_MIN_WAVES
#define RTG_FK_MIN_WAVES 0   // >0: min waves per SIMD asked of the streaming FK kernels (4: <= 128 VGPRs, 16 waves/CU)
#endif
#ifndef RTG_FK_ALIGNED_STORE
#define RTG_FK_ALIGNED_STORE 0   // 1: FK output rows leave as whole 64-byte sectors (chunk_store_aligned; measured 11-15 % slower); 0: per-window rows
#endif
#ifndef RTG_FK_REG_SLOTS
#define RTG_FK_REG_SLOTS (RTG_FK_ALIGNED_STORE ? 2 : 0)   // aligned stores need 8 KiB of carry LDS: slots move to VGPRs
#endif
#ifndef RTG_FK_NT_STORE
#define RTG_FK_NT_STORE 0   // 1: FK output rows leave with non-temporal stores (written once, never re-read here)
#endif
#ifndef RTG_DOF_FK_POS_REGS
#define RTG_DOF_FK_POS_REGS 1   // k_dof_fk positions staged through the rotation window (as RTG_FK_POS_REGS; measured +7-9 %)
#endif
#ifndef RTG_EXP_FK_COPY
#define RTG_EXP_FK_COPY 0   // measurement knob: k_fk_stream copies its windows out without the chain (wrong answers)
#endif
#ifndef RTG_EXP_FK_NOPOS
#define RTG_EXP_FK_NOPOS 0   // measurement knob: k_fk_stream writes no position rows (wrong answers)
#endif
// ---- used by rtg_math.cuh
#ifndef RTG_FAST_EXACT
#define RTG_FAST_EXACT 1
#endif
#ifndef RTG_FAST_NORM
#define RTG_FAST_NORM 1   // sqrt_clamp_rcp: one v_rsq_f64 + Goldschmidt / Newton for the norm and 1/norm (else cr_sqrt + rcp64)
#endif
#ifndef RTG_EXP_MULR_NOBRANCH
#define RTG_EXP_MULR_NOBRANCH 0   // measurement knob: mulr without its subnormal-quotient branch (wrong answers on rare inputs)
#endif
#ifndef RTG_EXP_NO_TABLE
#define RTG_EXP_NO_TABLE 0
#endif
#ifndef RTG_ANG_TAB_BITS
#define RTG_ANG_TAB_BITS 3
#endif
#ifndef RTG_SVD_DIV
#define RTG_SVD_DIV 1   // 1: the compiler's IEEE f32 division sequence (measured +6 %); 0: rcp64 + mulr
#endif
#ifndef RTG_SVD_SQRT
#define RTG_SVD_SQRT 0  // 0: cr_sqrt (v_sqrt_f64 + Newton); 1: the compiler's IEEE f32 sqrt sequence
#endif
#ifndef RTG_EXP_STUB_SVD
#define RTG_EXP_STUB_SVD 0   // measurement knob (tools/build_variants.sh): R = identity-ish, wrong answers
#endif
