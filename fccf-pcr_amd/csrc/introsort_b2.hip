// introsort_b2.hip — K1's sort kernels compiled a second time with 256-thread block-kernel
// workgroups that hold segments of up to 4,096 elements in LDS (41 KB; the rounds split
// every longer one), three per CU (156 VGPRs, no spills), for stage groups of several
// pairs: only introsort_block_b2 (the block kernel's launch) is taken from this
// translation unit; everything else is introsort.hip's (IS_KERNEL_VARIANT leaves out its
// host functions).  Against 512-thread workgroups over 8,192 elements at two per CU:
// k_is_block 545 -> 301 us per ten-cloud launch, pipelined c3 0.593 -> 0.548 ms per
// registration (profiles/r06u).
#define KT_TU 13  // ktrace.h source tag
#ifndef IS_B2_OT
#define IS_B2_OT 256
#endif
#ifndef IS_B2_LCAP
#define IS_B2_LCAP 4096
#endif
#ifndef IS_B2_PER_CU
#define IS_B2_PER_CU 3
#endif
#define IS_OT_VAL IS_B2_OT
#define IS_LCAP_VAL IS_B2_LCAP
#ifndef IS_B2_WPE
#define IS_B2_WPE 3  // (LDS allows three workgroups per CU: 3 waves per SIMD)
#endif
#define IS_BLOCK_WPE IS_B2_WPE
#define IS_KERNEL_VARIANT 1
#include "introsort.hip"
