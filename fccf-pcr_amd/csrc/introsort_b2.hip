// introsort_b2.hip — K1's sort kernels compiled a second time with 512-thread block-kernel
// workgroups at two per CU (128 VGPRs each), for stage groups of several pairs: only
// introsort_block_b2 (the block kernel's launch) is taken from this translation unit;
// everything else is introsort.hip's (IS_KERNEL_VARIANT leaves out its host functions).
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
#define IS_B2_WPE 4
#endif
#define IS_BLOCK_WPE IS_B2_WPE
#define IS_KERNEL_VARIANT 1
#include "introsort.hip"
