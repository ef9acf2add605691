// introsort_b2.hip — K1's sort kernels compiled a second time with 512-thread block-kernel
// workgroups at two per CU (128 VGPRs each), for stage groups of several pairs: only
// introsort_block_b2 (the block kernel's launch) is taken from this translation unit;
// everything else is introsort.hip's (IS_KERNEL_VARIANT leaves out its host functions).
#define KT_TU 13  // ktrace.h source tag
#define IS_OT_VAL 512
#define IS_BLOCK_WPE 4
#define IS_KERNEL_VARIANT 1
#include "introsort.hip"
