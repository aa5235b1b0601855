// search_kernels_pre.hip -- the Pre-mode fast_search<J, kModePre> kernels of
// libminehip, in a translation unit of their own so that the Makefile can build
// them with a different AMDGPU machine scheduler than the rest (see
// launch_fast_pre in search_kernels.hip and SCHEDFLAGS in the Makefile).
#define MH_PRE_TU 1
#include "search_kernels.hip"
