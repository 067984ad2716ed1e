// The key-switch kernels built from ntt.hip in a translation unit of their own (compile time:
// ntt.hip's instantiations are split over three files that build in parallel): the column-forward
// pass alone, the fused ModUp conversion + column pass (k_modup_col), the fused row-NTT + inner
// product (k_ks_row_inner) and the fused ModDown row pass (k_moddown_row).
#define FHE_NTT_KS_ONLY 1
#include "ntt.hip"
