// The standalone NTT row passes at E = 8 elements per thread: ntt.hip rebuilt with FHE_ELOG = 3,
// exporting only launch_ntt_row_e8 (ntt.hip, row_pass).  Half the VGPRs and LDS per wave of the
// E = 16 build, so twice the resident waves cover the per-row twiddle loads' L2 latency.
#define FHE_ELOG 3
#define FHE_NTT_ROW_ONLY 1
#include "ntt.hip"
