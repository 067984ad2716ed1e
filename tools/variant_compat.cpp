// Entry points added to include/fhecore.h after round 4, for A/B variants built from an older
// commit (tools/build_variant.sh with REV=<rev> COMPAT=1): the ctypes table binds every declared
// symbol, so an older library needs these to load. Each one keeps the older library's behaviour.
#include <cstdint>

// Older libraries run fhe_keyswitch / fhe_rotate / fhe_mul_relin over the whole batch in one pass.
extern "C" uint32_t fhe_keyswitch_pass_batch(const void*, uint32_t batch) { return batch; }
