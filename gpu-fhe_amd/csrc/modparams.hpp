// Per-modulus constants shared by the host table builders and the device kernels (plain C++: no
// HIP types, so the host-only sanitizer build, tests/cpp/host_sanitize.cpp, can use it too).
#pragma once
#include <stdint.h>

namespace fhe {

using u64 = uint64_t;
using u32 = uint32_t;
using u128 = unsigned __int128;

// One record per RNS limb (device and host share the layout).
struct ModParams {
  u64 q;
  u64 mu;    // Barrett: floor(2^(2 bitlen + 2) / q); 0 marks a wide modulus (q >= 2^61)
  u32 sh_a;  // bitlen - 1
  u32 sh_b;  // bitlen + 3  (= b - a)
  u64 qinv;  // Montgomery (R = 2^64): -q^-1 mod 2^64 for odd q, else 0
  u64 r64;   // 2^64 mod q, and its Shoup companion floor(r64 2^64 / q)
  u64 r64s;
  u64 ones;  // floor(2^64 / q): the Shoup companion of 1 (a 64-bit word mod q)
};

// A constant and its Shoup companion {w, floor(w 2^64 / q)}: the byte layout of the device's
// ulonglong2 table entries.
struct Pair64 {
  u64 x, y;
};

}  // namespace fhe
