// Host-side number theory and table construction for libfhecore (plain C++17, no HIP): moduli,
// roots, twiddle tables in the kernels' layout, base-conversion constants.  context.cpp and
// rns.hip upload what these build; tests/cpp/host_sanitize.cpp runs them under ASan/UBSan.
// Conventions follow SURVEY.md §8a' (psi = g^((q - 1) / 2N), g the smallest primitive root).
#pragma once
#include <string>
#include <vector>

#include "modparams.hpp"

namespace fhe {

u64 mulmod_u64(u64 a, u64 b, u64 q);
u64 powmod_u64(u64 b, u64 e, u64 q);
bool is_prime_u64(u64 n);
u64 find_psi(u64 q, u32 log_n);
u32 bitrev(u32 x, u32 bits);
ModParams make_mod_params(u64 q);
inline Pair64 shoup_pair(u64 w, u64 q) { return Pair64{w, (u64)(((u128)w << 64) / q)}; }

// The `count` largest primes q < 2^bits with q = 1 mod 2N, descending, after skipping `skip`.
// Returns false (and sets err) when the range is invalid or runs out of primes.
bool gen_moduli_host(u32 log_n, u32 count, u32 bits, u32 skip, u64* out, std::string& err);

// Per-limb NTT tables (ntt.hip): twf / twi [n] Shoup pairs of psi^brv(k) / psi^-brv(k), in the
// row passes' lane-major layout (lane_major_rows), and nfold [4]: N^-1, psi^-1 N^-1 and the same
// times R = 2^64 (the fused HomMult's Montgomery tensor).  psi is returned.  twf9 (optional): the
// forward table laid out for rows of the (log_n / 2 + 1) x rest split (the HomMult's 512 x 128
// forward at N = 2^16).
u64 ntt_tables(u64 q, u32 log_n, Pair64* twf, Pair64* twi, Pair64* nfold, Pair64* twf9 = nullptr);
// Row-pass twiddle layout: the low-bit round's stage segments of each n-entry table stored
// transposed (see host_tables.cpp); a permutation within each segment.  n1: column stages of the
// split (default log_n / 2); kb_last: stages of the low-bit round (default: ntt.hip Rounds').
void lane_major_rows(Pair64* tw, size_t entries, u32 log_n, int elog, int n1 = -1,
                     int kb_last = -1);

// Fast base conversion constants (rns.hip) for the source limbs [s0, s0 + S) of `mods`:
// inv[k] = Shoup pair of (S^_k)^-1 mod s_k; hat[k * M + t] = {S^_k mod t, S^_k 2^64 mod t} for
// every limb t of `mods` (M = mods.size()).
void conv_tables(const std::vector<u64>& mods, u32 s0, u32 S, std::vector<Pair64>& inv,
                 std::vector<Pair64>& hat);

}  // namespace fhe
