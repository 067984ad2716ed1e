// Host-side number theory and table construction (see host_tables.hpp).
#include "host_tables.hpp"

#include <algorithm>
#include <numeric>

namespace fhe {

u64 mulmod_u64(u64 a, u64 b, u64 q) { return (u64)((u128)a * b % q); }

u64 powmod_u64(u64 b, u64 e, u64 q) {
  u64 r = 1 % q;
  b %= q;
  while (e) {
    if (e & 1) r = mulmod_u64(r, b, q);
    b = mulmod_u64(b, b, q);
    e >>= 1;
  }
  return r;
}

bool is_prime_u64(u64 n) {
  static const u64 bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2) return false;
  for (u64 p : bases)
    if (n % p == 0) return n == p;
  u64 d = n - 1;
  int s = 0;
  while (!(d & 1)) {
    d >>= 1;
    ++s;
  }
  for (u64 a : bases) {
    u64 x = powmod_u64(a, d, n);
    if (x == 1 || x == n - 1) continue;
    bool composite = true;
    for (int r = 1; r < s && composite; ++r) {
      x = mulmod_u64(x, x, n);
      composite = x != n - 1;
    }
    if (composite) return false;
  }
  return true;
}

namespace {

u64 pollard_rho(u64 n) {
  if (!(n & 1)) return 2;
  for (u64 c = 1;; ++c) {
    u64 x = 2, y = 2, d = 1;
    while (d == 1) {
      x = (mulmod_u64(x, x, n) + c) % n;
      y = (mulmod_u64(y, y, n) + c) % n;
      y = (mulmod_u64(y, y, n) + c) % n;
      d = std::gcd(x > y ? x - y : y - x, n);
    }
    if (d != n) return d;
  }
}

void distinct_factors(u64 n, std::vector<u64>& out) {
  std::vector<u64> stack{n};
  while (!stack.empty()) {
    u64 m = stack.back();
    stack.pop_back();
    if (m == 1) continue;
    if (is_prime_u64(m)) {
      if (std::find(out.begin(), out.end(), m) == out.end()) out.push_back(m);
      continue;
    }
    u64 d = 0;
    for (u64 p = 2; p < 64 && !d; ++p)
      if (m % p == 0) d = p;
    if (!d) d = pollard_rho(m);
    stack.push_back(d);
    stack.push_back(m / d);
  }
}

}  // namespace

u64 find_psi(u64 q, u32 log_n) {
  std::vector<u64> fs;
  distinct_factors(q - 1, fs);
  u64 g = 2;
  for (;; ++g) {
    bool ok = true;
    for (u64 f : fs) ok = ok && powmod_u64(g, (q - 1) / f, q) != 1;
    if (ok) break;
  }
  return powmod_u64(g, (q - 1) / (2ull << log_n), q);
}

u32 bitrev(u32 x, u32 bits) {
  u32 r = 0;
  for (u32 i = 0; i < bits; ++i) {
    r = (r << 1) | (x & 1);
    x >>= 1;
  }
  return r;
}

ModParams make_mod_params(u64 q) {
  ModParams m{};
  m.q = q;
  const u32 bl = 64 - __builtin_clzll(q);
  // wide modulus (q >= 2^61): mu = 0 marks the exact paths (reduce128_wide, non-lazy butterflies)
  if (bl <= 61) {
    m.sh_a = bl - 1;
    m.sh_b = bl + 3;
    m.mu = (u64)(((u128)1 << (2 * bl + 2)) / q);
  }
  if (q & 1) {
    u64 inv = q;  // Newton: each step doubles the correct low bits (q * q = 1 mod 8)
    for (int i = 0; i < 5; ++i) inv *= 2 - q * inv;
    m.qinv = 0 - inv;
  }
  m.r64 = (u64)(((u128)1 << 64) % q);
  m.r64s = (u64)(((u128)m.r64 << 64) / q);
  m.ones = (u64)(((u128)1 << 64) / q);
  return m;
}

bool gen_moduli_host(u32 log_n, u32 count, u32 bits, u32 skip, u64* out, std::string& err) {
  if (log_n > 20 || bits < log_n + 3 || bits > 63) {
    err = "gen_moduli: bits out of range";
    return false;
  }
  const u64 step = 2ull << log_n;
  u64 q = (((1ull << bits) - 1) / step) * step + 1;
  if (q >= (1ull << bits)) q -= step;
  u32 found = 0;
  while (found < count + skip) {
    if (q <= step) {
      err = "gen_moduli: ran out of NTT-friendly primes";
      return false;
    }
    if (is_prime_u64(q)) {
      if (found >= skip) out[found - skip] = q;
      ++found;
    }
    q -= step;
  }
  return true;
}

// Row-pass twiddle layout (ntt.hip round_compute, ROWTAB).  The standalone and fused row passes
// split a row of R2 = 2^N2 points into rounds of at most 2^elog-point butterflies; in the round on
// the lowest position bits (the forward's last, the inverse's first) thread t of the row owns
// positions t 2^elog + [0, 2^elog), so at row stage st (bit b = N2 - 1 - st) it needs groups
// g = t W + sj, W = 2^(elog - b - 1), sj < W.  Those stages' segments [(R1 + r) 2^st, +2^st) of
// every limb's table are stored transposed -- entry g at sj TPS + t, TPS = R2 / 2^elog -- so one
// twiddle load instruction reads consecutive words across the wavefront's lanes.
void lane_major_rows(Pair64* tw, size_t entries, u32 log_n, int elog, int n1, int kb_last) {
  const u32 n = 1u << log_n;
  if (n1 < 0) n1 = (int)log_n / 2;
  const int n2 = (int)log_n - n1;
  const int nr = (n2 + elog - 1) / elog;
  if (kb_last < 0) kb_last = n2 / nr + (nr - 1 < n2 % nr ? 1 : 0);
  const u32 r1 = 1u << n1, tps = 1u << (n2 - elog);
  std::vector<Pair64> seg;
  for (size_t base = 0; base + n <= entries; base += n)
    for (int b = 0; b < kb_last; ++b) {
      const int st = n2 - 1 - b;
      const u32 w = 1u << (elog - b - 1), len = 1u << st;
      for (u32 r = 0; r < r1; ++r) {
        Pair64* p = tw + base + ((size_t)(r1 + r) << st);
        seg.assign(p, p + len);
        for (u32 g = 0; g < len; ++g) p[(g % w) * tps + g / w] = seg[g];
      }
    }
}

u64 ntt_tables(u64 q, u32 log_n, Pair64* twf, Pair64* twi, Pair64* nfold, Pair64* twf9) {
  const u64 n = 1ull << log_n;
  const u64 psi = find_psi(q, log_n), psi_inv = powmod_u64(psi, q - 2, q);
  std::vector<u64> pw(n), pwi(n);
  pw[0] = pwi[0] = 1;
  for (u64 k = 1; k < n; ++k) {
    pw[k] = mulmod_u64(pw[k - 1], psi, q);
    pwi[k] = mulmod_u64(pwi[k - 1], psi_inv, q);
  }
  for (u64 k = 0; k < n; ++k) {
    const u32 b = bitrev((u32)k, log_n);
    twf[k] = shoup_pair(pw[b], q);
    twi[k] = shoup_pair(pwi[b], q);
  }
  const u64 n_inv = powmod_u64(n % q, q - 2, q);
  const u64 r_mod = (u64)(((u128)1 << 64) % q);  // Montgomery R = 2^64 mod q
  const u64 nf1 = mulmod_u64(twi[1].x, n_inv, q);
  nfold[0] = shoup_pair(n_inv, q);
  nfold[1] = shoup_pair(nf1, q);
  nfold[2] = shoup_pair(mulmod_u64(n_inv, r_mod, q), q);  // HomMult: undo the tensor's R^-1
  nfold[3] = shoup_pair(mulmod_u64(nf1, r_mod, q), q);
  if (twf9) {  // the 512 x 128 split's forward rows (HomMult at N = 2^16: k_hm_col9 + 7-stage rows)
    std::copy(twf, twf + n, twf9);
    lane_major_rows(twf9, n, log_n, 4, (int)log_n / 2 + 1, 4);  // rounds 3 + 4 (SMALL_FIRST)
  }
  lane_major_rows(twf, n, log_n, 4);
  lane_major_rows(twi, n, log_n, 4);
  return psi;
}

void conv_tables(const std::vector<u64>& mods, u32 s0, u32 S, std::vector<Pair64>& inv,
                 std::vector<Pair64>& hat) {
  const u32 M = (u32)mods.size();
  inv.resize(S);
  hat.resize((size_t)S * M);
  for (u32 k = 0; k < S; ++k) {
    const u64 sk = mods[s0 + k];
    u64 h = 1;
    for (u32 i = 0; i < S; ++i)
      if (i != k) h = mulmod_u64(h, mods[s0 + i] % sk, sk);
    inv[k] = shoup_pair(powmod_u64(h, sk - 2, sk), sk);
    for (u32 t = 0; t < M; ++t) {
      const u64 tm = mods[t];
      u64 hm = 1;
      for (u32 i = 0; i < S; ++i)
        if (i != k) hm = mulmod_u64(hm, mods[s0 + i] % tm, tm);
      // {S^_k mod t, S^_k 2^64 mod t}: the plain word for the 128-bit sums of k_baseconv (S >= 8),
      // the Montgomery form for its Montgomery-reduced sums (S < 8)
      hat[(size_t)k * M + t] = Pair64{hm, (u64)(((u128)hm << 64) % tm)};
    }
  }
}

}  // namespace fhe
