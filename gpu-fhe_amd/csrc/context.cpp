// Host side of fhe_ctx: parameter validation, number theory and the device-resident tables
// (twiddles with Shoup companions, Barrett constants, base-conversion constants).
//
// The reference has no context -- MOD is passed on every call (/root/reference/arithmetic.py:3,7,11)
// and NTT takes no parameters at all (arithmetic.py:15).  The context here owns everything the
// kernels need per modulus so that the hot calls take only device pointers and sizes.
// Conventions follow SURVEY.md §8a' (psi = g^((q-1)/2N), g the smallest primitive root).
#include <algorithm>
#include <cstring>
#include <numeric>

#include "internal.hpp"

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

u32 bitrev(u32 x, u32 bits) {
  u32 r = 0;
  for (u32 i = 0; i < bits; ++i) {
    r = (r << 1) | (x & 1);
    x >>= 1;
  }
  return r;
}

// Row-pass twiddle layout (ntt.hip round_compute, ROWTAB).  The standalone and fused row passes
// split a row of R2 = 2^N2 points into rounds of at most 2^elog-point butterflies; in the round on
// the lowest position bits (the forward's last, the inverse's first) thread t of the row owns
// positions t 2^elog + [0, 2^elog), so at row stage st (bit b = N2 - 1 - st) it needs groups
// g = t W + sj, W = 2^(elog - b - 1), sj < W.  Those stages' segments [(R1 + r) 2^st, +2^st) of
// every limb's table are stored transposed -- entry g at sj TPS + t, TPS = R2 / 2^elog -- so one
// twiddle load instruction reads consecutive words across the wavefront's lanes.
void lane_major_rows(std::vector<ulonglong2>& tw, u32 log_n, int elog) {
  const u32 n = 1u << log_n;
  const int n1 = (int)log_n / 2, n2 = (int)log_n - n1;
  const int nr = (n2 + elog - 1) / elog;
  const int kb_last = n2 / nr + (nr - 1 < n2 % nr ? 1 : 0);
  const u32 r1 = 1u << n1, tps = 1u << (n2 - elog);
  std::vector<ulonglong2> seg;
  for (size_t base = 0; base < tw.size(); base += n)
    for (int b = 0; b < kb_last; ++b) {
      const int st = n2 - 1 - b;
      const u32 w = 1u << (elog - b - 1), len = 1u << st;
      for (u32 r = 0; r < r1; ++r) {
        ulonglong2* p = tw.data() + base + ((size_t)(r1 + r) << st);
        seg.assign(p, p + len);
        for (u32 g = 0; g < len; ++g) p[(g % w) * tps + g / w] = seg[g];
      }
    }
}

inline ulonglong2 shoup_pair(u64 w, u64 q) {
  ulonglong2 p;
  p.x = w;
  p.y = (u64)(((u128)w << 64) / q);
  return p;
}

template <class T>
int upload(T** dptr, const T* src, size_t count) {
  FHE_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(dptr), count * sizeof(T)));
  FHE_HIP_CHECK(hipMemcpy(*dptr, src, count * sizeof(T), hipMemcpyHostToDevice));
  return kOk;
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

int gen_moduli(u32 log_n, u32 count, u32 bits, u32 skip, u64* out) {
  if (bits < log_n + 3 || bits > 63) {
    set_error("gen_moduli: bits out of range");
    return kInvalid;
  }
  const u64 step = 2ull << log_n;
  u64 q = (((1ull << bits) - 1) / step) * step + 1;
  if (q >= (1ull << bits)) q -= step;
  u32 found = 0;
  while (found < count + skip) {
    if (q <= step) {
      set_error("gen_moduli: ran out of NTT-friendly primes");
      return kInvalid;
    }
    if (is_prime_u64(q)) {
      if (found >= skip) out[found - skip] = q;
      ++found;
    }
    q -= step;
  }
  return kOk;
}

int ctx_create(fhe_ctx** out, u32 log_n, const u64* q, u32 L, const u64* p, u32 K, u32 dnum,
               int device) {
  if (!out) {
    set_error("ctx_create: null out pointer");
    return kInvalid;
  }
  *out = nullptr;
  if (log_n < 10 || log_n > 17) {
    set_error("ctx_create: log_n must be in [10, 17]");
    return kUnsupported;
  }
  if (L == 0 || L > 64 || K > 16 || (K > 0 && (dnum == 0 || dnum > L))) {
    set_error("ctx_create: need 1 <= L <= 64, K <= 16, 1 <= dnum <= L when K > 0");
    return kInvalid;
  }
  const u64 n = 1ull << log_n;
  std::vector<u64> mods(q, q + L);
  if (K) mods.insert(mods.end(), p, p + K);
  for (size_t i = 0; i < mods.size(); ++i) {
    const u64 m = mods[i];
    if (m >= (1ull << 63) || m % (2 * n) != 1 || !is_prime_u64(m)) {
      set_error("ctx_create: modulus #" + std::to_string(i) + " = " + std::to_string(m) +
                " is not a prime < 2^63 with q = 1 mod 2N");
      return kInvalid;
    }
    for (size_t j = 0; j < i; ++j)
      if (mods[j] == m) {
        set_error("ctx_create: duplicate modulus " + std::to_string(m));
        return kInvalid;
      }
  }
  int ndev = 0;
  FHE_HIP_CHECK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    set_error("ctx_create: device index out of range");
    return kInvalid;
  }
  FHE_HIP_CHECK(hipSetDevice(device));

  int cus = 0;
  FHE_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  auto* c = new fhe_ctx();
  c->device = device;
  c->num_cus = cus;
  c->lz16 = true;
  c->wide = false;
  for (u64 m : mods) {
    c->lz16 = c->lz16 && m < (1ull << 60);
    c->wide = c->wide || m >= (1ull << 61);
  }
  c->log_n = log_n;
  c->n = n;
  c->L = L;
  c->K = K;
  c->dnum = K ? dnum : 0;
  c->alpha = K ? (L + dnum - 1) / dnum : 0;
  c->moduli = mods;
  const size_t M = mods.size();
  std::vector<ulonglong2> twf(M * n), twi(M * n), nfold(4 * M);
  c->psi.resize(M);
  c->mods_host.resize(M);
  std::vector<u64> pw(n), pwi(n);
  for (size_t i = 0; i < M; ++i) {
    const u64 m = mods[i];
    c->mods_host[i] = make_mod_params(m);
    const u64 psi = find_psi(m, log_n), psi_inv = powmod_u64(psi, m - 2, m);
    c->psi[i] = psi;
    pw[0] = pwi[0] = 1;
    for (u64 k = 1; k < n; ++k) {
      pw[k] = mulmod_u64(pw[k - 1], psi, m);
      pwi[k] = mulmod_u64(pwi[k - 1], psi_inv, m);
    }
    for (u64 k = 0; k < n; ++k) {
      const u32 b = bitrev((u32)k, log_n);
      twf[i * n + k] = shoup_pair(pw[b], m);
      twi[i * n + k] = shoup_pair(pwi[b], m);
    }
    const u64 n_inv = powmod_u64(n % m, m - 2, m);
    const u64 r_mod = (u64)(((u128)1 << 64) % m);  // Montgomery R = 2^64 mod q
    const u64 nf1 = mulmod_u64(twi[i * n + 1].x, n_inv, m);
    nfold[4 * i] = shoup_pair(n_inv, m);
    nfold[4 * i + 1] = shoup_pair(nf1, m);
    nfold[4 * i + 2] = shoup_pair(mulmod_u64(n_inv, r_mod, m), m);  // HomMult: undo R^-1
    nfold[4 * i + 3] = shoup_pair(mulmod_u64(nf1, r_mod, m), m);
  }
  lane_major_rows(twf, log_n, 4);
  lane_major_rows(twi, log_n, 4);
  int rc = kOk;
  if ((rc = upload(&c->d_mods, c->mods_host.data(), M)) ||
      (rc = upload(&c->d_tw_fwd, twf.data(), M * n)) ||
      (rc = upload(&c->d_tw_inv, twi.data(), M * n)) ||
      (rc = upload(&c->d_nfold, nfold.data(), 4 * M)) || (rc = build_rns_tables(c)) ||
      (rc = build_galois_tables(c))) {
    ctx_destroy(c);
    return rc;
  }
  *out = c;
  return kOk;
}

int ctx_destroy(fhe_ctx* c) {
  if (!c) return kOk;
  (void)hipSetDevice(c->device);
  if (c->aux_stream) (void)hipStreamDestroy(c->aux_stream);
  if (c->aux_fork) (void)hipEventDestroy(c->aux_fork);
  if (c->aux_join) (void)hipEventDestroy(c->aux_join);
  for (auto& t : c->bc_tables) (void)hipFree(t.second);
  for (void* ptr : {(void*)c->d_mods, (void*)c->d_tw_fwd, (void*)c->d_tw_inv, (void*)c->d_nfold, (void*)c->d_nfold_down,
                    (void*)c->d_modup_inv, (void*)c->d_modup_hat, (void*)c->d_moddown_inv,
                    (void*)c->d_moddown_hat, (void*)c->d_pinv, (void*)c->d_rs_tab,
                    (void*)c->d_rs_half, c->workspace})
    if (ptr) (void)hipFree(ptr);
  delete c;
  return kOk;
}

}  // namespace fhe
