/* Exact C restatement of the FHE polynomial-arithmetic hot path (TEST INFRASTRUCTURE ONLY).
 *
 * Role: the bit-exact CPU comparator for the HIP kernels at full sizes and the timed host
 * baseline ("kind": "port") in bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it; nothing in gpu-fhe_amd/ links or calls it.
 *
 * It restates oracle/pyoracle.py (itself pinned by the reference's golden vectors for
 * vec_add/vec_sub/vec_mul -- /root/reference/arithmetic.py:3-13 -- and by the O(N^2) NTT
 * definition of SURVEY.md §8a', since the reference's NTT/iNTT are identities,
 * arithmetic.py:15-19).  Every modular product is computed as an exact unsigned __int128
 * followed by a 128-bit % (twiddle products use Shoup with an exact correction step), so the
 * outputs are the canonical residues in [0, q) that define parity.
 *
 * Layout everywhere: u64 residues [poly][limb][N], limb-major, each limb contiguous.
 * Threading: OpenMP over (poly, limb) pairs.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;

/* ---------------------------------------------------------------- number theory */
static u64 mulmod(u64 a, u64 b, u64 q) { return (u64)((u128)a * b % q); }

static u64 powmod(u64 b, u64 e, u64 q) {
  u64 r = 1 % q;
  b %= q;
  while (e) {
    if (e & 1) r = mulmod(r, b, q);
    b = mulmod(b, b, q);
    e >>= 1;
  }
  return r;
}

static int is_prime(u64 n) {
  static const u64 bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2) return 0;
  for (int i = 0; i < 12; ++i)
    if (n % bases[i] == 0) return n == bases[i];
  u64 d = n - 1;
  int s = 0;
  while (!(d & 1)) { d >>= 1; ++s; }
  for (int i = 0; i < 12; ++i) {
    u64 x = powmod(bases[i], d, n);
    if (x == 1 || x == n - 1) continue;
    int comp = 1;
    for (int r = 1; r < s; ++r) {
      x = mulmod(x, x, n);
      if (x == n - 1) { comp = 0; break; }
    }
    if (comp) return 0;
  }
  return 1;
}

static u64 gcd64(u64 a, u64 b) { while (b) { u64 t = a % b; a = b; b = t; } return a; }

static u64 rho(u64 n) {
  if (!(n & 1)) return 2;
  for (u64 c = 1;; ++c) {
    u64 x = 2, y = 2, d = 1;
    while (d == 1) {
      x = (mulmod(x, x, n) + c) % n;
      y = (mulmod(y, y, n) + c) % n;
      y = (mulmod(y, y, n) + c) % n;
      d = gcd64(x > y ? x - y : y - x, n);
    }
    if (d != n) return d;
  }
}

/* distinct prime factors of n into fs (returns count) */
static int factor_distinct(u64 n, u64* fs) {
  u64 stack[128];
  int sp = 0, nf = 0;
  stack[sp++] = n;
  while (sp) {
    u64 m = stack[--sp];
    if (m == 1) continue;
    if (is_prime(m)) {
      int seen = 0;
      for (int i = 0; i < nf; ++i) seen |= fs[i] == m;
      if (!seen) fs[nf++] = m;
      continue;
    }
    u64 d = 0;
    for (u64 p = 2; p < 64 && !d; ++p)
      if (m % p == 0) d = p;
    if (!d) d = rho(m);
    stack[sp++] = d;
    stack[sp++] = m / d;
  }
  return nf;
}

u64 oracle_primitive_root(u64 q) {
  u64 fs[64];
  int nf = factor_distinct(q - 1, fs);
  for (u64 g = 2;; ++g) {
    int ok = 1;
    for (int i = 0; i < nf && ok; ++i) ok = powmod(g, (q - 1) / fs[i], q) != 1;
    if (ok) return g;
  }
}

u64 oracle_psi(u64 q, uint32_t log_n) {
  u64 n2 = 2ull << log_n;
  return powmod(oracle_primitive_root(q), (q - 1) / n2, q);
}

/* The `count` largest primes < 2^bits with q = 1 mod 2N, descending, after `skip`. */
int oracle_gen_moduli(uint32_t log_n, uint32_t count, uint32_t bits, uint32_t skip, u64* out) {
  u64 step = 2ull << log_n;
  u64 q = (((1ull << bits) - 1) / step) * step + 1;
  if (q >= (1ull << bits)) q -= step;
  uint32_t found = 0;
  while (found < count + skip) {
    if (q <= step) return -1;
    if (is_prime(q)) {
      if (found >= skip) out[found - skip] = q;
      ++found;
    }
    q -= step;
  }
  return 0;
}

static uint32_t bitrev(uint32_t x, uint32_t bits) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < bits; ++i) { r = (r << 1) | (x & 1); x >>= 1; }
  return r;
}

/* ---------------------------------------------------------------- twiddle tables */
typedef struct {
  u64 q;
  uint32_t log_n;
  u64* w;    /* psi^brv(k)          */
  u64* ws;   /* floor(w * 2^64 / q) */
  u64* wi;   /* psi^-brv(k)         */
  u64* wis;
  u64 n_inv;
} tables_t;

#define MAX_TABLES 256
static tables_t g_tab[MAX_TABLES];
static int g_ntab = 0;

/* The table cache.  Only prepare() (serial, before any parallel region of its caller) may build
 * or recycle entries; the parallel regions only look them up.  (Recycling inside get_tables, as
 * this file first did, could free a table an earlier prepare() of the same call had just built
 * once ~256 distinct moduli had passed through one process, and the parallel lookups then built
 * entries concurrently: wrong expected values in a long test session.) */
static const tables_t* find_tables(u64 q, uint32_t log_n) {
  for (int i = 0; i < g_ntab; ++i)
    if (g_tab[i].q == q && g_tab[i].log_n == log_n) return &g_tab[i];
  return NULL;
}

static const tables_t* get_tables(u64 q, uint32_t log_n) {
  const tables_t* found = find_tables(q, log_n);
  if (found) return found;
  if (g_ntab == MAX_TABLES) {
    fprintf(stderr, "fhe_oracle: table cache full outside prepare()\n");
    abort();
  }
  tables_t* t = &g_tab[g_ntab++];
  u64 n = 1ull << log_n;
  t->q = q;
  t->log_n = log_n;
  t->w = malloc(n * 8); t->ws = malloc(n * 8); t->wi = malloc(n * 8); t->wis = malloc(n * 8);
  u64 psi = oracle_psi(q, log_n), psi_inv = powmod(psi, q - 2, q);
  u64* pw = malloc(n * 8);
  u64* pwi = malloc(n * 8);
  pw[0] = pwi[0] = 1;
  for (u64 i = 1; i < n; ++i) { pw[i] = mulmod(pw[i - 1], psi, q); pwi[i] = mulmod(pwi[i - 1], psi_inv, q); }
  for (u64 k = 0; k < n; ++k) {
    uint32_t b = bitrev((uint32_t)k, log_n);
    t->w[k] = pw[b];
    t->wi[k] = pwi[b];
    t->ws[k] = (u64)(((u128)t->w[k] << 64) / q);
    t->wis[k] = (u64)(((u128)t->wi[k] << 64) / q);
  }
  free(pw); free(pwi);
  t->n_inv = powmod(n % q, q - 2, q);
  return t;
}

/* Shoup product x*w mod q for x < 2^64, w < q (exact: the estimate is corrected fully). */
static inline u64 shoup(u64 x, u64 w, u64 ws, u64 q) {
  u64 qh = (u64)(((u128)x * ws) >> 64);
  u64 r = x * w - qh * q;
  while (r >= q) r -= q;
  return r;
}

/* ---------------------------------------------------------------- NTT */
static void ntt_fwd_1(u64* a, const tables_t* t) {
  const u64 q = t->q;
  const u64 n = 1ull << t->log_n;
  u64 tt = n;
  for (u64 m = 1; m < n; m <<= 1) {
    tt >>= 1;
    for (u64 i = 0; i < m; ++i) {
      const u64 w = t->w[m + i], ws = t->ws[m + i];
      u64* x = a + 2 * i * tt;
      u64* y = x + tt;
      for (u64 j = 0; j < tt; ++j) {
        u64 u = x[j], v = shoup(y[j], w, ws, q);
        u64 s = u + v;
        x[j] = s >= q ? s - q : s;
        y[j] = u >= v ? u - v : u + q - v;
      }
    }
  }
}

static void ntt_inv_1(u64* a, const tables_t* t) {
  const u64 q = t->q;
  const u64 n = 1ull << t->log_n;
  u64 tt = 1;
  for (u64 m = n; m > 1; m >>= 1) {
    const u64 h = m >> 1;
    for (u64 i = 0; i < h; ++i) {
      const u64 w = t->wi[h + i], ws = t->wis[h + i];
      u64* x = a + 2 * i * tt;
      u64* y = x + tt;
      for (u64 j = 0; j < tt; ++j) {
        u64 u = x[j], v = y[j];
        u64 s = u + v;
        x[j] = s >= q ? s - q : s;
        y[j] = shoup(u >= v ? u - v : u + q - v, w, ws, q);
      }
    }
    tt <<= 1;
  }
  const u64 ni = t->n_inv, nis = (u64)(((u128)ni << 64) / q);
  for (u64 j = 0; j < n; ++j) a[j] = shoup(a[j], ni, nis, q);
}

static void prepare(uint32_t log_n, const u64* moduli, uint32_t L) {
  uint32_t missing = 0;
  for (uint32_t l = 0; l < L; ++l) missing += find_tables(moduli[l], log_n) == NULL;
  if (g_ntab + missing > MAX_TABLES) { /* recycle everything before building this call's tables */
    for (int i = 0; i < g_ntab; ++i) {
      free(g_tab[i].w); free(g_tab[i].ws); free(g_tab[i].wi); free(g_tab[i].wis);
    }
    g_ntab = 0;
  }
  for (uint32_t l = 0; l < L; ++l) get_tables(moduli[l], log_n);
}

/* data: [polys][L][N], in place. */
void oracle_ntt_fwd(u64* data, uint64_t polys, uint32_t log_n, const u64* moduli, uint32_t L) {
  prepare(log_n, moduli, L);
  const u64 n = 1ull << log_n;
#pragma omp parallel for schedule(dynamic)
  for (int64_t pl = 0; pl < (int64_t)(polys * L); ++pl)
    ntt_fwd_1(data + (u64)pl * n, get_tables(moduli[pl % L], log_n));
}

void oracle_ntt_inv(u64* data, uint64_t polys, uint32_t log_n, const u64* moduli, uint32_t L) {
  prepare(log_n, moduli, L);
  const u64 n = 1ull << log_n;
#pragma omp parallel for schedule(dynamic)
  for (int64_t pl = 0; pl < (int64_t)(polys * L); ++pl)
    ntt_inv_1(data + (u64)pl * n, get_tables(moduli[pl % L], log_n));
}

/* ---------------------------------------------------------------- coefficient-wise ops
 * rows x cols u64 matrices; row r uses modulus mods[r * mod_stride] (mod_stride 0 = scalar).
 * Exact for any u64 inputs and 1 < q < 2^64 (Python/numpy-object '%' semantics). */
void oracle_vec_op(int op, u64* out, const u64* a, const u64* b, uint64_t rows, uint64_t cols,
                   const u64* mods, uint64_t mod_stride) {
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < (int64_t)rows; ++r) {
    const u64 q = mods[r * mod_stride];
    for (u64 c = 0; c < cols; ++c) {
      const u64 x = a[r * cols + c], y = b[r * cols + c];
      u64 v;
      if (op == 0) v = (u64)(((u128)x + y) % q);
      else if (op == 1) { u64 xr = x % q, yr = y % q; v = xr >= yr ? xr - yr : xr + (q - yr); }
      else v = (u64)((u128)x * y % q);
      out[r * cols + c] = v;
    }
  }
}

/* ---------------------------------------------------------------- HomMult
 * a, b: [batch][2][L][N] coefficient form; d: [batch][3][L][N] coefficient form. */
void oracle_hommult(u64* d, const u64* a, const u64* b, uint64_t batch, uint32_t log_n,
                    const u64* moduli, uint32_t L) {
  prepare(log_n, moduli, L);
  const u64 n = 1ull << log_n, limb = n, ct = 2 * L * n;
#pragma omp parallel for schedule(dynamic)
  for (int64_t bl = 0; bl < (int64_t)(batch * L); ++bl) {
    const u64 bi = (u64)bl / L, l = (u64)bl % L;
    const tables_t* t = get_tables(moduli[l], log_n);
    const u64 q = t->q;
    u64* A0 = malloc(n * 8); u64* A1 = malloc(n * 8);
    u64* B0 = malloc(n * 8); u64* B1 = malloc(n * 8);
    memcpy(A0, a + bi * ct + l * limb, n * 8);
    memcpy(A1, a + bi * ct + (L + l) * limb, n * 8);
    memcpy(B0, b + bi * ct + l * limb, n * 8);
    memcpy(B1, b + bi * ct + (L + l) * limb, n * 8);
    ntt_fwd_1(A0, t); ntt_fwd_1(A1, t); ntt_fwd_1(B0, t); ntt_fwd_1(B1, t);
    u64* D0 = d + bi * 3 * L * n + l * limb;
    u64* D1 = D0 + L * n;
    u64* D2 = D1 + L * n;
    for (u64 j = 0; j < n; ++j) {
      D0[j] = mulmod(A0[j], B0[j], q);
      D1[j] = (u64)(((u128)mulmod(A0[j], B1[j], q) + mulmod(A1[j], B0[j], q)) % q);
      D2[j] = mulmod(A1[j], B1[j], q);
    }
    ntt_inv_1(D0, t); ntt_inv_1(D1, t); ntt_inv_1(D2, t);
    free(A0); free(A1); free(B0); free(B1);
  }
}

/* ---------------------------------------------------------------- RNS base conversion
 * Fast basis extension without correction (SURVEY.md §8a'), coefficient domain.
 * x: [S][N] over src moduli; out: [T][N] over dst moduli. */
void oracle_baseconv(u64* out, const u64* x, uint64_t n, const u64* src, uint32_t S,
                     const u64* dst, uint32_t T) {
  /* (S/s_i)^-1 mod s_i and (S/s_i) mod t, by products of residues */
  u64* hat_inv = malloc(S * 8);
  u64* hat_mod = malloc((u64)S * T * 8);
  for (uint32_t i = 0; i < S; ++i) {
    u64 h = 1;
    for (uint32_t k = 0; k < S; ++k)
      if (k != i) h = mulmod(h, src[k] % src[i], src[i]);
    hat_inv[i] = powmod(h, src[i] - 2, src[i]);
    for (uint32_t t = 0; t < T; ++t) {
      u64 hm = 1;
      for (uint32_t k = 0; k < S; ++k)
        if (k != i) hm = mulmod(hm, src[k] % dst[t], dst[t]);
      hat_mod[(u64)i * T + t] = hm;
    }
  }
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < (int64_t)n; ++j) {
    u64 y[64];
    for (uint32_t i = 0; i < S; ++i) y[i] = mulmod(x[(u64)i * n + j], hat_inv[i], src[i]);
    for (uint32_t t = 0; t < T; ++t) {
      u128 acc = 0;
      for (uint32_t i = 0; i < S; ++i) acc += (u128)y[i] * hat_mod[(u64)i * T + t] % dst[t];
      out[(u64)t * n + j] = (u64)(acc % dst[t]);
    }
  }
  free(hat_inv);
  free(hat_mod);
}

/* ---------------------------------------------------------------- hybrid key-switch
 * d2: [L][N] NTT form over Q; evk_b, evk_a: [dnum][L+K][N] NTT form over Q u P;
 * ks0, ks1: [L][N] NTT form over Q.  Digits are alpha = ceil(L/dnum) consecutive limbs. */
void oracle_keyswitch(u64* ks0, u64* ks1, const u64* d2, const u64* evk_b, const u64* evk_a,
                      uint32_t log_n, const u64* qs, uint32_t L, const u64* ps, uint32_t K,
                      uint32_t dnum) {
  const u64 n = 1ull << log_n;
  const uint32_t LK = L + K, alpha = (L + dnum - 1) / dnum;
  u64* mods = malloc(LK * 8);
  memcpy(mods, qs, L * 8);
  memcpy(mods + L, ps, K * 8);
  prepare(log_n, mods, LK);
  u64* c = malloc(L * n * 8);
  memcpy(c, d2, L * n * 8);
  oracle_ntt_inv(c, 1, log_n, qs, L);
  u64* acc0 = calloc(LK * n, 8);
  u64* acc1 = calloc(LK * n, 8);
  u64* ext = malloc(LK * n * 8);
  u64* tmp = malloc(LK * n * 8);
  u64* dstm = malloc(LK * 8);
  for (uint32_t j = 0; j < dnum; ++j) {
    const uint32_t lo = j * alpha, hi = lo + alpha < L ? lo + alpha : L;
    if (lo >= L) break;
    uint32_t T = 0;
    for (uint32_t i = 0; i < LK; ++i)
      if (i < lo || i >= hi) dstm[T++] = mods[i];
    oracle_baseconv(tmp, c + (u64)lo * n, n, qs + lo, hi - lo, dstm, T);
    for (uint32_t i = 0, k = 0; i < LK; ++i) {
      const u64* src = (i >= lo && i < hi) ? c + (u64)i * n : tmp + (u64)(k++) * n;
      memcpy(ext + (u64)i * n, src, n * 8);
    }
    oracle_ntt_fwd(ext, 1, log_n, mods, LK);
    const u64* eb = evk_b + (u64)j * LK * n;
    const u64* ea = evk_a + (u64)j * LK * n;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)LK; ++i) {
      const u64 q = mods[i];
      for (u64 k = 0; k < n; ++k) {
        const u64 idx = (u64)i * n + k;
        acc0[idx] = (u64)(((u128)ext[idx] * eb[idx] + acc0[idx]) % q);
        acc1[idx] = (u64)(((u128)ext[idx] * ea[idx] + acc1[idx]) % q);
      }
    }
  }
  /* ModDown both accumulators */
  u64 pinv[64];
  for (uint32_t i = 0; i < L; ++i) {
    u64 pm = 1;
    for (uint32_t k = 0; k < K; ++k) pm = mulmod(pm, ps[k] % qs[i], qs[i]);
    pinv[i] = powmod(pm, qs[i] - 2, qs[i]);
  }
  for (int which = 0; which < 2; ++which) {
    u64* acc = which ? acc1 : acc0;
    u64* out = which ? ks1 : ks0;
    u64* xp = malloc(K * n * 8);
    memcpy(xp, acc + (u64)L * n, K * n * 8);
    oracle_ntt_inv(xp, 1, log_n, ps, K);
    oracle_baseconv(tmp, xp, n, ps, K, qs, L);
    oracle_ntt_fwd(tmp, 1, log_n, qs, L);
    for (uint32_t i = 0; i < L; ++i) {
      const u64 q = qs[i];
      for (u64 k = 0; k < n; ++k) {
        const u64 idx = (u64)i * n + k;
        const u64 x = acc[idx], y = tmp[idx];
        out[idx] = mulmod(x >= y ? x - y : x + q - y, pinv[i], q);
      }
    }
    free(xp);
  }
  free(mods); free(c); free(acc0); free(acc1); free(ext); free(tmp); free(dstm);
}

/* ---------------------------------------------------------------- rotation sum, double hoisting
 * Restates oracle/pyoracle.py rotate_sum_hoisted (gpu-fhe_amd/csrc/galois.hip
 * launch_rotate_sum_hoisted): out = sum_r pt_r rot_{gal_r}(ct) with one ModUp of c1 and one
 * ModDown per accumulator.  ct, out: [2][L][N] NTT form over Q; keys_b, keys_a:
 * [count][dnum][L+K][N] (ignored where gal_r == 1, the unrotated term); pts: [count][L+K][N]
 * NTT form over Q u P. */
static u64 oracle_gather_src(u64 j, u64 k, uint32_t log_n) {
  const u64 n = 1ull << log_n;
  const u64 e = (2 * (u64)bitrev((uint32_t)j, log_n) + 1) * k % (2 * n);
  return bitrev((uint32_t)((e - 1) / 2), log_n);
}

void oracle_rotate_sum_hoisted(u64* out, const u64* ct, const uint32_t* gal, uint32_t count,
                               const u64* keys_b, const u64* keys_a, const u64* pts,
                               uint32_t log_n, const u64* qs, uint32_t L, const u64* ps,
                               uint32_t K, uint32_t dnum) {
  const u64 n = 1ull << log_n;
  const uint32_t LK = L + K, alpha = (L + dnum - 1) / dnum;
  const u64 ln = (u64)L * n, lkn = (u64)LK * n;
  const u64* c0 = ct;
  const u64* c1 = ct + ln;
  u64* mods = malloc(LK * 8);
  memcpy(mods, qs, L * 8);
  memcpy(mods + L, ps, K * 8);
  prepare(log_n, mods, LK);
  /* ModUp of c1: every digit extended to Q u P, NTT form (own rows: c1 itself) */
  u64* ext = malloc((u64)dnum * lkn * 8);
  u64* c = malloc(ln * 8);
  u64* tmp = malloc(lkn * 8);
  u64* dstm = malloc(LK * 8);
  memcpy(c, c1, ln * 8);
  oracle_ntt_inv(c, 1, log_n, qs, L);
  uint32_t nd = 0;
  for (uint32_t j = 0; j < dnum; ++j) {
    const uint32_t lo = j * alpha, hi = lo + alpha < L ? lo + alpha : L;
    if (lo >= L) break;
    ++nd;
    uint32_t T = 0;
    for (uint32_t i = 0; i < LK; ++i)
      if (i < lo || i >= hi) dstm[T++] = mods[i];
    oracle_baseconv(tmp, c + (u64)lo * n, n, qs + lo, hi - lo, dstm, T);
    u64* e = ext + (u64)j * lkn;
    for (uint32_t i = 0, k = 0; i < LK; ++i) {
      const u64* src = (i >= lo && i < hi) ? c + (u64)i * n : tmp + (u64)(k++) * n;
      memcpy(e + (u64)i * n, src, n * 8);
    }
    oracle_ntt_fwd(e, 1, log_n, mods, LK);
  }
  u64* a0 = calloc(lkn, 8);
  u64* a1 = calloc(lkn, 8);
  u64* s0 = calloc(ln, 8);
  u64* idx = malloc(n * 8);
  u64 pmod[64];
  for (uint32_t i = 0; i < L; ++i) {
    u64 pm = 1;
    for (uint32_t k = 0; k < K; ++k) pm = mulmod(pm, ps[k] % qs[i], qs[i]);
    pmod[i] = pm;
  }
  for (uint32_t r = 0; r < count; ++r) {
    const u64* pt = pts + (u64)r * lkn;
    if (gal[r] == 1) {
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < (int64_t)L; ++i) {
        const u64 q = qs[i];
        for (u64 k = 0; k < n; ++k) {
          const u64 x = (u64)i * n + k;
          s0[x] = (u64)(((u128)pt[x] * c0[x] + s0[x]) % q);
          a1[x] = (u64)(((u128)pt[x] * mulmod(pmod[i], c1[x], q) + a1[x]) % q);
        }
      }
      continue;
    }
    for (u64 k = 0; k < n; ++k) idx[k] = oracle_gather_src(k, gal[r], log_n);
    const u64* kb = keys_b + (u64)r * dnum * lkn;
    const u64* ka = keys_a + (u64)r * dnum * lkn;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)LK; ++i) {
      const u64 q = mods[i];
      for (u64 k = 0; k < n; ++k) {
        const u64 x = (u64)i * n + k, xs = (u64)i * n + idx[k];
        u64 t0 = 0, t1 = 0;
        for (uint32_t j = 0; j < nd; ++j) {
          const u64 v = ext[(u64)j * lkn + xs];
          t0 = (u64)(((u128)v * kb[(u64)j * lkn + x] + t0) % q);
          t1 = (u64)(((u128)v * ka[(u64)j * lkn + x] + t1) % q);
        }
        a0[x] = (u64)(((u128)pt[x] * t0 + a0[x]) % q);
        a1[x] = (u64)(((u128)pt[x] * t1 + a1[x]) % q);
        if (i < (int64_t)L) s0[x] = (u64)(((u128)pt[x] * c0[xs] + s0[x]) % q);
      }
    }
  }
  /* one ModDown per accumulator; out0 = s0 + ModDown(a0), out1 = ModDown(a1) */
  u64 pinv[64];
  for (uint32_t i = 0; i < L; ++i) pinv[i] = powmod(pmod[i], qs[i] - 2, qs[i]);
  u64* xp = malloc((u64)K * n * 8);
  for (int which = 0; which < 2; ++which) {
    const u64* acc = which ? a1 : a0;
    u64* o = out + (u64)which * ln;
    memcpy(xp, acc + ln, (u64)K * n * 8);
    oracle_ntt_inv(xp, 1, log_n, ps, K);
    oracle_baseconv(tmp, xp, n, ps, K, qs, L);
    oracle_ntt_fwd(tmp, 1, log_n, qs, L);
    for (uint32_t i = 0; i < L; ++i) {
      const u64 q = qs[i];
      for (u64 k = 0; k < n; ++k) {
        const u64 x = (u64)i * n + k, y = tmp[x], v = acc[x];
        u64 m = mulmod(v >= y ? v - y : v + q - y, pinv[i], q);
        if (!which) m = (u64)(((u128)m + s0[x]) % q);
        o[x] = m;
      }
    }
  }
  free(xp); free(idx); free(a0); free(a1); free(s0);
  free(mods); free(c); free(ext); free(tmp); free(dstm);
}
