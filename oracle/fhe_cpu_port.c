/* Tuned CPU port of the hot path (TEST / MEASUREMENT INFRASTRUCTURE ONLY): bench.py's
 * `cpu_baseline` ("kind": "port").  The exact checker stays oracle/fhe_oracle.c; this file is the
 * fair host baseline the GPU numbers are reported beside -- the same algorithms written the way a
 * tuned CPU library would:
 *   - twiddle tables with Shoup companions built once per (q, log_n) and cached;
 *   - Harvey lazy butterflies: forward values in [0, 4q), inverse in [0, 2q), one Shoup product
 *     (a 64x64 -> 128 multiply for the quotient, two 64-bit low products) per butterfly, no `%`;
 *   - the HomMult tensor by Montgomery REDC (R = 2^64) with R folded into the inverse NTT's N^-1,
 *     so no 128-bit division anywhere on the hot path;
 *   - no allocation per (ciphertext, limb): each OpenMP thread reuses one scratch buffer.
 * Outputs are canonical residues, bit-identical to the oracle (tests/test_oracle.py checks).
 * Spec: SURVEY.md §8a' (forward natural -> bit-reversed, psi^brv twiddles; inverse exact).
 * Nothing in gpu-fhe_amd/ links or calls it. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;

u64 oracle_psi(u64 q, uint32_t log_n); /* fhe_oracle.c (linked into the same library) */

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
static uint32_t bitrev(uint32_t x, uint32_t bits) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < bits; ++i) { r = (r << 1) | (x & 1); x >>= 1; }
  return r;
}

typedef struct {
  u64 q, qi; /* qi = q^-1 mod 2^64 */
  uint32_t log_n;
  u64 *w, *ws, *wi, *wis; /* psi^brv(k), psi^-brv(k) and Shoup companions */
  u64 ninv, ninvs;        /* N^-1 */
  u64 ninvr, ninvrs;      /* N^-1 R (the Montgomery tensor's R^-1 undone) */
} ptab_t;

#define MAX_PTAB 256
static ptab_t g_ptab[MAX_PTAB];
static int g_nptab = 0;

static inline u64 shoup_c(u64 w, u64 q) { return (u64)(((u128)w << 64) / q); }

/* Tables are built serially (prepare) before any parallel region reads them. */
/* Only prepare() builds or recycles entries (fhe_oracle.c get_tables: recycling here could free a
 * table the same call's prepare() had just built). */
static const ptab_t* find_ptab(u64 q, uint32_t log_n) {
  for (int i = 0; i < g_nptab; ++i)
    if (g_ptab[i].q == q && g_ptab[i].log_n == log_n) return &g_ptab[i];
  return NULL;
}

static const ptab_t* ptab(u64 q, uint32_t log_n) {
  const ptab_t* found = find_ptab(q, log_n);
  if (found) return found;
  if (g_nptab == MAX_PTAB) {
    fprintf(stderr, "fhe_cpu_port: table cache full outside prepare()\n");
    abort();
  }
  ptab_t* t = &g_ptab[g_nptab++];
  const u64 n = 1ull << log_n;
  t->q = q;
  t->log_n = log_n;
  u64 inv = q;
  for (int i = 0; i < 5; ++i) inv *= 2 - q * inv;
  t->qi = inv;
  t->w = malloc(n * 8); t->ws = malloc(n * 8); t->wi = malloc(n * 8); t->wis = malloc(n * 8);
  const u64 psi = oracle_psi(q, log_n), psi_inv = powmod(psi, q - 2, q);
  u64 p = 1, pi = 1;
  u64* pw = malloc(n * 8);
  u64* pwi = malloc(n * 8);
  for (u64 k = 0; k < n; ++k) { pw[k] = p; pwi[k] = pi; p = mulmod(p, psi, q); pi = mulmod(pi, psi_inv, q); }
  for (u64 k = 0; k < n; ++k) {
    const uint32_t b = bitrev((uint32_t)k, log_n);
    t->w[k] = pw[b]; t->ws[k] = shoup_c(pw[b], q);
    t->wi[k] = pwi[b]; t->wis[k] = shoup_c(pwi[b], q);
  }
  free(pw); free(pwi);
  t->ninv = powmod(n % q, q - 2, q);
  t->ninvs = shoup_c(t->ninv, q);
  t->ninvr = mulmod(t->ninv, (u64)(((u128)1 << 64) % q), q);
  t->ninvrs = shoup_c(t->ninvr, q);
  return t;
}

/* y w mod q up to one q: [0, 2q) for any 64-bit y */
static inline u64 shoup(u64 y, u64 w, u64 ws, u64 q) {
  const u64 h = (u64)(((u128)y * ws) >> 64);
  return y * w - h * q;
}

/* Forward, natural -> bit-reversed; lazy [0, 4q) between stages, canonical out. */
static void port_fwd_1(u64* a, const ptab_t* t) {
  const u64 q = t->q, q2 = 2 * q, n = 1ull << t->log_n;
  u64 tt = n;
  for (u64 m = 1; m < n; m <<= 1) {
    tt >>= 1;
    for (u64 i = 0; i < m; ++i) {
      const u64 w = t->w[m + i], ws = t->ws[m + i];
      u64* x = a + 2 * i * tt;
      u64* y = x + tt;
      for (u64 j = 0; j < tt; ++j) {
        u64 u = x[j];
        u = u >= q2 ? u - q2 : u;
        const u64 v = shoup(y[j], w, ws, q);
        x[j] = u + v;
        y[j] = u - v + q2;
      }
    }
  }
  for (u64 j = 0; j < n; ++j) {
    u64 v = a[j];
    v = v >= q2 ? v - q2 : v;
    a[j] = v >= q ? v - q : v;
  }
}

/* Inverse (Gentleman-Sande), bit-reversed -> natural; lazy [0, 2q); the last stage folds the
 * given N^-1 constant (ni, nis) into both outputs; canonical out. */
static void port_inv_1(u64* a, const ptab_t* t, u64 ni, u64 nis) {
  const u64 q = t->q, q2 = 2 * q, n = 1ull << t->log_n;
  u64 tt = 1;
  for (u64 m = n; m > 2; m >>= 1) {
    const u64 h = m >> 1;
    for (u64 i = 0; i < h; ++i) {
      const u64 w = t->wi[h + i], ws = t->wis[h + i];
      u64* x = a + 2 * i * tt;
      u64* y = x + tt;
      for (u64 j = 0; j < tt; ++j) {
        const u64 u = x[j], v = y[j];
        const u64 s = u + v;
        x[j] = s >= q2 ? s - q2 : s;
        y[j] = shoup(u - v + q2, w, ws, q);
      }
    }
    tt <<= 1;
  }
  /* last stage: w = psi^-brv(1) times N^-1 on the difference, N^-1 on the sum */
  const u64 w1 = mulmod(t->wi[1], ni, q), w1s = shoup_c(w1, q);
  u64* x = a;
  u64* y = a + tt;
  for (u64 j = 0; j < tt; ++j) {
    const u64 u = x[j], v = y[j];
    u64 s = shoup(u + v, ni, nis, q);
    u64 d = shoup(u - v + q2, w1, w1s, q);
    x[j] = s >= q ? s - q : s;
    y[j] = d >= q ? d - q : d;
  }
}

/* Montgomery REDC of a 128-bit t < q 2^64: t 2^-64 mod q in [0, 2q) (subtractive form). */
static inline u64 redc(u128 t, u64 q, u64 qi) {
  const u64 m = (u64)t * qi;
  return (u64)(t >> 64) + q - (u64)(((u128)m * q) >> 64);
}

static void prepare(uint32_t log_n, const u64* moduli, uint32_t L) {
  uint32_t missing = 0;
  for (uint32_t l = 0; l < L; ++l) missing += find_ptab(moduli[l], log_n) == NULL;
  if (g_nptab + missing > MAX_PTAB) { /* recycle everything before building this call's tables */
    for (int i = 0; i < g_nptab; ++i) {
      free(g_ptab[i].w); free(g_ptab[i].ws); free(g_ptab[i].wi); free(g_ptab[i].wis);
    }
    g_nptab = 0;
  }
  for (uint32_t l = 0; l < L; ++l) ptab(moduli[l], log_n);
}

/* data [polys][L][N] in place. */
void port_ntt_fwd(u64* data, uint64_t polys, uint32_t log_n, const u64* moduli, uint32_t L) {
  prepare(log_n, moduli, L);
  const u64 n = 1ull << log_n;
#pragma omp parallel for schedule(dynamic)
  for (int64_t pl = 0; pl < (int64_t)(polys * L); ++pl)
    port_fwd_1(data + (u64)pl * n, ptab(moduli[pl % L], log_n));
}

void port_ntt_inv(u64* data, uint64_t polys, uint32_t log_n, const u64* moduli, uint32_t L) {
  prepare(log_n, moduli, L);
  const u64 n = 1ull << log_n;
#pragma omp parallel for schedule(dynamic)
  for (int64_t pl = 0; pl < (int64_t)(polys * L); ++pl) {
    const ptab_t* t = ptab(moduli[pl % L], log_n);
    port_inv_1(data + (u64)pl * n, t, t->ninv, t->ninvs);
  }
}

/* a, b [batch][2][L][N] coefficient form -> d [batch][3][L][N] coefficient form (SURVEY §8a'). */
void port_hommult(u64* d, const u64* a, const u64* b, uint64_t batch, uint32_t log_n,
                  const u64* moduli, uint32_t L) {
  prepare(log_n, moduli, L);
  const u64 n = 1ull << log_n, ln = (u64)L * n;
#pragma omp parallel
  {
    u64* s = malloc(2 * n * 8); /* one scratch pair per thread, reused for every limb */
#pragma omp for schedule(dynamic)
    for (int64_t bl = 0; bl < (int64_t)(batch * L); ++bl) {
      const u64 bi = (u64)bl / L, l = (u64)bl % L;
      const ptab_t* t = ptab(moduli[l], log_n);
      const u64 q = t->q, qi = t->qi;
      u64* D0 = d + bi * 3 * ln + l * n;
      u64* D1 = D0 + ln;
      u64* D2 = D1 + ln;
      u64* A1 = s;
      u64* B1 = s + n;
      memcpy(D0, a + bi * 2 * ln + l * n, n * 8);        /* A0 */
      memcpy(A1, a + bi * 2 * ln + ln + l * n, n * 8);
      memcpy(D2, b + bi * 2 * ln + l * n, n * 8);        /* B0 */
      memcpy(B1, b + bi * 2 * ln + ln + l * n, n * 8);
      port_fwd_1(D0, t); port_fwd_1(A1, t); port_fwd_1(D2, t); port_fwd_1(B1, t);
      for (u64 j = 0; j < n; ++j) {
        const u64 a0 = D0[j], a1 = A1[j], b0 = D2[j], b1 = B1[j];
        u64 r0 = redc((u128)a0 * b0, q, qi);
        u64 r1 = redc((u128)a0 * b1 + (u128)a1 * b0, q, qi);
        u64 r2 = redc((u128)a1 * b1, q, qi);
        D0[j] = r0 >= q ? r0 - q : r0;
        D1[j] = r1 >= q ? r1 - q : r1;
        D2[j] = r2 >= q ? r2 - q : r2;
      }
      port_inv_1(D0, t, t->ninvr, t->ninvrs);
      port_inv_1(D1, t, t->ninvr, t->ninvrs);
      port_inv_1(D2, t, t->ninvr, t->ninvrs);
    }
    free(s);
  }
}

/* ---------------------------------------------------------------- hybrid key-switch (port)
 * The same algorithm as oracle_keyswitch (SURVEY.md §8a'; INTT d2 -> per digit ModUp + NTT ->
 * inner product with the key -> ModDown), written like a tuned CPU library: cached twiddle tables,
 * lazy Harvey NTTs, Shoup products for every constant factor, 128-bit sums reduced once by two
 * Shoup products (no `%`), one scratch row + two 128-bit accumulator rows per OpenMP thread, and
 * the batch's key shared.  d2, ks0, ks1 [batch][L][N] NTT form; evk_b, evk_a [dnum][L+K][N]. */

typedef struct { u64 q, r64, r64s, one_s; } red_t;  /* 2^64 mod q and its / 1's Shoup companions */

static red_t red_make(u64 q) {
  red_t r;
  r.q = q;
  r.r64 = (u64)(((u128)1 << 64) % q);
  r.r64s = shoup_c(r.r64, q);
  r.one_s = shoup_c(1, q);
  return r;
}

/* any 128-bit z mod q (q < 2^62): z_hi (2^64 mod q) + z_lo, each Shoup product in [0, 2q) */
static inline u64 red128(u128 z, const red_t* r) {
  const u64 q = r->q;
  u64 s = shoup((u64)(z >> 64), r->r64, r->r64s, q) + shoup((u64)z, 1, r->one_s, q);
  s = s >= 2 * q ? s - 2 * q : s;
  return s >= q ? s - q : s;
}

/* canonical x c mod q for a constant c with Shoup companion cs */
static inline u64 mulc(u64 x, u64 c, u64 cs, u64 q) {
  const u64 r = shoup(x, c, cs, q);
  return r >= q ? r - q : r;
}

void port_keyswitch(u64* ks0, u64* ks1, const u64* d2, const u64* evk_b, const u64* evk_a,
                    uint64_t batch, uint32_t log_n, const u64* qs, uint32_t L, const u64* ps,
                    uint32_t K, uint32_t dnum) {
  const u64 n = 1ull << log_n;
  if (L == 0 || K == 0 || dnum == 0 || L > 64 || K > 64) return; /* the constant tables below */
  const uint32_t LK = L + K, alpha = (L + dnum - 1) / dnum;
  u64* mods = malloc(LK * 8);
  memcpy(mods, qs, L * 8);
  memcpy(mods + L, ps, K * 8);
  prepare(log_n, mods, LK);
  red_t* red = malloc(LK * sizeof(red_t));
  for (uint32_t i = 0; i < LK; ++i) red[i] = red_make(mods[i]);
  /* ModUp constants: limb l of digit j = l / alpha: (D^_l)^-1 mod q_l, and D^_l mod m_t */
  u64* uinv = malloc(L * 8);
  u64* uinvs = malloc(L * 8);
  u64* uhat = malloc((u64)L * LK * 8);
  for (uint32_t l = 0; l < L; ++l) {
    const uint32_t lo = l / alpha * alpha, hi = lo + alpha < L ? lo + alpha : L;
    u64 h = 1;
    for (uint32_t k = lo; k < hi; ++k)
      if (k != l) h = mulmod(h, qs[k] % qs[l], qs[l]);
    uinv[l] = powmod(h, qs[l] - 2, qs[l]);
    uinvs[l] = shoup_c(uinv[l], qs[l]);
    for (uint32_t t = 0; t < LK; ++t) {
      u64 hm = 1;
      for (uint32_t k = lo; k < hi; ++k)
        if (k != l) hm = mulmod(hm, qs[k] % mods[t], mods[t]);
      uhat[(u64)l * LK + t] = hm;
    }
  }
  /* ModDown constants: (P^_k)^-1 mod p_k, P^_k mod q_i, P^-1 mod q_i */
  u64 dinv[64], dinvs[64], pinv[64], pinvs[64];
  u64* dhat = malloc((u64)K * L * 8);
  for (uint32_t k = 0; k < K; ++k) {
    u64 h = 1;
    for (uint32_t m = 0; m < K; ++m)
      if (m != k) h = mulmod(h, ps[m] % ps[k], ps[k]);
    dinv[k] = powmod(h, ps[k] - 2, ps[k]);
    dinvs[k] = shoup_c(dinv[k], ps[k]);
    for (uint32_t i = 0; i < L; ++i) {
      u64 hm = 1;
      for (uint32_t m = 0; m < K; ++m)
        if (m != k) hm = mulmod(hm, ps[m] % qs[i], qs[i]);
      dhat[(u64)k * L + i] = hm;
    }
  }
  for (uint32_t i = 0; i < L; ++i) {
    u64 pm = 1;
    for (uint32_t k = 0; k < K; ++k) pm = mulmod(pm, ps[k] % qs[i], qs[i]);
    pinv[i] = powmod(pm, qs[i] - 2, qs[i]);
    pinvs[i] = shoup_c(pinv[i], qs[i]);
  }
  u64* y = malloc((u64)L * n * 8);          /* ModUp sources [L][N] */
  u64* acc = malloc((u64)2 * LK * n * 8);  /* [2][LK][N] */
  u64* yp = malloc((u64)2 * K * n * 8);    /* ModDown sources [2][K][N] */
  for (u64 b = 0; b < batch; ++b) {
    const u64* d2b = d2 + b * L * n;
#pragma omp parallel for schedule(dynamic)
    for (int64_t l = 0; l < (int64_t)L; ++l) {
      const ptab_t* t = ptab(qs[l], log_n);
      u64* yl = y + (u64)l * n;
      memcpy(yl, d2b + (u64)l * n, n * 8);
      port_inv_1(yl, t, t->ninv, t->ninvs);
      for (u64 k = 0; k < n; ++k) yl[k] = mulc(yl[k], uinv[l], uinvs[l], qs[l]);
    }
#pragma omp parallel
    {
      u64* row = malloc(n * 8);
      u128* s0 = malloc(n * sizeof(u128));
      u128* s1 = malloc(n * sizeof(u128));
#pragma omp for schedule(dynamic)
      for (int64_t i = 0; i < (int64_t)LK; ++i) {
        const ptab_t* t = ptab(mods[i], log_n);
        memset(s0, 0, n * sizeof(u128));
        memset(s1, 0, n * sizeof(u128));
        for (uint32_t j = 0; j < dnum; ++j) {
          const uint32_t lo = j * alpha, hi = lo + alpha < L ? lo + alpha : L;
          if (lo >= L) break;
          const u64* x;
          if (i >= (int64_t)lo && i < (int64_t)hi) {
            x = d2b + (u64)i * n; /* the digit's own limb: d2 itself (NTT form) */
          } else {
            for (u64 k = 0; k < n; ++k) {
              u128 z = 0;
              for (uint32_t l = lo; l < hi; ++l) z += (u128)y[(u64)l * n + k] * uhat[(u64)l * LK + i];
              row[k] = red128(z, &red[i]);
            }
            port_fwd_1(row, t);
            x = row;
          }
          const u64* eb = evk_b + ((u64)j * LK + i) * n;
          const u64* ea = evk_a + ((u64)j * LK + i) * n;
          for (u64 k = 0; k < n; ++k) {
            s0[k] += (u128)x[k] * eb[k];
            s1[k] += (u128)x[k] * ea[k];
          }
        }
        u64* a0 = acc + (u64)i * n;
        u64* a1 = acc + ((u64)LK + i) * n;
        for (u64 k = 0; k < n; ++k) {
          a0[k] = red128(s0[k], &red[i]);
          a1[k] = red128(s1[k], &red[i]);
        }
      }
      free(row); free(s0); free(s1);
    }
    /* ModDown both accumulators: INTT + scale of the P rows, then per Q-limb convert, NTT, finish */
#pragma omp parallel for schedule(dynamic)
    for (int64_t hk = 0; hk < (int64_t)(2 * K); ++hk) {
      const uint32_t h = (uint32_t)hk / K, k = (uint32_t)hk % K;
      const ptab_t* t = ptab(ps[k], log_n);
      u64* x = yp + (u64)hk * n;
      memcpy(x, acc + ((u64)h * LK + L + k) * n, n * 8);
      port_inv_1(x, t, t->ninv, t->ninvs);
      for (u64 m = 0; m < n; ++m) x[m] = mulc(x[m], dinv[k], dinvs[k], ps[k]);
    }
#pragma omp parallel
    {
      u64* row = malloc(n * 8);
#pragma omp for schedule(dynamic)
      for (int64_t hi_ = 0; hi_ < (int64_t)(2 * L); ++hi_) {
        const uint32_t h = (uint32_t)hi_ / L, i = (uint32_t)hi_ % L;
        const ptab_t* t = ptab(qs[i], log_n);
        const u64 q = qs[i];
        for (u64 m = 0; m < n; ++m) {
          u128 z = 0;
          for (uint32_t k = 0; k < K; ++k) z += (u128)yp[((u64)h * K + k) * n + m] * dhat[(u64)k * L + i];
          row[m] = red128(z, &red[i]);
        }
        port_fwd_1(row, t);
        const u64* a = acc + ((u64)h * LK + i) * n;
        u64* out = (h ? ks1 : ks0) + (b * L + i) * n;
        for (u64 m = 0; m < n; ++m) {
          const u64 x = a[m], v = row[m];
          out[m] = mulc(x >= v ? x - v : x + q - v, pinv[i], pinvs[i], q);
        }
      }
      free(row);
    }
  }
  free(mods); free(red); free(uinv); free(uinvs); free(uhat); free(dhat); free(y); free(acc); free(yp);
}

/* ---------------------------------------------------------------- vec_add / vec_sub / vec_mul
 * The reference's coefficient-wise operators (/root/reference/arithmetic.py:3-13, exact
 * semantics) on canonical residues a, b, out [rows][cols], row r modulo mods[r], the way a tuned
 * CPU library would run them: OpenMP over rows, no `%` -- add / sub by one conditional
 * correction, mul by a 64x64 -> 128 product reduced by red128 (two Shoup products).  Timed as
 * bench.py --workload vec's cpu_baseline; checked against oracle_vec_op by tests/test_oracle.py. */
void port_vec_op(int op, u64* out, const u64* a, const u64* b, uint64_t rows, uint64_t cols,
                 const u64* mods) {
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < (int64_t)rows; ++r) {
    const u64 q = mods[r];
    const u64* x = a + (u64)r * cols;
    const u64* y = b + (u64)r * cols;
    u64* o = out + (u64)r * cols;
    if (op == 0) {
      for (u64 c = 0; c < cols; ++c) {
        const u64 s = x[c] + y[c];
        o[c] = s >= q ? s - q : s;
      }
    } else if (op == 1) {
      for (u64 c = 0; c < cols; ++c) o[c] = x[c] >= y[c] ? x[c] - y[c] : x[c] + q - y[c];
    } else {
      const red_t rd = red_make(q);
      for (u64 c = 0; c < cols; ++c) o[c] = red128((u128)x[c] * y[c], &rd);
    }
  }
}
