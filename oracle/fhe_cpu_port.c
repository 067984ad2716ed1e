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
static const ptab_t* ptab(u64 q, uint32_t log_n) {
  for (int i = 0; i < g_nptab; ++i)
    if (g_ptab[i].q == q && g_ptab[i].log_n == log_n) return &g_ptab[i];
  if (g_nptab == MAX_PTAB) {
    for (int i = 0; i < g_nptab; ++i) {
      free(g_ptab[i].w); free(g_ptab[i].ws); free(g_ptab[i].wi); free(g_ptab[i].wis);
    }
    g_nptab = 0;
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
