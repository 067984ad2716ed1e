// Negacyclic NTT / INTT and the fused ct x ct tensor (HomMult) for gfx950.
//
// Spec (SURVEY.md §8a'; the reference's NTT/iNTT are identities, /root/reference/arithmetic.py:15-19):
//   forward  NTT(a)[k] = sum_i a_i psi^((2 brv(k) + 1) i) mod q   natural in -> bit-reversed out
//   inverse  exact inverse (Gentleman-Sande), bit-reversed in -> natural out, N^-1 folded in.
// Restated bit-exactly by oracle/fhe_oracle.c (ntt_fwd_1 / ntt_inv_1).
//
// Structure ("two-pass", N = R1 x R2 with R1 = 2^floor(logN/2)):
//   column pass: the first log R1 CT stages only couple elements in the same column of the
//                R1 x R2 row-major view; a workgroup owns SUBS whole columns (a tile of R1 rows x
//                SUBS columns), stages it through LDS and runs the stages in registers;
//   row pass:    the last log R2 stages stay inside one contiguous row; a workgroup owns SUBS
//                whole rows.
// Inside a pass, each thread holds E = 16 elements of one sub-transform in VGPRs and runs up to
// 4 butterfly stages per LDS round trip (radix-16 rounds); twiddles come from the per-limb
// table psi^brv (16-byte {w, floor(w 2^64 / q)} Shoup pairs, L2-resident).  Butterflies are
// Harvey-lazy: forward values live in [0, 4q), inverse in [0, 2q); the last pass reduces to [0, q).
//
// HomMult (config 3) = 3 launches: column-forward on the 4 input polys -> one fused row kernel
// (row-forward x4, tensor d0 = A0B0, d1 = A0B1 + A1B0, d2 = A1B1 in LDS, row-inverse x3) ->
// column-inverse on the 3 output polys.
#include <type_traits>
#include <utility>

#include "internal.hpp"

namespace fhe {
namespace {

constexpr int kThreads = 256;
constexpr int kElog = 4;  // 16 elements per thread per round

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Round split of a 2^LOGR-point sub-transform into NR rounds of <= kElog stages.
template <int LOGR>
struct Rounds {
  static constexpr int NR = (LOGR + kElog - 1) / kElog;
  static constexpr int kb(int k) { return LOGR / NR + (k < LOGR % NR ? 1 : 0); }
  // bit positions covered by round k: forward rounds go top-down, inverse bottom-up
  static constexpr int lo_fwd(int k) {
    int hi = LOGR;
    for (int i = 0; i < k; ++i) hi -= kb(i);
    return hi - kb(k);
  }
  static constexpr int lo_inv(int k) {
    int lo = 0;
    for (int i = 0; i < k; ++i) lo += kb(i);
    return lo;
  }
};

// Which position bits of the sub-transform a thread's element index j owns in one round:
// bits [LO, LO + KB) are butterflied; the remaining kElog - KB bits of j take the lowest free
// positions; the thread index fills every other bit, ascending.
template <int LOGR, int KB, int LO>
struct Layout {
  static constexpr int E = 1 << kElog;
  static constexpr int ex_pos(int k) {
    int found = 0;
    for (int i = 0; i < LOGR; ++i) {
      if (i >= LO && i < LO + KB) continue;
      if (found == k) return i;
      ++found;
    }
    return -1;
  }
  static constexpr u32 jpos(int j) {
    u32 p = 0;
    for (int b = 0; b < KB; ++b)
      if ((j >> b) & 1) p |= 1u << (LO + b);
    for (int b = 0; b < kElog - KB; ++b)
      if ((j >> (KB + b)) & 1) p |= 1u << ex_pos(b);
    return p;
  }
  static constexpr u32 jmask = jpos(E - 1);
  static __device__ __forceinline__ u32 tpos(u32 t) {
    u32 p = 0;
    int k = 0;
#pragma unroll
    for (int i = 0; i < LOGR; ++i) {
      if ((jmask >> i) & 1) continue;
      p |= ((t >> k) & 1u) << i;
      ++k;
    }
    return p;
  }
};

enum Final : int { kNotFinal = 0, kFinalFwd = 1, kFinalInv = 2 };

// Maps a launch's poly index p to element offsets: p = g * pg + k reads src + g*sgs + k*sps and
// writes dst + g*dgs + k*dps (lets HomMult scatter a/b into its 4-slot workspace).
struct PolyMap {
  u32 pg;
  u64 sgs, sps, dgs, dps;
  __device__ __forceinline__ u64 src(u32 p) const { return (u64)(p / pg) * sgs + (u64)(p % pg) * sps; }
  __device__ __forceinline__ u64 dst(u32 p) const { return (u64)(p / pg) * dgs + (u64)(p % pg) * dps; }
};
static inline PolyMap flat_map(u64 pstride) { return PolyMap{1, pstride, 0, pstride, 0}; }

// One round: load 16 elements of this thread's sub-transform from LDS (element at position p
// lives at s[p * ps]), run the round's stages, store back.  `base` selects the twiddle rows:
// local stage st, group g reads tw[(base << st) + g] (base = 1 for the column pass,
// R1 + row for the row pass).
template <int LOGR, int KB, int LO, bool FWD, int FIN>
__device__ __forceinline__ void ntt_round(u64* __restrict__ s, const int ps, const u32 t,
                                          const ulonglong2* __restrict__ tw, const u32 base,
                                          const u64 q, const ulonglong2 nf0, const ulonglong2 nf1) {
  using Lay = Layout<LOGR, KB, LO>;
  constexpr int E = Lay::E;
  const u32 tp = Lay::tpos(t);
  const u64 q2 = 2 * q;
  u64 x[E];
#pragma unroll
  for (int j = 0; j < E; ++j) x[j] = s[(tp | Lay::jpos(j)) * ps];

  if constexpr (FWD) {
#pragma unroll
    for (int b = KB - 1; b >= 0; --b) {
      const int bitpos = LO + b;
      const int st = LOGR - 1 - bitpos;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        if (j & (1 << b)) continue;
        const int jj = j | (1 << b);
        const u32 g = (tp >> (bitpos + 1)) | (Lay::jpos(j) >> (bitpos + 1));
        const ulonglong2 w = tw[(base << st) + g];
        const u64 u = csub(x[j], q2);
        const u64 v = shoup_lazy(x[jj], w.x, w.y, q);
        x[j] = u + v;
        x[jj] = u - v + q2;
      }
    }
    if constexpr (FIN == kFinalFwd) {
#pragma unroll
      for (int j = 0; j < E; ++j) x[j] = csub(csub(x[j], q2), q);
    }
  } else {
#pragma unroll
    for (int b = 0; b < KB; ++b) {
      const int bitpos = LO + b;
      const int st = LOGR - 1 - bitpos;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        if (j & (1 << b)) continue;
        const int jj = j | (1 << b);
        const u64 u = x[j], v = x[jj];
        const u64 sum = u + v, dif = u - v + q2;
        if (FIN == kFinalInv && st == 0) {
          // last stage of the whole inverse: fold N^-1 (both outputs) and reduce to [0, q)
          x[j] = csub(shoup_lazy(sum, nf0.x, nf0.y, q), q);
          x[jj] = csub(shoup_lazy(dif, nf1.x, nf1.y, q), q);
        } else {
          const u32 g = (tp >> (bitpos + 1)) | (Lay::jpos(j) >> (bitpos + 1));
          const ulonglong2 w = tw[(base << st) + g];
          x[j] = csub(sum, q2);
          x[jj] = shoup_lazy(dif, w.x, w.y, q);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < E; ++j) s[(tp | Lay::jpos(j)) * ps] = x[j];
}

// All rounds of a 2^LOGR-point sub-transform held in LDS. Caller syncs before and after.
template <int LOGR, bool FWD, int FIN>
__device__ __forceinline__ void ntt_sub(u64* s, int ps, u32 t, bool active,
                                        const ulonglong2* __restrict__ tw, u32 base, u64 q,
                                        ulonglong2 nf0, ulonglong2 nf1) {
  using Rd = Rounds<LOGR>;
  static_for<0, Rd::NR>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int KB = Rd::kb(k);
    constexpr int LO = FWD ? Rd::lo_fwd(k) : Rd::lo_inv(k);
    constexpr int F = (k == Rd::NR - 1) ? FIN : kNotFinal;
    if (k > 0) __syncthreads();
    if (active) ntt_round<LOGR, KB, LO, FWD, F>(s, ps, t, tw, base, q, nf0, nf1);
  });
}

template <int LOGN>
struct Geo {
  static constexpr int N1 = LOGN / 2, N2 = LOGN - N1;
  static constexpr int R1 = 1 << N1, R2 = 1 << N2;  // R1 rows x R2 columns
  // column pass: SUBS_C columns per workgroup
  static constexpr int TPS_C = R1 >> kElog;
  static constexpr int SUBS_C = (kThreads / TPS_C) < R2 ? (kThreads / TPS_C) : R2;
  static constexpr int THR_C = SUBS_C * TPS_C;
  static constexpr int PAD_C = 1;
  static constexpr int LDS_C = R1 * (SUBS_C + PAD_C);
  static constexpr int TILES_C = R2 / SUBS_C;
  // row pass: SUBS_R rows per workgroup
  static constexpr int TPS_R = R2 >> kElog;
  static constexpr int SUBS_R = (kThreads / TPS_R) < R1 ? (kThreads / TPS_R) : R1;
  static constexpr int THR_R = SUBS_R * TPS_R;
  static constexpr int PAD_R = 1;
  static constexpr int LDS_R = SUBS_R * (R2 + PAD_R);
  static constexpr int TILES_R = R1 / SUBS_R;
  static_assert(N1 >= kElog - 1 && N2 >= kElog, "log N too small for this kernel family");
};

// Column pass. src/dst: [polys][nlimbs][N] with poly stride pstride; grid = polys*nlimbs*TILES_C.
template <int LOGN, bool FWD>
__global__ __launch_bounds__(kThreads) void k_ntt_col(const u64* __restrict__ src,
                                                      u64* __restrict__ dst, u32 nlimbs,
                                                      u32 limb0, PolyMap pm,
                                                      const ulonglong2* __restrict__ tw_all,
                                                      const ulonglong2* __restrict__ nfold,
                                                      const ModParams* __restrict__ mods) {
  using G = Geo<LOGN>;
  constexpr u64 N = 1ull << LOGN;
  __shared__ u64 lds[G::LDS_C];
  const u32 tile = blockIdx.x % G::TILES_C;
  const u32 pl = blockIdx.x / G::TILES_C;
  const u32 l = pl % nlimbs, p = pl / nlimbs;
  const u32 limb = limb0 + l;
  const u64 loc = (u64)l * N + (u64)tile * G::SUBS_C;
  const u64* sp = src + pm.src(p) + loc;
  u64* dp = dst + pm.dst(p) + loc;
  const u64 q = mods[limb].q;
  const ulonglong2* tw = tw_all + (u64)limb * N;
  const u32 tid = threadIdx.x;

  for (u32 e = tid; e < (u32)(G::R1 * G::SUBS_C); e += G::THR_C) {
    const u32 row = e / G::SUBS_C, col = e % G::SUBS_C;
    lds[row * (G::SUBS_C + G::PAD_C) + col] = sp[(u64)row * G::R2 + col];
  }
  __syncthreads();
  const u32 sub = tid % G::SUBS_C, t = tid / G::SUBS_C;
  ulonglong2 nf0 = {0, 0}, nf1 = {0, 0};
  if (!FWD) {
    nf0 = nfold[2 * limb];
    nf1 = nfold[2 * limb + 1];
  }
  ntt_sub<G::N1, FWD, FWD ? kNotFinal : kFinalInv>(lds + sub, G::SUBS_C + G::PAD_C, t, true, tw,
                                                   1u, q, nf0, nf1);
  __syncthreads();
  for (u32 e = tid; e < (u32)(G::R1 * G::SUBS_C); e += G::THR_C) {
    const u32 row = e / G::SUBS_C, col = e % G::SUBS_C;
    dp[(u64)row * G::R2 + col] = lds[row * (G::SUBS_C + G::PAD_C) + col];
  }
}

// Row pass. grid = polys*nlimbs*TILES_R.
template <int LOGN, bool FWD>
__global__ __launch_bounds__(kThreads) void k_ntt_row(const u64* __restrict__ src,
                                                      u64* __restrict__ dst, u32 nlimbs,
                                                      u32 limb0, PolyMap pm,
                                                      const ulonglong2* __restrict__ tw_all,
                                                      const ModParams* __restrict__ mods) {
  using G = Geo<LOGN>;
  constexpr u64 N = 1ull << LOGN;
  __shared__ u64 lds[G::LDS_R];
  const u32 tile = blockIdx.x % G::TILES_R;
  const u32 pl = blockIdx.x / G::TILES_R;
  const u32 l = pl % nlimbs, p = pl / nlimbs;
  const u32 limb = limb0 + l;
  const u64 loc = (u64)l * N + (u64)tile * G::SUBS_R * G::R2;
  const u64* sp = src + pm.src(p) + loc;
  u64* dp = dst + pm.dst(p) + loc;
  const u64 q = mods[limb].q;
  const ulonglong2* tw = tw_all + (u64)limb * N;
  const u32 tid = threadIdx.x;

  for (u32 e = tid; e < (u32)(G::SUBS_R * G::R2); e += G::THR_R)
    lds[(e / G::R2) * (G::R2 + G::PAD_R) + e % G::R2] = sp[e];
  __syncthreads();
  const u32 sub = tid % G::SUBS_R, t = tid / G::SUBS_R;
  const u32 row = tile * G::SUBS_R + sub;
  ntt_sub<G::N2, FWD, FWD ? kFinalFwd : kNotFinal>(lds + sub * (G::R2 + G::PAD_R), 1, t, true,
                                                   tw, (u32)G::R1 + row, q, {0, 0}, {0, 0});
  __syncthreads();
  for (u32 e = tid; e < (u32)(G::SUBS_R * G::R2); e += G::THR_R)
    dp[e] = lds[(e / G::R2) * (G::R2 + G::PAD_R) + e % G::R2];
}

// Fused HomMult row kernel: rows of the 4 column-transformed inputs (layout [batch][4][nlimbs][N]
// in `x`: A0, A1, B0, B1) -> row-forward, tensor, row-inverse -> d [batch][3][nlimbs][N].
template <int LOGN>
struct HmGeo {
  using G = Geo<LOGN>;
  static constexpr int TPS = G::TPS_R;
  static constexpr int ROWS = (kThreads / 4 / TPS) < 1 ? 1 : (kThreads / 4 / TPS);
  static constexpr int THR = 4 * ROWS * TPS;
  static constexpr int STRIDE = G::R2 + 1;
  static constexpr int SLOT = ROWS * STRIDE;
  static constexpr int TILES = G::R1 / ROWS;
};

template <int LOGN>
__global__ __launch_bounds__(kThreads) void k_hommult_row(const u64* __restrict__ x,
                                                          u64* __restrict__ d, u32 nlimbs,
                                                          u32 limb0,
                                                          const ulonglong2* __restrict__ twf,
                                                          const ulonglong2* __restrict__ twi,
                                                          const ModParams* __restrict__ mods) {
  using G = Geo<LOGN>;
  using H = HmGeo<LOGN>;
  constexpr u64 N = 1ull << LOGN;
  __shared__ u64 lds[4 * H::SLOT];
  const u32 tile = blockIdx.x % H::TILES;
  const u32 bl = blockIdx.x / H::TILES;
  const u32 l = bl % nlimbs, b = bl / nlimbs;
  const u32 limb = limb0 + l;
  const ModParams m = mods[limb];
  const u64 q = m.q;
  const u64 limbN = (u64)nlimbs * N;
  const u64 rowoff = (u64)l * N + (u64)tile * H::ROWS * G::R2;
  const u32 tid = threadIdx.x;
  constexpr u32 TILE_ELEMS = H::ROWS * G::R2;

  // load 4 polys
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const u64* src = x + ((u64)b * 4 + k) * limbN + rowoff;
    for (u32 e = tid; e < TILE_ELEMS; e += H::THR)
      lds[k * H::SLOT + (e / G::R2) * H::STRIDE + e % G::R2] = src[e];
  }
  __syncthreads();
  const u32 poly = tid / (H::ROWS * H::TPS);
  const u32 rem = tid % (H::ROWS * H::TPS);
  const u32 sub = rem % H::ROWS, t = rem / H::ROWS;
  const u32 row = tile * H::ROWS + sub;
  u64* my = lds + poly * H::SLOT + sub * H::STRIDE;
  ntt_sub<G::N2, true, kFinalFwd>(my, 1, t, true, twf + (u64)limb * N, (u32)G::R1 + row, q,
                                  {0, 0}, {0, 0});
  __syncthreads();
  // tensor in place: slots 0,1,2 <- d0, d1, d2
  for (u32 e = tid; e < TILE_ELEMS; e += H::THR) {
    const u32 li = (e / G::R2) * H::STRIDE + e % G::R2;
    const u64 a0 = lds[li], a1 = lds[H::SLOT + li];
    const u64 b0 = lds[2 * H::SLOT + li], b1 = lds[3 * H::SLOT + li];
    lds[li] = mulmod_barrett(a0, b0, m);
    lds[H::SLOT + li] = barrett_reduce((u128)a0 * b1 + (u128)a1 * b0, m);
    lds[2 * H::SLOT + li] = mulmod_barrett(a1, b1, m);
  }
  __syncthreads();
  ntt_sub<G::N2, false, kNotFinal>(my, 1, t, poly < 3, twi + (u64)limb * N, (u32)G::R1 + row, q,
                                   {0, 0}, {0, 0});
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    u64* out = d + ((u64)b * 3 + k) * limbN + rowoff;
    for (u32 e = tid; e < TILE_ELEMS; e += H::THR)
      out[e] = lds[k * H::SLOT + (e / G::R2) * H::STRIDE + e % G::R2];
  }
}


template <int LOGN>
int ntt_dispatch(const fhe_ctx* c, bool fwd, const u64* src, u64* dst, u32 polys, u64 pstride,
                 u32 limb0, u32 nlimbs, hipStream_t s) {
  using G = Geo<LOGN>;
  const u64 pl = (u64)polys * nlimbs;
  const PolyMap pm = flat_map(pstride);
  const dim3 gc((u32)(pl * G::TILES_C)), gr((u32)(pl * G::TILES_R));
  if (fwd) {
    k_ntt_col<LOGN, true><<<gc, G::THR_C, 0, s>>>(src, dst, nlimbs, limb0, pm, c->d_tw_fwd,
                                                 c->d_nfold, c->d_mods);
    prof_mark(s, "ntt_col_fwd");
    k_ntt_row<LOGN, true><<<gr, G::THR_R, 0, s>>>(dst, dst, nlimbs, limb0, pm, c->d_tw_fwd,
                                                 c->d_mods);
    prof_mark(s, "ntt_row_fwd");
  } else {
    k_ntt_row<LOGN, false><<<gr, G::THR_R, 0, s>>>(src, dst, nlimbs, limb0, pm, c->d_tw_inv,
                                                  c->d_mods);
    prof_mark(s, "ntt_row_inv");
    k_ntt_col<LOGN, false><<<gc, G::THR_C, 0, s>>>(dst, dst, nlimbs, limb0, pm, c->d_tw_inv,
                                                  c->d_nfold, c->d_mods);
    prof_mark(s, "ntt_col_inv");
  }
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}

template <int LOGN>
int hommult_dispatch(const fhe_ctx* c, u64* d, const u64* a, const u64* b, u32 batch, u32 limb0,
                     u32 nlimbs, u64* x, hipStream_t s) {
  using G = Geo<LOGN>;
  using H = HmGeo<LOGN>;
  constexpr u64 N = 1ull << LOGN;
  const u64 limbN = (u64)nlimbs * N;
  // x: [batch][4][nlimbs][N] workspace; A0, A1 -> slots 0, 1; B0, B1 -> slots 2, 3.
  const PolyMap to_x{2, 2 * limbN, limbN, 4 * limbN, limbN};
  const dim3 gc((u32)((u64)batch * 2 * nlimbs * G::TILES_C));
  k_ntt_col<LOGN, true><<<gc, G::THR_C, 0, s>>>(a, x, nlimbs, limb0, to_x, c->d_tw_fwd,
                                               c->d_nfold, c->d_mods);
  prof_mark(s, "hm_col_fwd_a");
  k_ntt_col<LOGN, true><<<gc, G::THR_C, 0, s>>>(b, x + 2 * limbN, nlimbs, limb0, to_x,
                                               c->d_tw_fwd, c->d_nfold, c->d_mods);
  prof_mark(s, "hm_col_fwd_b");
  const dim3 gh((u32)((u64)batch * nlimbs * H::TILES));
  k_hommult_row<LOGN><<<gh, H::THR, 0, s>>>(x, d, nlimbs, limb0, c->d_tw_fwd, c->d_tw_inv,
                                            c->d_mods);
  prof_mark(s, "hm_row_tensor");
  const dim3 gi((u32)((u64)batch * 3 * nlimbs * G::TILES_C));
  k_ntt_col<LOGN, false><<<gi, G::THR_C, 0, s>>>(d, d, nlimbs, limb0, flat_map(limbN),
                                                c->d_tw_inv, c->d_nfold, c->d_mods);
  prof_mark(s, "hm_col_inv");
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}

}  // namespace

#define FHE_LOGN_CASES(X) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17)

int launch_ntt(const fhe_ctx* c, bool forward, const u64* src, u64* dst, u32 polys, u64 pstride,
               u32 limb0, u32 nlimbs, hipStream_t s) {
  if ((u64)polys * nlimbs == 0) return kOk;
  switch (c->log_n) {
#define X(n) \
  case n:    \
    return ntt_dispatch<n>(c, forward, src, dst, polys, pstride, limb0, nlimbs, s);
    FHE_LOGN_CASES(X)
#undef X
  }
  set_error("unsupported log_n");
  return kUnsupported;
}

size_t hommult_workspace_bytes(const fhe_ctx* c, u32 batch, u32 nlimbs) {
  return (size_t)batch * 4 * nlimbs * c->n * sizeof(u64);
}

int launch_hommult(const fhe_ctx* c, u64* d, const u64* a, const u64* b, u32 batch, u32 limb0,
                   u32 nlimbs, void* ws, hipStream_t s) {
  if ((u64)batch * nlimbs == 0) return kOk;
  u64* x = static_cast<u64*>(ws);
  switch (c->log_n) {
#define X(n) \
  case n:    \
    return hommult_dispatch<n>(c, d, a, b, batch, limb0, nlimbs, x, s);
    FHE_LOGN_CASES(X)
#undef X
  }
  set_error("unsupported log_n");
  return kUnsupported;
}

}  // namespace fhe
