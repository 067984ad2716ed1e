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
// lazy (round_compute): forward values live below H q, inverse in [0, 3q) between stages and
// passes; the last pass reduces to [0, q).
//
// HomMult (config 3) = 3 launches: column-forward of a and b's 4 polys -> one fused row kernel
// (row-forward x4, tensor d0 = A0B0, d1 = A0B1 + A1B0, d2 = A1B1 in LDS, row-inverse x3) ->
// column-inverse on the 3 output polys.  Moduli of 61-63 bits take exact butterflies (H = 2).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "internal.hpp"

namespace fhe {
namespace {

// log2 of the elements a thread holds per round: 16, rounds of up to 4 stages.  (E = 8 standalone
// row passes measured faster until their stores and twiddle loads were made contiguous, then 10 %
// slower; context.cpp lane_major_rows lays the row twiddles out for this E.)
constexpr int kElog = 4;
constexpr int kE = 1 << kElog;
constexpr int kThreads = 4096 / kE;  // 16 sub-transforms of 256 points per workgroup
// Column-pass workgroup size: 16 columns per 256 threads at N = 2^16.  (512 threads, i.e. wider
// tiles, measured -4 % on the N = 2^17 ntt-batch column pass and +9 % on the HomMult column
// inverse; 256 kept everywhere.)
constexpr int kColThreads = kThreads;

// Occupancy the register allocator / scheduler may assume (waves per SIMD): LDS caps these kernels
// at 4 workgroups (16 waves) per CU, so a lower target costs no waves and lets the scheduler spend
// VGPRs on interleaving independent butterflies; anything above 128 VGPRs would cost waves.
#define FHE_KATTR \
  __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 8)))

// Butterfly arithmetic (measured choices; DESIGN.md §3, §8 keep the alternatives' numbers):
//  * Shoup with the 3-product quotient estimate (shoup_q3, products in [0, 3q)) and lazy ranges:
//    forward values below H q (fwd_range), inverse in [0, 3q) (sum mod 3q, (u - v + 3q) w).  Needs
//    8q < 2^64, i.e. q < 2^61; wider moduli take the exact H = 2 form;
//  * the forward CT butterfly folds its X-operand into the product's remainder chain
//    (shoup_q3_add): one 64-bit add fewer per butterfly;
//  * conditional subtractions by sign-mask select (csub_fast);
//  * the forward row passes store their last round in linear order through the LDS (pass_run
//    XOUT: ntt-batch row-forward 20.7 -> 19.0 ms, ModDown finish 255 -> 190 us) and the inverse
//    row pass loads its first round the same way (121.5 -> 118.3 us).

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Round split of a 2^LOGR-point sub-transform into NR rounds of <= 2^EL-point stages; the longer
// rounds come first, or last with SMALL_FIRST (the HomMult's 7-stage forward rows: 3 + 4, so the
// first round's loads and the last round's low bits are whole 16-byte pairs / 16-element runs).
template <int LOGR, int EL = kElog, bool SMALL_FIRST = false>
struct Rounds {
  static constexpr int NR = (LOGR + EL - 1) / EL;
  static constexpr int kb(int k) {
    return LOGR / NR + ((SMALL_FIRST ? NR - 1 - k : k) < LOGR % NR ? 1 : 0);
  }
  // bit positions covered by round k: forward rounds go top-down, inverse bottom-up
  static constexpr int lo_fwd(int k) {
    int hi = LOGR;
    for (int i = 0; i < k; ++i) hi -= kb(i);
    return hi - kb(k);
  }
  // the inverse runs the forward's rounds in mirror order (bottom bits first)
  static constexpr int kb_inv(int k) { return kb(NR - 1 - k); }
  static constexpr int lo_inv(int k) { return lo_fwd(NR - 1 - k); }
};

// Which position bits of the sub-transform a thread's element index j owns in one round:
// bits [LO, LO + KB) are butterflied; the remaining kElog - KB bits of j take the lowest free
// positions; the thread index fills every other bit, ascending.
template <int LOGR, int KB, int LO, int EL = kElog>
struct Layout {
  static constexpr int E = 1 << EL;
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
    for (int b = 0; b < EL - KB; ++b)
      if ((j >> (KB + b)) & 1) p |= 1u << ex_pos(b);
    return p;
  }
  static constexpr u32 jmask = jpos(E - 1);
  // every thread-index bit sits below the butterflied bits: a stage's twiddle group then depends on
  // the element index only (wave-uniform), as in the column passes' top-bit rounds
  static constexpr bool kTpBelow = ((jmask >> LO) + 1) == (1u << (LOGR - LO));
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

// kFinalFwd reduces the last forward stage to [0, q); kFinalFwd2 only to [0, 2q) (the fused
// HomMult tensor: its Montgomery products accept operands below 2q).
// kFinalInvS30: kFinalInv, then each canonical output in Sum30's split form split30(x) (the
// key-switch's INTTs whose outputs only feed k_modup_col's conversions: it reads them pre-split).
enum Final : int { kNotFinal = 0, kFinalFwd = 1, kFinalInv = 2, kFinalFwd2 = 3, kFinalInvS30 = 4 };

// LDS exchange fences.  A row sub-transform's threads all sit in one wavefront, so the row
// kernels only need wavefront-scope ordering of their LDS traffic (DS instructions of one wave
// execute in issue order): no s_barrier, and waves drift apart freely, overlapping one wave's
// global loads with another's butterflies.  The column pass spans waves and uses the block barrier.
enum Sync : int { kBlockSync = 0, kWaveSync = 1 };
template <int S>
__device__ __forceinline__ void lds_sync() {
  if constexpr (S == kBlockSync) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// XCD-aware block -> (limb, rest) split for the row passes.  Their twiddles are per (limb, row):
// 2 MiB of forward + inverse table per limb, so when every XCD sees every limb the 4 MiB L2 of
// an XCD thrashes and the re-reads go out to the Infinity Cache (measured: 1.5x the algorithmic
// read traffic of hm_row_tensor at 8 limbs).  Workgroups are dealt round-robin to the 8 XCDs, so
// tying the limb to blockIdx % 8 keeps each limb's table on one XCD's L2.  Placement only
// affects speed: every (limb, rest) pair is still covered exactly once for any nlimbs.
// With more than 8 limbs an XCD owns nlimbs / 8 of them and walks them one after another (the limb
// changes every `per_limb` = items / nlimbs of its blocks), so only one limb's table is hot in its
// L2 at a time.
__device__ __forceinline__ void xcd_limb_split(u32 b, u32 nlimbs, u32 per_limb, u32& limb,
                                               u32& rest) {
  constexpr u32 kXcd = 8;
  if (nlimbs % kXcd == 0) {
    const u32 hi = b / kXcd;
    limb = b % kXcd + kXcd * (hi / per_limb);
    rest = hi % per_limb;
  } else if (kXcd % nlimbs == 0) {
    const u32 per = kXcd / nlimbs;  // XCDs per limb
    limb = (b % kXcd) % nlimbs;
    rest = (b / kXcd) * per + (b % kXcd) / nlimbs;
  } else {
    limb = b % nlimbs;
    rest = b / nlimbs;
  }
}

// Maps a launch's poly index p to element offsets: p = g * pg + k reads src + g*sgs + k*sps and
// writes dst + g*dgs + k*dps (lets HomMult scatter a/b into its 4-slot workspace).
// With alt > 0, the polys k >= alt of each group read the second source at k - alt instead
// (HomMult's column-forward reads a's two polys and b's two polys of a ciphertext in one launch).
struct PolyMap {
  u32 pg;
  u64 sgs, sps, dgs, dps;
  u32 alt = 0;
  __device__ __forceinline__ u64 src(u32 p) const { return (u64)(p / pg) * sgs + (u64)(p % pg) * sps; }
  __device__ __forceinline__ u64 dst(u32 p) const { return (u64)(p / pg) * dgs + (u64)(p % pg) * dps; }
  __device__ __forceinline__ bool second(u32 p) const { return alt != 0 && p % pg >= alt; }
  __device__ __forceinline__ u64 src2(u32 p) const {
    return (u64)(p / pg) * sgs + (u64)(p % pg - alt) * sps;
  }
};
static inline PolyMap flat_map(u64 pstride) { return PolyMap{1, pstride, 0, pstride, 0, 0}; }

// The distinct twiddles of one round: butterfly (stage b, pair j) uses twiddle group
// g = (tp | jpos(j)) >> (LO + b + 1); slot[b][j] numbers the distinct (b, g - tp part) pairs and
// rep[] keeps one representative j per slot.
template <int LOGR, int KB, int LO, int EL = kElog>
struct TwSlots {
  using Lay = Layout<LOGR, KB, LO, EL>;
  static constexpr int E = 1 << EL;
  struct Tab {
    int ns = 0;
    int slot[EL][E] = {};
    int rep_b[EL * E] = {}, rep_j[EL * E] = {};
  };
  static constexpr Tab make() {
    Tab t{};
    for (int b = 0; b < KB; ++b)
      for (int j = 0; j < E; ++j) {
        if (j & (1 << b)) continue;
        const u32 key = Lay::jpos(j) >> (LO + b + 1);
        int found = -1;
        for (int s = 0; s < t.ns; ++s)
          if (t.rep_b[s] == b && (Lay::jpos(t.rep_j[s]) >> (LO + b + 1)) == key) found = s;
        if (found < 0) {
          found = t.ns++;
          t.rep_b[found] = b;
          t.rep_j[found] = j;
        }
        t.slot[b][j] = found;
      }
    return t;
  }
  static constexpr Tab T = make();
};

// Twiddle load through an explicitly global pointer: the opaque-base asm in pass_run hides the
// address space, and a flat load would also count against lgkmcnt, making every LDS wait of the
// round wait for the twiddles too.
typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ ulonglong2 ld_tw(const ulonglong2* p) {
  const u64x2_t v = *(const __attribute__((address_space(1))) u64x2_t*)p;
  return make_ulonglong2(v.x, v.y);
}

// Conditional subtraction in the butterflies: sign-mask select (csub_fast: one 64-bit add, an
// arithmetic shift and two v_bfi, no VCC) instead of a 64-bit compare, two v_cndmask and a borrow
// chain.  Needs |x - m| < 2^63, which every range here satisfies.
__device__ __forceinline__ u64 csubk(u64 x, u64 m) {
  // -m as an opaque uniform: otherwise x + (0 - m) folds back into a borrow chain (sub_co/subb,
  // two instructions) instead of one v_lshl_add_u64
  u64 nm = 0 - m;
  asm("" : "+s"(nm));
  return csub_fast(x, nm);
}

// Forward lazy ranges, in units of q.  A CT stage maps X-operands below r q to
// outputs below (r' + 3) q, where r' = r unless r + 3 would exceed the headroom H (values must stay
// below H q <= 2^64), in which case X is first reduced (r' = fwd_reduced(H)).  H = 8 (q < 2^61):
// one subtraction of 4q, at every stage once warm.  H = 16 (lz16 contexts: every q < 2^60 and
// within 1/16 below a power of two): the top-bits estimate x - (x >> s) q, s = bitlength(q), which
// takes any x < 16q below 2q at the cost of one subtraction, so a reduction every fifth stage.
constexpr int fwd_reduced(int H) { return H == 16 ? 2 : H / 2; }
constexpr int fwd_stage_out(int r, int H) { return (r + 3 > H ? fwd_reduced(H) : r) + 3; }

// x - floor(x / 2^s) q for x < 16 q, q in [2^s - 2^(s-4), 2^s), 33 <= s <= 60 (fhe_ctx::lz16):
// k = x >> s <= x / q and x - k q < x (2^s - q) / 2^s + q < 2q.  Computed as
// (x mod 2^s) + k c with c = 2^s - q < 2^(s-4) <= 2^56 (nq = -q mod 2^64, so c = nq + 2^s), all in
// the 32-bit halves: k and the masked high word by two 32-bit ops, one v_mad_u64_u32 for k c_lo
// into {lo x, masked hi} and k c_hi (c_hi < 2^24) by v_mad_u32_u24 into the high word.  No sum
// exceeds 2^61.  (x + k nq as a 32 x 64-bit product cost a 64-bit shift, two mads and two
// register-pair moves: 8 issue slots against 5.)  HALVES = false keeps that product form: the
// inverse column passes, which are latency- rather than issue-bound, measured 4 % slower with the
// halves form's dependent mads (HomMult column inverse 0.318 -> 0.331 ms), the issue-bound row
// kernels and forward passes 0.8-1.2 % faster.
template <bool HALVES = true>
__device__ __forceinline__ u64 top_bits(u64 x, u32 s, u64 nq) {
  if constexpr (!HALVES) return x + (u64)(u32)(x >> s) * nq;
  const u64 c = nq + (1ull << s);  // uniform
  const u32 sh = s - 32;
  const u32 hi = (u32)(x >> 32);
  const u32 k = hi >> sh;
  const u32 hm = hi & ((1u << sh) - 1);
  const u64 r = mad_u64_u32(k, (u32)c, ((u64)hm << 32) | (u32)x);
  return ((u64)(__umul24(k, (u32)(c >> 32)) + (u32)(r >> 32)) << 32) | (u32)r;
}
constexpr int fwd_range(int r0, int stages, int H) {
  int r = r0;
  for (int i = 0; i < stages; ++i) r = fwd_stage_out(r, H);
  return r;
}

// Inverse lazy ranges for H = 16 (lz16 contexts: values up to 16q fit, top_bits applies), in
// units of q: the range of element j before local stage k of a GS round whose inputs are below 3q.
// Both elements of a pair (j, j | 1 << b) share it (ranges depend only on the bits already
// processed).  The difference leaves below 3q (Shoup); the sum leaves unreduced, below 2r q, except
// that a pair at r = 12 is first taken below 2q by top_bits.  Per 16-element round: 6 reductions
// in the stages + 8 at the end (every element above 3q back below 2q for the exchange) instead of
// 32 conditional subtractions.
constexpr int gs_red(int r) { return r > 8 ? 2 : r; }
constexpr int gs_in(int j, int k) {
  int r = 3;
  for (int b = 0; b < k; ++b) r = ((j >> b) & 1) ? 3 : 2 * gs_red(r);
  return r;
}

// Runs one round's butterfly stages on the 16 values a thread holds in registers.
// Element j sits at sub-transform position tp | Lay::jpos(j).  `base` selects the twiddle rows:
// local stage st, group g reads tw[(base << st) + g] (base = 1 for the column pass, R1 + row for
// the row pass).
// GATHER = false leaves the twiddle loads to the scheduler, next to their butterflies (better for
// the column pass, whose twiddles are few and shared); true issues them all first (the row passes:
// per-lane twiddles from L2, whose latency then overlaps instead of stalling each stage).
// ROWTAB: the twiddles come from a row table region (base = R1 + row), whose low-bit-round stages
// are stored lane-major.
// PRE0 (forward, k_modup_col): the operands of stage 0's products arrive already multiplied by
// its twiddle (the base conversion folds it into its constants), so stage 0 only adds.
template <int LOGR, int KB, int LO, bool FWD, int FIN, bool GATHER = false, int H = 8,
          int RIN = 8, bool ROWTAB = GATHER, bool CHAIN = GATHER, bool PRE0 = false,
          int EL = kElog>
__device__ __forceinline__ void round_compute(u64 (&x)[1 << EL], const u32 tp,
                                              const ulonglong2* __restrict__ tw, const u32 base,
                                              const u64 q, const ulonglong2 nf0,
                                              const ulonglong2 nf1) {
  using Lay = Layout<LOGR, KB, LO, EL>;
  using TS = TwSlots<LOGR, KB, LO, EL>;
  constexpr int E = Lay::E;
  ulonglong2 tws[GATHER && TS::T.ns > 0 ? TS::T.ns : 1];
  if constexpr (GATHER) {
    static_for<0, TS::T.ns>([&](auto sc) {
      constexpr int sl = decltype(sc)::value;
      constexpr int b = TS::T.rep_b[sl];
      constexpr int bitpos = LO + b;
      constexpr int st = LOGR - 1 - bitpos;
      if constexpr (!((FIN == kFinalInv || FIN == kFinalInvS30) && st == 0)) {  // folds N^-1 instead
        // natural group index: g = t W + sj, W = 2^(kElog - bitpos - 1) (the low-bit round has
        // tp = t << kElog); the row tables store those stages lane-major (host_tables.cpp
        // lane_major_rows), so the load index is sj TPS + t and a wavefront reads contiguous words
        const u32 sj = Lay::jpos(TS::T.rep_j[sl]) >> (bitpos + 1);
        const u32 g = (ROWTAB && LO == 0) ? sj * ((1u << LOGR) / E) + (tp >> EL)
                                          : (tp >> (bitpos + 1)) | sj;
        tws[sl] = ld_tw(tw + (base << st) + g);
      }
    });
    asm volatile("" ::: "memory");
  }
  static_assert(GATHER || !(ROWTAB && LO == 0), "lane-major row twiddles are gathered");
  auto twiddle = [&](int b, int j, int bitpos, int st) {
    if constexpr (GATHER) return tws[TS::T.slot[b][j]];
    // (kTpBelow: tp >> (bitpos + 1) is 0, written out so the address is visibly uniform and the
    // pair can come through the scalar cache into SGPRs)
    const u32 g = (Lay::kTpBelow ? 0u : (tp >> (bitpos + 1))) | (Lay::jpos(j) >> (bitpos + 1));
    return ld_tw(tw + (base << st) + g);
  };
  const u64 q2 = 2 * q, nq = 0 - q;
  // 3q as an opaque uniform: otherwise u + 3q is strength-reduced into a mad per butterfly
  u64 q3 = 3 * q;
  asm("" : "+s"(q3));
  if constexpr (FWD && H == 2) {
    // wide moduli (2^61 <= q < 2^63, ctx->wide): no lazy headroom.  Values stay below 2q:
    // u = x mod q, v = (w x') mod q by the exact-quotient Shoup product (any 64-bit x', [0, 2q)
    // then one subtraction), outputs u + v and u - v + q, both in [0, 2q).
    static_for<0, KB>([&](auto sc) {
      constexpr int b = KB - 1 - decltype(sc)::value;
      const int bitpos = LO + b;
      const int st = LOGR - 1 - bitpos;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        if (j & (1 << b)) continue;
        const int jj = j | (1 << b);
        const ulonglong2 w = twiddle(b, j, bitpos, st);
        const u64 u = csubk(x[j], q);
        const u64 v = csubk(shoup_fast(x[jj], w.x, w.y, nq), q);
        x[j] = u + v;
        x[jj] = u - v + q;
      }
    });
    if constexpr (FIN == kFinalFwd) {
#pragma unroll
      for (int j = 0; j < E; ++j) x[j] = csubk(x[j], q);
    }
  } else if constexpr (FWD) {
    // CT: X-operands below r q (the static range of this stage, fwd_range), reduced by H/2 q
    // only when the stage would outgrow H q; v = w x[jj] in [0, 3q); outputs below (r' + 3) q
    const u64 qh = (u64)(H / 2) * q;
    const u32 sb = 64 - __builtin_clzll(q);  // bitlength of q (H = 16 top-bits reductions)
    static_for<0, KB>([&](auto sc) {
      constexpr int done = decltype(sc)::value;
      constexpr int b = KB - 1 - done;
      constexpr int rin = fwd_range(RIN, done, H);
      constexpr bool reduce = rin + 3 > H;
      constexpr int bitpos = LO + b;
      constexpr int st = LOGR - 1 - bitpos;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        if (j & (1 << b)) continue;
        const int jj = j | (1 << b);
        const ulonglong2 w = twiddle(b, j, bitpos, st);
        u64 u = x[j];
        if constexpr (reduce) u = H == 16 ? top_bits(u, sb, nq) : csubk(u, qh);
        FHE_OPAQUE(u);  // keeps 2u + 3q one v_lshl_add_u64 (not distributed over the select)
        // u + v straight out of the remainder chain; u - v + 3q = (2u + 3q) - (u + v)
        u64 s;
        if constexpr (PRE0 && st == 0) {
          (void)w;
          s = u + x[jj];  // x[jj] = w v below 2q: u + w v below (r + 2) q, u - w v + 3q below (r + 3) q
        } else {
          s = shoup_q3_add<CHAIN>(x[jj], w.x, w.y, nq, u);
        }
        FHE_OPAQUE(s);
        x[j] = s;
        u64 t2 = (u << 1) + q3;
        FHE_OPAQUE(t2);
        x[jj] = t2 - s;
      }
    });
    if constexpr (FIN == kFinalFwd || FIN == kFinalFwd2) {
      // from below r_out q down to [0, q) (kFinalFwd) or [0, 2q) (kFinalFwd2) by halving steps
      constexpr int rout = fwd_range(RIN, KB, H);
      constexpr int stop = FIN == kFinalFwd ? 1 : 2;
      // a modulus within 1/16 below 2^s (s = its bitlength: every lz16 modulus; for H = 8, s = 60
      // is tested): one top-bits estimate instead of up to three halving steps.  Kept a
      // wave-uniform runtime test even where H = 16 guarantees it: with the branch resolved at
      // compile time the fused HomMult kernel's allocation spills 31 VGPRs (2 with the branch).
      const u32 sf = H == 16 ? sb : 60;
      if (rout > 4 && rout <= 16 && (q >> (sf - 4)) == 15) {
#pragma unroll
        for (int j = 0; j < E; ++j) {
          x[j] = top_bits(x[j], sf, nq);
          if constexpr (FIN == kFinalFwd) x[j] = csubk(x[j], q);
        }
      } else {
#pragma unroll
        for (int j = 0; j < E; ++j) {
          static_for<0, 5>([&](auto ci) {
            constexpr int c = 16 >> decltype(ci)::value;  // 16, 8, 4, 2, 1
            if constexpr (c >= stop && c < rout) x[j] = csubk(x[j], (u64)c * q);
          });
        }
      }
    }
  } else if constexpr (H == 2) {
    // wide GS: canonical inputs; sum mod q, (u - v + q) w by the exact Shoup product, reduced
    static_for<0, KB>([&](auto bc) {
      constexpr int b = decltype(bc)::value;
      constexpr int bitpos = LO + b;
      constexpr int st = LOGR - 1 - bitpos;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        if (j & (1 << b)) continue;
        const int jj = j | (1 << b);
        const u64 u = x[j], v = x[jj];
        const u64 sum = u + v, dif = u - v + q;
        if constexpr (FIN == kFinalInv && st == 0) {
          x[j] = csubk(shoup_fast(sum, nf0.x, nf0.y, nq), q);
          x[jj] = csubk(shoup_fast(dif, nf1.x, nf1.y, nq), q);
        } else {
          const ulonglong2 w = twiddle(b, j, bitpos, st);
          x[j] = csubk(sum, q);
          x[jj] = csubk(shoup_fast(dif, w.x, w.y, nq), q);
        }
      }
    });
  } else if constexpr (H == 16) {
    // GS with lazy sums (gs_in): inputs in [0, 3q); each pair at r q: sum u + v below 2r q,
    // (u - v + r q) w -> [0, 3q); the round ends with every element back in [0, 3q)
    const u32 sb = 64 - __builtin_clzll(q);  // bitlength of q (top_bits)
    u64 q4 = 4 * q, q6 = 6 * q, q8 = 8 * q;
    asm("" : "+s"(q4));
    asm("" : "+s"(q6));
    asm("" : "+s"(q8));
    constexpr bool kLast = FIN == kFinalInv || FIN == kFinalInvS30;
    static_for<0, KB>([&](auto bc) {
      constexpr int b = decltype(bc)::value;
      constexpr int bitpos = LO + b;
      constexpr int st = LOGR - 1 - bitpos;
      static_for<0, E>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (!(j & (1 << b))) {
          constexpr int jj = j | (1 << b);
          constexpr int r = gs_in(j, b), rr = gs_red(r);
          u64 u = x[j], v = x[jj];
          if constexpr (rr != r) {
            u = top_bits<GATHER>(u, sb, nq);
            v = top_bits<GATHER>(v, sb, nq);
          }
          static_assert(rr == 2 || rr == 3 || rr == 4 || rr == 6 || rr == 8, "GS range");
          const u64 off = rr == 2 ? q2 : rr == 3 ? q3 : rr == 4 ? q4 : rr == 6 ? q6 : q8;
          const u64 sum = u + v, dif = u - v + off;
          if constexpr (kLast && st == 0) {
            // last stage of the whole inverse: fold N^-1 (both outputs) by the exact-quotient
            // product ([0, 2q)) and reduce to [0, q)
            x[j] = csubk(shoup_fast(sum, nf0.x, nf0.y, nq), q);
            x[jj] = csubk(shoup_fast(dif, nf1.x, nf1.y, nq), q);
          } else {
            const ulonglong2 w = twiddle(b, j, bitpos, st);
            x[j] = sum;
            x[jj] = shoup_q3<CHAIN>(dif, w.x, w.y, nq);
          }
        }
      });
    });
    if constexpr (kLast) {
      if constexpr (FIN == kFinalInvS30) {
#pragma unroll
        for (int j = 0; j < E; ++j) x[j] = split30(x[j]);
      }
    } else {
      static_for<0, E>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (gs_in(j, KB) > 3) x[j] = top_bits<GATHER>(x[j], sb, nq);
      });
    }
  } else {
    // GS: inputs in [0, 3q); sum -> [0, 3q); (u - v + 3q) w -> [0, 3q)
    static_for<0, KB>([&](auto bc) {
      constexpr int b = decltype(bc)::value;
      constexpr int bitpos = LO + b;
      constexpr int st = LOGR - 1 - bitpos;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        if (j & (1 << b)) continue;
        const int jj = j | (1 << b);
        const u64 u = x[j], v = x[jj];
        const u64 sum = u + v, dif = u - v + q3;
        if constexpr ((FIN == kFinalInv || FIN == kFinalInvS30) && st == 0) {
          // last stage of the whole inverse: fold N^-1 (both outputs) and reduce to [0, q)
          x[j] = csubk(csubk(shoup_q3<GATHER>(sum, nf0.x, nf0.y, nq), q2), q);
          x[jj] = csubk(csubk(shoup_q3<GATHER>(dif, nf1.x, nf1.y, nq), q2), q);
        } else {
          const ulonglong2 w = twiddle(b, j, bitpos, st);
          x[j] = csubk(sum, q3);
          x[jj] = shoup_q3<GATHER>(dif, w.x, w.y, nq);
        }
      }
    });
    if constexpr (FIN == kFinalInvS30) {
#pragma unroll
      for (int j = 0; j < E; ++j) x[j] = split30(x[j]);
    }
  }
}

// Whether a round's kE positions are tp + 0..kE-1 (contiguous words: 16-byte accesses).
template <class Lay>
constexpr bool contiguous16() {
  for (int j = 0; j < Lay::E; ++j)
    if (Lay::jpos(j) != (u32)j) return false;
  return true;
}

// Global-memory views of one sub-transform.  Column pass: position p at base[p * R2] (lanes run
// over adjacent columns, so every access is coalesced).  Row pass: position p at base[p].
// `base` is wave-uniform and `lane` the per-lane element offset, so every access is an SGPR base
// (the position's constant part folded in by the scalar unit) plus one 32-bit VGPR offset: no
// per-element 64-bit address registers.
// (Accesses go through explicitly global pointers: when the base pointer comes out of an item
// decode the compiler may lose its address space and emit flat accesses, which also count against
// lgkmcnt and so make every LDS wait wait for them.)
using gptr_u64 = __attribute__((address_space(1))) u64*;
using gptr_u128 = __attribute__((address_space(1))) u64x2_t*;
// NT views: non-temporal loads / stores for data streamed once through a working set larger
// than the caches.  HomMult's fused row kernel and its column-inverse pass use them (measured
// +1.5-2 % HomMult/s at batch 16-64: column inverse -6 %, fused kernel -2 %); the standalone NTT
// does not (its second pass re-reads what the first wrote, and the Infinity Cache serves part of
// it: non-temporal there costs 20 %).
template <bool NT, class P>
__device__ __forceinline__ auto gld(P p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, class P, class V>
__device__ __forceinline__ void gst(P p, V v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}
template <int STRIDE, bool NT = false, bool NTS = NT>
struct GView {
  u64* base;
  u32 lane;
  template <class Lay>
  __device__ __forceinline__ void load(u64 (&x)[Lay::E], u32 tp) const {
    const u32 off = lane + tp * STRIDE;
    if constexpr (STRIDE == 1 && contiguous16<Lay>()) {
      const gptr_u128 v = (gptr_u128)(base + off);
#pragma unroll
      for (int j = 0; j < Lay::E / 2; ++j) {
        const u64x2_t w = gld<NT>(v + j);
        x[2 * j] = w.x;
        x[2 * j + 1] = w.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < Lay::E; ++j)
        x[j] = gld<NT>((gptr_u64)(base + (u64)Lay::jpos(j) * STRIDE) + off);
    }
  }
  template <class Lay>
  __device__ __forceinline__ void store(const u64 (&x)[Lay::E], u32 tp) const {
    const u32 off = lane + tp * STRIDE;
    if constexpr (STRIDE == 1 && contiguous16<Lay>()) {
      const gptr_u128 v = (gptr_u128)(base + off);
#pragma unroll
      for (int j = 0; j < Lay::E / 2; ++j) gst<NTS>(v + j, u64x2_t{x[2 * j], x[2 * j + 1]});
    } else {
#pragma unroll
      for (int j = 0; j < Lay::E; ++j)
        gst<NTS>((gptr_u64)(base + (u64)Lay::jpos(j) * STRIDE) + off, x[j]);
    }
  }
  // Linear store of a row: thread t of the row's TPS threads owns positions 2 t + 2 TPS jj
  // (+ 0, 1), so each 16-byte store instruction covers 16 TPS contiguous bytes of the row.
  template <u32 TPS>
  __device__ __forceinline__ void load_lin(u64 (&x)[kE], u32 t) const {
    static_assert(STRIDE == 1, "rows only");
    const gptr_u128 v = (gptr_u128)(base + lane) + t;
#pragma unroll
    for (int jj = 0; jj < kE / 2; ++jj) {
      const u64x2_t w = gld<NT>(v + jj * TPS);
      x[2 * jj] = w.x;
      x[2 * jj + 1] = w.y;
    }
  }
  struct NoPre {};
  template <u32 TPS>
  __device__ __forceinline__ NoPre pre_lin(u32) const {
    return {};
  }
  template <u32 TPS>
  __device__ __forceinline__ void store_lin(const u64 (&x)[kE], u32 t, NoPre = {}) const {
    static_assert(STRIDE == 1, "rows only");
    const gptr_u128 v = (gptr_u128)(base + lane) + t;
#pragma unroll
    for (int jj = 0; jj < kE / 2; ++jj) gst<NTS>(v + jj * TPS, u64x2_t{x[2 * jj], x[2 * jj + 1]});
  }
};

// LDS view of one sub-transform: position p at s[p * PS + (PAD16 ? p >> 4 : 0)].
template <int PS, bool PAD16>
struct LView {
  u64* s;
  __device__ __forceinline__ u32 idx(u32 p) const { return p * PS + (PAD16 ? (p >> 4) : 0); }
  template <class Lay>
  __device__ __forceinline__ void load(u64 (&x)[Lay::E], u32 tp) const {
#pragma unroll
    for (int j = 0; j < Lay::E; ++j) x[j] = s[idx(tp | Lay::jpos(j))];
  }
  template <class Lay>
  __device__ __forceinline__ void store(const u64 (&x)[Lay::E], u32 tp) const {
#pragma unroll
    for (int j = 0; j < Lay::E; ++j) s[idx(tp | Lay::jpos(j))] = x[j];
  }
};

// LDS view of the column pass: position p of column `sub` (base s = lds + sub) in a tile of S
// columns, no padding.  S >= 32: rows of S words, and a half-wavefront (32 lanes = 32 columns)
// touches 32 distinct banks.  S = 16 (N1 = 8): rows pair into 32-word blocks, and the half each
// row takes is swapped by bit 4 of p, so both exchange patterns (p = t + 16 j and p = 16 t + j,
// t and t + 1 in one half-wavefront) land in different halves.  32 KB per workgroup instead of
// 34 KB with a pad column: 5 workgroups per CU instead of 4.
// SW: the position bit that picks the half-block; kElog (bit 4) for E = 16 threads.  With E = 32
// (the 512-row HomMult column pass, k_hm_col9) the second round's threads sit 32 positions apart,
// so the swap bit is 5 there (model-checked with the layouts, tests/test_modarith_model.py).
template <int S, int SW = kElog>
struct LViewC {
  u64* s;
  __device__ __forceinline__ u32 idx(u32 p) const {
    if constexpr (S >= 32) return p * S;
    return (p >> 1) * 32 + (((p ^ (p >> SW)) & 1u) << 4);
  }
  template <class Lay>
  __device__ __forceinline__ void load(u64 (&x)[Lay::E], u32 tp) const {
#pragma unroll
    for (int j = 0; j < Lay::E; ++j) x[j] = s[idx(tp | Lay::jpos(j))];
  }
  template <class Lay>
  __device__ __forceinline__ void store(const u64 (&x)[Lay::E], u32 tp) const {
#pragma unroll
    for (int j = 0; j < Lay::E; ++j) s[idx(tp | Lay::jpos(j))] = x[j];
  }
};

// Column-pass round exchange through half the tile's LDS (pass_run HALF).  A split bit SB of the
// position is an element bit in the writing round's layout and a thread bit -- uniform per
// wavefront (t = threadIdx.x / SUBS) -- in the reading round's: the forward's top bit, the
// inverse's bit 3 (the top bit of its first round).  The tile's two halves (positions with bit
// SB = h) then go through one buffer, positions compressed to LOGR - 1 bits, in phase h: every
// thread writes its 8 half-h elements; barrier; the threads of half h read all 16 of theirs.
// The half-0 readers still owe their half-1 elements to phase 1, so they read into x after
// copying those 8 values to y.  16 KB per tile instead of 32 KB at LOGR = 8, 16 columns: LDS no
// longer caps the column passes at 5 workgroups per CU.  Every layout pair is conflict-free in
// the LDS banks (same cycles as the full-tile exchange) and is model-checked in
// tests/test_modarith_model.py::test_half_exchange_layouts.  The caller has no LDS access
// outstanding on the buffer.
template <u32 WJ, u32 RJ>
constexpr int half_split_bit() {
  for (int b = 31; b >= 0; --b)
    if (((WJ & ~RJ) >> b) & 1u) return b;
  return -1;
}
template <int SB>
__device__ __forceinline__ u32 half_pos(u32 p) {
  return (p & ((1u << SB) - 1)) | ((p >> (SB + 1)) << SB);
}
template <int LOGR, class LayW, class LayR, class LV>
__device__ __forceinline__ void half_exchange(u64 (&x)[LayW::E], const LV& lv, u32 t) {
  constexpr int kE = LayW::E;
  static_assert(LayR::E == kE, "one element count for both rounds");
  constexpr int SB = half_split_bit<LayW::jmask, LayR::jmask>();
  static_assert(SB >= 0 && SB < LOGR, "no element bit of the writer is a thread bit of the reader");
  constexpr u32 S = 1u << SB;
  const u32 tpw = LayW::tpos(t), tpr = LayR::tpos(t);
  const bool hr = (tpr & S) != 0;  // this thread's half as a reader (wave-uniform)
  u64 y[kE];
  static_for<0, 2>([&](auto hc) {
    constexpr u32 h = decltype(hc)::value;
    if constexpr (h == 1) __syncthreads();  // phase 0's reads are done
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      if (((LayW::jpos(j) & S) != 0) != (h == 1)) continue;
      // the half-0 readers hold their half-1 elements in y (phase 0 replaced x)
      lv.s[lv.idx(half_pos<SB>(tpw | LayW::jpos(j)))] = (h == 1 && !hr) ? y[j] : x[j];
    }
    __syncthreads();
    if (hr == (h == 1)) {
#pragma unroll
      for (int j = 0; j < kE; ++j) {
        if (h == 0) y[j] = x[j];
        x[j] = lv.s[lv.idx(half_pos<SB>(tpr | LayR::jpos(j)))];
      }
    }
  });
}

// Round-0 global load of one sub-transform into registers.
template <int LOGR, bool FWD, int EL = kElog, class GIn>
__device__ __forceinline__ void pass_load(const GIn& gin, u32 t, u64 (&x)[1 << EL]) {
  using Rd = Rounds<LOGR, EL>;
  using Lay = Layout<LOGR, FWD ? Rd::kb(0) : Rd::kb_inv(0), FWD ? Rd::lo_fwd(0) : Rd::lo_inv(0),
                     EL>;
  gin.template load<Lay>(x, Lay::tpos(t));
}

// The rest of a 2^LOGR-point pass on values pass_load brought in: rounds exchange through LDS,
// the last round stores straight to global memory.  Every thread of the LDS-sharing group must
// call it (it contains the exchange fences).
// H / R0: forward headroom and input range of the pass (fwd_range), in units of q.
// XOUT: the last round goes out through the LDS in linear order (GView::store_lin) instead of
// straight from registers, whose last-round positions are E consecutive words per thread, so a
// direct store instruction writes 16 of every 16 E bytes across 16 E * 64 bytes.
// HALF: the column passes' one exchange (two rounds) through half the tile's LDS (half_exchange).
template <int LOGR, bool FWD, int FIN, int SYNC, bool GATHER, int H, int R0, bool XOUT = false,
          bool CHAIN = GATHER, bool HALF = false, bool PRE0 = false, int EL = kElog, class GOut,
          class LV>
__device__ __forceinline__ void pass_run(u64 (&x)[1 << EL], const GOut& gout, const LV& lv, u32 t,
                                         const ulonglong2* __restrict__ tw, u32 base, u64 q,
                                         ulonglong2 nf0, ulonglong2 nf1) {
  using Rd = Rounds<LOGR, EL>;
  static_for<0, Rd::NR>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int KB = FWD ? Rd::kb(k) : Rd::kb_inv(k);
    constexpr int LO = FWD ? Rd::lo_fwd(k) : Rd::lo_inv(k);
    constexpr int F = (k == Rd::NR - 1) ? FIN : kNotFinal;
    constexpr int RIN = fwd_range(R0, Rd::lo_fwd(0) + Rd::kb(0) - (LO + KB), H);  // stages before
    using Lay = Layout<LOGR, KB, LO, EL>;
    const u32 tp = Lay::tpos(t);
    static_assert(!HALF || (Rd::NR == 2 && SYNC == kBlockSync), "half exchange: column, 2 rounds");
    static_assert(!XOUT || EL == kElog, "linear row stores: 16 elements per thread");
    if constexpr (k > 0 && !HALF) {  // (HALF: half_exchange already loaded this round's layout)
      lds_sync<SYNC>();
      lv.template load<Lay>(x, tp);
    }
    // an opaque twiddle base per round keeps the scheduler from hoisting every round's twiddle
    // loads to the top (the gathered row passes: their VGPRs would cost occupancy or spill); the
    // column pass's few shared twiddles are left to the scheduler
    const ulonglong2* twk = tw;
    if constexpr (GATHER) asm volatile("" : "+s"(twk));
    round_compute<LOGR, KB, LO, FWD, F, GATHER, H, RIN, GATHER, CHAIN, PRE0 && k == 0, EL>(
        x, tp, twk, base, q, nf0, nf1);
    if constexpr (k == Rd::NR - 1) {
      if constexpr (XOUT) {
        constexpr u32 TPS = (1u << LOGR) / kE;
        // an output view that reads operands at the store positions (FinishView's acc rows)
        // issues those loads here, so they are in flight during the LDS transposition
        const auto pre = gout.template pre_lin<TPS>(t);
        lds_sync<SYNC>();
        lv.template store<Lay>(x, tp);
        lds_sync<SYNC>();
#pragma unroll
        for (int jj = 0; jj < kE / 2; ++jj) {
          const u32 p = 2 * t + 2 * TPS * jj;
          x[2 * jj] = lv.s[lv.idx(p)];
          x[2 * jj + 1] = lv.s[lv.idx(p + 1)];
        }
        gout.template store_lin<TPS>(x, t, pre);
      } else {
        gout.template store<Lay>(x, tp);
      }
    } else if constexpr (HALF) {
      constexpr int KN = FWD ? Rd::kb(k + 1) : Rd::kb_inv(k + 1);
      constexpr int LN = FWD ? Rd::lo_fwd(k + 1) : Rd::lo_inv(k + 1);
      half_exchange<LOGR, Lay, Layout<LOGR, KN, LN, EL>>(x, lv, t);
    } else {
      // the (free) wave-local fence before round 0's store keeps the row passes' LDS stores
      // together after the butterflies, which measured faster than letting them interleave
      if (k > 0 || SYNC == kWaveSync) lds_sync<SYNC>();
      lv.template store<Lay>(x, tp);
    }
  });
}

template <int LOGN>
struct Geo {
  static constexpr int N1 = LOGN / 2, N2 = LOGN - N1;
  static constexpr int R1 = 1 << N1, R2 = 1 << N2;  // R1 rows x R2 columns
  // column pass: SUBS_C columns per workgroup, lanes run over columns
  static constexpr int TPS_C = R1 >> kElog;
  static constexpr int SUBS_C = (kColThreads / TPS_C) < R2 ? (kColThreads / TPS_C) : R2;
  static constexpr int THR_C = SUBS_C * TPS_C;
  static constexpr int LDS_C = R1 * SUBS_C;  // LViewC: no padding
  static_assert(SUBS_C == 16 || SUBS_C >= 32, "column LDS layout assumes 16 or >= 32 columns");
  // the column passes exchange through half the tile (half_exchange) where their two rounds are
  // 4 + 4 stages over 16 columns (N = 2^16, 2^17): 16 KB per workgroup
  static constexpr bool HALF_C = N1 == 8 && SUBS_C == 16;
  static constexpr int LDS_CF = HALF_C ? LDS_C / 2 : LDS_C;
  static constexpr int TILES_C = R2 / SUBS_C;
  // row pass: SUBS_R rows per workgroup, lanes run along a row
  static constexpr int TPS_R = R2 >> kElog;
  static constexpr int SUBS_R = (kThreads / TPS_R) < R1 ? (kThreads / TPS_R) : R1;
  static constexpr int THR_R = SUBS_R * TPS_R;
  static constexpr int RS = R2 + R2 / 16;  // LDS row stride (one pad word per 16)
  static constexpr int LDS_R = SUBS_R * RS;
  static constexpr int TILES_R = R1 / SUBS_R;
  static_assert(N1 >= kElog - 1 && N2 >= kElog, "log N too small for this kernel family");
};

// Column pass, one workgroup per item (p, l, tile) of src/dst [polys][nlimbs][N] via PolyMap.
// NTL / NTS: non-temporal loads of the source / stores of the destination (see GView).
// (Persistent grids looping over items with a register prefetch of the next one measured slower:
// vmcnt retires in issue order, so every twiddle wait also waited for the prefetch, and the
// prefetch registers pushed the column kernel into spills -- DESIGN.md §8.)
// FI: the inverse's final stage (kFinalInv, or kFinalInvS30 for split30 outputs).
// R0: the forward's input range (units of q) its lazy schedule starts from.  The row pass that
// follows must assume the same R0: fwd_range is not monotonic in it (an earlier reduction can leave
// a smaller bound), so the key-switch / rescale row kernels, which assume 2 (k_modup_col's
// outputs), get column passes scheduled from 2 as well (col_fwd_pass, k_rescale_col).
// One column tile (poly p, limb l, tile) of a column pass (the body of k_ntt_col; lds: G::LDS_CF
// words).
template <int LOGN, bool FWD, int H, bool NTL, bool NTS, int FI, int R0>
__device__ __forceinline__ void col_tile(u64* lds, const u64* __restrict__ src,
                                         const u64* __restrict__ src2, u64* __restrict__ dst,
                                         u32 limb0, const PolyMap& pm, u32 p, u32 l, u32 tile,
                                         const ulonglong2* __restrict__ tw_all,
                                         const ulonglong2* __restrict__ nfold,
                                         const ModParams* __restrict__ mods) {
  using G = Geo<LOGN>;
  constexpr u64 N = 1ull << LOGN;
  const u32 sub = threadIdx.x % G::SUBS_C, t = threadIdx.x / G::SUBS_C;
  const LViewC<G::SUBS_C> lv{lds + sub};
  const u64 loc = (u64)l * N + (u64)tile * G::SUBS_C;
  const u64* s = (pm.second(p) ? src2 + pm.src2(p) : src + pm.src(p)) + loc;
  const u32 limb = __builtin_amdgcn_readfirstlane(limb0 + l);
  u64 x[kE];
  pass_load<G::N1, FWD>(GView<G::R2, NTL>{const_cast<u64*>(s), sub}, t, x);
  ulonglong2 nf0 = {0, 0}, nf1 = {0, 0};
  if (!FWD) {
    nf0 = nfold[4 * limb];
    nf1 = nfold[4 * limb + 1];
  }
  pass_run<G::N1, FWD, FWD ? kNotFinal : FI, kBlockSync, false, H, R0, false, false, G::HALF_C>(
      x, GView<G::R2, false, NTS>{dst + pm.dst(p) + loc, sub}, lv, t, tw_all + (u64)limb * N, 1u,
      mods[limb].q, nf0, nf1);
}

template <int LOGN, bool FWD, int H = 8, bool NTL = false, bool NTS = false, int FI = kFinalInv,
          int R0 = 1>
__global__ __launch_bounds__(kColThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_ntt_col(
    const u64* __restrict__ src, const u64* __restrict__ src2, u64* __restrict__ dst, u32 nlimbs,
    u32 limb0, PolyMap pm, u32 items, const ulonglong2* __restrict__ tw_all,
    const ulonglong2* __restrict__ nfold, const ModParams* __restrict__ mods) {
  using G = Geo<LOGN>;
  __shared__ u64 lds[G::LDS_CF];
  const u32 it = blockIdx.x;
  if (it >= items) return;
  // XCD-grouped placement: workgroups are dealt to the 8 XCDs round-robin, so XCD x takes the
  // poly-limbs pl = x mod 8 and runs all TILES_C column tiles of one back to back.  Adjacent
  // 128-byte row segments then come from one XCD close together in time (DRAM page locality):
  // tools/microbench/colcopy.hip, this access pattern 5.30 -> 5.85 TB/s; with 8 | nlimbs the limb
  // (and its twiddles) is also tied to the XCD.  Otherwise tiles fastest over all XCDs.  (All 8
  // XCDs sweeping one poly-limb's tiles together instead: HomMult column forward +3.4 %, column
  // inverse +2.4 %, configs[4] column pass +6 %; profiles/r03_row_order_ab.txt.)
  u32 tile, pl;
  if ((items / G::TILES_C) % 8 == 0) {
    const u32 k = it / 8;
    tile = k % G::TILES_C;
    pl = (k / G::TILES_C) * 8 + it % 8;
  } else {
    tile = it % G::TILES_C;
    pl = it / G::TILES_C;
  }
  col_tile<LOGN, FWD, H, NTL, NTS, FI, R0>(lds, src, src2, dst, limb0, pm, pl / nlimbs,
                                           pl % nlimbs, tile, tw_all, nfold, mods);
}

// One row tile (poly p, limb l, tile) of a row pass (the body of k_ntt_row; lds: G::LDS_R words).
// The forward stores its last round in linear order through the LDS (XOUT); the inverse loads its
// first round that way.
template <int LOGN, bool FWD, int H, bool NTL, bool NTS, int R0 = 1>
__device__ __forceinline__ void row_tile(u64* lds, const u64* __restrict__ src,
                                         u64* __restrict__ dst, u32 limb0, const PolyMap& pm,
                                         u32 p, u32 l, u32 tile,
                                         const ulonglong2* __restrict__ tw_all,
                                         const ModParams* __restrict__ mods) {
  using G = Geo<LOGN>;
  constexpr u64 N = 1ull << LOGN;
  static_assert(64 % G::TPS_R == 0, "a row must not straddle wavefronts");
  const u32 t = threadIdx.x % G::TPS_R, sub = threadIdx.x / G::TPS_R;
  const LView<1, true> lv{lds + sub * G::RS};
  const u32 row0 = tile * G::SUBS_R;
  const u64 loc = (u64)l * N + (u64)row0 * G::R2;
  const u32 limb = __builtin_amdgcn_readfirstlane(limb0 + l);
  const u32 lane = sub * G::R2;
  const GView<1, NTL> gin{const_cast<u64*>(src) + pm.src(p) + loc, lane};
  u64 x[kE];
  if constexpr (!FWD) {
    // the inverse's round 0 owns E consecutive words per thread: load the row linearly and
    // redistribute through the LDS (the mirror of pass_run's XOUT store)
    using Rd = Rounds<G::N2>;
    using Lay0 = Layout<G::N2, Rd::kb_inv(0), Rd::lo_inv(0)>;
    gin.template load_lin<G::TPS_R>(x, t);
#pragma unroll
    for (int jj = 0; jj < kE / 2; ++jj) {
      const u32 q = 2 * t + 2 * G::TPS_R * jj;
      lv.s[lv.idx(q)] = x[2 * jj];
      lv.s[lv.idx(q + 1)] = x[2 * jj + 1];
    }
    lds_sync<kWaveSync>();
    lv.template load<Lay0>(x, Lay0::tpos(t));
  } else {
    pass_load<G::N2, FWD>(gin, t, x);
  }
  pass_run<G::N2, FWD, FWD ? kFinalFwd : kNotFinal, kWaveSync, true, H, fwd_range(R0, G::N1, H),
           FWD>(x, GView<1, false, NTS>{dst + pm.dst(p) + loc, lane}, lv, t,
                tw_all + (u64)limb * N, (u32)G::R1 + row0 + sub, mods[limb].q, {0, 0}, {0, 0});
}

// Row pass, one workgroup per item (l, p, tile): the limb follows the XCD (its row twiddles stay
// in that XCD's L2) and the tile varies fastest, so an XCD streams each poly-limb's rows front to
// back.  (Poly fastest, which re-read a row's twiddles sooner: row passes 8 % slower,
// profiles/r03_row_order_ab.txt.)
// R0: the input range (units of q) the preceding column pass was scheduled from (fwd_range); 2 after
// k_modup_col (the hoisted ModUp's row pass, launch_ntt_row_fwd_r2)
template <int LOGN, bool FWD, int H = 8, bool NTL = false, bool NTS = false, int R0 = 1>
__global__ FHE_KATTR void k_ntt_row(const u64* __restrict__ src, u64* __restrict__ dst, u32 nlimbs,
                                    u32 limb0, PolyMap pm, u32 items,
                                    const ulonglong2* __restrict__ tw_all,
                                    const ModParams* __restrict__ mods) {
  using G = Geo<LOGN>;
  __shared__ u64 lds[G::LDS_R];
  const u32 it = blockIdx.x;
  if (it >= items) return;
  u32 l, rest;
  xcd_limb_split(it, nlimbs, items / nlimbs, l, rest);
  row_tile<LOGN, FWD, H, NTL, NTS, R0>(lds, src, dst, limb0, pm, rest / G::TILES_R, l,
                                   rest % G::TILES_R, tw_all, mods);
}

// HomMult column forward on the 512 x 128 view of N = 2^16 (the first 9 of the 16 stages; the fused
// row kernel then runs 7 on 128-word rows, k_hommult_row S9): 32 elements per thread in two rounds
// of 5 + 4 stages with one exchange through half the tile (LViewC swap bit 5: both rounds' access
// patterns conflict-free), tiles of 16 columns x 512 rows (256 threads, 16 per column), 32 KB of
// LDS.  Moves a stage of the 4 forward polys out of the issue-bound row kernel into this
// HBM-bound pass (the 2^9 x 2^7 split).  Same item placement and poly map as
// k_ntt_col (a's and b's polys into the 4-slot workspace).
constexpr int kC9Log = 9, kC9El = 5, kC9R2 = 128, kC9Subs = 16, kC9Tiles = kC9R2 / kC9Subs;
// Occupancy: 4 waves per SIMD (104 VGPRs, no spill).  At 5 (96 VGPRs + 60 B of scratch) the pass
// took 0.452 instead of 0.389 ms (profiles/r06_split9_ab.txt); an exchange by column halves (waves
// 0-1 / 2-3 taking turns through a full-column buffer, no pending elements) still spilled at 5
// waves: 0.947 ms (profiles/r06_col9_xhalf_ab.txt); the second round's twiddles from an LDS copy
// (either exchange, 4 or 5 waves) 0.43-0.46 ms against 0.40 (profiles/r06_col9_lds_twiddles_ab.txt).
template <int H>
__global__ __launch_bounds__(kColThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) void
k_hm_col9(const u64* __restrict__ src, const u64* __restrict__ src2, u64* __restrict__ dst,
          u32 nlimbs, u32 limb0, PolyMap pm, u32 items, const ulonglong2* __restrict__ tw_all,
          const ModParams* __restrict__ mods) {
  constexpr u64 N = 1ull << 16;
  static_assert(kC9Subs * (1 << (kC9Log - kC9El)) == kColThreads, "16 threads per column");
  __shared__ u64 lds[(1 << kC9Log) * kC9Subs / 2];
  const u32 it = blockIdx.x;
  if (it >= items) return;
  u32 tile, pl;
  if ((items / kC9Tiles) % 8 == 0) {  // XCD-grouped, as k_ntt_col
    const u32 k = it / 8;
    tile = k % kC9Tiles;
    pl = (k / kC9Tiles) * 8 + it % 8;
  } else {
    tile = it % kC9Tiles;
    pl = it / kC9Tiles;
  }
  const u32 p = pl / nlimbs, l = pl % nlimbs;
  const u64 loc = (u64)l * N + (u64)tile * kC9Subs;
  const u64* s = (pm.second(p) ? src2 + pm.src2(p) : src + pm.src(p)) + loc;
  const u32 limb = __builtin_amdgcn_readfirstlane(limb0 + l);
  u64 x[1 << kC9El];
  const u32 sub = threadIdx.x % kC9Subs, t = threadIdx.x / kC9Subs;
  const LViewC<kC9Subs, 5> lv{lds + sub};
  pass_load<kC9Log, true, kC9El>(GView<kC9R2, true>{const_cast<u64*>(s), sub}, t, x);
  pass_run<kC9Log, true, kNotFinal, kBlockSync, false, H, 1, false, false, true, false, kC9El>(
      x, GView<kC9R2>{dst + pm.dst(p) + loc, sub}, lv, t, tw_all + (u64)limb * N, 1u,
      mods[limb].q, {0, 0}, {0, 0});
}

// Fused HomMult row kernel: rows of the 4 column-transformed inputs (layout [batch][4][nlimbs][N]
// in `x`: A0, A1, B0, B1) -> row-forward, tensor, row-inverse -> d [batch][3][nlimbs][N].
// Thread groups g = 0..3 own one polynomial each; after the forward rows every group writes its
// canonical values to LDS slot g, groups 0..2 then form d_g from the slots at the same positions
// and run the inverse rows (group 3 idles through them).
template <int LOGN>
struct HmGeo {
  using G = Geo<LOGN>;
  static constexpr int TPS = G::TPS_R;
  static constexpr int LANES_ROW = 4 * TPS;                  // 4 polys x TPS threads per row
  static constexpr int ROWS = kThreads / LANES_ROW;          // rows per workgroup
  static constexpr int THR = ROWS * LANES_ROW;
  static constexpr int ROWW = 4 * G::RS;                     // LDS words per row (4 slots)
  static constexpr int TILES = G::R1 / ROWS;
  static_assert(64 % LANES_ROW == 0 || LANES_ROW % 64 == 0, "row group vs wavefront");
  // Thread group g = one polynomial spread over whole wavefronts ("poly-major"), so during the
  // 3-poly inverse the 4th group is a whole idle wave (its SIMD slots go to other waves) instead
  // of idle lanes inside every wave (measured: VALUBusy ~100 % with 77 % lane utilisation).
  // A polynomial's rows then sit in one wavefront, so its round exchanges stay wave-local and
  // only the tensor (reading all four slots) needs the block barrier.
  static constexpr int SYNC_TENSOR = kBlockSync;
  static constexpr int SYNC_ROUND = kWaveSync;
};

// Cache policy (measured per access): non-temporal workspace reads / output writes
// in the fused HomMult kernel and its column inverse (-2 % / -6 %), non-temporal a, b reads in the
// HomMult column forward (read once, +0.7 % HomMult/s), non-temporal stores / loads of the
// key-switch's extended rows (written by k_modup_col, read once by k_ks_row_inner: fused row
// kernel -6 %).  The standalone NTT stays cached: its second pass re-reads what the first wrote,
// and the Infinity Cache serves part of it (non-temporal there: -5 ... -8 % NTT/s).
constexpr bool kHmNT = true;
constexpr bool kKsNT = true;

// S9 (N = 2^16, after k_hm_col9): the forward rows are the 512 x 128 split's 7-stage rows, two
// per 256-word row (its 16 threads: 8 per half), with twf the d_tw_fwd9 layout; the tensor and the
// inverse are unchanged (the forward's last values go to LDS in its own layout, the tensor reads
// them in the inverse's first-round layout).
template <int LOGN, int HR = 8, bool S9 = false>
__global__ FHE_KATTR void k_hommult_row(const u64* __restrict__ x,
                                                          u64* __restrict__ d, u32 nlimbs,
                                                          u32 limb0,
                                                          const ulonglong2* __restrict__ twf,
                                                          const ulonglong2* __restrict__ twi,
                                                          const ModParams* __restrict__ mods) {
  using G = Geo<LOGN>;
  using H = HmGeo<LOGN>;
  using Rd = Rounds<G::N2>;
  constexpr u64 N = 1ull << LOGN;
  __shared__ u64 lds[H::ROWS * H::ROWW];
  u32 l, rest;
  xcd_limb_split(blockIdx.x, nlimbs, gridDim.x / nlimbs, l, rest);
  // tile fastest: an XCD's workgroups stream each poly-limb's rows front to back (DRAM page
  // locality; the limb's row twiddles stay in that XCD's L2 either way).  Measured against
  // ciphertext fastest: hm_row_tensor 0.684 -> 0.668 ms, standalone row passes -8 %; against all
  // 8 XCDs sweeping one poly-limb together (tile t on XCD t mod 8): -0.8 % on this kernel, row
  // passes +1-4 %, the N = 2^17 row pass +15 % (profiles/r03_row_order_ab.txt)
  const u32 b = rest / H::TILES, tile = rest % H::TILES;
  const u32 limb = limb0 + l;
  const ModParams m = mods[limb];
  const u64 q = m.q;
  const u64 limbN = (u64)nlimbs * N;
  // [poly][row][lane]; which wave gets which poly rotates per workgroup: the wave that idles
  // through the 3-poly inverse must not land on the same SIMD in every workgroup
  u32 grp = (threadIdx.x / (H::ROWS * H::TPS) + blockIdx.x) % 4;
  const u32 sub = (threadIdx.x / H::TPS) % H::ROWS;
  const u32 t = threadIdx.x % H::TPS;
  const u32 row = tile * H::ROWS + sub;
  const u64 loc = (u64)l * N + (u64)row * G::R2;
  const ulonglong2* tf = twf + (u64)limb * N;
  const ulonglong2* ti = twi + (u64)limb * N;
  const u32 base = (u32)G::R1 + row;
  u64* rowlds = lds + sub * H::ROWW;
  const LView<1, true> own{rowlds + grp * G::RS};
  constexpr int SY = H::SYNC_ROUND, ST = H::SYNC_TENSOR;

  // forward row pass: round 0 from global, rounds exchange through LDS, last round stays in VGPRs
  u64 v[kE];
  // the tensor reads every slot in the inverse's first-round layout (the 256 split's last forward
  // layout as well)
  using LayT = Layout<G::N2, Rd::kb_inv(0), Rd::lo_inv(0)>;
  const u32 tpT = LayT::tpos(t);
  if constexpr (S9) {
    static_assert(LOGN == 16, "the 512 x 128 split is built for N = 2^16");
    // rounds of 3 + 4 stages: the first round's elements pair into adjacent words (its spare
    // element bit is position 0), so it loads 16-byte pairs, 256 contiguous bytes per row; the
    // last round is the 16-element low-bit round of the 256 split (lane-major twiddles, kb 4)
    using R7 = Rounds<G::N2 - 1, kElog, true>;
    static_assert(R7::NR == 2 && R7::kb(0) == 3 && R7::lo_fwd(0) == 4 && R7::lo_fwd(1) == 0,
                  "3 + 4 stages");
    const u32 h7 = t >> 3, t7 = t & 7;  // half of the 256-word row, thread within it
    const LView<1, true> own7{rowlds + grp * G::RS + h7 * (128 + 8)};
    const u32 base7 = 2u * (u32)G::R1 + 2 * row + h7;  // row 2 row + h7 of the 512-row view
    const ulonglong2* tf9 = twf + (u64)limb * N;
    static_for<0, R7::NR>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int KB = R7::kb(k);
      constexpr int LO = R7::lo_fwd(k);
      constexpr int F = (k == R7::NR - 1) ? (HR == 2 ? kFinalFwd : kFinalFwd2) : kNotFinal;
      constexpr int RIN = fwd_range(fwd_range(1, G::N1 + 1, HR), G::N2 - 1 - (LO + KB), HR);
      using Lay = Layout<G::N2 - 1, KB, LO>;
      const u32 tp = Lay::tpos(t7);
      if constexpr (k == 0) {
        static_assert(Lay::jpos(kE / 2) == 1, "the spare element bit is position 0");
        const gptr_u128 gin = (gptr_u128)(const_cast<u64*>(x) + ((u64)b * 4 + grp) * limbN + loc +
                                          h7 * 128 + tp);
#pragma unroll
        for (int j = 0; j < kE / 2; ++j) {
          const u64x2_t w2 = gld<kHmNT>(gin + Lay::jpos(j) / 2);
          v[j] = w2.x;
          v[j + kE / 2] = w2.y;
        }
      } else {
        lds_sync<SY>();
        own7.template load<Lay>(v, tp);
      }
      round_compute<G::N2 - 1, KB, LO, true, F, true, HR, RIN>(v, tp, tf9, base7, q, {0, 0},
                                                                {0, 0});
      // every round's values back to the slot (the last one's for the tensor)
      if (k > 0) lds_sync<SY>();
      own7.template store<Lay>(v, tp);
    });
  } else {
    static_assert(Rd::lo_fwd(Rd::NR - 1) == Rd::lo_inv(0) && Rd::kb(Rd::NR - 1) == Rd::kb_inv(0),
                  "tensor layout must match the last forward round");
    static_for<0, Rd::NR>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int KB = Rd::kb(k);
      constexpr int LO = Rd::lo_fwd(k);
      // wide moduli: canonical forward outputs (4 q^2 would exceed q R for q > 2^62)
      constexpr int F = (k == Rd::NR - 1) ? (HR == 2 ? kFinalFwd : kFinalFwd2) : kNotFinal;
      constexpr int RIN = fwd_range(fwd_range(1, G::N1, HR), G::N2 - (LO + KB), HR);
      using Lay = Layout<G::N2, KB, LO>;
      const u32 tp = Lay::tpos(t);
      if constexpr (k == 0) {
        const GView<1, kHmNT> gin{const_cast<u64*>(x) + ((u64)b * 4 + grp) * limbN + loc, 0};
        gin.template load<Lay>(v, tp);
      } else {
        lds_sync<SY>();
        own.template load<Lay>(v, tp);
      }
      round_compute<G::N2, KB, LO, true, F, true, HR, RIN>(v, tp, tf, base, q, {0, 0}, {0, 0});
      if constexpr (k < Rd::NR - 1) {
        if (k > 0) lds_sync<SY>();
        own.template store<Lay>(v, tp);
      }
    });
    // tensor: publish canonical A0, A1, B0, B1 at the last forward layout
    lds_sync<SY>();
    own.template store<LayT>(v, tpT);
  }
  lds_sync<ST>();
  // Montgomery products of the forward outputs (in [0, 2q)): t R^-1 in [0, 2q), which the inverse
  // rows take (inputs below 3q); R is folded back in with N^-1 by the column inverse.  d1's sum of
  // two products stays below 8q^2 < q R (q < 2^61).
  // Poly-major groups are whole wavefronts, so the group switch is a uniform branch per wave.
  grp = __builtin_amdgcn_readfirstlane(grp);
  const bool active = grp < 3;
  const u32 aoff = grp == 2 ? G::RS : 0, boff = grp == 2 ? 3 * G::RS : 2 * G::RS;
  // subtractive REDC (mont_redc): no carry-in term, 3 VALU fewer per element than the additive one
  u64 qi = 0 - m.qinv;  // q^-1 mod 2^64
  asm("" : "+s"(qi));
  if constexpr (HR == 16) {
    // every modulus < 2^60: operands below 2^61, hand-written partial products and REDC
    // (d1 -42 %, d0 / d2 -26 % static VALU)
    if (grp == 1) {
#pragma unroll
      for (int j = 0; j < kE; ++j) {
        const u32 idx = own.idx(tpT | LayT::jpos(j));
        u64 tlo, thi;
        mul2_wide61(rowlds[idx], rowlds[3 * G::RS + idx], rowlds[G::RS + idx],
                    rowlds[2 * G::RS + idx], tlo, thi);
        v[j] = mont_redc_x(tlo, thi, q, qi);
      }
    } else if (active) {
#pragma unroll
      for (int j = 0; j < kE; ++j) {
        const u32 idx = own.idx(tpT | LayT::jpos(j));
        u64 tlo, thi;
        mul_wide61(rowlds[aoff + idx], rowlds[boff + idx], tlo, thi);
        v[j] = mont_redc_x(tlo, thi, q, qi);
      }
    }
  } else if (grp == 1) {
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      const u32 idx = own.idx(tpT | LayT::jpos(j));
      const u128 t = (u128)rowlds[idx] * rowlds[3 * G::RS + idx] +
                     (u128)rowlds[G::RS + idx] * rowlds[2 * G::RS + idx];
      v[j] = mont_redc((u64)t, (u64)(t >> 64), q, qi);
    }
  } else if (active) {
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      const u32 idx = own.idx(tpT | LayT::jpos(j));
      const u128 t = (u128)rowlds[aoff + idx] * rowlds[boff + idx];
      v[j] = mont_redc((u64)t, (u64)(t >> 64), q, qi);
    }
  }
  if constexpr (HR == 2) {  // the wide inverse takes canonical inputs
#pragma unroll
    for (int j = 0; j < kE; ++j) v[j] = csubk(v[j], q);
  }
  // inverse row pass: its first round butterflies the low bits, the layout the tensor used
  static_assert(Rd::lo_fwd(Rd::NR - 1) == Rd::lo_inv(0) && Rd::kb(Rd::NR - 1) == Rd::kb_inv(0),
                "tensor layout must match the first inverse round");
  static_for<0, Rd::NR>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int KB = Rd::kb_inv(k);
    constexpr int LO = Rd::lo_inv(k);
    using Lay = Layout<G::N2, KB, LO>;
    const u32 tp = Lay::tpos(t);
    if constexpr (k > 0) {
      lds_sync<SY>();
      if (active) own.template load<Lay>(v, tp);
    }
    if (active) round_compute<G::N2, KB, LO, false, kNotFinal, true, HR>(v, tp, ti, base, q, {0, 0}, {0, 0});
    if constexpr (k == Rd::NR - 1) {
      const GView<1, kHmNT> gout{d + ((u64)b * 3 + grp) * limbN + loc, 0};
      // (a linear 16-byte store through the own slot, pass_run's XOUT: 0.660 -> 0.665 ms,
      // profiles/r06_hm_xout_ab.txt)
      if (active) gout.template store<Lay>(v, tp);
    } else {
      // the first store into this slot must wait until every group has read it for the tensor
      lds_sync<(k == 0 ? ST : SY)>();
      if (active) own.template store<Lay>(v, tp);
    }
  });
}

// Up to 4 digits of one ModUp in one launch (kernel argument).  Digit k owns the blocks from
// blk0 on; its source row j of ciphertext b is at y + b ybs + o[j], its T target rows go to ext.
struct ModUpDigit {
  u64 o[4];
  u64* ext;
  const ulonglong2* hat;
  u32 T, skip_at, skip_len, blk0;
};
struct ModUpDigits {
  ModUpDigit d[4];
  u32 n;
};

// ModUp column pass (key-switch): the column-forward pass of every extended row of one digit,
// reading its input straight from the digit's S pre-scaled source rows y_k = [x_k (D^_k)^-1]_{d_k}
// (coefficient form: the key-switch's own INTT of d2 folds the factor in (d_nfold_up), else
// rns.hip k_modup_scale makes them) and converting on the fly:
//   x = sum_k y_k (D^_k mod t) mod t   (sum < S 2^61 t < t 2^64: Sum30, one Montgomery reduction;
//                                       hat[k hs + t].y = D^_k 2^64 mod t)
// so the extended rows are never written in coefficient form (SURVEY §8a' ModUp; the unfused path
// is k_baseconv + k_ntt_col).  Items (target row, ciphertext, column tile) are dealt XCD-major,
// target fastest: an XCD converts every target of a (ciphertext, tile) while the S source tiles are
// hot in its L2.  Target tr -> row r = tr < skip_at ? tr : tr + skip_len (the digit's own rows are
// skipped) -> limb r < n0 ? base0 + r : base1 + (r - n0).  Every digit of a ModUp runs in this
// one launch (md.n digits with the same S, block ranges in digit order: no launch tail per digit).
// Targets per workgroup: the S source tiles are loaded once and converted for kModupTG targets.
// 1: two targets per workgroup (half the source loads) hold both converted tiles through the
// first target's pass, 128 VGPRs with spills: ModUp 0.50 -> 0.60 ms (profiles/
// r05_modup_targets_per_wg_ab.txt).
constexpr u32 kModupTG = 1;
template <int LOGN, int H, int S>
__global__ __launch_bounds__(kColThreads) __attribute__((amdgpu_waves_per_eu(
    4, 8))) void k_modup_col(const u64* __restrict__ y, u64 ybs, const ModUpDigits md, u64 rn,
                             u32 n0, u32 base0, u32 base1, u32 batch, u32 hs,
                             const ulonglong2* __restrict__ tw_all,
                             const ModParams* __restrict__ mods) {
  using G = Geo<LOGN>;
  using Rd = Rounds<G::N1>;
  using Lay0 = Layout<G::N1, Rd::kb(0), Rd::lo_fwd(0)>;
  constexpr u64 N = 1ull << LOGN;
  constexpr u32 TG = kModupTG;
  __shared__ u64 lds[G::LDS_CF];
  const u32 sub = threadIdx.x % G::SUBS_C, t = threadIdx.x / G::SUBS_C;
  const LViewC<G::SUBS_C> lv{lds + sub};
  u32 di = 0;
#pragma unroll
  for (u32 k = 1; k < 4; ++k)
    if (k < md.n && blockIdx.x >= md.d[k].blk0) di = k;
  const ModUpDigit& dg = md.d[di];
  const u32 T = dg.T, skip_at = dg.skip_at, skip_len = dg.skip_len;
  const u32 TP = (T + TG - 1) / TG;  // target groups
  u64* __restrict__ ext = dg.ext;
  const ulonglong2* __restrict__ hat = dg.hat;
  const u32 blk = blockIdx.x - dg.blk0;
  const u32 nbt = batch * G::TILES_C;
  u32 tg, bt;
  // (Tile-major per XCD instead, as k_ntt_col's placement -- a (target, ciphertext) pair's 16
  // tiles back to back on one XCD, the sources then read by every XCD: ModUp 0.252 -> 0.277 ms,
  // profiles/r03_row_order_ab.txt)
  if (nbt % 8 == 0) {  // every digit's block range then starts at a multiple of 8
    const u32 xcd = blk % 8, k8 = blk / 8;
    tg = k8 % TP;
    bt = xcd + 8 * (k8 / TP);
  } else {
    tg = blk % TP;
    bt = blk / TP;
  }
  const u32 b = bt / G::TILES_C, tile = bt % G::TILES_C;
  u32 rr[TG], limbs[TG];
  bool live[TG];
#pragma unroll
  for (u32 g = 0; g < TG; ++g) {
    const u32 tr = tg * TG + g;
    live[g] = tr < T;
    rr[g] = tr < skip_at ? tr : tr + skip_len;
    limbs[g] = __builtin_amdgcn_readfirstlane(rr[g] < n0 ? base0 + rr[g] : base1 + (rr[g] - n0));
  }
  const u32 tp = Lay0::tpos(t);
  const gptr_u64 yb = (gptr_u64)(y + (u64)b * ybs + (u64)tile * G::SUBS_C + sub);
  u64 x[TG][kE];
  // Stage 0 of the column-forward pass multiplies the upper half of the rows (position bit
  // N1 - 1) by its one twiddle w0 = psi^(N/2): the tables carry {h, h w0 mod t} pairs (rns.hip
  // build_rns_tables), so those rows are converted straight into w0 x and stage 0 only adds
  // (pass_run PRE0): 8 Shoup products per thread fewer.
  auto upper = [](int j) { return ((Lay0::jpos(j) >> (G::N1 - 1)) & 1u) != 0; };
  if constexpr (H == 16) {
    // lz16 (every modulus < 2^60): plain sources, the S-term sum on 32-bit halves (dot_wide61:
    // no splitting, the low column's carries from the mads) and the subtractive REDC into (0, 2q)
    // (mont_redc: mont_redc_x's carry-mask asm does not survive this kernel's register allocation)
    u64 hk[TG][S], hw[TG][S], qq[TG], qi[TG];
#pragma unroll
    for (u32 g = 0; g < TG; ++g) {
#pragma unroll
      for (int k = 0; k < S; ++k) {
        const ulonglong2 h = hat[(u64)k * hs + limbs[g]];
        hk[g][k] = h.x;
        hw[g][k] = h.y;
      }
      qq[g] = mods[limbs[g]].q;
      qi[g] = 0 - mods[limbs[g]].qinv;  // q^-1 mod 2^64
    }
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      const u64 i = (u64)(tp | Lay0::jpos(j)) * G::R2;
      u64 ys[S];
#pragma unroll
      for (int k = 0; k < S; ++k) ys[k] = yb[dg.o[k] + i];
#pragma unroll
      for (u32 g = 0; g < TG; ++g) {
        u64 tlo, thi;
        dot_wide61<S>(ys, upper(j) ? hw[g] : hk[g], tlo, thi);
        x[g][j] = mont_redc(tlo, thi, qq[g], qi[g]);  // (0, 2q): the pass takes inputs below 2q
      }
    }
  } else {
    // the constants' 30-bit pieces (Sum30: four v_mad_u64_u32 per term; sources arrive pre-split,
    // ks_split30)
    u64 h2[TG][S], h2w[TG][S];
#pragma unroll
    for (u32 g = 0; g < TG; ++g) {
#pragma unroll
      for (int k = 0; k < S; ++k) {
        const ulonglong2 h = hat[(u64)k * hs + limbs[g]];
        h2[g][k] = split30(h.x);
        h2w[g][k] = split30(h.y);
      }
    }
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      const u64 i = (u64)(tp | Lay0::jpos(j)) * G::R2;
      u64 ys[S];
#pragma unroll
      for (int k = 0; k < S; ++k) ys[k] = yb[dg.o[k] + i];
#pragma unroll
      for (u32 g = 0; g < TG; ++g) {
        Sum30 acc;
#pragma unroll
        for (int k = 0; k < S; ++k) acc.add(ys[k], upper(j) ? h2w[g][k] : h2[g][k]);
        const ModParams& mg = mods[limbs[g]];
        x[g][j] = acc.mont_lazy(mg.q, mg.qinv);  // [0, 2q): the pass takes inputs below 2q
      }
    }
  }
  // mad-chain remainders (CHAIN) although this is a column pass: unlike the latency-bound column
  // passes of the NTTs, this one is VALU-bound (the conversion products): ModUp -1.1 %, ModDown
  // conversion pass -1 % same-box (profiles/r03_modup_chain_ab.txt)
  static_for<0, (int)TG>([&](auto gc) {
    constexpr int g = decltype(gc)::value;
    if (!live[g]) return;  // workgroup-uniform
    if (g > 0) __syncthreads();  // the previous target's exchange reads are done
    const u32 lg = __builtin_amdgcn_readfirstlane(limbs[g]);
    const u32 rg = __builtin_amdgcn_readfirstlane(rr[g]);
    pass_run<G::N1, true, kNotFinal, kBlockSync, false, H, 2, false, true, G::HALF_C, true>(
        x[g], GView<G::R2, false, kKsNT>{ext + (u64)b * rn + (u64)rg * N + (u64)tile * G::SUBS_C, sub},
        lv, t, tw_all + (u64)lg * N, 1u, mods[lg].q, {0, 0}, {0, 0});
  });
}

// ModDown's last step fused into the row-forward pass of the conversion NTT (key-switch):
// conv [2][batch][nq][N] arrives column-passed; each row finishes its forward NTT in registers
// and, instead of storing NTT(conv), stores out_h = (acc_h - NTT(conv_h)) P^-1 mod q straight into
// ks0 / ks1 [batch][nq][N] (acc_h [batch][rows][N], its own Q-limb rows first).  Saves the
// NTT-form conv round trip and the separate finish pass (rns.hip k_moddown_finish).
struct FinishView {
  u64* out;
  const u64* acc;
  const u64* add;  // the KsEpilogue's addend rows, or null
  u32 lane;
  u64 q;
  ulonglong2 pinv;
  u32 gal = 0;    // != 0: the addend is read through sigma_gal (hoisted rotation: sigma(c0))
  u32 rbase = 0;  // slot of add[0] within its poly
  u32 log_n = 0;
  __device__ __forceinline__ u64 fin(u64 a, u64 x) const {
    return csub(shoup_lazy(a + q - x, pinv.x, pinv.y, q), q);
  }
  __device__ __forceinline__ u32 gal_src(u32 i) const {
    const u32 sh = 32 - log_n;
    const u32 g = ((2 * (__builtin_bitreverse32(i) >> sh) + 1) * gal) & ((2u << log_n) - 1);
    return __builtin_bitreverse32((g - 1) >> 1) >> sh;
  }
  __device__ __forceinline__ u64x2_t plus(u64x2_t r, u32 off) const {
    if (!add) return r;  // kernel-argument uniform
    u64x2_t a;
    if (gal) {  // kernel-argument uniform; the sources of a row stay inside its aligned block
      const __attribute__((address_space(1))) u64* base =
          (const __attribute__((address_space(1))) u64*)(add - rbase);
      a = u64x2_t{base[gal_src(rbase + off)], base[gal_src(rbase + off + 1)]};
    } else {
      a = *(const __attribute__((address_space(1))) u64x2_t*)(add + off);
    }
    return u64x2_t{csub(r.x + a.x, q), csub(r.y + a.y, q)};
  }
  template <class Lay>
  __device__ __forceinline__ void store(const u64 (&x)[kE], u32 tp) const {
    static_assert(contiguous16<Lay>(), "the last forward row round is contiguous");
    const u32 off = lane + tp;
    const gptr_u128 a = (gptr_u128)(acc + off);
    const gptr_u128 o = (gptr_u128)(out + off);
#pragma unroll
    for (int j = 0; j < kE / 2; ++j) {
      const u64x2_t av = a[j];
      o[j] = plus(u64x2_t{fin(av.x, x[2 * j]), fin(av.y, x[2 * j + 1])}, off + 2 * j);
    }
  }
  struct Pre {
    u64x2_t a[kE / 2];
  };
  template <u32 TPS>
  __device__ __forceinline__ Pre pre_lin(u32 t) const {
    Pre pre;
    const gptr_u128 a = (gptr_u128)(acc + lane) + t;
#pragma unroll
    for (int jj = 0; jj < kE / 2; ++jj) pre.a[jj] = a[jj * TPS];
    return pre;
  }
  template <u32 TPS>
  __device__ __forceinline__ void store_lin(const u64 (&x)[kE], u32 t, const Pre& pa) const {
    const gptr_u128 o = (gptr_u128)(out + lane) + t;
#pragma unroll
    for (int jj = 0; jj < kE / 2; ++jj) {
      const u64x2_t av = pa.a[jj];
      o[jj * TPS] = plus(u64x2_t{fin(av.x, x[2 * jj]), fin(av.y, x[2 * jj + 1])},
                         lane + 2 * (t + jj * TPS));
    }
  }
};

template <int LOGN, int H>
__global__ FHE_KATTR void k_moddown_row(const u64* __restrict__ conv, u64* __restrict__ ks0,
                                        u64* __restrict__ ks1, const u64* __restrict__ acc,
                                        u64 acc_ws, u32 rows, u32 nq, u32 limb0, u32 batch,
                                        u32 items, u32 halves,
                                        const ulonglong2* __restrict__ pinv,
                                        const ulonglong2* __restrict__ tw_all,
                                        const ModParams* __restrict__ mods, KsEpilogue ep) {
  using G = Geo<LOGN>;
  constexpr u64 N = 1ull << LOGN;
  __shared__ u64 lds[G::LDS_R];
  const u32 t = threadIdx.x % G::TPS_R, sub = threadIdx.x / G::TPS_R;
  const LView<1, true> lv{lds + sub * G::RS};
  const u32 it = blockIdx.x;
  if (it >= items) return;
  (void)halves;  // items = nq * halves * batch * TILES_R
  u32 l, rest;
  xcd_limb_split(it, nq, items / nq, l, rest);
  const u32 p = rest / G::TILES_R, tile = rest % G::TILES_R;  // tile fastest, as k_ntt_row
  const u32 h = p / batch, b = p % batch;
  const u32 row0 = tile * G::SUBS_R;
  const u32 limb = __builtin_amdgcn_readfirstlane(limb0 + l);
  const u64 q = mods[limb].q;
  const u32 lane = sub * G::R2;
  const u64 rloc = (u64)row0 * G::R2;
  u64 x[kE];
  pass_load<G::N2, true>(GView<1>{const_cast<u64*>(conv) + ((u64)p * nq + l) * N + rloc, lane}, t,
                         x);
  const u64* add = h ? ep.add1 : ep.add0;
  const FinishView fo{(h ? ks1 : ks0) + (u64)b * ep.out_bs + (u64)l * N + rloc,
                      acc + (h ? acc_ws : 0) + ((u64)b * rows + l) * N + rloc,
                      add ? add + (u64)b * ep.add_bs + (u64)l * N + rloc : nullptr, lane, q,
                      pinv[limb], ep.add_gal, (u32)rloc, (u32)LOGN};
  // column-passed by k_modup_col (inputs below 2q) or k_ntt_col (below q)
  pass_run<G::N2, true, kFinalFwd, kWaveSync, true, H, fwd_range(2, G::N1, H), true>(
      x, fo, lv, t, tw_all + (u64)limb * N, (u32)G::R1 + row0 + sub, q, {0, 0}, {0, 0});
}

// Fused key-switch row kernel: the row-forward NTT of every ModUp digit plus the inner product
// with the evaluation key, so the extended digits never go back to HBM in NTT form and no separate
// inner-product pass re-reads them (SURVEY §8a' key-switch; the unfused path is k_ntt_row per digit
// + k_ks_inner in rns.hip).  Workgroup = (row r of Q u P, ciphertext b, tile of H::ROWS rows of the
// R1 x R2 view); thread group g = digit j (whole wavefronts, as in k_hommult_row):
//   * if row r's limb belongs to digit j, its value is d2 itself: the NTT-form d2_own row, loaded;
//   * else ext_j's column-forward row: the row-forward stages run in registers / LDS, with no
//     final reduction (the products are accumulated as 128-bit integers, any 64-bit operand);
// all digits publish to LDS slot j; then every thread combines 4 of its 16 positions for both
// outputs: acc{0,1} = sum_j x_j * evk{b,a}[j][r] (128-bit sums of DNUM products, one reduce128).
// Rows: r < nq -> own Q-limb base0 + r, else special limb base1 + (r - nq).
// MONT (lz16 only): the ext rows arrive times R = 2^64 (k_modup_col with d_modup_hat_rw), the own
// digit's d2 rows are taken times R here (by its otherwise idle wave), and each output is one
// subtractive REDC of the 128-bit sum (R^-1 cancels the factor) plus one subtraction, instead of
// reduce128's two Shoup products and three subtractions.
// PINV != 0 (ModDown follows, rns.hip fused_down): the special rows (r >= nq) of both
// accumulators take the first pass of ModDown's INTT here, the inverse row pass, while the
// workgroup still holds whole rows; they are stored row-inverted, and only the column inverse is
// left to launch (launch_ntt_col_inv): no separate row-pass launch and no HBM round trip for it.
template <int LOGN, int HR, int DNUM, bool MONT = false>
__global__ FHE_KATTR void k_ks_row_inner(u64* __restrict__ acc, u64 acc_ws,
                                         const u64* __restrict__ ext, u64 ext_ds,
                                         const u64* __restrict__ d2_own,
                                         const u64* __restrict__ evk_b,
                                         const u64* __restrict__ evk_a, u32 rows, u32 nq,
                                         u32 row0, u32 nrows,
                                         u32 base0, u32 base1, u32 alpha, u32 L, u32 batch,
                                         u32 pinv, const ulonglong2* __restrict__ rscale,
                                         const ulonglong2* __restrict__ twf,
                                         const ulonglong2* __restrict__ twi,
                                         const ModParams* __restrict__ mods) {
  static_assert(DNUM >= 1 && DNUM <= 4, "one thread group per digit, four groups");
  using G = Geo<LOGN>;
  using H = HmGeo<LOGN>;
  using Rd = Rounds<G::N2>;
  constexpr u64 N = 1ull << LOGN;
  __shared__ u64 lds[H::ROWS * H::ROWW];
  // Placement: tile t goes to XCD t mod 8, and the 8 XCDs sweep one (row, ciphertext) together,
  // the TILES / 8 tiles of each XCD back to back, ciphertexts of a row next: a row's ext words
  // stream contiguously, and an XCD's share of the row's key words and twiddles (its tiles) stays
  // in its L2 for all `batch` ciphertexts.  (Ciphertext fastest per (row, tile), round 2: this
  // kernel 3.5 % slower, profiles/r03_row_order_ab.txt.)  gridDim.x = rows * TILES * batch.
  u32 b, r, tile;
  if (H::TILES % 8 == 0) {
    const u32 xcd = blockIdx.x % 8, k8 = blockIdx.x / 8;
    constexpr u32 T8 = H::TILES / 8;
    tile = xcd + 8 * (k8 % T8);
    const u32 rb = k8 / T8;
    b = rb % batch;
    r = row0 + rb / batch;
  } else {  // small N: too few tiles to deal out by XCD
    r = row0 + blockIdx.x % nrows;
    b = (blockIdx.x / nrows) % batch;
    tile = blockIdx.x / (nrows * batch);
  }
  const u32 limb = r < nq ? base0 + r : base1 + (r - nq);
  const ModParams m = mods[limb];
  const u64 q = m.q;
  const u64 rn = (u64)rows * N;
  // digit-major thread groups (whole wavefronts), as k_hommult_row's poly-major layout
  const u32 grp = __builtin_amdgcn_readfirstlane(threadIdx.x / (H::ROWS * H::TPS));
  const u32 sub = (threadIdx.x / H::TPS) % H::ROWS, t = threadIdx.x % H::TPS;
  const u32 row = tile * H::ROWS + sub;
  const u64 loc = (u64)row * G::R2;
  const u32 base = (u32)G::R1 + row;
  u64* rowlds = lds + sub * H::ROWW;
  const LView<1, true> own_slot{rowlds + grp * G::RS};
  constexpr int SY = H::SYNC_ROUND;
  using LayT = Layout<G::N2, Rd::kb(Rd::NR - 1), Rd::lo_fwd(Rd::NR - 1)>;
  const u32 tpT = LayT::tpos(t);
  const bool is_own = limb < L && grp == limb / alpha;  // wave-uniform
  u64 v[kE];
  if (grp < (u32)DNUM) {
    if (is_own) {
      // d2 is already in NTT form: straight into the LDS slot, read in linear order
      const GView<1> gin{const_cast<u64*>(d2_own) + ((u64)b * nq + r) * N + loc, 0};
      gin.template load_lin<H::TPS>(v, t);
      if constexpr (MONT) {
        // v R mod q into [0, 2q) (Shoup by R mod q: [0, 3q), one subtraction): the inner
        // product's operands must stay below 2^61.  (R P^-1 with rscale: ModDown's P^-1 folded)
        const u64 nq = 0 - q;
        const ulonglong2 rs = rscale ? rscale[limb] : make_ulonglong2(m.r64, m.r64s);
#pragma unroll
        for (int j = 0; j < kE; ++j) v[j] = csubk(shoup_q3(v[j], rs.x, rs.y, nq), q);
      }
#pragma unroll
      for (int jj = 0; jj < kE / 2; ++jj) {
        const u32 p = 2 * t + 2 * H::TPS * jj;
        own_slot.s[own_slot.idx(p)] = v[2 * jj];
        own_slot.s[own_slot.idx(p + 1)] = v[2 * jj + 1];
      }
    } else {
      const ulonglong2* tf = twf + (u64)limb * N;
      static_for<0, Rd::NR>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int KB = Rd::kb(k);
        constexpr int LO = Rd::lo_fwd(k);
        // column-passed by k_modup_col (inputs below 2q: mont_lazy) or k_ntt_col (below q)
        constexpr int RIN = fwd_range(fwd_range(2, G::N1, HR), G::N2 - (LO + KB), HR);
        using Lay = Layout<G::N2, KB, LO>;
        const u32 tp = Lay::tpos(t);
        if constexpr (k == 0) {
          const GView<1, kKsNT> gin{const_cast<u64*>(ext) + (u64)grp * ext_ds + (u64)b * rn + (u64)r * N + loc, 0};
          gin.template load<Lay>(v, tp);
        } else {
          lds_sync<SY>();
          own_slot.template load<Lay>(v, tp);
        }
        // lz16: the last round reduces to [0, 2q) for the hand-written inner product (dot_wide61)
        constexpr int F = (HR == 16 && k == Rd::NR - 1) ? kFinalFwd2 : kNotFinal;
        round_compute<G::N2, KB, LO, true, F, true, HR, RIN>(v, tp, tf, base, q, {0, 0}, {0, 0});
        if constexpr (k < Rd::NR - 1) {
          if (k > 0) lds_sync<SY>();
          own_slot.template store<Lay>(v, tp);
        }
      });
      lds_sync<SY>();
      own_slot.template store<LayT>(v, tpT);
    }
  }
  // combine: the workgroup's ROWS x R2 positions are re-dealt so that each thread takes CW
  // consecutive positions of one row and a wavefront covers contiguous words (coalesced 16-byte
  // key loads and output stores).  The key words do not depend on the other digits' rows, so
  // every thread issues its loads before the barrier: they are in flight while the slower
  // digits finish their NTTs (and the own digit's wave, which only loaded d2, waits for them).
  constexpr int CW = (H::ROWS * G::R2) / H::THR;
  static_assert(CW == 4 || CW == 2 || CW == 8, "combine width");
  const u32 cpos0 = threadIdx.x * CW;
  const u32 crow = cpos0 / G::R2, cpos = cpos0 % G::R2;
  const u64 okey = (u64)r * N + (u64)(tile * H::ROWS + crow) * G::R2 + cpos;
  const u64* lrow = lds + crow * H::ROWW;
  u64x2_t kbv[CW / 2][DNUM], kav[CW / 2][DNUM];
#pragma unroll
  for (int e = 0; e < CW; e += 2) {
#pragma unroll
    for (int d = 0; d < DNUM; ++d) {
      kbv[e / 2][d] = *(const __attribute__((address_space(1))) u64x2_t*)(evk_b + (u64)d * rn + okey + e);
      kav[e / 2][d] = *(const __attribute__((address_space(1))) u64x2_t*)(evk_a + (u64)d * rn + okey + e);
    }
  }
  __syncthreads();
  u64 o0[CW], o1[CW];
  u64 qi = 0 - m.qinv;  // q^-1 mod 2^64 (MONT)
  asm("" : "+s"(qi));
  if constexpr (HR == 16) {
#pragma unroll
    for (int e = 0; e < CW; e += 2) {
      u64 x0[DNUM], x1[DNUM], kb0[DNUM], kb1[DNUM], ka0[DNUM], ka1[DNUM];
#pragma unroll
      for (int d = 0; d < DNUM; ++d) {
        const u64x2_t kb = kbv[e / 2][d], ka = kav[e / 2][d];
        const u32 p = cpos + e;
        x0[d] = lrow[d * G::RS + p + (p >> 4)];
        x1[d] = lrow[d * G::RS + (p + 1) + ((p + 1) >> 4)];
        kb0[d] = kb.x;
        kb1[d] = kb.y;
        ka0[d] = ka.x;
        ka1[d] = ka.y;
      }
      u64 tl, th;
      if constexpr (MONT) {
        // sum < DNUM 2q q <= 8 q^2 < q 2^64: REDC into (0, 2q), then canonical
        dot_wide61<DNUM>(x0, kb0, tl, th);
        o0[e] = csubk(mont_redc_x(tl, th, q, qi), q);
        dot_wide61<DNUM>(x1, kb1, tl, th);
        o0[e + 1] = csubk(mont_redc_x(tl, th, q, qi), q);
        dot_wide61<DNUM>(x0, ka0, tl, th);
        o1[e] = csubk(mont_redc_x(tl, th, q, qi), q);
        dot_wide61<DNUM>(x1, ka1, tl, th);
        o1[e + 1] = csubk(mont_redc_x(tl, th, q, qi), q);
      } else {
        dot_wide61<DNUM>(x0, kb0, tl, th);
        o0[e] = reduce128(tl, th, m);
        dot_wide61<DNUM>(x1, kb1, tl, th);
        o0[e + 1] = reduce128(tl, th, m);
        dot_wide61<DNUM>(x0, ka0, tl, th);
        o1[e] = reduce128(tl, th, m);
        dot_wide61<DNUM>(x1, ka1, tl, th);
        o1[e + 1] = reduce128(tl, th, m);
      }
    }
  } else {
#pragma unroll
  for (int e = 0; e < CW; e += 2) {
    u128 s0[2] = {0, 0}, s1[2] = {0, 0};
#pragma unroll
    for (int d = 0; d < DNUM; ++d) {
      const u64x2_t kb = kbv[e / 2][d], ka = kav[e / 2][d];
      const u32 p = cpos + e;
      const u64 x0 = lrow[d * G::RS + p + (p >> 4)];
      const u64 x1 = lrow[d * G::RS + (p + 1) + ((p + 1) >> 4)];
      s0[0] += (u128)x0 * kb.x;
      s0[1] += (u128)x1 * kb.y;
      s1[0] += (u128)x0 * ka.x;
      s1[1] += (u128)x1 * ka.y;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      o0[e + h] = reduce128((u64)s0[h], (u64)(s0[h] >> 64), m);
      o1[e + h] = reduce128((u64)s1[h], (u64)(s1[h] >> 64), m);
    }
  }
  }
  if (pinv && r >= nq) {  // workgroup-uniform
    // o0 / o1 of row crow -> slots 0 / 1 of that row in linear order (every wave's combine reads
    // are done first); then wave h runs the inverse row pass of accumulator h's 4 rows
    static_assert(CW == 4 && H::ROWS * H::TPS == 64, "one row per wave in the combine");
    const LView<1, true> s0{lds + crow * H::ROWW}, s1{lds + crow * H::ROWW + G::RS};
    __syncthreads();
#pragma unroll
    for (int e = 0; e < CW; ++e) {
      s0.s[s0.idx(cpos + e)] = o0[e];
      s1.s[s1.idx(cpos + e)] = o1[e];
    }
    __syncthreads();
    const u32 h = threadIdx.x / 64;  // wave index (uniform)
    if (h < 2) {
      using Lay0 = Layout<G::N2, Rd::kb_inv(0), Rd::lo_inv(0)>;
      const LView<1, true> lv{rowlds + h * G::RS};
      u64 x[kE];
      lv.template load<Lay0>(x, Lay0::tpos(t));
      pass_run<G::N2, false, kNotFinal, kWaveSync, true, HR, fwd_range(1, G::N1, HR)>(
          x, GView<1>{acc + h * acc_ws + (u64)b * rn + (u64)r * N + loc, 0}, lv, t,
          twi + (u64)limb * N, base, q, {0, 0}, {0, 0});
    }
    return;
  }
  gptr_u128 a0 = (gptr_u128)(acc + (u64)b * rn + okey);
  gptr_u128 a1 = (gptr_u128)(acc + acc_ws + (u64)b * rn + okey);
#pragma unroll
  for (int e = 0; e < CW; e += 2) {
    a0[e / 2] = u64x2_t{o0[e], o0[e + 1]};
    a1[e / 2] = u64x2_t{o1[e], o1[e + 1]};
  }
}

// The key-switch's Q rows with ModDown's finish in the same workgroup (lz16 contexts with P^-1
// folded into the constants, rns.hip pscale): launched after the special rows (k_ks_row_inner
// with PINV over rows [nq, rows)) and ModDown's conversion (k_modup_col: conv [2][batch][nq][N],
// column-passed), so NTT(conv) can be taken here instead of in k_moddown_row, and the
// accumulators' Q rows never go to HBM:
//   * the own digit's wave, which had only d2 to load, runs conv_0's row-forward pass into its LDS
//     slot; the combine reads the own digit's d2 words straight from global memory (times R P^-1);
//   * out_0 = acc_0 - NTT(conv_0) mod q (+ the epilogue's addend) is stored at once, acc_1 stays in
//     registers while one wave (an idle one when DNUM < 4, else wave 0 after a barrier) runs
//     conv_1's row-forward pass, then out_1.
// Same placement and thread groups as k_ks_row_inner; gridDim.x = nq * TILES * batch.
template <int LOGN, int DNUM>
__global__ FHE_KATTR void k_ks_row_fin(const u64* __restrict__ ext, u64 ext_ds,
                                       const u64* __restrict__ d2_own,
                                       const u64* __restrict__ evk_b,
                                       const u64* __restrict__ evk_a, u32 rows, u32 nq,
                                       u32 base0, u32 alpha, u32 L, u32 batch,
                                       const ulonglong2* __restrict__ rscale,
                                       const u64* __restrict__ conv, u64* __restrict__ ks0,
                                       u64* __restrict__ ks1, KsEpilogue ep,
                                       const ulonglong2* __restrict__ twf,
                                       const ModParams* __restrict__ mods) {
  static_assert(DNUM >= 1 && DNUM <= 4, "one thread group per digit, four groups");
  constexpr int HR = 16;
  using G = Geo<LOGN>;
  using H = HmGeo<LOGN>;
  using Rd = Rounds<G::N2>;
  constexpr u64 N = 1ull << LOGN;
  __shared__ u64 lds[H::ROWS * H::ROWW];
  u32 b, r, tile;
  if (H::TILES % 8 == 0) {
    const u32 xcd = blockIdx.x % 8, k8 = blockIdx.x / 8;
    constexpr u32 T8 = H::TILES / 8;
    tile = xcd + 8 * (k8 % T8);
    const u32 rb = k8 / T8;
    b = rb % batch;
    r = rb / batch;
  } else {
    r = blockIdx.x % nq;
    b = (blockIdx.x / nq) % batch;
    tile = blockIdx.x / (nq * batch);
  }
  const u32 limb = base0 + r;  // a Q row: its limb is this rank's own
  const ModParams m = mods[limb];
  const u64 q = m.q;
  const u64 rn = (u64)rows * N;
  const u32 grp = __builtin_amdgcn_readfirstlane(threadIdx.x / (H::ROWS * H::TPS));
  const u32 sub = (threadIdx.x / H::TPS) % H::ROWS, t = threadIdx.x % H::TPS;
  const u32 row = tile * H::ROWS + sub;
  const u64 loc = (u64)row * G::R2;
  const u32 base = (u32)G::R1 + row;
  u64* rowlds = lds + sub * H::ROWW;
  constexpr int SY = H::SYNC_ROUND;
  using LayT = Layout<G::N2, Rd::kb(Rd::NR - 1), Rd::lo_fwd(Rd::NR - 1)>;
  const u32 tpT = LayT::tpos(t);
  const u32 od = __builtin_amdgcn_readfirstlane(limb / alpha);  // the own digit (< DNUM)
  const ulonglong2* tf = twf + (u64)limb * N;
  // row-forward pass of a column-passed row (inputs below 2q) into LDS slot `slot`; FIN: the last
  // round's reduction (canonical for conv, [0, 2q) for the inner product's operands)
  auto row_fwd = [&](const u64* src, u32 slot, auto fin) {
    constexpr int FINAL = decltype(fin)::value;
    const LView<1, true> sl{rowlds + slot * G::RS};
    u64 v[kE];
    static_for<0, Rd::NR>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int KB = Rd::kb(k);
      constexpr int LO = Rd::lo_fwd(k);
      constexpr int RIN = fwd_range(fwd_range(2, G::N1, HR), G::N2 - (LO + KB), HR);
      using Lay = Layout<G::N2, KB, LO>;
      const u32 tp = Lay::tpos(t);
      if constexpr (k == 0) {
        const GView<1, kKsNT> gin{const_cast<u64*>(src) + loc, 0};
        gin.template load<Lay>(v, tp);
      } else {
        lds_sync<SY>();
        sl.template load<Lay>(v, tp);
      }
      constexpr int F = k == Rd::NR - 1 ? FINAL : kNotFinal;
      round_compute<G::N2, KB, LO, true, F, true, HR, RIN>(v, tp, tf, base, q, {0, 0}, {0, 0});
      if constexpr (k < Rd::NR - 1) {
        if (k > 0) lds_sync<SY>();
        sl.template store<Lay>(v, tp);
      }
    });
    lds_sync<SY>();
    sl.template store<LayT>(v, tpT);
  };
  using FinC = std::integral_constant<int, kFinalFwd>;
  using FinX = std::integral_constant<int, kFinalFwd2>;
  const u64* conv0 = conv + ((u64)b * nq + r) * N;
  const u64* conv1 = conv + ((u64)(batch + b) * nq + r) * N;
  if (grp < (u32)DNUM) {
    if (grp == od) row_fwd(conv0, grp, FinC{});
    else row_fwd(ext + (u64)grp * ext_ds + (u64)b * rn + (u64)r * N, grp, FinX{});
  } else if (grp == (u32)DNUM) {
    row_fwd(conv1, grp, FinC{});  // an idle wave (DNUM < 4) takes conv_1 now
  }
  // combine operands: keys and the own digit's d2 words, issued before the barrier
  constexpr int CW = (H::ROWS * G::R2) / H::THR;
  static_assert(CW == 4 && H::ROWS * H::TPS == 64, "one row per wave in the combine");
  const u32 cpos0 = threadIdx.x * CW;
  const u32 crow = cpos0 / G::R2, cpos = cpos0 % G::R2;
  const u64 orow = (u64)(tile * H::ROWS + crow) * G::R2 + cpos;  // position within the poly
  const u64 okey = (u64)r * N + orow;
  u64* lrow = lds + crow * H::ROWW;
  u64x2_t kbv[CW / 2][DNUM], kav[CW / 2][DNUM], dv[CW / 2];
#pragma unroll
  for (int e = 0; e < CW; e += 2) {
#pragma unroll
    for (int d = 0; d < DNUM; ++d) {
      kbv[e / 2][d] = *(const __attribute__((address_space(1))) u64x2_t*)(evk_b + (u64)d * rn + okey + e);
      kav[e / 2][d] = *(const __attribute__((address_space(1))) u64x2_t*)(evk_a + (u64)d * rn + okey + e);
    }
    dv[e / 2] = *(const __attribute__((address_space(1))) u64x2_t*)(d2_own + ((u64)b * nq + r) * N + orow + e);
  }
  __syncthreads();
  u64 qi = 0 - m.qinv;  // q^-1 mod 2^64
  asm("" : "+s"(qi));
  const ulonglong2 rs = rscale[limb];  // R P^-1 mod q
  const u64 nqm = 0 - q;
  auto at = [&](u32 slot, u32 p) { return lrow[slot * G::RS + p + (p >> 4)]; };
  u64 o1[CW], f0[CW];
#pragma unroll
  for (int e = 0; e < CW; e += 2) {
    u64 x0[DNUM], x1[DNUM], kb0[DNUM], kb1[DNUM], ka0[DNUM], ka1[DNUM];
    // the own digit's slot holds NTT(conv_0): its operand is d2 R P^-1 instead, in [0, 2q)
    const u64 xo0 = csubk(shoup_q3(dv[e / 2].x, rs.x, rs.y, nqm), q);
    const u64 xo1 = csubk(shoup_q3(dv[e / 2].y, rs.x, rs.y, nqm), q);
#pragma unroll
    for (int d = 0; d < DNUM; ++d) {
      const u64x2_t kb = kbv[e / 2][d], ka = kav[e / 2][d];
      const u32 p = cpos + e;
      x0[d] = (u32)d == od ? xo0 : at(d, p);
      x1[d] = (u32)d == od ? xo1 : at(d, p + 1);
      kb0[d] = kb.x;
      kb1[d] = kb.y;
      ka0[d] = ka.x;
      ka1[d] = ka.y;
    }
    u64 tl, th;
    // sum < DNUM 2q q <= 8 q^2 < q 2^64: REDC into (0, 2q), then canonical
    dot_wide61<DNUM>(x0, kb0, tl, th);
    const u64 a00 = csubk(mont_redc_x(tl, th, q, qi), q);
    dot_wide61<DNUM>(x1, kb1, tl, th);
    const u64 a01 = csubk(mont_redc_x(tl, th, q, qi), q);
    dot_wide61<DNUM>(x0, ka0, tl, th);
    o1[e] = csubk(mont_redc_x(tl, th, q, qi), q);
    dot_wide61<DNUM>(x1, ka1, tl, th);
    o1[e + 1] = csubk(mont_redc_x(tl, th, q, qi), q);
    // out_0 = acc_0 - NTT(conv_0): both already carry P^-1
    f0[e] = csub(a00 + q - at(od, cpos + e), q);
    f0[e + 1] = csub(a01 + q - at(od, cpos + e + 1), q);
  }
  const u64 rloc = (u64)tile * H::ROWS * G::R2;
  const u64 obase = (u64)b * ep.out_bs + (u64)r * N + rloc;
  const u64 abase = (u64)b * ep.add_bs + (u64)r * N + rloc;
  const u32 off = crow * G::R2 + cpos;
  auto emit = [&](u64* out, const u64* add, const u64 (&f)[CW]) {
    const FinishView fv{out + obase, nullptr, add ? add + abase : nullptr, 0, q, {0, 0},
                        ep.add_gal, (u32)rloc, (u32)LOGN};
    const gptr_u128 o = (gptr_u128)(out + obase + off);
#pragma unroll
    for (int e = 0; e < CW; e += 2) o[e / 2] = fv.plus(u64x2_t{f[e], f[e + 1]}, off + e);
  };
  emit(ks0, ep.add0, f0);
  u64 f1[CW];
  if constexpr (DNUM == 4) {
    // acc_1 waits in slot 1 (free once every combine read is done) while wave 0 runs conv_1's
    // row pass into slot 0: no registers held across that pass
    __syncthreads();
#pragma unroll
    for (int e = 0; e < CW; ++e) lrow[1 * G::RS + (cpos + e) + ((cpos + e) >> 4)] = o1[e];
    if (grp == 0) row_fwd(conv1, 0u, FinC{});
    __syncthreads();
#pragma unroll
    for (int e = 0; e < CW; ++e) f1[e] = csub(at(1, cpos + e) + q - at(0, cpos + e), q);
  } else {
#pragma unroll
    for (int e = 0; e < CW; ++e) f1[e] = csub(o1[e] + q - at(DNUM, cpos + e), q);
  }
  emit(ks1, ep.add1, f1);
}

// One workgroup per item, rounded up to a multiple of 8 so item -> XCD placement holds (surplus
// workgroups exit at once).
inline u64 item_blocks(u64 items) { return (items + 7) / 8 * 8; }
inline dim3 item_grid(u64 items) { return dim3((u32)item_blocks(items)); }

// The inverse passes' H: the lazy inverse does not depend on the forward headroom (one build for
// H = 8 and 16); wide contexts (H = 2) take the exact one.
constexpr int inv_h(int hd) { return hd; }

// Row pass of a standalone NTT over [polys][nlimbs][N] (src poly stride sp -> dst stride dp).
template <int LOGN, int HD>
void row_pass(const fhe_ctx* c, bool fwd, const u64* src, u64 sp, u64* dst, u64 dp, u32 polys,
              u32 limb0, u32 nlimbs, hipStream_t s) {
  using G = Geo<LOGN>;
  const u64 ir = (u64)polys * nlimbs * G::TILES_R;
  const PolyMap pm{1, sp, 0, dp, 0, 0};
  const ulonglong2* twf = c->d_tw_fwd;
  const ulonglong2* twi = c->d_tw_inv;
  if (fwd)  // the forward's second pass
    k_ntt_row<LOGN, true, HD>
        <<<item_grid(ir), G::THR_R,
           0, s>>>(src, dst, nlimbs, limb0, pm, (u32)ir, twf, c->d_mods);
  else  // the inverse's first pass
    k_ntt_row<LOGN, false, inv_h(HD)>
        <<<item_grid(ir), G::THR_R,
           0, s>>>(src, dst, nlimbs, limb0, pm, (u32)ir, twi, c->d_mods);
}

#if !FHE_NTT_KS_ONLY
template <int LOGN, int HD>
int ntt_dispatch(const fhe_ctx* c, bool fwd, const u64* src, u64 spstride, u64* dst,
                 u64 dpstride, u32 polys, u32 limb0, u32 nlimbs, hipStream_t s,
                 const ulonglong2* nfold, bool split) {
  using G = Geo<LOGN>;
  const u64 pl = (u64)polys * nlimbs;
  const PolyMap pm{1, spstride, 0, dpstride, 0, 0};
  // the second pass runs in place on dst
  const PolyMap pd = flat_map(dpstride);
  const u64 ic = pl * G::TILES_C;
  if (int rc = check_grid(item_blocks(ic), G::THR_C, 1, 1, "ntt")) return rc;
  if (int rc = check_grid(item_blocks(pl * G::TILES_R), G::THR_R, 1, 1, "ntt")) return rc;
  // Transforms far larger than the Infinity Cache (configs[4]: 32 GiB per call) stream every
  // access (non-temporal loads and stores in both passes): the intermediate is evicted before the
  // row pass reads it anyway.  configs[4] forward 1.139-1.140 -> 1.204-1.205 M NTT/s same-box
  // (+5.7 %; only the column pass's source / the row pass's output streamed: +3 %;
  // profiles/r05_ntt_stream_ab.txt).  Smaller ones stay cached: their second pass re-reads the
  // first pass's output from the Infinity Cache (non-temporal there: -5 ... -8 %, round 3).
  const bool stream = pl * G::R1 * G::R2 * 8 > (1ull << 30);
  if (fwd && stream) {
    k_ntt_col<LOGN, true, HD, true, true>
        <<<item_grid(ic),
           G::THR_C, 0, s>>>(src, nullptr, dst, nlimbs, limb0, pm, (u32)ic, c->d_tw_fwd,
                             c->d_nfold, c->d_mods);
    prof_mark(s, "ntt_col_fwd");
    const u64 ir = pl * G::TILES_R;
    k_ntt_row<LOGN, true, HD, true, true>
        <<<item_grid(ir), G::THR_R,
           0, s>>>(dst, dst, nlimbs, limb0, pd, (u32)ir, c->d_tw_fwd, c->d_mods);
    prof_mark(s, "ntt_row_fwd");
  } else if (fwd) {
    k_ntt_col<LOGN, true, HD>
        <<<item_grid(ic),
           G::THR_C, 0, s>>>(src, nullptr, dst, nlimbs, limb0, pm, (u32)ic, c->d_tw_fwd,
                             c->d_nfold, c->d_mods);
    prof_mark(s, "ntt_col_fwd");
    row_pass<LOGN, HD>(c, true, dst, dpstride, dst, dpstride, polys, limb0, nlimbs, s);
    prof_mark(s, "ntt_row_fwd");
  } else {
    // the inverse streams the same way above 1 GiB (plain outputs; the split30 form feeds the
    // key-switch, whose passes stay below 256 MiB): 4 GiB same-box, row pass -2.8 %, column pass
    // -4.6 % (profiles/r05_intt_stream.txt)
    const bool stream_inv = stream && !split;
    if (stream_inv) {
      const u64 ir = pl * G::TILES_R;
      k_ntt_row<LOGN, false, inv_h(HD), true, true>
          <<<item_grid(ir), G::THR_R, 0, s>>>(src, dst, nlimbs, limb0, pm, (u32)ir, c->d_tw_inv,
                                              c->d_mods);
    } else {
      row_pass<LOGN, HD>(c, false, src, spstride, dst, dpstride, polys, limb0, nlimbs, s);
    }
    prof_mark(s, "ntt_row_inv");
    const ulonglong2* nf = nfold ? nfold : c->d_nfold;
    if constexpr (HD != 2) {
      if (split) {  // outputs for k_modup_col only (narrow contexts: split30 needs x < 2^61)
        k_ntt_col<LOGN, false, inv_h(HD), false, false, kFinalInvS30>
            <<<item_grid(ic), G::THR_C, 0, s>>>(dst, nullptr, dst, nlimbs, limb0, pd, (u32)ic,
                                                c->d_tw_inv, nf, c->d_mods);
        prof_mark(s, "ntt_col_inv");
        FHE_HIP_CHECK(hipGetLastError());
        return kOk;
      }
    } else if (split) {
      set_error("split30 INTT outputs need every modulus < 2^61");
      return kUnsupported;
    }
    if (stream_inv) {
      k_ntt_col<LOGN, false, inv_h(HD), true, true>
          <<<item_grid(ic), G::THR_C, 0, s>>>(dst, nullptr, dst, nlimbs, limb0, pd, (u32)ic,
                                              c->d_tw_inv, nf, c->d_mods);
      prof_mark(s, "ntt_col_inv");
      FHE_HIP_CHECK(hipGetLastError());
      return kOk;
    }
    k_ntt_col<LOGN, false, inv_h(HD)>
        <<<item_grid(ic),
           G::THR_C, 0, s>>>(dst, nullptr, dst, nlimbs, limb0, pd, (u32)ic, c->d_tw_inv, nf,
                             c->d_mods);
    prof_mark(s, "ntt_col_inv");
  }
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}

template <int LOGN, int HD>
int hommult_dispatch(const fhe_ctx* c, u64* d, const u64* a, const u64* b, u32 batch, u32 limb0,
                     u32 nlimbs, u64* x, hipStream_t s) {
  using G = Geo<LOGN>;
  using H = HmGeo<LOGN>;
  constexpr u64 N = 1ull << LOGN;
  const u64 limbN = (u64)nlimbs * N;
  // x: [batch][4][nlimbs][N] workspace; A0, A1 -> slots 0, 1; B0, B1 -> slots 2, 3: one launch
  // over the 4 polys of every ciphertext pair (group of 4: slots 0, 1 from a, slots 2, 3 from b)
  const PolyMap to_x{4, 2 * limbN, limbN, 4 * limbN, limbN, 2};
  const u64 ic = (u64)batch * 4 * nlimbs * G::TILES_C;
  if (int rc = check_grid(item_blocks(ic), G::THR_C, 1, 1, "hommult")) return rc;
  if (int rc = check_grid((u64)batch * nlimbs * H::TILES, H::THR, 1, 1, "hommult")) return rc;
  constexpr bool FL = true;  // a, b are read once: non-temporal
  const dim3 gh((u32)((u64)batch * nlimbs * H::TILES));
  // N = 2^16: the forward split 9 + 7 (k_hm_col9: 32 elements per thread, the row kernel's
  // forward rows one stage shorter); other sizes 8 + 8 (log N / 2 each)
  bool split9 = false;
  if constexpr (LOGN == 16 && HD != 2) split9 = c->d_tw_fwd9 != nullptr;
  if (split9) {
    if constexpr (LOGN == 16 && HD != 2) {
      const u64 i9 = (u64)batch * 4 * nlimbs * kC9Tiles;
      k_hm_col9<HD><<<item_grid(i9), kColThreads, 0, s>>>(a, b, x, nlimbs, limb0, to_x, (u32)i9,
                                                          c->d_tw_fwd, c->d_mods);
      prof_mark(s, "hm_col_fwd");
      k_hommult_row<LOGN, HD, true><<<gh, H::THR, 0, s>>>(x, d, nlimbs, limb0, c->d_tw_fwd9,
                                                          c->d_tw_inv, c->d_mods);
      prof_mark(s, "hm_row_tensor");
    }
  } else {
    k_ntt_col<LOGN, true, HD, FL><<<item_grid(ic),
                                    G::THR_C, 0, s>>>(a, b, x, nlimbs, limb0, to_x, (u32)ic,
                                                      c->d_tw_fwd, c->d_nfold, c->d_mods);
    prof_mark(s, "hm_col_fwd");
    k_hommult_row<LOGN, HD><<<gh, H::THR, 0, s>>>(x, d, nlimbs, limb0, c->d_tw_fwd,
                                                      c->d_tw_inv, c->d_mods);
    prof_mark(s, "hm_row_tensor");
  }
  const u64 ii = (u64)batch * 3 * nlimbs * G::TILES_C;
  // the Montgomery tensor left a factor R^-1: fold R in with N^-1 (entries 2, 3 of d_nfold)
  k_ntt_col<LOGN, false, inv_h(HD), kHmNT, kHmNT>
      <<<item_grid(ii),
         G::THR_C, 0, s>>>(d, nullptr, d, nlimbs, limb0, flat_map(limbN), (u32)ii, c->d_tw_inv,
                           c->d_nfold + 2, c->d_mods);
  prof_mark(s, "hm_col_inv");
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}
// Rescale (NTT form): the spread of the last limb over the other limbs folded into the
// column-forward pass.  last [polys][N] holds INTT(x_last); the tile of limb l (l < nq, the last
// limb is nq) loads last's columns and spreads them in registers,
//   v = ((last + h) mod q_last - h) mod q_l,  h = q_last / 2   (galois.hip k_rescale_spread, the
// path of wide contexts)
// before the column-forward stages, writing dst [polys][nq][N]: no spread pass and no re-read of
// its output.  The row pass is k_moddown_row with the q_last^-1 table (the finish).
template <int LOGN, int H>
__global__ __launch_bounds__(kColThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) void
k_rescale_col(const u64* __restrict__ last, u64* __restrict__ dst, u32 nq, u32 items,
              const u64* __restrict__ half, const ulonglong2* __restrict__ tw_all,
              const ModParams* __restrict__ mods) {
  using G = Geo<LOGN>;
  constexpr u64 N = 1ull << LOGN;
  __shared__ u64 lds[G::LDS_CF];
  const u32 sub = threadIdx.x % G::SUBS_C, t = threadIdx.x / G::SUBS_C;
  const LViewC<G::SUBS_C> lv{lds + sub};
  const u32 it = blockIdx.x;
  if (it >= items) return;
  // placement: with 8 | polys, XCD x takes the polys p = x mod 8 and runs the nq limbs of one
  // (p, tile) back to back, so last's column tile comes from HBM once and from the XCD's L2 for
  // the other limbs; otherwise limbs fastest over all XCDs
  const u32 polys = items / (nq * G::TILES_C);
  u32 tile, l, p;
  if (polys % 8 == 0) {
    const u32 k = it / 8;
    l = k % nq;
    tile = (k / nq) % G::TILES_C;
    p = (k / (nq * G::TILES_C)) * 8 + it % 8;
  } else {
    l = it % nq;
    tile = (it / nq) % G::TILES_C;
    p = it / (nq * G::TILES_C);
  }
  l = __builtin_amdgcn_readfirstlane(l);
  const u32 pl = p * nq + l;
  const u64 col = (u64)tile * G::SUBS_C;
  u64 x[kE];
  pass_load<G::N1, true>(GView<G::R2>{const_cast<u64*>(last) + (u64)p * N + col, sub}, t, x);
  const ModParams ml = mods[nq], mi = mods[l];
  const u64 h = ml.q >> 1, mh = mi.q - half[l];
#pragma unroll
  for (int j = 0; j < kE; ++j) x[j] = csub(reduce_word(csub(x[j] + h, ml.q), mi) + mh, mi.q);
  // scheduled from 2 (inputs are below q): the range k_moddown_row assumes
  pass_run<G::N1, true, kNotFinal, kBlockSync, false, H, 2, false, false, G::HALF_C>(
      x, GView<G::R2>{dst + (u64)pl * N + col, sub}, lv, t, tw_all + (u64)l * N, 1u, mi.q,
      {0, 0}, {0, 0});
}

template <int LOGN, int HD>
int rescale_col_dispatch(const fhe_ctx* c, const u64* last, u64* dst, u32 polys, u32 nq,
                         const u64* half, hipStream_t s) {
  using G = Geo<LOGN>;
  const u64 ic = (u64)polys * nq * G::TILES_C;
  if (int rc = check_grid(item_blocks(ic), G::THR_C, 1, 1, "rescale_col")) return rc;
  k_rescale_col<LOGN, HD><<<item_grid(ic), G::THR_C, 0, s>>>(last, dst, nq, (u32)ic, half,
                                                            c->d_tw_fwd, c->d_mods);
  return kOk;
}
#endif  // !FHE_NTT_KS_ONLY

}  // namespace

#define FHE_LOGN_CASES(X) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17)

#if FHE_NTT_KS_ONLY

namespace {
// The fused key-switch kernels rely on lazy ranges and 128-bit sums that need q < 2^61; wide
// contexts take the unfused key-switch (rns.hip), which never calls these launchers.
int wide_unsupported() {
  set_error("fused key-switch kernels need every modulus < 2^61");
  return kUnsupported;
}
template <int LOGN, int HD>
int col_fwd_pass(const fhe_ctx* c, const u64* src, u64 sp, u64* dst, u64 dp, u32 polys,
                 u32 limb0, u32 nlimbs, hipStream_t s) {
  using G = Geo<LOGN>;
  const u64 ic = (u64)polys * nlimbs * G::TILES_C;
  if (int rc = check_grid(item_blocks(ic), G::THR_C, 1, 1, "ntt_col_fwd")) return rc;
  const PolyMap pm{1, sp, 0, dp, 0, 0};
  // scheduled from 2: the row kernels that follow (k_ks_row_inner, k_moddown_row) assume it
  k_ntt_col<LOGN, true, HD, false, false, kFinalInv, 2><<<item_grid(ic),
                              G::THR_C, 0, s>>>(src, nullptr, dst, nlimbs, limb0, pm, (u32)ic,
                                                c->d_tw_fwd, c->d_nfold, c->d_mods);
  return kOk;
}

template <int LOGN, int HD>
int ks_row_inner_dispatch(const fhe_ctx* c, const KsRowArgs& a, hipStream_t s) {
  using H = HmGeo<LOGN>;
  const u32 nrows = a.nrows ? a.nrows : a.rows;
  if (int rc = check_grid((u64)nrows * a.batch * H::TILES, H::THR, 1, 1, "ks_row_inner")) return rc;
  const dim3 g((u32)((u64)nrows * a.batch * H::TILES));
  switch (c->dnum) {
#define D(k)                                                                                    \
  case k:                                                                                       \
    if (HD == 16 && a.mont)                                                                     \
      k_ks_row_inner<LOGN, HD, k, HD == 16><<<g, H::THR, 0, s>>>(                               \
          a.acc, a.acc_ws, a.ext, a.ext_ds, a.d2_own, a.evk_b, a.evk_a, a.rows, a.nq, a.row0,   \
          nrows, a.base0, a.base1, a.alpha, a.L, a.batch, a.pinv, a.rscale, c->d_tw_fwd,       \
          c->d_tw_inv, c->d_mods);                                                              \
    else                                                                                        \
      k_ks_row_inner<LOGN, HD, k><<<g, H::THR, 0, s>>>(                                         \
          a.acc, a.acc_ws, a.ext, a.ext_ds, a.d2_own, a.evk_b, a.evk_a, a.rows, a.nq, a.row0,   \
          nrows, a.base0, a.base1, a.alpha, a.L, a.batch, a.pinv, a.rscale, c->d_tw_fwd,       \
          c->d_tw_inv, c->d_mods);                                                              \
    break;
    D(1) D(2) D(3) D(4)
#undef D
    default:
      set_error("ks_row_inner: dnum > 4");
      return kUnsupported;
  }
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}
}  // namespace

int launch_ntt_col_fwd(const fhe_ctx* c, const u64* src, u64 spstride, u64* dst, u64 dpstride,
                       u32 polys, u32 limb0, u32 nlimbs, hipStream_t s) {
  if ((u64)polys * nlimbs == 0) return kOk;
  if (c->wide) return wide_unsupported();
  switch (c->log_n) {
#define X(n)                                                                                 \
  case n:                                                                                    \
    if (int rc = c->lz16 ? col_fwd_pass<n, 16>(c, src, spstride, dst, dpstride, polys, limb0, \
                                                nlimbs, s)                                   \
                         : col_fwd_pass<n, 8>(c, src, spstride, dst, dpstride, polys, limb0,  \
                                              nlimbs, s))                                    \
      return rc;                                                                             \
    FHE_HIP_CHECK(hipGetLastError());                                                       \
    return kOk;
    FHE_LOGN_CASES(X)
#undef X
  }
  set_error("unsupported log_n");
  return kUnsupported;
}

// The row-forward pass over rows that k_modup_col column-passed (its schedule starts from 2):
// canonical NTT-form outputs, in place or out of place.  The hoisted ModUp (rotations, rotation sums)
// runs it over each digit's extended rows.
int launch_ntt_row_fwd_r2(const fhe_ctx* c, const u64* src, u64 spstride, u64* dst, u64 dpstride,
                          u32 polys, u32 limb0, u32 nlimbs, hipStream_t s) {
  if ((u64)polys * nlimbs == 0) return kOk;
  if (c->wide) return wide_unsupported();
  switch (c->log_n) {
#define X(n)                                                                                      \
  case n: {                                                                                       \
    using G = Geo<n>;                                                                             \
    const u64 ir = (u64)polys * nlimbs * G::TILES_R;                                              \
    if (int rc = check_grid(item_blocks(ir), G::THR_R, 1, 1, "ntt_row_fwd")) return rc;           \
    const PolyMap pm{1, spstride, 0, dpstride, 0, 0};                                             \
    if (c->lz16)                                                                                  \
      k_ntt_row<n, true, 16, false, false, 2><<<item_grid(ir), G::THR_R, 0, s>>>(                 \
          src, dst, nlimbs, limb0, pm, (u32)ir, c->d_tw_fwd, c->d_mods);                          \
    else                                                                                          \
      k_ntt_row<n, true, 8, false, false, 2><<<item_grid(ir), G::THR_R, 0, s>>>(                  \
          src, dst, nlimbs, limb0, pm, (u32)ir, c->d_tw_fwd, c->d_mods);                          \
    FHE_HIP_CHECK(hipGetLastError());                                                             \
    return kOk;                                                                                   \
  }
    FHE_LOGN_CASES(X)
#undef X
  }
  set_error("unsupported log_n");
  return kUnsupported;
}

namespace {
// a[0..n) share everything but the per-digit fields (yoff, ext, T, skip_*, hat): one launch
template <int LOGN, int HD>
int modup_col_dispatch(const fhe_ctx* c, const ModUpColArgs* a, u32 n, hipStream_t s) {
  using G = Geo<LOGN>;
  ModUpDigits md{};
  md.n = n;
  u64 blocks = 0;
  for (u32 k = 0; k < n; ++k) {
    ModUpDigit& d = md.d[k];
    for (int j = 0; j < 4; ++j) d.o[j] = a[k].yoff[j];
    d.ext = a[k].ext;
    d.hat = a[k].hat;
    d.T = a[k].T;
    d.skip_at = a[k].skip_at;
    d.skip_len = a[k].skip_len;
    d.blk0 = (u32)blocks;
    blocks += (u64)((a[k].T + kModupTG - 1) / kModupTG) * a[k].batch * G::TILES_C;
    if (int rc = check_grid(blocks, G::THR_C, 1, 1, "modup_col")) return rc;
  }
  const ModUpColArgs& a0 = a[0];
  const dim3 g((u32)blocks);
  switch (a0.S) {
#define D(k)                                                                                   \
  case k:                                                                                      \
    k_modup_col<LOGN, HD, k><<<g, G::THR_C, 0, s>>>(a0.y, a0.ybs, md, a0.rn, a0.n0, a0.base0, \
                                                    a0.base1, a0.batch, a0.hs, c->d_tw_fwd,    \
                                                    c->d_mods);                                \
    break;
    D(1) D(2) D(3) D(4)
#undef D
    default:
      set_error("modup_col: digits of more than 4 limbs take the unfused path");
      return kUnsupported;
  }
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}
}  // namespace

namespace {
int launch_modup_group(const fhe_ctx* c, const ModUpColArgs* a, u32 n, hipStream_t s) {
  switch (c->log_n) {
#define X(n_) \
  case n_:    \
    return c->lz16 ? modup_col_dispatch<n_, 16>(c, a, n, s) : modup_col_dispatch<n_, 8>(c, a, n, s);
    FHE_LOGN_CASES(X)
#undef X
  }
  set_error("unsupported log_n");
  return kUnsupported;
}
}  // namespace

int launch_modup_cols(const fhe_ctx* c, const ModUpColArgs* a, u32 n, hipStream_t s) {
  if (c->wide) return wide_unsupported();
  // digits with no targets launch nothing; consecutive digits whose shared fields agree (always,
  // within one key-switch, except a last digit with fewer limbs) go in one launch
  ModUpColArgs live[4];
  u32 m = 0;
  for (u32 k = 0; k < n; ++k) {
    const ModUpColArgs& x = a[k];
    if ((u64)x.T * x.batch == 0) continue;
    const bool joins = m > 0 && m < 4 && x.y == live[0].y && x.ybs == live[0].ybs &&
                       x.rn == live[0].rn && x.S == live[0].S && x.n0 == live[0].n0 &&
                       x.base0 == live[0].base0 && x.base1 == live[0].base1 &&
                       x.batch == live[0].batch && x.hs == live[0].hs;
    if (m > 0 && !joins) {
      if (int rc = launch_modup_group(c, live, m, s)) return rc;
      m = 0;
    }
    live[m++] = x;
  }
  return m ? launch_modup_group(c, live, m, s) : kOk;
}

int launch_modup_col(const fhe_ctx* c, const ModUpColArgs& a, hipStream_t s) {
  return launch_modup_cols(c, &a, 1, s);
}

namespace {
template <int LOGN, int HD>
int moddown_row_dispatch(const fhe_ctx* c, const ModDownRowArgs& a, hipStream_t s) {
  using G = Geo<LOGN>;
  const u64 items = (u64)a.halves * a.batch * a.nq * G::TILES_R;
  if (int rc = check_grid(item_blocks(items), G::THR_R, 1, 1, "moddown_row")) return rc;
  k_moddown_row<LOGN, HD><<<dim3((u32)((items + 7) / 8 * 8)), G::THR_R, 0, s>>>(
      a.conv, a.ks0, a.ks1, a.acc, a.acc_ws, a.rows, a.nq, a.limb0, a.batch, (u32)items, a.halves,
      a.pinv ? a.pinv : c->d_pinv, c->d_tw_fwd, c->d_mods, a.ep);
  return kOk;
}
}  // namespace

int launch_moddown_row(const fhe_ctx* c, const ModDownRowArgs& a, hipStream_t s) {
  if ((u64)a.batch * a.nq == 0) return kOk;
  if (c->wide) return wide_unsupported();
  switch (c->log_n) {
#define X(n)                                                                                   \
  case n:                                                                                      \
    if (int rc = c->lz16 ? moddown_row_dispatch<n, 16>(c, a, s)                              \
                         : moddown_row_dispatch<n, 8>(c, a, s))                               \
      return rc;                                                                               \
    FHE_HIP_CHECK(hipGetLastError());                                                         \
    return kOk;
    FHE_LOGN_CASES(X)
#undef X
  }
  set_error("unsupported log_n");
  return kUnsupported;
}

namespace {
template <int LOGN>
int ks_row_fin_dispatch(const fhe_ctx* c, const KsFinArgs& a, hipStream_t s) {
  using H = HmGeo<LOGN>;
  if (int rc = check_grid((u64)a.nq * a.batch * H::TILES, H::THR, 1, 1, "ks_row_fin")) return rc;
  const dim3 g((u32)((u64)a.nq * a.batch * H::TILES));
  switch (c->dnum) {
#define D(k)                                                                                     \
  case k:                                                                                        \
    k_ks_row_fin<LOGN, k><<<g, H::THR, 0, s>>>(a.ext, a.ext_ds, a.d2_own, a.evk_b, a.evk_a,     \
                                               a.rows, a.nq, a.base0, a.alpha, a.L, a.batch,     \
                                               a.rscale, a.conv, a.ks0, a.ks1, a.ep, c->d_tw_fwd, \
                                               c->d_mods);                                       \
    break;
    D(1) D(2) D(3) D(4)
#undef D
    default:
      set_error("ks_row_fin: dnum > 4");
      return kUnsupported;
  }
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}
}  // namespace

int launch_ks_row_fin(const fhe_ctx* c, const KsFinArgs& a, hipStream_t s) {
  if ((u64)a.nq * a.batch == 0) return kOk;
  if (c->wide || !c->lz16) {
    set_error("ks_row_fin: needs an lz16 context (every modulus below 2^60)");
    return kUnsupported;
  }
  switch (c->log_n) {
#define X(n) \
  case n:    \
    return ks_row_fin_dispatch<n>(c, a, s);
    FHE_LOGN_CASES(X)
#undef X
  }
  set_error("unsupported log_n");
  return kUnsupported;
}

int launch_ks_row_inner(const fhe_ctx* c, const KsRowArgs& a, hipStream_t s) {
  if ((u64)a.rows * a.batch == 0) return kOk;
  if (c->wide) return wide_unsupported();
  switch (c->log_n) {
#define X(n) \
  case n:    \
    return c->lz16 ? ks_row_inner_dispatch<n, 16>(c, a, s) : ks_row_inner_dispatch<n, 8>(c, a, s);
    FHE_LOGN_CASES(X)
#undef X
  }
  set_error("unsupported log_n");
  return kUnsupported;
}

#else

int launch_ntt(const fhe_ctx* c, bool forward, const u64* src, u64* dst, u32 polys, u64 pstride,
               u32 limb0, u32 nlimbs, hipStream_t s) {
  return launch_ntt_strided(c, forward, src, pstride, dst, pstride, polys, limb0, nlimbs, s);
}

int launch_ntt_strided(const fhe_ctx* c, bool forward, const u64* src, u64 spstride, u64* dst,
                       u64 dpstride, u32 polys, u32 limb0, u32 nlimbs, hipStream_t s,
                       const ulonglong2* nfold, bool split) {
  if ((u64)polys * nlimbs == 0) return kOk;
  switch (c->log_n) {
#define X(n) \
  case n:    \
    return c->wide   ? ntt_dispatch<n, 2>(c, forward, src, spstride, dst, dpstride, polys, limb0, \
                                          nlimbs, s, nfold, split)                              \
           : c->lz16 ? ntt_dispatch<n, 16>(c, forward, src, spstride, dst, dpstride, polys, limb0, \
                                           nlimbs, s, nfold, split)                             \
                     : ntt_dispatch<n, 8>(c, forward, src, spstride, dst, dpstride, polys, limb0,  \
                                          nlimbs, s, nfold, split);
    FHE_LOGN_CASES(X)
#undef X
  }
  set_error("unsupported log_n");
  return kUnsupported;
}

namespace {
template <int LOGN, int HD>
int col_inv_dispatch(const fhe_ctx* c, const u64* src, u64 spstride, u64* dst, u64 dpstride,
                     u32 polys, u32 limb0, u32 nlimbs, hipStream_t s, const ulonglong2* nfold,
                     bool split) {
  using G = Geo<LOGN>;
  const u64 ic = (u64)polys * nlimbs * G::TILES_C;
  if (int rc = check_grid(item_blocks(ic), G::THR_C, 1, 1, "ntt_col_inv")) return rc;
  const PolyMap pm{1, spstride, 0, dpstride, 0, 0};
  const ulonglong2* nf = nfold ? nfold : c->d_nfold;
  if constexpr (HD != 2) {
    if (split) {
      k_ntt_col<LOGN, false, inv_h(HD), false, false, kFinalInvS30>
          <<<item_grid(ic), G::THR_C, 0, s>>>(src, nullptr, dst, nlimbs, limb0, pm, (u32)ic,
                                              c->d_tw_inv, nf, c->d_mods);
      prof_mark(s, "ntt_col_inv");
      return kOk;
    }
  } else if (split) {
    set_error("split30 INTT outputs need every modulus < 2^61");
    return kUnsupported;
  }
  k_ntt_col<LOGN, false, inv_h(HD)><<<item_grid(ic), G::THR_C, 0, s>>>(
      src, nullptr, dst, nlimbs, limb0, pm, (u32)ic, c->d_tw_inv, nf, c->d_mods);
  prof_mark(s, "ntt_col_inv");
  return kOk;
}
}  // namespace

int launch_ntt_col_inv(const fhe_ctx* c, const u64* src, u64 spstride, u64* dst, u64 dpstride,
                       u32 polys, u32 limb0, u32 nlimbs, hipStream_t s, const ulonglong2* nfold,
                       bool split) {
  if ((u64)polys * nlimbs == 0) return kOk;
  int rc = kUnsupported;
  switch (c->log_n) {
#define X(n)                                                                                     \
  case n:                                                                                        \
    rc = c->wide   ? col_inv_dispatch<n, 2>(c, src, spstride, dst, dpstride, polys, limb0,      \
                                            nlimbs, s, nfold, split)                            \
         : c->lz16 ? col_inv_dispatch<n, 16>(c, src, spstride, dst, dpstride, polys, limb0,     \
                                             nlimbs, s, nfold, split)                           \
                   : col_inv_dispatch<n, 8>(c, src, spstride, dst, dpstride, polys, limb0,      \
                                            nlimbs, s, nfold, split);                           \
    break;
    FHE_LOGN_CASES(X)
#undef X
    default:
      set_error("unsupported log_n");
      return kUnsupported;
  }
  if (rc) return rc;
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}

size_t hommult_workspace_bytes(const fhe_ctx* c, u32 batch, u32 nlimbs) {
  return (size_t)batch * 4 * nlimbs * c->n * sizeof(u64);
}

static int hommult_chunk(const fhe_ctx* c, u64* d, const u64* a, const u64* b, u32 batch,
                         u32 limb0, u32 nlimbs, u64* x, hipStream_t s) {
  switch (c->log_n) {
#define X(n) \
  case n:    \
    return c->wide   ? hommult_dispatch<n, 2>(c, d, a, b, batch, limb0, nlimbs, x, s)  \
           : c->lz16 ? hommult_dispatch<n, 16>(c, d, a, b, batch, limb0, nlimbs, x, s) \
                     : hommult_dispatch<n, 8>(c, d, a, b, batch, limb0, nlimbs, x, s);
    FHE_LOGN_CASES(X)
#undef X
  }
  set_error("unsupported log_n");
  return kUnsupported;
}

// (Measured no gain, DESIGN.md §8: two half-batch pipelines on two streams, 37.2k vs 36.9k
// HomMult/s; chunks of 4-16 ciphertexts so the workspace stays in the Infinity Cache, -1 ... -11 %
// (launch tails in the column passes); those chunks alternating over two streams, +0.5 %.)
int launch_hommult(const fhe_ctx* c, u64* d, const u64* a, const u64* b, u32 batch, u32 limb0,
                   u32 nlimbs, void* ws, hipStream_t s) {
  if ((u64)batch * nlimbs == 0) return kOk;
  return hommult_chunk(c, d, a, b, batch, limb0, nlimbs, static_cast<u64*>(ws), s);
}

int launch_rescale_col(const fhe_ctx* c, const u64* last, u64* dst, u32 polys, u32 nq,
                       const u64* half, hipStream_t s) {
  if ((u64)polys * nq == 0) return kOk;
  if (c->wide) {
    set_error("rescale_col: the fused rescale needs every modulus < 2^61");
    return kUnsupported;
  }
  switch (c->log_n) {
#define X(n)                                                  \
  case n:                                                     \
    if (int rc = c->lz16 ? rescale_col_dispatch<n, 16>(c, last, dst, polys, nq, half, s) \
                         : rescale_col_dispatch<n, 8>(c, last, dst, polys, nq, half, s))  \
      return rc;                                              \
    FHE_HIP_CHECK(hipGetLastError());                         \
    return kOk;
    FHE_LOGN_CASES(X)
#undef X
  }
  set_error("unsupported log_n");
  return kUnsupported;
}

#endif  // FHE_NTT_KS_ONLY

}  // namespace fhe
