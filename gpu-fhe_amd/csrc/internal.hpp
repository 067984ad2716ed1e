// Library-internal context and launcher declarations for libfhecore (not installed).
#pragma once
#include <algorithm>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <mutex>
#include <vector>

#include "host_tables.hpp"
#include "modarith.hpp"

namespace fhe {

// Status codes shared with include/fhecore.h.
enum Status : int {
  kOk = 0,
  kInvalid = -1,
  kNoMem = -2,
  kDevice = -3,
  kUnsupported = -4,
};

void set_error(const std::string& msg);
// Records a timing mark after a launch when fhe_prof_begin() is active (prof.cpp).
void prof_mark(hipStream_t s, const char* name);

// Launch-size guard, called by every launcher before its first launch: the dispatch packet
// counts work-items along x in 32 bits, and y / z hold at most 65535 workgroups; the launchers
// narrow their grids to u32, so a size beyond either is refused (FHE_EINVAL) here rather than
// silently truncated.  (At these kernels' 16 elements per work-item, x overflows only past 2^36
// residues, more than HBM holds; y / z carry batch / poly counts, reachable at small N.)
constexpr uint64_t kMaxGridYZ = 65535;
inline int check_grid(uint64_t blocks_x, uint64_t threads, uint64_t y, uint64_t z,
                      const char* who) {
  if (blocks_x * threads >= (1ull << 32) || blocks_x >= (1ull << 32) || y > kMaxGridYZ ||
      z > kMaxGridYZ) {
    set_error(std::string(who) + ": launch too large (grid " + std::to_string(blocks_x) + " x " +
              std::to_string(y) + " x " + std::to_string(z) + " of " + std::to_string(threads) +
              " threads): split the call");
    return kInvalid;
  }
  return kOk;
}


}  // namespace fhe

// Immutable after fhe_ctx_create, except for the lazily grown internal workspace.
struct fhe_ctx {
  int device = 0;
  int num_cus = 0;  // compute units of `device` (one-generation grids of the item-loop kernels)
  // every modulus < 2^60 and within 1/16 below a power of two: NTTs run lazy up to 16q with
  // top-bits reductions (ntt.hip fwd_range, top_bits, gs_in)
  bool lz16 = false;
  // some modulus in [2^61, 2^63): exact (non-lazy) butterflies, HD = 2 in ntt.hip, and the
  // unfused key-switch (rns.hip)
  bool wide = false;
  uint32_t log_n = 0;
  uint64_t n = 0;
  uint32_t L = 0, K = 0, dnum = 0, alpha = 0;
  std::vector<uint64_t> moduli;  // L Q-primes then K P-primes
  std::vector<uint64_t> psi;     // primitive 2N-th roots, per modulus
  std::vector<fhe::ModParams> mods_host;

  fhe::ModParams* d_mods = nullptr;  // [L + K]
  ulonglong2* d_tw_fwd = nullptr;    // [L + K][N] (psi^brv(k), Shoup)
  ulonglong2* d_tw_inv = nullptr;    // [L + K][N] (psi^-brv(k), Shoup)
  // [L][N] the forward table with the row layout of the 512 x 128 split (N = 2^16, narrow
  // contexts; the HomMult's 7-stage forward rows after k_hm_col9), else null
  ulonglong2* d_tw_fwd9 = nullptr;
  // (both tables: the row-pass stages of the low-bit round are stored lane-major, context.cpp
  // lane_major_rows)
  // [L + K][4] Shoup pairs: N^-1, psi^-1 N^-1 (last inverse stage), and the same times
  // R = 2^64 (HomMult's inverse, undoing the Montgomery tensor's R^-1)
  ulonglong2* d_nfold = nullptr;
  // rescale: [L][L] Shoup pairs of q_l^-1 mod q_i and (q_l / 2) mod q_i, row l = last limb
  ulonglong2* d_rs_tab = nullptr;
  uint64_t* d_rs_half = nullptr;

  // Hybrid key-switch base-conversion constants (rns.hip), Shoup pairs, device resident.
  // Digit j covers Q-limbs [j * alpha, min(L, (j + 1) * alpha)).
  ulonglong2* d_modup_inv = nullptr;    // [dnum][alpha]        (D^_k)^-1 mod q_k
  ulonglong2* d_modup_hat = nullptr;    // [dnum][alpha][L + K] D^_k mod t  (by ctx limb t)
  // the fused conversions' tables (ntt.hip k_modup_col): {h, h w0 mod t} with h the .y word of
  // d_modup_hat (_w), of its Montgomery-scaled form D^_k 2^128 mod t (_rw: the fused lz16 ModUp
  // then emits the extended rows times R = 2^64, so k_ks_row_inner's inner product reduces by one
  // REDC; built on the host only), of d_moddown_hat (_w), and w0 = psi_t^(N/2), the twiddle of
  // the column-forward pass's stage 0, folded in for the rows that stage multiplies
  ulonglong2* d_modup_hat_w = nullptr;    // [dnum][alpha][L + K]
  ulonglong2* d_modup_hat_rw = nullptr;   // [dnum][alpha][L + K]
  ulonglong2* d_moddown_hat_w = nullptr;  // [K][L + K]
  // the same with P^-1 mod q folded into every Q-limb column (ModDown's P^-1 taken by the
  // conversions and the accumulators instead of the finish: rns.hip pscale), and R P^-1 mod q_i
  // for the own digit's d2 rows
  ulonglong2* d_modup_hat_rwp = nullptr;   // [dnum][alpha][L + K]
  ulonglong2* d_moddown_hat_wp = nullptr;  // [K][L + K]
  ulonglong2* d_rpinv = nullptr;           // [L]
  ulonglong2* d_moddown_inv = nullptr;  // [K]                  (P^_k)^-1 mod p_k
  ulonglong2* d_moddown_hat = nullptr;  // [K][L + K]           P^_k mod q_i
  ulonglong2* d_pinv = nullptr;         // [L]                  P^-1 mod q_i
  // fold table for ModDown's INTT of the P rows (entries of limbs L..L+K-1): N^-1 (P^_k)^-1 and
  // psi^-N/2 N^-1 (P^_k)^-1, so the INTT emits the scaled conversion inputs directly
  ulonglong2* d_nfold_down = nullptr;   // [L + K][4]
  // fold table for the INTT of d2 ahead of a key-switch (entries of limbs 0..L-1): N^-1 (D^_k)^-1
  // and psi^-N/2 N^-1 (D^_k)^-1 of limb k's digit, so the INTT emits ModUp's scaled inputs
  ulonglong2* d_nfold_up = nullptr;     // [L + K][4]

  void* workspace = nullptr;
  size_t workspace_bytes = 0;
  // the stream that last took the internal workspace (a call on another stream waits for the
  // device first: capi.cpp ensure_ws)
  hipStream_t ws_stream = nullptr;
  bool ws_used = false;
  std::mutex ws_mutex;
  // fhe_baseconv's conversion tables per source range (s0, S): device [S] inv + [S][L + K] hat,
  // built on first use (rns.hip launch_baseconv) and freed with the context
  std::mutex bc_mutex;
  std::vector<std::pair<uint64_t, ulonglong2*>> bc_tables;
};

namespace fhe {

// ---- launchers (ntt.hip) ---------------------------------------------------------------
// data layout [polys][nlimbs][N] with poly stride `pstride` (elements); limb l uses table limb0 + l.
int launch_ntt(const fhe_ctx* c, bool forward, const u64* src, u64* dst, u32 polys, u64 pstride,
               u32 limb0, u32 nlimbs, hipStream_t s);
// the same with separate source / destination poly strides
// (nfold: the inverse's last-stage fold table [limb][4], default c->d_nfold; split: the inverse
// writes split30(x) -- Sum30's 30-bit pieces -- for k_modup_col, which reads its sources that way)
int launch_ntt_strided(const fhe_ctx* c, bool forward, const u64* src, u64 spstride, u64* dst,
                       u64 dpstride, u32 polys, u32 limb0, u32 nlimbs, hipStream_t s,
                       const ulonglong2* nfold = nullptr, bool split = false);
// The second (column) pass of an inverse NTT alone, src [polys][nlimbs][N] (stride spstride,
// already row-inverted, e.g. by k_ks_row_inner PINV) -> dst (stride dpstride); nfold / split as
// launch_ntt_strided.
int launch_ntt_col_inv(const fhe_ctx* c, const u64* src, u64 spstride, u64* dst, u64 dpstride,
                       u32 polys, u32 limb0, u32 nlimbs, hipStream_t s,
                       const ulonglong2* nfold = nullptr, bool split = false);
// Column-forward pass only (first half of a forward NTT; the key-switch's fused row kernel
// finishes it).
int launch_ntt_col_fwd(const fhe_ctx* c, const u64* src, u64 spstride, u64* dst, u64 dpstride,
                       u32 polys, u32 limb0, u32 nlimbs, hipStream_t s);
// the row-forward pass after k_modup_col (input range scheduled from 2), canonical outputs
int launch_ntt_row_fwd_r2(const fhe_ctx* c, const u64* src, u64 spstride, u64* dst, u64 dpstride,
                          u32 polys, u32 limb0, u32 nlimbs, hipStream_t s);
// Fused key-switch row kernel (ntt.hip, k_ks_row_inner): row-forward NTT of every ModUp digit's
// column-passed rows + inner product with the key.  ext [dnum][batch][rows][N] (digit stride
// ext_ds words), d2_own [batch][nq][N] NTT form, evk [dnum][rows][N], acc [2][batch][rows][N]
// (second half at acc + acc_ws); row r -> limb r < nq ? base0 + r : base1 + r - nq.
struct KsRowArgs {
  u64* acc;
  u64 acc_ws;
  const u64* ext;
  u64 ext_ds;
  const u64* d2_own;
  const u64* evk_b;
  const u64* evk_a;
  u32 rows, nq, base0, base1, alpha, L, batch;
  // ext rows carry a factor R = 2^64 (the fused lz16 ModUp with d_modup_hat_rw): the inner product
  // takes the own digit's d2 rows times R as well and reduces each 128-bit sum by one Montgomery
  // REDC (R^-1) instead of reduce128
  bool mont = false;
  // the special rows leave row-inverted (the first pass of ModDown's INTT, k_ks_row_inner PINV):
  // the caller follows with launch_ntt_col_inv only
  u32 pinv = 0;
  // per-limb Shoup pairs of the factor the own digit's d2 rows are taken times (MONT); null: R
  // (ModParams::r64).  R P^-1 when ModDown's P^-1 is folded into the accumulators (rns.hip pscale)
  const ulonglong2* rscale = nullptr;
  // the rows this launch covers: [row0, row0 + nrows) (nrows 0: all rows)
  u32 row0 = 0, nrows = 0;
};
int launch_ks_row_inner(const fhe_ctx* c, const KsRowArgs& a, hipStream_t s);
// ModUp column pass (ntt.hip, k_modup_col): converts a digit's S pre-scaled source rows
// y [batch][S][N] into each of its T target rows and runs their column-forward pass, writing the
// column-passed rows into ext [batch][rows][N] (row stride N, ciphertext stride rn words).
struct ModUpColArgs {
  const u64* y;   // source row k of ciphertext b at y + b ybs + yoff[k]
  u64 ybs;
  u64 yoff[4];
  u64* ext;
  u64 rn;
  u32 S, T, skip_at, skip_len, n0, base0, base1, batch;
  // this digit's conversion table: hat[k hs + limb] = {h, h w0} (fhe_ctx::d_modup_hat_w)
  const ulonglong2* hat;
  u32 hs;
};
int launch_modup_col(const fhe_ctx* c, const ModUpColArgs& a, hipStream_t s);
// several digits (n <= 4) of one ModUp: one launch for each run of digits with the same S and
// shared fields
int launch_modup_cols(const fhe_ctx* c, const ModUpColArgs* a, u32 n, hipStream_t s);
// ModDown finish fused into the conversion NTT's row-forward pass (ntt.hip, k_moddown_row): conv
// [2][batch][nq][N] column-passed -> ks{0,1} [batch][nq][N] = (acc - NTT(conv)) P^-1 mod q.
// Optional epilogue of a key-switch's ModDown finish: the outputs of ciphertext b land at
// ks{0,1} + b * out_bs (rows of N words), and with add{0,1} set the finish writes
// add_h[b * add_bs + row N + i] + ks_h mod q instead of ks_h -- the relinearisation / rotation
// combine folded into the last pass (no separate read of ks0 / ks1).  Defaults: contiguous
// [batch][nlimbs][N] outputs, nothing added.
struct KsEpilogue {
  u64 out_bs = 0;  // 0: nlimbs * N
  const u64* add0 = nullptr;
  const u64* add1 = nullptr;
  u64 add_bs = 0;
  u32 add_gal = 0;  // != 0: add rows read through sigma_add_gal's NTT-domain gather (k_moddown_row)
};
// The Q rows with ModDown's finish (ntt.hip k_ks_row_fin; lz16 with P^-1 folded, after the P rows,
// their column inverse and ModDown's conversion): ks{0,1} [batch][nq][N] (+ the epilogue)
struct KsFinArgs {
  const u64* ext;
  u64 ext_ds;
  const u64* d2_own;
  const u64* evk_b;
  const u64* evk_a;
  u32 rows, nq, base0, alpha, L, batch;
  const ulonglong2* rscale;  // R P^-1 per limb
  const u64* conv;           // [2][batch][nq][N], column-passed
  u64* ks0;
  u64* ks1;
  KsEpilogue ep;  // out_bs resolved
};
int launch_ks_row_fin(const fhe_ctx* c, const KsFinArgs& a, hipStream_t s);
// Hoisted rotations (galois.hip launch_rotate_hoisted): modup_only runs ModUp alone and leaves the
// NTT-form digits in the workspace's ext region; otherwise the key-switch skips ModUp and reads
// those digits (and d2_own) through sigma_galois inside the inner product (unfused kernels).
// Whether a key-switch finishes in k_moddown_row (which can gather its addend, add_gal)
inline bool ks_fused(const fhe_ctx* c) { return c->dnum <= 4 && !c->wide; }
// The hoisted rotation's inner step takes the fused ModDown (whose finish can gather sigma(c0))
inline bool ks_hoist_fused_down(const fhe_ctx* c) { return c->K <= 4 && c->dnum <= 4 && !c->wide; }
struct KsHoist {
  bool modup_only = false;
  u32 galois = 0;
  u64* ydn = nullptr;  // [2 batch][K][N] scratch for the fused ModDown (the ext region is taken)
  // the caller has filled the accumulators (ks_acc_region) itself: ModDown only (the rotation
  // sum, galois.hip launch_rotate_sum_hoisted)
  bool acc_ready = false;
};
// The key-switch workspace's regions (keyswitch_workspace_bytes): ext [dnum][batch][rows][N], then
// the accumulators acc [2][batch][rows][N], rows = nlimbs + K
inline u64* ks_acc_region(const fhe_ctx* c, void* ws, u32 nlimbs, u32 batch) {
  return static_cast<u64*>(ws) + (u64)c->dnum * batch * (nlimbs + c->K) * c->n;
}
struct ModDownRowArgs {
  const u64* conv;
  u64* ks0;
  u64* ks1;
  const u64* acc;
  u64 acc_ws;
  u32 rows, nq, limb0, batch;
  KsEpilogue ep;  // out_bs resolved (non-zero)
  // 2: the key-switch's two accumulators (h = 0 -> ks0, 1 -> ks1; conv [2][batch][nq][N]);
  // 1: one set of polys (ks0 only, conv [batch][nq][N]), as the NTT-form rescale uses it
  u32 halves = 2;
  const ulonglong2* pinv = nullptr;  // per-limb Shoup pairs of the divisor's inverse; null: P^-1
};
int launch_moddown_row(const fhe_ctx* c, const ModDownRowArgs& a, hipStream_t s);
// NTT-form rescale, spread + column-forward pass in one (ntt.hip, k_rescale_col): last [polys][N]
// (coefficient form of limb nq) -> dst [polys][nq][N] column-passed; half = rescale half table.
int launch_rescale_col(const fhe_ctx* c, const u64* last, u64* dst, u32 polys, u32 nq,
                       const u64* half, hipStream_t s);
// Fused ct x ct tensor: a, b [batch][2][nlimbs][N] coefficient form -> d [batch][3][nlimbs][N].
int launch_hommult(const fhe_ctx* c, u64* d, const u64* a, const u64* b, u32 batch, u32 limb0,
                   u32 nlimbs, void* ws, hipStream_t s);
size_t hommult_workspace_bytes(const fhe_ctx* c, u32 batch, u32 nlimbs);

// ---- launchers (elementwise.hip) -------------------------------------------------------
enum VecOp : int { kAdd = 0, kSub = 1, kMul = 2 };
int launch_vec_ctx(const fhe_ctx* c, int op, u64* out, const u64* a, const u64* b, u32 polys,
                   u32 limb0, u32 nlimbs, hipStream_t s);
// moduli records inline in the kernel arguments (generic vec ops with few distinct moduli)
constexpr int kArgMods = 32;
struct ModArgs {
  ModParams m[kArgMods];
};
// row r uses d_mods[r * mod_stride], or inl.m[r * mod_stride] when d_mods is null
int launch_vec_mod(int op, u64* out, const u64* a, const u64* b, u64 rows, u64 cols,
                   const ModParams* d_mods, const ModArgs& inl, u64 mod_stride, int signed_in,
                   hipStream_t s);

// ---- launchers (rns.hip) --------------------------------------------------------------
// Per-rank body of the hybrid key-switch (SURVEY.md §8a', §8e) over `batch` ciphertexts sharing
// one key: c_all [batch][L][N] coefficient form of the whole d2 (all-gathered), d2_own
// [batch][nlimbs][N] NTT form of this rank's Q-limbs [limb0, limb0 + nlimbs), evk_b/evk_a
// [dnum][nlimbs + K][N] NTT form (own Q-limbs then P).  ks0/ks1 [batch][nlimbs][N] NTT form.
int launch_keyswitch_shard(const fhe_ctx* c, u64* ks0, u64* ks1, const u64* c_all,
                           const u64* d2_own, const u64* evk_b, const u64* evk_a, u32 limb0,
                           u32 nlimbs, u32 batch, void* ws, hipStream_t s);
// Where a key-switch finds the coefficient-form d2 of every Q-limb: element (b, l, i) at
// ptr + b bs + (l / lpr) rs + (l % lpr) N + i.  Contiguous [batch][L][N]: lpr = L, bs = L N.
// The rank-major output of an all-gather over G ranks of c = ceil(L / G) limbs each,
// [G][batch][c][N] (the last ranks' blocks padded): lpr = c, rs = batch c N, bs = c N.
struct CAll {
  const u64* ptr;
  u32 lpr;
  u64 rs, bs;
  static CAll contiguous(const u64* p, u32 L, u64 n) { return CAll{p, L, 0, (u64)L * n}; }
  static CAll ranked(const u64* p, u32 L, u32 ranks, u32 batch, u64 n) {
    const u32 c = (L + ranks - 1) / ranks;
    return CAll{p, c, (u64)batch * c * n, (u64)c * n};
  }
  u64 off(u32 l, u64 n) const { return (u64)(l / lpr) * rs + (u64)(l % lpr) * n; }
  // "prepared" input: every Q-limb k already scaled by (D^_k)^-1 of its digit (the INTT that made
  // it folded the factor into its last stage, d_nfold_up), so ModUp's scaling pass is skipped
  bool scaled = false;
};
// Whether a key-switch on this context takes the fused ModUp (conversion inside the column pass),
// which can read a prepared (pre-scaled) input: dnum <= 4, digits of <= 4 limbs, q < 2^61.
inline bool ks_prepared(const fhe_ctx* c) {
  return c->K > 0 && c->dnum <= 4 && c->alpha <= 4 && !c->wide;
}
// The fused conversions' source format (k_modup_col): lz16 contexts (every q < 2^60) read plain
// residues (dot_wide61 on 32-bit halves); the others read Sum30's 30-bit pieces (split30), which
// the INTTs and k_modup_scale feeding them emit directly.
inline bool ks_split30(const fhe_ctx* c) { return !c->lz16; }

// The single-device key-switch paths (fhe_keyswitch, mul-relin, rotate) run a batch in passes of
// at most this many bytes of INTT(d2), the size of the Infinity Cache: ModUp then reads its
// sources from the cache the INTT just wrote.  Measured at N = 2^16, L = 16 (8 MiB of d2 per
// ciphertext): ModUp 16.2 us per ciphertext up to batch 32, 19-21 us at 40-64, every other kernel
// linear in the batch.
constexpr size_t kKsPassBytes = 256ull << 20;
inline uint32_t ks_pass_batch(const fhe_ctx* c, uint32_t batch) {
  const uint64_t per = (uint64_t)c->L * c->n * sizeof(uint64_t);
  return batch ? (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(batch, kKsPassBytes / per)) : 0;
}
int launch_keyswitch_shard(const fhe_ctx* c, u64* ks0, u64* ks1, const CAll& call,
                           const u64* d2_own, const u64* evk_b, const u64* evk_a, u32 limb0,
                           u32 nlimbs, u32 batch, void* ws, hipStream_t s,
                           const KsEpilogue* ep = nullptr, const KsHoist* hoist = nullptr);
size_t keyswitch_workspace_bytes(const fhe_ctx* c, u32 nlimbs, u32 batch);
// The key-switch aliasing rule (include/fhecore.h): each output span (out_words from ks0 / ks1)
// either is d2 itself (same start, the contiguous layout: `contiguous`, out_words == d2_words) or
// does not overlap d2's d2_words; with contiguous outputs ks0 and ks1 must not overlap each other
// (the epilogue layouts interleave their rows by design).  FHE_EINVAL otherwise, nothing launched.
inline bool spans_overlap(const u64* a, u64 na, const u64* b, u64 nb) {
  return na && nb && a < b + nb && b < a + na;
}
inline int ks_check_alias(const u64* ks0, const u64* ks1, const u64* d2, u64 d2_words,
                          u64 out_words, bool contiguous, const char* who) {
  const char* name[2] = {"ks0", "ks1"};
  const u64* out[2] = {ks0, ks1};
  for (int h = 0; h < 2; ++h) {
    const bool in_place = out[h] == d2 && contiguous && out_words == d2_words;
    if (!in_place && spans_overlap(out[h], out_words, d2, d2_words)) {
      set_error(std::string(who) + ": " + name[h] +
                " overlaps d2 without being d2 itself (outputs are either d2, in place, or "
                "disjoint from it)");
      return kInvalid;
    }
  }
  if (contiguous && spans_overlap(ks0, out_words, ks1, out_words)) {
    set_error(std::string(who) + ": ks0 and ks1 overlap");
    return kInvalid;
  }
  return kOk;
}
// Fast basis extension between contiguous ctx limb ranges: in [S][N] over limbs [s0, s0+S),
// out [T][N] over limbs [t0, t0+T) (ranges disjoint).
int launch_baseconv(const fhe_ctx* c, u64* out, const u64* in, u32 s0, u32 S, u32 t0, u32 T,
                    hipStream_t s);

// ---- launchers (galois.hip): SURVEY.md §8(f) row 1 -------------------------------------
int build_galois_tables(fhe_ctx* c);
// sigma_k on [polys][nlimbs][N] rows (poly strides pin / pout), NTT or coefficient form
int launch_automorphism(const fhe_ctx* c, u64* out, u64 pout, const u64* in, u64 pin, u32 polys,
                        u32 limb0, u32 nlimbs, u32 galois_elt, bool ntt, hipStream_t s);
// divide-and-round by q_{nl-1}: in [polys][nl][N] (Q-limbs 0..nl-1) -> out [polys][nl-1][N]
int launch_rescale(const fhe_ctx* c, u64* out, const u64* in, u32 polys, u32 nl, bool ntt,
                   void* ws, hipStream_t s);
size_t rescale_workspace_bytes(const fhe_ctx* c, u32 polys, u32 nl);
// in/out [batch][2][L][N] NTT form; rot_b/rot_a [dnum][L + K][N] (key for sigma_k(s) -> s)
int launch_rotate(const fhe_ctx* c, u64* out, const u64* in, u32 galois_elt, const u64* rot_b,
                  const u64* rot_a, u32 batch, void* ws, hipStream_t s);
size_t rotate_workspace_bytes(const fhe_ctx* c, u32 batch);
// `count` rotations of the same ciphertexts sharing one ModUp: out [count][batch][2][L][N],
// galois[r] with its key rot_b[r] / rot_a[r] (host arrays of device pointers)
int launch_rotate_hoisted(const fhe_ctx* c, u64* out, const u64* in, const u32* galois,
                          const u64* const* rot_b, const u64* const* rot_a, u32 count, u32 batch,
                          void* ws, hipStream_t s);
size_t rotate_hoisted_workspace_bytes(const fhe_ctx* c, u32 batch);
// Double-hoisted rotation sum: out [batch][2][L][N] = sum_r pt[r] rot_{galois[r]}(in), one ModUp
// and one ModDown; pt[r] [L + K][N] NTT form (host array of device pointers); galois[r] == 1 is
// the unrotated term (no key).  count <= kRotSumMax.
constexpr u32 kRotSumMax = 16;
int launch_rotate_sum_hoisted(const fhe_ctx* c, u64* out, const u64* in, const u32* galois,
                              const u64* const* rot_b, const u64* const* rot_a,
                              const u64* const* pt, u32 count, u32 batch, void* ws,
                              hipStream_t s);
size_t rotate_sum_hoisted_workspace_bytes(const fhe_ctx* c, u32 batch);
// sum_r rot_{galois[r]}(cts[r]) over different ciphertexts [batch][2][L][N] with one ModDown
int launch_rotate_sum_multi(const fhe_ctx* c, u64* out, const u64* const* cts, const u32* galois,
                            const u64* const* rot_b, const u64* const* rot_a, u32 count,
                            u32 batch, void* ws, hipStream_t s);
size_t rotate_sum_multi_workspace_bytes(const fhe_ctx* c, u32 count, u32 batch);
// out = sum_g rot_{giant[g]}(sum_b pt[g n1 + b] rot_{baby[b]}(in)), both hoistings
int launch_linear_transform(const fhe_ctx* c, u64* out, const u64* in, u32 n1, u32 n2,
                            const u32* baby, const u64* const* baby_b, const u64* const* baby_a,
                            const u32* giant, const u64* const* giant_b,
                            const u64* const* giant_a, const u64* const* pt, u32 batch, void* ws,
                            hipStream_t s);
size_t linear_transform_workspace_bytes(const fhe_ctx* c, u32 n2, u32 batch);

// ---- launchers (pipeline.hip): SURVEY.md §8(f) row 4 -----------------------------------
int launch_mul_relin(const fhe_ctx* c, u64* out, const u64* a, const u64* b, const u64* evk_b,
                     const u64* evk_a, u32 batch, bool rescale, void* ws, hipStream_t s);
size_t mul_relin_workspace_bytes(const fhe_ctx* c, u32 batch);

// caller workspace, else the context's internal one grown to `bytes` (capi.cpp); an error while
// `s` is capturing a graph
int ensure_ws(const fhe_ctx* c, size_t bytes, void** ws, hipStream_t s);

// ---- host (context.cpp) ----------------------------------------------------------------
int ctx_create(fhe_ctx** out, u32 log_n, const u64* q, u32 L, const u64* p, u32 K, u32 dnum,
               int device);
int ctx_destroy(fhe_ctx* c);
int gen_moduli(u32 log_n, u32 count, u32 bits, u32 skip, u64* out);
int build_rns_tables(fhe_ctx* c);

}  // namespace fhe

#define FHE_HIP_CHECK(expr)                                                             \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      fhe::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                \
      return fhe::kDevice;                                                              \
    }                                                                                   \
  } while (0)
