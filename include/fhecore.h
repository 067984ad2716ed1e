/* libfhecore -- MI355X-native (gfx950) FHE polynomial-arithmetic core: C ABI.
 *
 * This is the drop-in boundary for the reference's hot path.  The reference
 * (Kelly-Zhe/GPU-FHE @ 2025-02-12) is a Python/numpy module whose whole operator surface is
 *     vec_add(a, b, MOD)   /root/reference/arithmetic.py:3-5
 *     vec_sub(a, b, MOD)   /root/reference/arithmetic.py:7-9
 *     vec_mul(a, b, MOD)   /root/reference/arithmetic.py:11-13   (= poly_mul_pointwise)
 *     NTT(x), iNTT(x)      /root/reference/arithmetic.py:15-19   (identity stubs there)
 *     poly_add(a, b, MOD)  /root/reference/ polynomial.py:3-5
 * Each entry point below names the reference function it replaces; the Python shim in
 * gpu-fhe_amd/arithmetic.py and gpu-fhe_amd/polynomial.py binds them by ctypes under the
 * reference's own names.  Components the north star names but the
 * reference lacks (Shoup/Barrett modmul, RNS base conversion, key-switch, HomMult) follow
 * the build-defined spec of SURVEY.md §8a'.
 *
 * Conventions
 *  - Return 0 on success, a negative FHE_E* code on error; fhe_last_error() (thread-local)
 *    describes the last failure.  No entry point aborts or throws.
 *  - Every data pointer is DEVICE memory owned by the caller.  Residues are uint64 in
 *    layout [poly][limb][N] (limb-major, each limb's N coefficients contiguous).
 *  - `stream` is a hipStream_t (NULL = the legacy default stream).  Launches are
 *    asynchronous and capture-safe (no allocation or synchronisation inside) unless noted.
 *  - A context is immutable after creation: calls on different streams may share it.  Passing
 *    workspace == NULL uses the context's internal workspace: a call on a different stream
 *    than the previous such call first waits for the device (hipDeviceSynchronize), so calls
 *    issued one after another never overlap on it; host threads calling concurrently must each
 *    pass their own workspace.
 *  - limb0 / nlimbs select a contiguous window of the context's Q-limbs (RNS-limb sharding).
 */
#ifndef FHECORE_H
#define FHECORE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FHE_OK 0
#define FHE_EINVAL (-1)
#define FHE_ENOMEM (-2)
#define FHE_EDEVICE (-3)
#define FHE_EUNSUPPORTED (-4)

typedef struct fhe_ctx fhe_ctx;
typedef void* fhe_stream_t; /* hipStream_t */

/* Thread-local description of the last error ("" if none). */
const char* fhe_last_error(void);
/* Library version string. */
const char* fhe_version(void);

/* ---- parameters (host only) -------------------------------------------------------- */
/* The `count` largest primes q < 2^bits with q = 1 (mod 2^(log_n+1)), descending, after skipping
 * `skip` (SURVEY.md §8a' modulus chain; special primes P continue the same list). */
int fhe_gen_moduli(uint32_t log_n, uint32_t count, uint32_t bits, uint32_t skip, uint64_t* out);

/* ---- context ------------------------------------------------------------------------ */
/* Creates a context on HIP device `device` for ring degree N = 2^log_n (10 <= log_n <= 17) with
 * Q-primes q[0..L) and special primes p[0..K) (K may be 0: no key-switch) and dnum gadget digits.
 * Every modulus must be a distinct prime < 2^61 with q = 1 (mod 2N).
 * Precomputes psi^brv twiddles (psi = g^((q-1)/2N), g the smallest primitive root), Shoup
 * companions, Barrett constants and key-switch base-conversion tables; uploads them.
 * Replaces: nothing in the reference (it passes MOD per call, arithmetic.py:3). */
int fhe_ctx_create(fhe_ctx** ctx, uint32_t log_n, const uint64_t* q, uint32_t L,
                   const uint64_t* p, uint32_t K, uint32_t dnum, int device);
int fhe_ctx_destroy(fhe_ctx* ctx);
/* Copies the L + K moduli (Q then P) and their psi roots to host arrays (either may be NULL). */
int fhe_ctx_moduli(const fhe_ctx* ctx, uint64_t* moduli, uint64_t* psi);
/* log_n, L, K, dnum, device. */
int fhe_ctx_shape(const fhe_ctx* ctx, uint32_t* log_n, uint32_t* L, uint32_t* K, uint32_t* dnum,
                  int* device);
/* Grows the context's internal workspace to >= bytes (allocates; not capture-safe). */
int fhe_ctx_reserve(fhe_ctx* ctx, size_t bytes);

/* ---- coefficient-wise ops on canonical residues ------------------------------------- */
/* out = (a op b) mod q_{limb0 + l} for every poly and limb l in [0, nlimbs); inputs in [0, q).
 * out may alias a or b.  Replaces vec_add / vec_sub / vec_mul (arithmetic.py:3-13) and
 * poly_add (' polynomial.py':3-5, with polys = 2). */
int fhe_vec_add(const fhe_ctx* ctx, uint64_t* out, const uint64_t* a, const uint64_t* b,
                uint32_t polys, uint32_t limb0, uint32_t nlimbs, fhe_stream_t stream);
int fhe_vec_sub(const fhe_ctx* ctx, uint64_t* out, const uint64_t* a, const uint64_t* b,
                uint32_t polys, uint32_t limb0, uint32_t nlimbs, fhe_stream_t stream);
int fhe_vec_mul(const fhe_ctx* ctx, uint64_t* out, const uint64_t* a, const uint64_t* b,
                uint32_t polys, uint32_t limb0, uint32_t nlimbs, fhe_stream_t stream);

/* Generic form used by the reference-shaped Python API: a, b, out are rows x cols matrices;
 * row r uses modulus mods[r * mod_stride] (mod_stride 0 = one scalar MOD).  `mods` is a HOST
 * array; inputs may be any uint64 (signed_in = 1: any int64), moduli any value in [2, 2^64).
 * Result = Python's exact (a op b) % MOD.  op: 0 add, 1 sub, 2 mul.
 * Up to 32 distinct modulus records (a scalar MOD, or a column of <= 32 rows) travel in the
 * kernel arguments: no allocation or synchronisation, capture-safe.  Longer modulus columns
 * allocate a stream-ordered table and synchronise `stream`. */
int fhe_vec_op_mod(int op, uint64_t* out, const uint64_t* a, const uint64_t* b, uint64_t rows,
                   uint64_t cols, const uint64_t* mods, uint64_t mod_stride, int signed_in,
                   int device, fhe_stream_t stream);

/* ---- negacyclic NTT ------------------------------------------------------------------ */
/* In place on data [polys][nlimbs][N]; limb l uses q_{limb0 + l} (limb0 + nlimbs <= L + K, so
 * P-limbs are addressable too).  Forward: natural -> bit-reversed order,
 * NTT(a)[k] = sum_i a_i psi^((2 brv(k) + 1) i); inverse: exact inverse incl. N^-1.
 * Inputs canonical in [0, q); outputs canonical.  Replaces NTT / iNTT (arithmetic.py:15-19). */
int fhe_ntt_fwd(const fhe_ctx* ctx, uint64_t* data, uint32_t polys, uint32_t limb0,
                uint32_t nlimbs, fhe_stream_t stream);
int fhe_ntt_inv(const fhe_ctx* ctx, uint64_t* data, uint32_t polys, uint32_t limb0,
                uint32_t nlimbs, fhe_stream_t stream);
/* Out of place: dst = NTT(src) / INTT(src), both [polys][nlimbs][N]; src is left untouched (the
 * first pass reads src and writes dst, the second runs in place on dst -- no copy).  dst == src is
 * the in-place call; other overlaps are undefined. */
int fhe_ntt_fwd_to(const fhe_ctx* ctx, uint64_t* dst, const uint64_t* src, uint32_t polys,
                   uint32_t limb0, uint32_t nlimbs, fhe_stream_t stream);
int fhe_ntt_inv_to(const fhe_ctx* ctx, uint64_t* dst, const uint64_t* src, uint32_t polys,
                   uint32_t limb0, uint32_t nlimbs, fhe_stream_t stream);

/* ---- ct x ct homomorphic multiplication (tensor) ----------------------------------------
 * a, b: [batch][2][nlimbs][N] coefficient form; d: [batch][3][nlimbs][N] coefficient form with
 * d0 = a0 b0, d1 = a0 b1 + a1 b0, d2 = a1 b1 in Z_q[X]/(X^N + 1) (NTT -> pointwise -> INTT).
 * workspace: >= fhe_hommult_workspace(ctx, batch, nlimbs) bytes of device memory, or NULL.
 * Replaces the caller-composed NTT -> vec_mul/vec_add -> iNTT chain (SURVEY.md §3 stack 4). */
size_t fhe_hommult_workspace(const fhe_ctx* ctx, uint32_t batch, uint32_t nlimbs);
int fhe_hommult(const fhe_ctx* ctx, uint64_t* d, const uint64_t* a, const uint64_t* b,
                uint32_t batch, uint32_t limb0, uint32_t nlimbs, void* workspace,
                fhe_stream_t stream);

/* ---- RNS base conversion ---------------------------------------------------------------
 * Fast basis extension (no correction) from ctx limbs [s0, s0+S) to [t0, t0+T) (disjoint),
 * coefficient domain: in [S][N] -> out [T][N].  S <= 16.  The conversion tables of a
 * (s0, S) source range are built and uploaded on its first use and cached on the context (that
 * first call synchronises `stream`); later calls neither allocate nor synchronise. */
int fhe_baseconv(const fhe_ctx* ctx, uint64_t* out, const uint64_t* in, uint32_t s0, uint32_t S,
                 uint32_t t0, uint32_t T, fhe_stream_t stream);

/* ---- hybrid key-switch (relinearisation) -------------------------------------------------
 * `batch` ciphertexts share one key.  Single-device form: d2 [batch][L][N] NTT form over Q;
 * evk_b, evk_a [dnum][L + K][N] NTT form over Q u P; ks0, ks1 [batch][L][N] NTT form:
 * ks0 + ks1 s = d2 s'' + small (SURVEY.md §8a').  The key is read once per batch.
 * Sharded form (one rank of G): c_all [batch][L][N] = INTT(d2) all-gathered (coefficient form),
 * d2_own [batch][nlimbs][N] NTT form of Q-limbs [limb0, limb0 + nlimbs), evk slices
 * [dnum][nlimbs + K][N] (own Q-limbs then all K P-limbs); outputs [batch][nlimbs][N].  The
 * sharded outputs of G ranks concatenate to the single-device result bit for bit.
 * fhe_keyswitch (and fhe_mul_relin, fhe_rotate) run the batch in passes of at most 256 MiB of
 * d2 (the Infinity Cache), so the internal workspace is sized for one pass; a caller's workspace
 * of the documented *_workspace(ctx, ..., batch) bytes is always large enough.
 * Aliasing (every key-switch entry point, incl. the _shard, _dist and _loopback forms): ks0 and
 * ks1 may each be d2 (d2_own) itself -- the in-place call, same start pointer -- or must not
 * overlap it at all; ks0 and ks1 must not overlap each other.  Any other overlap returns
 * FHE_EINVAL before anything is launched.  c_all / c_gathered, the keys and the workspace must
 * not overlap the outputs (not checked). */
size_t fhe_keyswitch_workspace(const fhe_ctx* ctx, uint32_t nlimbs, uint32_t batch);
/* The pass size of fhe_keyswitch / fhe_rotate / fhe_mul_relin for `batch` ciphertexts:
 * min(batch, the ciphertexts whose L limbs fit 256 MiB), at least 1 (0 for batch 0).  A workspace
 * of fhe_keyswitch_workspace(ctx, L, pass) (fhe_rotate_workspace(ctx, pass),
 * fhe_mul_relin_workspace(ctx, pass)) bytes is enough for any batch those calls split into passes
 * of that size. */
uint32_t fhe_keyswitch_pass_batch(const fhe_ctx* ctx, uint32_t batch);
int fhe_keyswitch(const fhe_ctx* ctx, uint64_t* ks0, uint64_t* ks1, const uint64_t* d2,
                  const uint64_t* evk_b, const uint64_t* evk_a, uint32_t batch, void* workspace,
                  fhe_stream_t stream);
int fhe_keyswitch_shard(const fhe_ctx* ctx, uint64_t* ks0, uint64_t* ks1, const uint64_t* c_all,
                        const uint64_t* d2_own, const uint64_t* evk_b, const uint64_t* evk_a,
                        uint32_t limb0, uint32_t nlimbs, uint32_t batch, void* workspace,
                        fhe_stream_t stream);

/* ---- multi-GPU: the limb-sharded key-switch over RCCL ---------------------
 * One process per GPU.  Rank r of G owns Q-limbs [r c, min((r + 1) c, L)), c = ceil(L / G)
 * (fhe_comm_shard), plus the K special limbs of the key.  A communicator is created from a
 * unique id that rank 0 makes (fhe_comm_get_unique_id) and the caller distributes out of band
 * (e.g. a torch.distributed broadcast), one fhe_comm_create per rank on its device.
 * fhe_keyswitch_dist: d2_own [batch][nlimbs][N] NTT form of the rank's limbs, evk_b / evk_a
 * [dnum][nlimbs + K][N] (own Q-limbs then all K P-limbs) -> ks0, ks1 [batch][nlimbs][N] NTT
 * form.  INTT of the own limbs, one all-gather of the coefficient-form d2 per chunk of the batch
 * (`chunks` pieces, 0 = default 4; each chunk's transfer runs on the communicator's stream and
 * overlaps the previous chunk's key-switch), then the local key-switch: the G ranks' outputs
 * concatenate to fhe_keyswitch's bit for bit.  Every rank must call it with the same batch and
 * chunks; one call at a time per communicator.
 * fhe_keyswitch_shard_ranked: the local step alone, on an all-gather output already in the
 * rank-major layout [ranks][batch][c][N] (blocks of the last ranks padded to c limbs). */
#define FHE_COMM_ID_BYTES 128
typedef struct fhe_comm_s* fhe_comm_t;
int fhe_comm_get_unique_id(uint8_t* id);
int fhe_comm_create(fhe_comm_t* comm, const uint8_t* id, int nranks, int rank, int device);
int fhe_comm_destroy(fhe_comm_t comm);
int fhe_comm_shard(const fhe_ctx* ctx, fhe_comm_t comm, uint32_t* limb0, uint32_t* nlimbs);
size_t fhe_keyswitch_dist_workspace(const fhe_ctx* ctx, fhe_comm_t comm, uint32_t batch,
                                    uint32_t chunks);
int fhe_keyswitch_dist(const fhe_ctx* ctx, fhe_comm_t comm, uint64_t* ks0, uint64_t* ks1,
                       const uint64_t* d2_own, const uint64_t* evk_b, const uint64_t* evk_a,
                       uint32_t batch, uint32_t chunks, void* workspace, fhe_stream_t stream);
int fhe_keyswitch_shard_ranked(const fhe_ctx* ctx, uint64_t* ks0, uint64_t* ks1,
                               const uint64_t* c_gathered, uint32_t ranks, const uint64_t* d2_own,
                               const uint64_t* evk_b, const uint64_t* evk_a, uint32_t limb0,
                               uint32_t nlimbs, uint32_t batch, void* workspace,
                               fhe_stream_t stream);
/* Per-chunk all-gather durations (ms, HIP events on the communicator's stream) of the last
 * fhe_keyswitch_dist call on `comm`: waits for that call's gathers; *count = its chunk count. */
int fhe_comm_gather_ms(fhe_comm_t comm, float* ms, uint32_t cap, uint32_t* count);

/* The placement plan fhe_keyswitch_dist follows (host only: no device access, callable without a
 * GPU).  Rank `rank` of `ranks` owns Q-limbs [limb0, limb0 + nlimbs); the batch is cut into
 * `chunks` chunks of `chunk_batch` ciphertexts (the last one possibly shorter, none empty); per
 * chunk every rank contributes one block of chunk_batch x width x N words (width = ceil(L / ranks),
 * padded on ranks owning fewer limbs), and the all-gather leaves the blocks rank-major in a region
 * of gather_words words: [chunks][ranks][chunk_batch][width][N].
 * fhe_dist_plan_chunk: the chunk's first ciphertext and length.
 * fhe_dist_plan_send_word: word offset in the gather region where this rank writes row (ciphertext
 * b, own limb j); fhe_dist_plan_read_word: where the key-switch reads row (b, Q-limb l) -- the
 * addressing its kernels use.  UINT64_MAX for an out-of-range argument. */
typedef struct fhe_dist_plan {
  uint32_t L, log_n, ranks, rank, batch;
  uint32_t limb0, nlimbs, width;
  uint32_t chunks, chunk_batch;
  uint64_t block_words, gather_words;
} fhe_dist_plan;
int fhe_dist_plan_make(fhe_dist_plan* plan, uint32_t L, uint32_t log_n, uint32_t ranks,
                       uint32_t rank, uint32_t batch, uint32_t chunks);
int fhe_dist_plan_chunk(const fhe_dist_plan* plan, uint32_t k, uint32_t* b0, uint32_t* bn);
uint64_t fhe_dist_plan_send_word(const fhe_dist_plan* plan, uint32_t b, uint32_t j);
uint64_t fhe_dist_plan_read_word(const fhe_dist_plan* plan, uint32_t b, uint32_t l);

/* fhe_keyswitch_dist for `ranks` ranks run one after another on this context's device (a
 * loopback communicator: the ranks' INTTs write one shared gather region, which is exactly what
 * the all-gather would leave on every rank).  Executes the G-rank plan, offsets and chunking of
 * fhe_keyswitch_dist on one GPU; per-rank arguments are host arrays of `ranks` device pointers
 * (ranks owning no limb may pass NULL), laid out as fhe_keyswitch_dist's. */
size_t fhe_keyswitch_dist_loopback_workspace(const fhe_ctx* ctx, uint32_t ranks, uint32_t batch,
                                             uint32_t chunks);
int fhe_keyswitch_dist_loopback(const fhe_ctx* ctx, uint32_t ranks, uint64_t* const* ks0,
                                uint64_t* const* ks1, const uint64_t* const* d2_own,
                                const uint64_t* const* evk_b, const uint64_t* const* evk_a,
                                uint32_t batch, uint32_t chunks, void* workspace,
                                fhe_stream_t stream);

/* Hybrid partition of a key-switch batch over `ranks` GPUs: `groups` ciphertext groups of
 * g = ranks / groups limb shards each (groups | ranks).  Rank r is limb shard r % g of group r / g;
 * group k takes the job's ciphertexts [batch0, batch0 + batch) (contiguous, ceil(job batch /
 * groups) per group, the last ones possibly shorter or empty) and runs the limb-sharded
 * key-switch above among its own g ranks: `plan` is fhe_dist_plan_make(L, log_n, g, r % g, batch,
 * chunks), the all-gather stays inside the group (the caller creates one communicator per group,
 * g ranks, with fhe_comm_create), and per-rank work is ~ batch (L / g + K) instead of the
 * limb-only job batch (L / ranks + K).  groups = 1 is the limb-only partition (the default);
 * groups = ranks replicates nothing but the key: each GPU key-switches whole ciphertexts, no
 * collective.  Host only, callable without a GPU. */
typedef struct fhe_dist_hybrid {
  uint32_t ranks, groups, g;
  uint32_t group, shard;   /* rank / g, rank % g */
  uint32_t batch0, batch;  /* the group's ciphertexts within the job's batch */
  fhe_dist_plan plan;      /* the group's limb plan for this rank */
} fhe_dist_hybrid;
int fhe_dist_hybrid_make(fhe_dist_hybrid* h, uint32_t L, uint32_t log_n, uint32_t ranks,
                         uint32_t groups, uint32_t rank, uint32_t batch, uint32_t chunks);
/* The hybrid partition's ranks run one after another on this device (per group: the loopback
 * above over its g ranks and its ciphertexts).  Per-rank host arrays of device pointers, rank r's
 * d2_own / ks0 / ks1 being [group batch][nlimbs_r][N] of its group's ciphertexts and its limbs;
 * `batch` is the job's.  The per-rank outputs equal fhe_keyswitch's rows (group k's ciphertexts,
 * shard s's limbs) bit for bit. */
size_t fhe_keyswitch_dist_hybrid_loopback_workspace(const fhe_ctx* ctx, uint32_t ranks,
                                                    uint32_t groups, uint32_t batch,
                                                    uint32_t chunks);
int fhe_keyswitch_dist_hybrid_loopback(const fhe_ctx* ctx, uint32_t ranks, uint32_t groups,
                                       uint64_t* const* ks0, uint64_t* const* ks1,
                                       const uint64_t* const* d2_own,
                                       const uint64_t* const* evk_b,
                                       const uint64_t* const* evk_a, uint32_t batch,
                                       uint32_t chunks, void* workspace, fhe_stream_t stream);

/* ---- rescale and rotation (not in the reference) ---------------------
 * Standard RNS-CKKS operations on this library's layout, restated by oracle/pyoracle.py
 * (rescale_coeff / rescale_ntt, automorphism_*, rotate).
 * fhe_rescale: divide-and-round by the last modulus.  in [polys][nlimbs][N] over Q-limbs
 * 0 .. nlimbs-1 (2 <= nlimbs <= L) -> out [polys][nlimbs-1][N], out_i = floor((X + q_l/2) / q_l)
 * mod q_i for the CRT value X; ntt_form selects NTT or coefficient form for both (the NTT form
 * needs a workspace of fhe_rescale_workspace bytes; NULL = internal). */
size_t fhe_rescale_workspace(const fhe_ctx* ctx, uint32_t polys, uint32_t nlimbs);
int fhe_rescale(const fhe_ctx* ctx, uint64_t* out, const uint64_t* in, uint32_t polys,
                uint32_t nlimbs, int ntt_form, void* workspace, fhe_stream_t stream);
/* fhe_automorphism: sigma_k(a)(X) = a(X^k) for an odd Galois element k < 2N, on
 * [polys][nlimbs][N] rows over limbs [limb0, limb0 + nlimbs), NTT or coefficient form (a slot
 * permutation, resp. a signed coefficient permutation).  out must not alias in.  Rotating the
 * slots by r uses k = 5^r mod 2N, conjugation k = 2N - 1. */
int fhe_automorphism(const fhe_ctx* ctx, uint64_t* out, const uint64_t* in, uint32_t polys,
                     uint32_t limb0, uint32_t nlimbs, uint32_t galois_elt, int ntt_form,
                     fhe_stream_t stream);
/* fhe_rotate: in, out [batch][2][L][N] NTT form over Q (out must not overlap in at all:
 * FHE_EINVAL -- the finish reads c0 through sigma while other workgroups write out);
 * out = (sigma_k c0 + KS0(sigma_k c1), KS1(sigma_k c1)) with rot_b, rot_a [dnum][L + K][N] the
 * key-switch key from sigma_k(s) to s (NTT form, as for fhe_keyswitch). */
size_t fhe_rotate_workspace(const fhe_ctx* ctx, uint32_t batch);
int fhe_rotate(const fhe_ctx* ctx, uint64_t* out, const uint64_t* in, uint32_t galois_elt,
               const uint64_t* rot_b, const uint64_t* rot_a, uint32_t batch, void* workspace,
               fhe_stream_t stream);

/* fhe_rotate_hoisted: `count` rotations of the same ciphertexts sharing one ModUp (hoisting:
 * the INTT, base conversion and NTT of c1's digits run once; each rotation reads them through
 * its automorphism inside the inner product).  in [batch][2][L][N] NTT form over Q; out
 * [count][batch][2][L][N] (must not overlap in); galois_elts[r] with its key rot_b[r], rot_a[r]
 * ([dnum][L + K][N] device pointers in host arrays, as for fhe_rotate).  Each output decrypts to
 * sigma_k(m) like fhe_rotate's, but is not bit-identical to it (ModUp of sigma(c1) differs from
 * sigma of ModUp(c1) by multiples of the digit moduli); restated by oracle/pyoracle.py
 * rotate_hoisted. */
size_t fhe_rotate_hoisted_workspace(const fhe_ctx* ctx, uint32_t batch);
int fhe_rotate_hoisted(const fhe_ctx* ctx, uint64_t* out, const uint64_t* in,
                       const uint32_t* galois_elts, const uint64_t* const* rot_b,
                       const uint64_t* const* rot_a, uint32_t count, uint32_t batch,
                       void* workspace, fhe_stream_t stream);

/* fhe_rotate_sum_hoisted: out = sum_r pt[r] * rot_{galois_elts[r]}(in) over `count` (1..16)
 * terms -- the inner loop of a baby-step / giant-step linear transform (CKKS bootstrapping's
 * CoeffToSlot / SlotToCoeff) -- with one ModUp of c1 and ONE ModDown per output polynomial
 * (double hoisting: each rotation's key-switch accumulators are multiplied by pt[r] and summed in
 * the extended basis Q u P before ModDown).  in, out [batch][2][L][N] NTT form over Q (out must
 * not overlap in); pt[r] [L + K][N] NTT form over Q u P (the diagonal, encoded over the extended
 * basis); galois_elts[r] == 1 is the unrotated term and takes no key (rot_b[r] / rot_a[r] may be
 * null there).  Decrypts to sum_r pt_r sigma_r(m) up to one ModDown's rounding; not bit-identical
 * to summing fhe_rotate_hoisted outputs.  Restated by oracle/pyoracle.py rotate_sum_hoisted.
 * Contexts with dnum <= 8. */
size_t fhe_rotate_sum_hoisted_workspace(const fhe_ctx* ctx, uint32_t batch);
int fhe_rotate_sum_hoisted(const fhe_ctx* ctx, uint64_t* out, const uint64_t* in,
                           const uint32_t* galois_elts, const uint64_t* const* rot_b,
                           const uint64_t* const* rot_a, const uint64_t* const* pt,
                           uint32_t count, uint32_t batch, void* workspace, fhe_stream_t stream);

/* fhe_rotate_sum_multi: out = sum_r rot_{galois_elts[r]}(cts[r]) over `count` (1..16) DIFFERENT
 * ciphertexts (each [batch][2][L][N] NTT form over Q) with ONE ModDown: a ModUp of each rotated
 * term's own c1 (the workspace holds every term's digits), then one pass forming all the gathered
 * inner products in Q u P (the giant-step sum of a baby-step / giant-step linear transform).  galois_elts[r] == 1 adds cts[r] unrotated (no key; rot_b[r] /
 * rot_a[r] may be null).  out must not overlap any cts[r].  Decrypts to sum_r sigma_r(m_r) up to one
 * ModDown's rounding.  Restated by oracle/pyoracle.py rotate_sum_multi.  Contexts with dnum <= 8. */
size_t fhe_rotate_sum_multi_workspace(const fhe_ctx* ctx, uint32_t count, uint32_t batch);
int fhe_rotate_sum_multi(const fhe_ctx* ctx, uint64_t* out, const uint64_t* const* cts,
                         const uint32_t* galois_elts, const uint64_t* const* rot_b,
                         const uint64_t* const* rot_a, uint32_t count, uint32_t batch,
                         void* workspace, fhe_stream_t stream);

/* fhe_linear_transform: the baby-step / giant-step plaintext-matrix product of CKKS bootstrapping
 * (CoeffToSlot / SlotToCoeff) with both hoistings:
 *   out = sum_{g < n2} rot_{giant_elts[g]}( sum_{b < n1} pt[g n1 + b] * rot_{baby_elts[b]}(in) ),
 * n1, n2 in 1..16; pt[g n1 + b] [L + K][N] NTT form over Q u P (the diagonals, pre-rotated by the
 * caller as BSGS requires); element 1 in either list is an unrotated step (its keys may be null).
 * ONE ModUp of in's c1 serves every baby step; each giant step's inner sum is exactly
 * fhe_rotate_sum_hoisted(in, baby_elts, baby keys, pt[g n1 ..]) and the outer sum exactly
 * fhe_rotate_sum_multi of those.  in, out [batch][2][L][N] NTT form; out must not overlap in.
 * Restated by oracle/pyoracle.py linear_transform. */
size_t fhe_linear_transform_workspace(const fhe_ctx* ctx, uint32_t n2, uint32_t batch);
int fhe_linear_transform(const fhe_ctx* ctx, uint64_t* out, const uint64_t* in, uint32_t n1,
                         uint32_t n2, const uint32_t* baby_elts, const uint64_t* const* baby_b,
                         const uint64_t* const* baby_a, const uint32_t* giant_elts,
                         const uint64_t* const* giant_b, const uint64_t* const* giant_a,
                         const uint64_t* const* pt, uint32_t batch, void* workspace,
                         fhe_stream_t stream);

/* ---- wire format (not in the reference) ------------------------------
 * A self-describing little-endian blob for any [polys][nlimbs][N] residue tensor over context
 * limbs [limb0, limb0 + nlimbs) -- ciphertexts, keys, plaintexts: "FHEC", version 1, flags (bit 0
 * NTT form), log_n, polys, limb0, nlimbs, the nlimbs moduli, the residues, an FNV-1a-64 checksum
 * (layout in gpu-fhe_amd/csrc/serialize.cpp).  fhe_serialize copies device -> host and
 * synchronises `stream`.  fhe_deserialize validates the blob against the context (N, moduli,
 * checksum, every residue below its modulus) before copying host -> device; with dev == NULL it
 * only validates and reports the shape, so a caller can size the device buffer (dev_words). */
size_t fhe_serialized_size(const fhe_ctx* ctx, uint32_t polys, uint32_t nlimbs);
int fhe_serialize(const fhe_ctx* ctx, const uint64_t* dev, uint32_t polys, uint32_t limb0,
                  uint32_t nlimbs, int ntt_form, void* host_buf, size_t buf_size,
                  fhe_stream_t stream);
int fhe_deserialize(const fhe_ctx* ctx, const void* host_buf, size_t size, uint64_t* dev,
                    size_t dev_words, uint32_t* polys, uint32_t* limb0, uint32_t* nlimbs,
                    int* ntt_form, fhe_stream_t stream);

/* ---- sampling, keys, encryption (not in the reference) ---------------
 * Counter-based Philox4x32-10 randomness: every sample is a function of (seed, tag, poly, limb,
 * coefficient), restated bit for bit by oracle/pyoracle.py.  kind: 0 uniform mod q, 1 ternary
 * {-1, 0, 1}, 2 centred binomial eta = 21 (small kinds: one integer per coefficient on every limb).
 * Keys are NTT form: sk [L + K][N] (all context limbs); pk [2][L][N] = (-a s + e, a);
 * switch key [2][dnum][L + K][N] = (b part, a part) from s_from ([L + K][N], NTT form: s^2 for
 * relinearisation, sigma_k(s) for rotation by Galois element k) to s -- the layout fhe_keyswitch,
 * fhe_rotate and fhe_mul_relin take as (evk_b, evk_a).  Ciphertexts [2][L][N] NTT form;
 * plaintexts [L][N] NTT form.  fhe_decrypt: pt = c0 + c1 s over the first nlimbs Q-limbs of
 * `batch` ciphertexts [batch][2][nlimbs][N].
 * SECURITY: the seed is the whole nonce.  Encryption randomness (u, e0, e1, and a for fhe_encrypt_sk)
 * and a switch key's a_j are pure functions of (seed, fixed tag), so two encryptions under one key
 * with the same seed have identical masks (their difference reveals pt1 - pt2), and two switch keys
 * generated from one seed share a_j.  Never repeat a seed per secret key: draw it from a CSPRNG or
 * a per-key monotonically increasing counter.  The explicit seed exists so tests are reproducible. */
int fhe_sample(const fhe_ctx* ctx, uint64_t* out, uint32_t polys, uint32_t limb0,
               uint32_t nlimbs, int kind, uint64_t seed, uint32_t tag, fhe_stream_t stream);
int fhe_keygen_secret(const fhe_ctx* ctx, uint64_t* sk, uint64_t seed, fhe_stream_t stream);
int fhe_keygen_public(const fhe_ctx* ctx, uint64_t* pk, const uint64_t* sk, uint64_t seed,
                      fhe_stream_t stream);
int fhe_keygen_switch(const fhe_ctx* ctx, uint64_t* key, const uint64_t* sk,
                      const uint64_t* s_from, uint64_t seed, fhe_stream_t stream);
int fhe_encrypt(const fhe_ctx* ctx, uint64_t* ct, const uint64_t* pt, const uint64_t* pk,
                uint64_t seed, void* workspace, fhe_stream_t stream);
int fhe_encrypt_sk(const fhe_ctx* ctx, uint64_t* ct, const uint64_t* pt, const uint64_t* sk,
                   uint64_t seed, fhe_stream_t stream);
int fhe_decrypt(const fhe_ctx* ctx, uint64_t* pt, const uint64_t* ct, const uint64_t* sk,
                uint32_t batch, uint32_t nlimbs, fhe_stream_t stream);

/* ---- fused multiply -> relinearise -> rescale ------------------------
 * a, b [batch][2][L][N] NTT form; evk_b, evk_a [dnum][L + K][N] the relinearisation key (NTT
 * form, as for fhe_keyswitch).  out = Relin(a x b) [batch][2][L][N], or with rescale != 0 its
 * divide-and-round by q_{L-1}, [batch][2][L-1][N]; NTT form.  Restated by oracle mul_relin. */
size_t fhe_mul_relin_workspace(const fhe_ctx* ctx, uint32_t batch);
int fhe_mul_relin(const fhe_ctx* ctx, uint64_t* out, const uint64_t* a, const uint64_t* b,
                  const uint64_t* evk_b, const uint64_t* evk_a, uint32_t batch, int rescale,
                  void* workspace, fhe_stream_t stream);

/* ---- HIP graphs: capture a sequence of libfhecore calls on `stream` and replay it -----------
 * Between fhe_graph_begin and fhe_graph_end every call that takes a workspace must be given an
 * explicit one: with workspace == NULL a call returns FHE_EINVAL while the stream is capturing
 * (the context's internal workspace may be reallocated later, which would leave the graph
 * pointing at freed memory).  Replays reuse the captured pointers, so every buffer a captured
 * call touches must outlive the graph. */
typedef struct fhe_graph_s* fhe_graph_t;
int fhe_graph_begin(fhe_stream_t stream);
int fhe_graph_end(fhe_stream_t stream, fhe_graph_t* graph);
int fhe_graph_launch(fhe_graph_t graph, fhe_stream_t stream);
int fhe_graph_destroy(fhe_graph_t graph);

/* ---- timing marks (measurement support, not part of the reference surface) ------------------
 * fhe_prof_begin records a HIP event on `stream`, then every kernel this host thread launches
 * through libfhecore records one more event after itself (up to max_marks).  fhe_prof_end waits
 * for the last event and returns the per-launch elapsed times (ms) and the kernel names,
 * newline-separated, in launch order. */
int fhe_prof_begin(uint32_t max_marks, fhe_stream_t stream);
int fhe_prof_end(float* elapsed_ms, uint32_t cap, uint32_t* count, char* names, size_t names_cap);

#ifdef __cplusplus
}
#endif

#endif /* FHECORE_H */
