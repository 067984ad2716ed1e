// Multi-GPU key-switch at the C ABI: RNS limbs sharded over the ranks of an RCCL
// communicator, one all-gather per key-switch -- over xGMI between the GPUs of a node.
//
// Rank r of G owns Q-limbs [r c, min((r + 1) c, L)), c = ceil(L / G), of every ciphertext, plus
// the key rows of those limbs and of all K special primes.  fhe_keyswitch_dist:
//   1. INTT of the rank's d2 limbs, straight into its block of the gather buffer;
//   2. one ncclAllGather (in place) of the coefficient-form d2 -> [G][chunk][c][N] on every rank;
//   3. ModUp / NTT / inner product / ModDown of the rank's limbs (launch_keyswitch_shard, reading
//      the rank-major gather layout directly: CAll::ranked -- no reorder copy).
// The batch is split into chunks: chunk k + 1's INTT is queued on the caller's stream right
// before chunk k's key-switch, its all-gather runs on the communicator's own stream as soon as
// that INTT is done, and the caller's stream waits for a chunk's gather only right before its
// key-switch, so chunk k + 1's transfer overlaps chunk k's key-switch (and at most two chunks of
// gathered d2 are live, which keeps ModUp's sources in the Infinity Cache).
// Every offset comes from one host-side plan (fhe_dist_plan_*, exported so that the CPU suite
// checks it for G = 1..8 without a GPU), and fhe_keyswitch_dist_loopback runs the same plan and
// the same per-chunk steps for G virtual ranks on one device (the GPU suite's G > 1 path).
// The reference has no communication code at all (/root/reference/arithmetic.py:1 is its only
// import); the sharded algorithm is restated by oracle/pyoracle.py keyswitch_shard.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fhecore.h"
#include "internal.hpp"

struct fhe_comm_s {
  ncclComm_t nccl = nullptr;
  int nranks = 1, rank = 0, device = 0;
  hipStream_t stream = nullptr;  // the all-gathers
  static constexpr int kMaxChunks = 16;
  hipEvent_t ev_intt[kMaxChunks] = {}, ev_gather[kMaxChunks] = {};
  // timing events around each chunk's all-gather on `stream` (fhe_comm_gather_ms)
  hipEvent_t ev_g0[kMaxChunks] = {}, ev_g1[kMaxChunks] = {};
  uint32_t last_chunks = 0;
};

namespace fhe {
namespace {

#define FHE_NCCL_CHECK(expr)                                                              \
  do {                                                                                    \
    ncclResult_t r_ = (expr);                                                             \
    if (r_ != ncclSuccess) {                                                              \
      set_error(std::string(#expr) + ": " + ncclGetErrorString(r_));                      \
      return kDevice;                                                                     \
    }                                                                                     \
  } while (0)

constexpr uint64_t kBad = ~0ull;

u32 shard_width(u32 L, u32 G) { return (L + G - 1) / G; }

void shard_of(u32 L, u32 G, u32 r, u32* limb0, u32* nlimbs) {
  const u32 c = shard_width(L, G);
  const u32 lo = std::min(L, r * c);
  *limb0 = lo;
  *nlimbs = std::min(L, lo + c) - lo;
}

// The chunk's view of the gather region: CAll::ranked over one chunk's [G][cb][c][N] blocks --
// the addressing launch_keyswitch_shard's kernels use for the source rows.
CAll chunk_call(const fhe_dist_plan& p, const u64* gather, u32 k) {
  return CAll::ranked(gather + (u64)k * p.ranks * p.block_words, p.L, p.ranks, p.chunk_batch,
                      1ull << p.log_n);
}

// One chunk's INTT of this rank's own limbs into its send block (what ncclAllGather sends).
int dist_intt_chunk(const fhe_ctx* ctx, const fhe_dist_plan& p, u32 k, const u64* d2_own,
                    u64* gather, hipStream_t s) {
  u32 b0, bn;
  fhe_dist_plan_chunk(&p, k, &b0, &bn);
  if (!p.nlimbs || !bn) return kOk;
  const u64 n = ctx->n;
  // the gathered d2 is the prepared ModUp input when the fused ModUp applies: each rank's INTT
  // folds (D^_k)^-1 of its limbs' digits into its last stage
  const bool prep = ks_prepared(ctx);
  return launch_ntt_strided(ctx, false, d2_own + (u64)b0 * p.nlimbs * n, (u64)p.nlimbs * n,
                            gather + fhe_dist_plan_send_word(&p, b0, 0), (u64)p.width * n, bn,
                            p.limb0, p.nlimbs, s, prep ? ctx->d_nfold_up : nullptr,
                            prep && ks_split30(ctx));
}

// One chunk's local key-switch once its gather has landed.
int dist_ks_chunk(const fhe_ctx* ctx, const fhe_dist_plan& p, u32 k, u64* ks0, u64* ks1,
                  const u64* d2_own, const u64* evk_b, const u64* evk_a, const u64* gather,
                  void* kws, hipStream_t s) {
  u32 b0, bn;
  fhe_dist_plan_chunk(&p, k, &b0, &bn);
  if (!p.nlimbs || !bn) return kOk;
  CAll call = chunk_call(p, gather, k);
  call.scaled = ks_prepared(ctx);
  const u64 off = (u64)b0 * p.nlimbs * ctx->n;
  return launch_keyswitch_shard(ctx, ks0 + off, ks1 + off, call, d2_own + off, evk_b, evk_a,
                                p.limb0, p.nlimbs, bn, kws, s);
}

size_t dist_workspace(const fhe_ctx* ctx, const fhe_dist_plan& p, u32 max_nlimbs) {
  return p.gather_words * sizeof(u64) + keyswitch_workspace_bytes(ctx, max_nlimbs, p.chunk_batch);
}

}  // namespace
}  // namespace fhe

using namespace fhe;

extern "C" {

int fhe_dist_plan_make(fhe_dist_plan* p, uint32_t L, uint32_t log_n, uint32_t G, uint32_t r,
                       uint32_t batch, uint32_t chunks) {
  if (!p || L == 0 || G == 0 || r >= G || log_n > 30) {
    set_error("fhe_dist_plan_make: need L >= 1, 0 <= rank < ranks");
    return kInvalid;
  }
  *p = fhe_dist_plan{};
  p->L = L;
  p->log_n = log_n;
  p->ranks = G;
  p->rank = r;
  p->batch = batch;
  shard_of(L, G, r, &p->limb0, &p->nlimbs);
  p->width = shard_width(L, G);
  // nc chunks of cb ciphertexts (the last one possibly shorter, none empty); 0 = default 4
  const u32 b = std::max(batch, 1u);
  const u32 want = std::max(1u, std::min({chunks ? chunks : 4u, b, (u32)fhe_comm_s::kMaxChunks}));
  p->chunk_batch = (b + want - 1) / want;
  p->chunks = (b + p->chunk_batch - 1) / p->chunk_batch;
  p->block_words = (u64)p->chunk_batch * p->width << log_n;
  p->gather_words = (u64)p->chunks * G * p->block_words;
  return kOk;
}

int fhe_dist_plan_chunk(const fhe_dist_plan* p, uint32_t k, uint32_t* b0, uint32_t* bn) {
  if (!p || !b0 || !bn || k >= p->chunks) {
    set_error("fhe_dist_plan_chunk: chunk out of range");
    return kInvalid;
  }
  *b0 = std::min(p->batch, k * p->chunk_batch);
  *bn = std::min(p->batch, *b0 + p->chunk_batch) - *b0;
  return kOk;
}

uint64_t fhe_dist_plan_send_word(const fhe_dist_plan* p, uint32_t b, uint32_t j) {
  if (!p || b >= p->batch || j >= p->nlimbs) return kBad;
  const u32 k = b / p->chunk_batch, bi = b % p->chunk_batch;
  const u64 n = 1ull << p->log_n;
  // the INTT of chunk k writes this rank's rows at poly stride width N into its block
  return ((u64)k * p->ranks + p->rank) * p->block_words + ((u64)bi * p->width + j) * n;
}

uint64_t fhe_dist_plan_read_word(const fhe_dist_plan* p, uint32_t b, uint32_t l) {
  if (!p || b >= p->batch || l >= p->L) return kBad;
  const u32 k = b / p->chunk_batch, bi = b % p->chunk_batch;
  // exactly the kernels' addressing: chunk k's CAll::ranked view, ciphertext bi, limb l
  const CAll call = CAll::ranked(nullptr, p->L, p->ranks, p->chunk_batch, 1ull << p->log_n);
  return (u64)k * p->ranks * p->block_words + (u64)bi * call.bs + call.off(l, 1ull << p->log_n);
}

int fhe_comm_get_unique_id(uint8_t* id) {
  if (!id) {
    set_error("fhe_comm_get_unique_id: null output");
    return kInvalid;
  }
  static_assert(sizeof(ncclUniqueId) == FHE_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId uid;
  FHE_NCCL_CHECK(ncclGetUniqueId(&uid));
  std::memcpy(id, &uid, sizeof(uid));
  return kOk;
}

int fhe_comm_create(fhe_comm_t* comm, const uint8_t* id, int nranks, int rank, int device) {
  if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks) {
    set_error("fhe_comm_create: need an id, 0 <= rank < nranks");
    return kInvalid;
  }
  *comm = nullptr;
  FHE_HIP_CHECK(hipSetDevice(device));
  auto* c = new fhe_comm_s();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, uid, rank);
  if (r != ncclSuccess) {
    set_error(std::string("fhe_comm_create: ncclCommInitRank: ") + ncclGetErrorString(r));
    delete c;
    return kDevice;
  }
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  for (int k = 0; k < fhe_comm_s::kMaxChunks && e == hipSuccess; ++k) {
    e = hipEventCreateWithFlags(&c->ev_intt[k], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_gather[k], hipEventDisableTiming);
    // timing-only events: no system-scope fence (no L2 writeback / invalidate at each record)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_g0[k], hipEventDisableSystemFence);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_g1[k], hipEventDisableSystemFence);
  }
  if (e != hipSuccess) {
    set_error(std::string("fhe_comm_create: ") + hipGetErrorString(e));
    fhe_comm_destroy(c);
    return kDevice;
  }
  *comm = c;
  return kOk;
}

int fhe_comm_destroy(fhe_comm_t c) {
  if (!c) return kOk;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (int k = 0; k < fhe_comm_s::kMaxChunks; ++k) {
    for (hipEvent_t ev : {c->ev_intt[k], c->ev_gather[k], c->ev_g0[k], c->ev_g1[k]})
      if (ev) (void)hipEventDestroy(ev);
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->nccl) (void)ncclCommDestroy(c->nccl);
  delete c;
  return kOk;
}

int fhe_comm_shard(const fhe_ctx* ctx, fhe_comm_t comm, uint32_t* limb0, uint32_t* nlimbs) {
  if (!ctx || !comm || !limb0 || !nlimbs) {
    set_error("fhe_comm_shard: null argument");
    return kInvalid;
  }
  shard_of(ctx->L, (u32)comm->nranks, (u32)comm->rank, limb0, nlimbs);
  return kOk;
}

int fhe_comm_gather_ms(fhe_comm_t comm, float* ms, uint32_t cap, uint32_t* count) {
  if (!comm || !count || (cap && !ms)) {
    set_error("fhe_comm_gather_ms: null argument");
    return kInvalid;
  }
  *count = comm->last_chunks;
  for (u32 k = 0; k < std::min(cap, comm->last_chunks); ++k) {
    FHE_HIP_CHECK(hipEventSynchronize(comm->ev_g1[k]));
    FHE_HIP_CHECK(hipEventElapsedTime(&ms[k], comm->ev_g0[k], comm->ev_g1[k]));
  }
  return kOk;
}

size_t fhe_keyswitch_dist_workspace(const fhe_ctx* ctx, fhe_comm_t comm, uint32_t batch,
                                    uint32_t chunks) {
  if (!ctx || !comm) return 0;
  fhe_dist_plan p;
  if (fhe_dist_plan_make(&p, ctx->L, ctx->log_n, (u32)comm->nranks, (u32)comm->rank, batch,
                         chunks))
    return 0;
  return dist_workspace(ctx, p, p.nlimbs);
}

int fhe_keyswitch_dist(const fhe_ctx* ctx, fhe_comm_t comm, uint64_t* ks0, uint64_t* ks1,
                       const uint64_t* d2_own, const uint64_t* evk_b, const uint64_t* evk_a,
                       uint32_t batch, uint32_t chunks, void* ws, fhe_stream_t stream) {
  if (!ctx || !comm) {
    set_error("fhe_keyswitch_dist: null context or communicator");
    return kInvalid;
  }
  if (ctx->K == 0) {
    set_error("fhe_keyswitch_dist: context has no special primes (K = 0)");
    return kInvalid;
  }
  if (comm->device != ctx->device) {
    // the gathers and their events would run on one device, the kernels on another
    set_error("fhe_keyswitch_dist: communicator on device " + std::to_string(comm->device) +
              ", context on device " + std::to_string(ctx->device));
    return kInvalid;
  }
  comm->last_chunks = 0;
  if (batch == 0) return kOk;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  fhe_dist_plan p;
  int rc;
  if ((rc = fhe_dist_plan_make(&p, ctx->L, ctx->log_n, (u32)comm->nranks, (u32)comm->rank, batch,
                               chunks)))
    return rc;
  // whole batch: chunk k's outputs must not land on a later chunk's d2 (fhecore.h aliasing rule)
  const u64 own_words = (u64)batch * p.nlimbs * ctx->n;
  if ((rc = ks_check_alias(ks0, ks1, d2_own, own_words, own_words, true, "fhe_keyswitch_dist")))
    return rc;
  if ((rc = ensure_ws(ctx, dist_workspace(ctx, p, p.nlimbs), &ws, s))) return rc;
  u64* gather = static_cast<u64*>(ws);  // [nc][G][cb][cw][N]
  void* kws = gather + p.gather_words;
  // 1 + 2: a chunk's INTT into its send block, then its gather on the comm stream.  With one
  // chunk nothing could overlap the gather, so it runs on the caller's stream: a cross-stream
  // event hand-off costs ~40 us of idle GPU per call (measured).
  const bool own_stream = p.chunks > 1;
  const hipStream_t gs = own_stream ? comm->stream : s;
  auto issue = [&](u32 k) -> int {
    int r;
    if ((r = dist_intt_chunk(ctx, p, k, d2_own, gather, s))) return r;
    u64* gbuf = gather + (u64)k * p.ranks * p.block_words;
    if (own_stream) {
      FHE_HIP_CHECK(hipEventRecord(comm->ev_intt[k], s));
      FHE_HIP_CHECK(hipStreamWaitEvent(gs, comm->ev_intt[k], 0));
    }
    FHE_HIP_CHECK(hipEventRecord(comm->ev_g0[k], gs));
    FHE_NCCL_CHECK(ncclAllGather(gbuf + (u64)p.rank * p.block_words, gbuf, p.block_words,
                                 ncclUint64, comm->nccl, gs));
    FHE_HIP_CHECK(hipEventRecord(comm->ev_g1[k], gs));
    if (own_stream) FHE_HIP_CHECK(hipEventRecord(comm->ev_gather[k], gs));
    return kOk;
  };
  // 3: chunk k's key-switch once its gather has landed, with chunk k + 1's INTT queued just
  // before it (its gather overlaps this key-switch) and no further: only two chunks of gathered
  // d2 are live at a time, so ModUp reads its sources from the Infinity Cache the gather just
  // wrote instead of from HBM (all INTTs first left every chunk but the last evicted once the
  // gathered batch outgrew the cache: DESIGN.md §8)
  // The "ks_dist_intt" mark covers chunk 0's INTT (+ gather on the caller's stream) only: chunk
  // k + 1's INTT is queued inside chunk k's key-switch, so its time counts in that chunk's marks.
  if ((rc = issue(0))) return rc;
  prof_mark(s, "ks_dist_intt");
  for (u32 k = 0; k < p.chunks; ++k) {
    if (k + 1 < p.chunks && (rc = issue(k + 1))) return rc;
    if (own_stream) FHE_HIP_CHECK(hipStreamWaitEvent(s, comm->ev_gather[k], 0));
    if ((rc = dist_ks_chunk(ctx, p, k, ks0, ks1, d2_own, evk_b, evk_a, gather, kws, s)))
      return rc;
  }
  comm->last_chunks = p.chunks;
  return kOk;
}

size_t fhe_keyswitch_dist_loopback_workspace(const fhe_ctx* ctx, uint32_t ranks, uint32_t batch,
                                             uint32_t chunks) {
  if (!ctx || ranks == 0) return 0;
  fhe_dist_plan p;
  if (fhe_dist_plan_make(&p, ctx->L, ctx->log_n, ranks, 0, batch, chunks)) return 0;
  return dist_workspace(ctx, p, p.width);  // rank 0 owns a full block of width limbs
}

int fhe_keyswitch_dist_loopback(const fhe_ctx* ctx, uint32_t ranks, uint64_t* const* ks0,
                                uint64_t* const* ks1, const uint64_t* const* d2_own,
                                const uint64_t* const* evk_b, const uint64_t* const* evk_a,
                                uint32_t batch, uint32_t chunks, void* ws, fhe_stream_t stream) {
  if (!ctx || ranks == 0 || !ks0 || !ks1 || !d2_own || !evk_b || !evk_a) {
    set_error("fhe_keyswitch_dist_loopback: null context or per-rank array, or zero ranks");
    return kInvalid;
  }
  if (ctx->K == 0) {
    set_error("fhe_keyswitch_dist_loopback: context has no special primes (K = 0)");
    return kInvalid;
  }
  if (batch == 0) return kOk;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<fhe_dist_plan> plan(ranks);
  int rc;
  for (u32 r = 0; r < ranks; ++r) {
    if ((rc = fhe_dist_plan_make(&plan[r], ctx->L, ctx->log_n, ranks, r, batch, chunks)))
      return rc;
    if (plan[r].nlimbs && (!ks0[r] || !ks1[r] || !d2_own[r] || !evk_b[r] || !evk_a[r])) {
      set_error("fhe_keyswitch_dist_loopback: null pointer for rank " + std::to_string(r));
      return kInvalid;
    }
    const u64 own_words = (u64)batch * plan[r].nlimbs * ctx->n;
    if ((rc = ks_check_alias(ks0[r], ks1[r], d2_own[r], own_words, own_words, true,
                             "fhe_keyswitch_dist_loopback")))
      return rc;
  }
  if ((rc = ensure_ws(ctx, fhe_keyswitch_dist_loopback_workspace(ctx, ranks, batch, chunks), &ws,
                      s)))
    return rc;
  u64* gather = static_cast<u64*>(ws);  // one region shared by the virtual ranks
  void* kws = gather + plan[0].gather_words;
  // every rank's INTT writes its own blocks: the region then holds what an in-place all-gather
  // leaves on each rank
  for (u32 k = 0; k < plan[0].chunks; ++k)
    for (u32 r = 0; r < ranks; ++r)
      if ((rc = dist_intt_chunk(ctx, plan[r], k, d2_own[r], gather, s))) return rc;
  for (u32 k = 0; k < plan[0].chunks; ++k)
    for (u32 r = 0; r < ranks; ++r)
      if ((rc = dist_ks_chunk(ctx, plan[r], k, ks0[r], ks1[r], d2_own[r], evk_b[r], evk_a[r],
                              gather, kws, s)))
        return rc;
  return kOk;
}

// ---- hybrid partition: `groups` ciphertext groups x g = ranks / groups limb shards -----------
int fhe_dist_hybrid_make(fhe_dist_hybrid* h, uint32_t L, uint32_t log_n, uint32_t ranks,
                         uint32_t groups, uint32_t rank, uint32_t batch, uint32_t chunks) {
  if (!h || groups == 0 || ranks == 0 || ranks % groups || rank >= ranks) {
    set_error("fhe_dist_hybrid_make: need groups | ranks and 0 <= rank < ranks");
    return kInvalid;
  }
  *h = fhe_dist_hybrid{};
  h->ranks = ranks;
  h->groups = groups;
  h->g = ranks / groups;
  // group k = ranks [k g, (k + 1) g): a limb plan of g ranks over the group's ciphertexts
  h->group = rank / h->g;
  h->shard = rank % h->g;
  const u32 cb = (batch + groups - 1) / groups;
  h->batch0 = std::min(batch, h->group * cb);
  h->batch = std::min(batch, h->batch0 + cb) - h->batch0;
  return fhe_dist_plan_make(&h->plan, L, log_n, h->g, h->shard, h->batch, chunks);
}

size_t fhe_keyswitch_dist_hybrid_loopback_workspace(const fhe_ctx* ctx, uint32_t ranks,
                                                    uint32_t groups, uint32_t batch,
                                                    uint32_t chunks) {
  if (!ctx || ranks == 0 || groups == 0 || ranks % groups) return 0;
  // groups run one after another on the shared workspace: group 0 has the most ciphertexts
  fhe_dist_hybrid h;
  if (fhe_dist_hybrid_make(&h, ctx->L, ctx->log_n, ranks, groups, 0, batch, chunks)) return 0;
  return fhe_keyswitch_dist_loopback_workspace(ctx, h.g, std::max(h.batch, 1u), chunks);
}

int fhe_keyswitch_dist_hybrid_loopback(const fhe_ctx* ctx, uint32_t ranks, uint32_t groups,
                                       uint64_t* const* ks0, uint64_t* const* ks1,
                                       const uint64_t* const* d2_own,
                                       const uint64_t* const* evk_b,
                                       const uint64_t* const* evk_a, uint32_t batch,
                                       uint32_t chunks, void* ws, fhe_stream_t stream) {
  if (!ctx || ranks == 0 || groups == 0 || ranks % groups || !ks0 || !ks1 || !d2_own || !evk_b ||
      !evk_a) {
    set_error("fhe_keyswitch_dist_hybrid_loopback: null argument, or groups does not divide ranks");
    return kInvalid;
  }
  if (batch == 0) return kOk;
  if (!ws) {  // one internal workspace for every group, sized once (the groups run in order)
    int rc = ensure_ws(ctx, fhe_keyswitch_dist_hybrid_loopback_workspace(ctx, ranks, groups, batch,
                                                                         chunks),
                       &ws, static_cast<hipStream_t>(stream));
    if (rc) return rc;
  }
  const u32 g = ranks / groups;
  for (u32 k = 0; k < groups; ++k) {
    fhe_dist_hybrid h;
    if (int rc = fhe_dist_hybrid_make(&h, ctx->L, ctx->log_n, ranks, groups, k * g, batch, chunks))
      return rc;
    // the group's g ranks: an independent limb-sharded key-switch of its ciphertexts
    if (int rc = fhe_keyswitch_dist_loopback(ctx, g, ks0 + k * g, ks1 + k * g, d2_own + k * g,
                                             evk_b + k * g, evk_a + k * g, h.batch, chunks, ws,
                                             stream))
      return rc;
  }
  return kOk;
}

int fhe_keyswitch_shard_ranked(const fhe_ctx* ctx, uint64_t* ks0, uint64_t* ks1,
                               const uint64_t* c_gathered, uint32_t ranks, const uint64_t* d2_own,
                               const uint64_t* evk_b, const uint64_t* evk_a, uint32_t limb0,
                               uint32_t nlimbs, uint32_t batch, void* ws, fhe_stream_t stream) {
  if (!ctx || ranks == 0) {
    set_error("fhe_keyswitch_shard_ranked: null context or zero ranks");
    return kInvalid;
  }
  const u32 cw = shard_width(ctx->L, ranks);
  u32 lo, nl;
  shard_of(ctx->L, ranks, limb0 / cw, &lo, &nl);
  if (limb0 % cw || lo != limb0 || nl != nlimbs || nlimbs == 0) {
    set_error("fhe_keyswitch_shard_ranked: limb window is not a rank's shard [r c, min((r+1) c, L))");
    return kInvalid;
  }
  const hipStream_t s = static_cast<hipStream_t>(stream);
  int rc;
  if ((rc = ensure_ws(ctx, keyswitch_workspace_bytes(ctx, nlimbs, batch), &ws, s))) return rc;
  return launch_keyswitch_shard(ctx, ks0, ks1, CAll::ranked(c_gathered, ctx->L, ranks, batch, ctx->n),
                                d2_own, evk_b, evk_a, limb0, nlimbs, batch, ws, s);
}

}  // extern "C"
