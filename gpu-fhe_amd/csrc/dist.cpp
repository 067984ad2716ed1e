// Multi-GPU key-switch at the C ABI: RNS limbs sharded over the ranks of an RCCL
// communicator, one all-gather per key-switch -- over xGMI between the GPUs of a node.
//
// Rank r of G owns Q-limbs [r c, min((r + 1) c, L)), c = ceil(L / G), of every ciphertext, plus
// the key rows of those limbs and of all K special primes.  fhe_keyswitch_dist:
//   1. INTT of the rank's d2 limbs, straight into its block of the gather buffer;
//   2. one ncclAllGather (in place) of the coefficient-form d2 -> [G][chunk][c][N] on every rank;
//   3. ModUp / NTT / inner product / ModDown of the rank's limbs (launch_keyswitch_shard, reading
//      the rank-major gather layout directly: CAll::ranked -- no reorder copy).
// The batch is split into chunks: the INTTs of every chunk are queued first on the caller's
// stream, each chunk's all-gather runs on the communicator's own stream as soon as its INTT is
// done, and the caller's stream waits for a chunk's gather only right before its key-switch, so
// chunk k + 1's transfer overlaps chunk k's key-switch.
// The reference has no communication code at all (/root/reference/arithmetic.py:1 is its only
// import); the sharded algorithm is restated by oracle/pyoracle.py keyswitch_shard.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "../../include/fhecore.h"
#include "internal.hpp"

struct fhe_comm_s {
  ncclComm_t nccl = nullptr;
  int nranks = 1, rank = 0, device = 0;
  hipStream_t stream = nullptr;  // the all-gathers
  static constexpr int kMaxChunks = 16;
  hipEvent_t ev_intt[kMaxChunks] = {}, ev_gather[kMaxChunks] = {};
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

u32 shard_width(u32 L, u32 G) { return (L + G - 1) / G; }

void shard_of(u32 L, u32 G, u32 r, u32* limb0, u32* nlimbs) {
  const u32 c = shard_width(L, G);
  const u32 lo = std::min(L, r * c);
  *limb0 = lo;
  *nlimbs = std::min(L, lo + c) - lo;
}

// Split a batch into nc chunks of cb ciphertexts (the last one possibly shorter, none empty).
void chunking(u32 batch, u32 chunks, u32* nc, u32* cb) {
  const u32 want = std::max(1u, std::min({chunks ? chunks : 4u, std::max(batch, 1u),
                                           (u32)fhe_comm_s::kMaxChunks}));
  *cb = (std::max(batch, 1u) + want - 1) / want;
  *nc = (std::max(batch, 1u) + *cb - 1) / *cb;
}

}  // namespace
}  // namespace fhe

using namespace fhe;

extern "C" {

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
    if (c->ev_intt[k]) (void)hipEventDestroy(c->ev_intt[k]);
    if (c->ev_gather[k]) (void)hipEventDestroy(c->ev_gather[k]);
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

size_t fhe_keyswitch_dist_workspace(const fhe_ctx* ctx, fhe_comm_t comm, uint32_t batch,
                                    uint32_t chunks) {
  if (!ctx || !comm) return 0;
  u32 limb0, nl;
  shard_of(ctx->L, (u32)comm->nranks, (u32)comm->rank, &limb0, &nl);
  const u32 cw = shard_width(ctx->L, (u32)comm->nranks);
  u32 nc, cb;
  chunking(batch, chunks, &nc, &cb);
  const size_t gather = (size_t)nc * comm->nranks * cb * cw * ctx->n * sizeof(u64);
  return gather + keyswitch_workspace_bytes(ctx, nl, cb);
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
  if (batch == 0) return kOk;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const u32 G = (u32)comm->nranks, r = (u32)comm->rank, L = ctx->L;
  u32 limb0, nl;
  shard_of(L, G, r, &limb0, &nl);
  const u32 cw = shard_width(L, G);
  u32 nc, cb;
  chunking(batch, chunks, &nc, &cb);
  const u64 n = ctx->n, blk = (u64)cb * cw * n;  // one rank's block of one chunk
  int rc;
  if ((rc = ensure_ws(ctx, fhe_keyswitch_dist_workspace(ctx, comm, batch, chunks), &ws, s)))
    return rc;
  u64* gather = static_cast<u64*>(ws);  // [nc][G][cb][cw][N]
  // the gathered d2 is the prepared ModUp input when the fused ModUp applies: each rank's INTT
  // folds (D^_k)^-1 of its limbs' digits into its last stage
  const bool prep = ks_prepared(ctx);
  void* kws = gather + (u64)nc * G * blk;
  // 1 + 2: every chunk's INTT into its send block, then its gather on the comm stream
  for (u32 k = 0; k < nc; ++k) {
    const u32 b0 = k * cb, bn = std::min(batch, b0 + cb) - b0;
    u64* gbuf = gather + (u64)k * G * blk;
    if (nl && bn &&
        (rc = launch_ntt_strided(ctx, false, d2_own + (u64)b0 * nl * n, (u64)nl * n,
                                 gbuf + (u64)r * blk, (u64)cw * n, bn, limb0, nl, s,
                                 prep ? ctx->d_nfold_up : nullptr,
                                 prep && ks_split30(ctx))))
      return rc;
    FHE_HIP_CHECK(hipEventRecord(comm->ev_intt[k], s));
    FHE_HIP_CHECK(hipStreamWaitEvent(comm->stream, comm->ev_intt[k], 0));
    FHE_NCCL_CHECK(ncclAllGather(gbuf + (u64)r * blk, gbuf, blk, ncclUint64, comm->nccl,
                                 comm->stream));
    FHE_HIP_CHECK(hipEventRecord(comm->ev_gather[k], comm->stream));
  }
  prof_mark(s, "ks_dist_intt");
  // 3: each chunk's key-switch once its gather has landed
  for (u32 k = 0; k < nc; ++k) {
    const u32 b0 = k * cb, bn = std::min(batch, b0 + cb) - b0;
    FHE_HIP_CHECK(hipStreamWaitEvent(s, comm->ev_gather[k], 0));
    if (!nl || !bn) continue;
    CAll call = CAll::ranked(gather + (u64)k * G * blk, L, G, cb, n);
    call.scaled = prep;
    const u64 off = (u64)b0 * nl * n;
    if ((rc = launch_keyswitch_shard(ctx, ks0 + off, ks1 + off, call, d2_own + off, evk_b, evk_a,
                                     limb0, nl, bn, kws, s)))
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
