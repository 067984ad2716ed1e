// Fused multiply -> relinearise -> rescale pipeline and HIP-graph capture:
// the CKKS ct x ct product as it is used in practice, everything in NTT form:
//   d = (a0 b0, a0 b1 + a1 b0, a1 b1)            elementwise tensor (k_tensor_ntt)
//   (ks0, ks1) = KeySwitch(d2, relin key)          the batched hybrid key-switch (rns.hip)
//   ct = (d0 + ks0, d1 + ks1)                      folded into the key-switch's ModDown finish
//                                                  (KsEpilogue: no separate combine pass)
//   [optional] ct = Rescale(ct)                    divide-and-round by the last modulus (galois.hip)
// Restated by oracle/pyoracle.py (mul_relin); not in the reference, whose only ciphertext
// operation is poly_add (/root/reference/ polynomial.py:3-5).  The launches never allocate or
// synchronise given a workspace, so the whole pipeline can be captured into a hipGraph once and
// replayed (fhe_graph_*), removing per-launch host overhead from repeated small-batch calls.
#include "../../include/fhecore.h"
#include "internal.hpp"

namespace fhe {
namespace {


// a, b [batch][2][L][N] NTT form, canonical -> d0, d1 into d [batch][2][L][N] and d2 into its own
// contiguous [batch][L][N] (the key-switch's operand, no gather copy).  Grid: x over coefficient
// pairs (16-byte accesses), y = limb, z = ciphertext.  a, b are read once and d0, d1 are read back
// only by the key-switch's finish, long after they left the caches: non-temporal; d2 stays cached
// for the INTT that reads it next.
typedef u64 vu64x2 __attribute__((ext_vector_type(2)));
constexpr int kTensorThreads = 128;
__global__ __launch_bounds__(kTensorThreads) void k_tensor_ntt(u64* __restrict__ d,
                                                               u64* __restrict__ d2,
                                                               const u64* __restrict__ a,
                                                               const u64* __restrict__ b, u32 L,
                                                               u32 log_n,
                                                               const ModParams* __restrict__ mods) {
  const u64 n = 1ull << log_n, ln = (u64)L * n;
  const u64 c = 2 * ((u64)blockIdx.x * blockDim.x + threadIdx.x);
  const u32 l = blockIdx.y;
  const u64 bt = blockIdx.z;
  const ModParams m = mods[l];
  const u64 off = bt * 2 * ln + (u64)l * n + c;
  auto ld = [](const u64* p) { return __builtin_nontemporal_load(reinterpret_cast<const vu64x2*>(p)); };
  const vu64x2 a0 = ld(a + off), a1 = ld(a + off + ln), b0 = ld(b + off), b1 = ld(b + off + ln);
  vu64x2 o0, o1, o2;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const u128 t0 = (u128)a0[h] * b0[h], t2 = (u128)a1[h] * b1[h];
    const u128 t1 = (u128)a0[h] * b1[h] + (u128)a1[h] * b0[h];
    o0[h] = reduce128_any((u64)t0, (u64)(t0 >> 64), m);
    o1[h] = reduce128_any((u64)t1, (u64)(t1 >> 64), m);
    o2[h] = reduce128_any((u64)t2, (u64)(t2 >> 64), m);
  }
  u64* o = d + bt * 2 * ln + (u64)l * n + c;
  __builtin_nontemporal_store(o0, reinterpret_cast<vu64x2*>(o));
  __builtin_nontemporal_store(o1, reinterpret_cast<vu64x2*>(o + ln));
  *reinterpret_cast<vu64x2*>(d2 + bt * ln + (u64)l * n + c) = o2;
}

}  // namespace

size_t mul_relin_workspace_bytes(const fhe_ctx* c, u32 batch) {
  const size_t ln = (size_t)c->L * c->n * sizeof(u64);
  // d0, d1 [2], relinearised ct before the rescale [2], d2 [1] (the key-switch's finish may run in
  // the same kernel as its reads of d2, k_ks_row_fin, so d2 cannot park in the output), the
  // rescale's own [2 L N] workspace, the key-switch's workspace (its tail holds INTT(d2))
  return (size_t)batch * ln * (2 + 2 + 1) + rescale_workspace_bytes(c, 2 * batch, c->L) +
         keyswitch_workspace_bytes(c, c->L, batch);
}

int launch_mul_relin(const fhe_ctx* c, u64* out, const u64* a, const u64* b, const u64* evk_b,
                     const u64* evk_a, u32 batch, bool rescale, void* ws, hipStream_t s) {
  if (c->K == 0) {
    set_error("mul_relin: context has no special primes (K = 0)");
    return kInvalid;
  }
  if (rescale && c->L < 2) {
    set_error("mul_relin: rescale needs L >= 2");
    return kInvalid;
  }
  if (batch == 0) return kOk;
  const u32 L = c->L;
  const u64 n = c->n, ln = (u64)L * n;
  // Infinity-Cache-sized passes (ks_pass_batch), each in the front of the workspace
  if (const u32 pass = ks_pass_batch(c, batch); pass < batch) {
    const u64 out_bs = 2 * (u64)(rescale ? L - 1 : L) * n;
    for (u32 b0 = 0; b0 < batch; b0 += pass) {
      if (int rc = launch_mul_relin(c, out + b0 * out_bs, a + b0 * 2 * ln, b + b0 * 2 * ln, evk_b,
                                    evk_a, std::min(pass, batch - b0), rescale, ws, s))
        return rc;
    }
    return kOk;
  }
  u64* d = static_cast<u64*>(ws);        // [batch][2][L][N]: d0, d1
  u64* rl = d + 2 * batch * ln;          // [batch][2][L][N] relinearised, before the rescale
  u64* d2 = rl + 2 * batch * ln;         // [batch][L][N] d2, NTT form, the key-switch's input
  u64* rws = d2 + batch * ln;            // rescale workspace
  u64* kws = reinterpret_cast<u64*>(reinterpret_cast<char*>(rws) +
                                    rescale_workspace_bytes(c, 2 * batch, L));
  const u64 tb = n / 2 / kTensorThreads;  // N >= 2^10: whole blocks of coefficient pairs
  if (int rc = check_grid(tb, kTensorThreads, L, batch, "tensor_ntt")) return rc;
  const dim3 g((u32)tb, L, batch);
  k_tensor_ntt<<<g, kTensorThreads, 0, s>>>(d, d2, a, b, L, c->log_n, c->d_mods);
  FHE_HIP_CHECK(hipGetLastError());
  prof_mark(s, "tensor_ntt");
  // d2 = d[b][2]: gather to a contiguous [batch][L][N] operand for the key-switch (its INTT lands
  // at the tail of the key-switch workspace, as in fhe_keyswitch)
  const size_t kbytes = keyswitch_workspace_bytes(c, L, batch);
  u64* c_all = reinterpret_cast<u64*>(reinterpret_cast<char*>(kws) + kbytes) - batch * ln;
  int rc;
  const bool prep = ks_prepared(c);  // the INTT emits ModUp's scaled inputs
  if ((rc = launch_ntt_strided(c, false, d2, ln, c_all, ln, batch, 0, L, s,
                               prep ? c->d_nfold_up : nullptr, prep && ks_split30(c))))
    return rc;
  CAll call = CAll::contiguous(c_all, L, n);
  call.scaled = prep;
  // the relinearised ciphertext (d0 + ks0, d1 + ks1) straight out of the ModDown finish
  // ([batch][2][L][N] outputs and addends, 2 L N apart per ciphertext)
  u64* dst = rescale ? rl : out;
  KsEpilogue ep;
  ep.out_bs = 2 * ln;
  ep.add0 = d;
  ep.add1 = d + ln;
  ep.add_bs = 2 * ln;
  if ((rc = launch_keyswitch_shard(c, dst, dst + ln, call, d2, evk_b, evk_a, 0, L, batch, kws, s,
                                   &ep)))
    return rc;
  prof_mark(s, "relin_keyswitch");
  if (rescale) {
    if ((rc = launch_rescale(c, out, rl, 2 * batch, L, true, rws, s))) return rc;
    prof_mark(s, "rescale");
  }
  return kOk;
}

}  // namespace fhe

// ---- HIP graphs: capture any sequence of libfhecore calls on a stream, replay it -------------
extern "C" {

int fhe_graph_begin(fhe_stream_t stream) {
  FHE_HIP_CHECK(hipStreamBeginCapture(static_cast<hipStream_t>(stream),
                                      hipStreamCaptureModeThreadLocal));
  return fhe::kOk;
}

int fhe_graph_end(fhe_stream_t stream, fhe_graph_t* graph) {
  if (!graph) {
    fhe::set_error("fhe_graph_end: null graph pointer");
    return fhe::kInvalid;
  }
  *graph = nullptr;
  hipGraph_t g = nullptr;
  FHE_HIP_CHECK(hipStreamEndCapture(static_cast<hipStream_t>(stream), &g));
  hipGraphExec_t ge = nullptr;
  const hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    fhe::set_error(std::string("fhe_graph_end: hipGraphInstantiate: ") + hipGetErrorString(e));
    return fhe::kDevice;
  }
  *graph = reinterpret_cast<fhe_graph_t>(ge);
  return fhe::kOk;
}

int fhe_graph_launch(fhe_graph_t graph, fhe_stream_t stream) {
  if (!graph) {
    fhe::set_error("fhe_graph_launch: null graph");
    return fhe::kInvalid;
  }
  FHE_HIP_CHECK(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph),
                               static_cast<hipStream_t>(stream)));
  return fhe::kOk;
}

int fhe_graph_destroy(fhe_graph_t graph) {
  if (graph) FHE_HIP_CHECK(hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph)));
  return fhe::kOk;
}

}  // extern "C"
