// extern "C" entry points of libfhecore (declared in include/fhecore.h): argument checking,
// error reporting and workspace handling around the HIP launchers.
#include "../../include/fhecore.h"

#include <algorithm>
#include <string>

#include "internal.hpp"

namespace fhe {

namespace {
thread_local std::string g_last_error;

inline hipStream_t hs(fhe_stream_t s) { return static_cast<hipStream_t>(s); }

int check_window(const fhe_ctx* c, uint32_t limb0, uint32_t nlimbs, uint32_t limit,
                 const char* who) {
  if (!c) {
    set_error(std::string(who) + ": null context");
    return kInvalid;
  }
  if ((uint64_t)limb0 + nlimbs > limit) {
    set_error(std::string(who) + ": limb window [" + std::to_string(limb0) + ", " +
              std::to_string(limb0 + nlimbs) + ") exceeds " + std::to_string(limit) + " limbs");
    return kInvalid;
  }
  return kOk;
}

}  // namespace

// Internal workspace (grows on demand).  Refused while `s` is capturing a graph: growing it would
// free memory a captured graph still points at, and a graph sharing it with eager calls on other
// streams would race them, so captured calls must bring their own workspace.
// Calls on different streams are ordered: a call whose stream differs from the last user's first
// waits (host side, hipDeviceSynchronize) until the device has finished what was queued before it,
// which includes the last call's launches since calls sharing the internal workspace are issued
// one after another by the host (concurrent host threads must pass their own workspaces,
// fhecore.h).  The last user's stream is not touched again: the caller may have destroyed it.
// Growing the buffer waits the same way before the old one is freed.  The waits, frees and
// allocations run on the context's device whatever device the calling thread has current
// (DeviceScope), so a multi-GPU host thread cannot wait on, or allocate from, the wrong GPU.
// use = false (fhe_ctx_reserve) only sizes the buffer: no stream takes it.
namespace {

// Makes `dev` current for the scope and restores the caller's device after.
struct DeviceScope {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceScope(int dev) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int acquire_ws(fhe_ctx* c, size_t bytes, hipStream_t s, bool use) {
  DeviceScope dev(c->device);
  FHE_HIP_CHECK(dev.err);
  std::lock_guard<std::mutex> lock(c->ws_mutex);
  const bool grow = c->workspace_bytes < bytes;
  if (c->ws_used && ((use && c->ws_stream != s) || grow)) FHE_HIP_CHECK(hipDeviceSynchronize());
  if (grow) {
    if (c->workspace) FHE_HIP_CHECK(hipFree(c->workspace));
    c->workspace = nullptr;
    c->workspace_bytes = 0;
    FHE_HIP_CHECK(hipMalloc(&c->workspace, bytes));
    c->workspace_bytes = bytes;
  }
  if (use) {
    c->ws_stream = s;
    c->ws_used = true;
  }
  return kOk;
}

}  // namespace

int ensure_ws(const fhe_ctx* cc, size_t bytes, void** ws, hipStream_t s) {
  if (*ws) return kOk;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  FHE_HIP_CHECK(hipStreamIsCapturing(s, &st));
  if (st != hipStreamCaptureStatusNone) {
    set_error("workspace == NULL while the stream is capturing a graph: pass a workspace");
    return kInvalid;
  }
  auto* c = const_cast<fhe_ctx*>(cc);
  int rc = acquire_ws(c, bytes, s, true);
  if (rc) return rc;
  *ws = c->workspace;
  return kOk;
}

void set_error(const std::string& msg) { g_last_error = msg; }

}  // namespace fhe

using namespace fhe;

extern "C" {

const char* fhe_last_error(void) { return g_last_error.c_str(); }

const char* fhe_version(void) { return "fhecore 0.1 (gfx950)"; }

int fhe_gen_moduli(uint32_t log_n, uint32_t count, uint32_t bits, uint32_t skip, uint64_t* out) {
  if (!out && count) {
    set_error("fhe_gen_moduli: null output");
    return kInvalid;
  }
  return gen_moduli(log_n, count, bits, skip, out);
}

int fhe_ctx_create(fhe_ctx** ctx, uint32_t log_n, const uint64_t* q, uint32_t L,
                   const uint64_t* p, uint32_t K, uint32_t dnum, int device) {
  if (!q || (K && !p)) {
    set_error("fhe_ctx_create: null modulus array");
    return kInvalid;
  }
  try {
    return ctx_create(ctx, log_n, q, L, p, K, dnum, device);
  } catch (const std::exception& e) {
    set_error(std::string("fhe_ctx_create: ") + e.what());
    return kNoMem;
  }
}

int fhe_ctx_destroy(fhe_ctx* ctx) { return ctx_destroy(ctx); }

int fhe_ctx_moduli(const fhe_ctx* c, uint64_t* moduli, uint64_t* psi) {
  if (!c) {
    set_error("fhe_ctx_moduli: null context");
    return kInvalid;
  }
  for (size_t i = 0; i < c->moduli.size(); ++i) {
    if (moduli) moduli[i] = c->moduli[i];
    if (psi) psi[i] = c->psi[i];
  }
  return kOk;
}

int fhe_ctx_shape(const fhe_ctx* c, uint32_t* log_n, uint32_t* L, uint32_t* K, uint32_t* dnum,
                  int* device) {
  if (!c) {
    set_error("fhe_ctx_shape: null context");
    return kInvalid;
  }
  if (log_n) *log_n = c->log_n;
  if (L) *L = c->L;
  if (K) *K = c->K;
  if (dnum) *dnum = c->dnum;
  if (device) *device = c->device;
  return kOk;
}

int fhe_ctx_reserve(fhe_ctx* c, size_t bytes) {
  if (!c) {
    set_error("fhe_ctx_reserve: null context");
    return kInvalid;
  }
  return acquire_ws(c, bytes, nullptr, false);
}

static int vec_ctx(int op, const fhe_ctx* c, uint64_t* out, const uint64_t* a, const uint64_t* b,
                   uint32_t polys, uint32_t limb0, uint32_t nlimbs, fhe_stream_t s,
                   const char* who) {
  int rc = check_window(c, limb0, nlimbs, c ? c->L + c->K : 0, who);
  if (rc) return rc;
  if ((!out || !a || !b) && (uint64_t)polys * nlimbs) {
    set_error(std::string(who) + ": null data pointer");
    return kInvalid;
  }
  return launch_vec_ctx(c, op, out, a, b, polys, limb0, nlimbs, hs(s));
}

int fhe_vec_add(const fhe_ctx* c, uint64_t* out, const uint64_t* a, const uint64_t* b,
                uint32_t polys, uint32_t limb0, uint32_t nlimbs, fhe_stream_t s) {
  return vec_ctx(kAdd, c, out, a, b, polys, limb0, nlimbs, s, "fhe_vec_add");
}
int fhe_vec_sub(const fhe_ctx* c, uint64_t* out, const uint64_t* a, const uint64_t* b,
                uint32_t polys, uint32_t limb0, uint32_t nlimbs, fhe_stream_t s) {
  return vec_ctx(kSub, c, out, a, b, polys, limb0, nlimbs, s, "fhe_vec_sub");
}
int fhe_vec_mul(const fhe_ctx* c, uint64_t* out, const uint64_t* a, const uint64_t* b,
                uint32_t polys, uint32_t limb0, uint32_t nlimbs, fhe_stream_t s) {
  return vec_ctx(kMul, c, out, a, b, polys, limb0, nlimbs, s, "fhe_vec_mul");
}

int fhe_vec_op_mod(int op, uint64_t* out, const uint64_t* a, const uint64_t* b, uint64_t rows,
                   uint64_t cols, const uint64_t* mods, uint64_t mod_stride, int signed_in,
                   int device, fhe_stream_t s) {
  if (op < kAdd || op > kMul) {
    set_error("fhe_vec_op_mod: op must be 0 (add), 1 (sub) or 2 (mul)");
    return kInvalid;
  }
  if (rows * cols == 0) return kOk;
  if (!out || !a || !b || !mods) {
    set_error("fhe_vec_op_mod: null pointer");
    return kInvalid;
  }
  const uint64_t nm = mod_stride ? (rows - 1) * mod_stride + 1 : 1;
  for (uint64_t i = 0; i < nm; ++i)
    if (mods[i] < 2) {
      set_error("fhe_vec_op_mod: modulus must be >= 2");
      return kInvalid;
    }
  FHE_HIP_CHECK(hipSetDevice(device));
  if (nm <= (uint64_t)kArgMods) {  // the common case: moduli by value, nothing allocated or synced
    ModArgs inl{};
    for (uint64_t i = 0; i < nm; ++i) inl.m[i] = make_mod_params(mods[i]);
    return launch_vec_mod(op, out, a, b, rows, cols, nullptr, inl, mod_stride, signed_in, hs(s));
  }
  std::vector<ModParams> mp(nm);
  for (uint64_t i = 0; i < nm; ++i) mp[i] = make_mod_params(mods[i]);
  ModParams* d = nullptr;
  FHE_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&d), nm * sizeof(ModParams), hs(s)));
  FHE_HIP_CHECK(hipMemcpyAsync(d, mp.data(), nm * sizeof(ModParams), hipMemcpyHostToDevice, hs(s)));
  const int rc = launch_vec_mod(op, out, a, b, rows, cols, d, ModArgs{}, mod_stride, signed_in,
                                hs(s));
  FHE_HIP_CHECK(hipStreamSynchronize(hs(s)));  // mp must outlive the async copy
  FHE_HIP_CHECK(hipFreeAsync(d, hs(s)));
  return rc;
}

int fhe_ntt_fwd(const fhe_ctx* c, uint64_t* data, uint32_t polys, uint32_t limb0,
                uint32_t nlimbs, fhe_stream_t s) {
  int rc = check_window(c, limb0, nlimbs, c ? c->L + c->K : 0, "fhe_ntt_fwd");
  if (rc) return rc;
  return launch_ntt(c, true, data, data, polys, (uint64_t)nlimbs * c->n, limb0, nlimbs, hs(s));
}

int fhe_ntt_inv(const fhe_ctx* c, uint64_t* data, uint32_t polys, uint32_t limb0,
                uint32_t nlimbs, fhe_stream_t s) {
  int rc = check_window(c, limb0, nlimbs, c ? c->L + c->K : 0, "fhe_ntt_inv");
  if (rc) return rc;
  return launch_ntt(c, false, data, data, polys, (uint64_t)nlimbs * c->n, limb0, nlimbs, hs(s));
}

int fhe_ntt_fwd_to(const fhe_ctx* c, uint64_t* dst, const uint64_t* src, uint32_t polys,
                   uint32_t limb0, uint32_t nlimbs, fhe_stream_t s) {
  int rc = check_window(c, limb0, nlimbs, c ? c->L + c->K : 0, "fhe_ntt_fwd_to");
  if (rc) return rc;
  return launch_ntt(c, true, src, dst, polys, (uint64_t)nlimbs * c->n, limb0, nlimbs, hs(s));
}

int fhe_ntt_inv_to(const fhe_ctx* c, uint64_t* dst, const uint64_t* src, uint32_t polys,
                   uint32_t limb0, uint32_t nlimbs, fhe_stream_t s) {
  int rc = check_window(c, limb0, nlimbs, c ? c->L + c->K : 0, "fhe_ntt_inv_to");
  if (rc) return rc;
  return launch_ntt(c, false, src, dst, polys, (uint64_t)nlimbs * c->n, limb0, nlimbs, hs(s));
}

size_t fhe_hommult_workspace(const fhe_ctx* c, uint32_t batch, uint32_t nlimbs) {
  return c ? hommult_workspace_bytes(c, batch, nlimbs) : 0;
}

int fhe_hommult(const fhe_ctx* c, uint64_t* d, const uint64_t* a, const uint64_t* b,
                uint32_t batch, uint32_t limb0, uint32_t nlimbs, void* ws, fhe_stream_t s) {
  int rc = check_window(c, limb0, nlimbs, c ? c->L : 0, "fhe_hommult");
  if (rc) return rc;
  if ((rc = ensure_ws(c, hommult_workspace_bytes(c, batch, nlimbs), &ws, hs(s)))) return rc;
  return launch_hommult(c, d, a, b, batch, limb0, nlimbs, ws, hs(s));
}

int fhe_baseconv(const fhe_ctx* c, uint64_t* out, const uint64_t* in, uint32_t s0, uint32_t S,
                 uint32_t t0, uint32_t T, fhe_stream_t s) {
  if (!c) {
    set_error("fhe_baseconv: null context");
    return kInvalid;
  }
  return launch_baseconv(c, out, in, s0, S, t0, T, hs(s));
}

size_t fhe_keyswitch_workspace(const fhe_ctx* c, uint32_t nlimbs, uint32_t batch) {
  return c ? keyswitch_workspace_bytes(c, nlimbs, batch) : 0;
}

uint32_t fhe_keyswitch_pass_batch(const fhe_ctx* c, uint32_t batch) {
  return c ? ks_pass_batch(c, batch) : 0;
}

int fhe_keyswitch_shard(const fhe_ctx* c, uint64_t* ks0, uint64_t* ks1, const uint64_t* c_all,
                        const uint64_t* d2_own, const uint64_t* evk_b, const uint64_t* evk_a,
                        uint32_t limb0, uint32_t nlimbs, uint32_t batch, void* ws,
                        fhe_stream_t s) {
  int rc = check_window(c, limb0, nlimbs, c ? c->L : 0, "fhe_keyswitch_shard");
  if (rc) return rc;
  if ((rc = ensure_ws(c, keyswitch_workspace_bytes(c, nlimbs, batch), &ws, hs(s)))) return rc;
  return launch_keyswitch_shard(c, ks0, ks1, c_all, d2_own, evk_b, evk_a, limb0, nlimbs, batch,
                                ws, hs(s));
}

int fhe_keyswitch(const fhe_ctx* c, uint64_t* ks0, uint64_t* ks1, const uint64_t* d2,
                  const uint64_t* evk_b, const uint64_t* evk_a, uint32_t batch, void* ws,
                  fhe_stream_t s) {
  int rc = check_window(c, 0, c ? c->L : 0, c ? c->L : 0, "fhe_keyswitch");
  if (rc) return rc;
  if (batch == 0) return kOk;
  const uint64_t ct_words = (uint64_t)c->L * c->n;
  // the whole batch at once: a pass must not overwrite a later pass's d2 (per-pass checks in the
  // launcher would miss an output shifted onto the next pass's input)
  if ((rc = ks_check_alias(ks0, ks1, d2, batch * ct_words, batch * ct_words, true,
                           "fhe_keyswitch")))
    return rc;
  const uint32_t pass = ks_pass_batch(c, batch);  // Infinity-Cache-sized passes
  const size_t bytes = keyswitch_workspace_bytes(c, c->L, pass);
  if ((rc = ensure_ws(c, bytes, &ws, hs(s)))) return rc;
  // c_all = INTT(d2) of one pass lives at the tail of the workspace (out of place: no copy of d2)
  const size_t call = (size_t)pass * ct_words * sizeof(uint64_t);
  uint64_t* c_all = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + bytes - call);
  // a prepared input when the fused ModUp applies: the INTT folds (D^_k)^-1 into its last stage
  const bool prep = ks_prepared(c);
  CAll src = CAll::contiguous(c_all, c->L, c->n);
  src.scaled = prep;
  for (uint32_t b0 = 0; b0 < batch; b0 += pass) {
    const uint32_t bn = std::min(pass, batch - b0);
    const uint64_t off = (uint64_t)b0 * ct_words;
    if ((rc = launch_ntt_strided(c, false, d2 + off, ct_words, c_all, ct_words, bn, 0, c->L, hs(s),
                                 prep ? c->d_nfold_up : nullptr, prep && ks_split30(c))))
      return rc;
    if ((rc = launch_keyswitch_shard(c, ks0 + off, ks1 + off, src, d2 + off, evk_b, evk_a, 0, c->L,
                                     bn, ws, hs(s))))
      return rc;
  }
  return kOk;
}

size_t fhe_rescale_workspace(const fhe_ctx* c, uint32_t polys, uint32_t nlimbs) {
  return c ? rescale_workspace_bytes(c, polys, nlimbs) : 0;
}

int fhe_rescale(const fhe_ctx* c, uint64_t* out, const uint64_t* in, uint32_t polys,
                uint32_t nlimbs, int ntt_form, void* ws, fhe_stream_t s) {
  int rc = check_window(c, 0, nlimbs, c ? c->L : 0, "fhe_rescale");
  if (rc) return rc;
  if (ntt_form && (rc = ensure_ws(c, rescale_workspace_bytes(c, polys, nlimbs), &ws, hs(s)))) return rc;
  return launch_rescale(c, out, in, polys, nlimbs, ntt_form != 0, ws, hs(s));
}

int fhe_automorphism(const fhe_ctx* c, uint64_t* out, const uint64_t* in, uint32_t polys,
                     uint32_t limb0, uint32_t nlimbs, uint32_t galois_elt, int ntt_form,
                     fhe_stream_t s) {
  int rc = check_window(c, limb0, nlimbs, c ? c->L + c->K : 0, "fhe_automorphism");
  if (rc) return rc;
  if (out == in && polys && nlimbs) {
    set_error("fhe_automorphism: out must not alias in");
    return kInvalid;
  }
  const uint64_t stride = (uint64_t)nlimbs * c->n;
  return launch_automorphism(c, out, stride, in, stride, polys, limb0, nlimbs, galois_elt,
                             ntt_form != 0, hs(s));
}

size_t fhe_rotate_workspace(const fhe_ctx* c, uint32_t batch) {
  return c ? rotate_workspace_bytes(c, batch) : 0;
}

int fhe_rotate(const fhe_ctx* c, uint64_t* out, const uint64_t* in, uint32_t galois_elt,
               const uint64_t* rot_b, const uint64_t* rot_a, uint32_t batch, void* ws,
               fhe_stream_t s) {
  int rc = check_window(c, 0, c ? c->L : 0, c ? c->L : 0, "fhe_rotate");
  if (rc) return rc;
  // the finish reads c0 through sigma (any word of its row block) while other workgroups write
  // out: any overlap of the two [batch][2][L][N] spans races, not just out == in
  const uint64_t span = (uint64_t)batch * 2 * c->L * c->n;
  if (spans_overlap(out, span, in, span)) {
    set_error("fhe_rotate: out must not overlap in");
    return kInvalid;
  }
  if ((rc = ensure_ws(c, rotate_workspace_bytes(c, ks_pass_batch(c, batch)), &ws, hs(s)))) return rc;
  return launch_rotate(c, out, in, galois_elt, rot_b, rot_a, batch, ws, hs(s));
}

size_t fhe_rotate_hoisted_workspace(const fhe_ctx* c, uint32_t batch) {
  return c ? rotate_hoisted_workspace_bytes(c, batch) : 0;
}

int fhe_rotate_hoisted(const fhe_ctx* c, uint64_t* out, const uint64_t* in,
                       const uint32_t* galois_elts, const uint64_t* const* rot_b,
                       const uint64_t* const* rot_a, uint32_t count, uint32_t batch, void* ws,
                       fhe_stream_t s) {
  int rc = check_window(c, 0, c ? c->L : 0, c ? c->L : 0, "fhe_rotate_hoisted");
  if (rc) return rc;
  if (count && (!galois_elts || !rot_b || !rot_a)) {
    set_error("fhe_rotate_hoisted: null Galois element or key array");
    return kInvalid;
  }
  for (uint32_t r = 0; r < count; ++r)
    if (!rot_b[r] || !rot_a[r]) {  // the kernels would dereference it on the device
      set_error("fhe_rotate_hoisted: null key pointer for rotation " + std::to_string(r));
      return kInvalid;
    }
  const uint64_t span = (uint64_t)count * batch * 2 * c->L * c->n;
  if (span && in < out + span && out < in + (uint64_t)batch * 2 * c->L * c->n) {
    set_error("fhe_rotate_hoisted: out must not overlap in");
    return kInvalid;
  }
  if ((rc = ensure_ws(c, rotate_hoisted_workspace_bytes(c, batch), &ws, hs(s)))) return rc;
  return launch_rotate_hoisted(c, out, in, galois_elts, rot_b, rot_a, count, batch, ws, hs(s));
}

size_t fhe_rotate_sum_hoisted_workspace(const fhe_ctx* c, uint32_t batch) {
  return c ? rotate_sum_hoisted_workspace_bytes(c, batch) : 0;
}

int fhe_rotate_sum_hoisted(const fhe_ctx* c, uint64_t* out, const uint64_t* in,
                           const uint32_t* galois_elts, const uint64_t* const* rot_b,
                           const uint64_t* const* rot_a, const uint64_t* const* pt,
                           uint32_t count, uint32_t batch, void* ws, fhe_stream_t s) {
  int rc = check_window(c, 0, c ? c->L : 0, c ? c->L : 0, "fhe_rotate_sum_hoisted");
  if (rc) return rc;
  if (count == 0 || count > kRotSumMax) {
    set_error("fhe_rotate_sum_hoisted: count must be 1..16");
    return kInvalid;
  }
  if (!galois_elts || !pt || ((!rot_b || !rot_a) && std::any_of(galois_elts, galois_elts + count,
                                                                 [](uint32_t g) { return g != 1; }))) {
    set_error("fhe_rotate_sum_hoisted: null Galois element, plaintext or key array");
    return kInvalid;
  }
  for (uint32_t r = 0; r < count; ++r) {
    // the kernels would dereference them on the device; the unrotated term (1) takes no key
    if (!pt[r] || (galois_elts[r] != 1 && (!rot_b[r] || !rot_a[r]))) {
      set_error("fhe_rotate_sum_hoisted: null plaintext or key pointer for term " +
                std::to_string(r));
      return kInvalid;
    }
  }
  const uint64_t span = (uint64_t)batch * 2 * c->L * c->n;
  if (spans_overlap(out, span, in, span)) {
    set_error("fhe_rotate_sum_hoisted: out must not overlap in");
    return kInvalid;
  }
  if ((rc = ensure_ws(c, rotate_sum_hoisted_workspace_bytes(c, batch), &ws, hs(s)))) return rc;
  return launch_rotate_sum_hoisted(c, out, in, galois_elts, rot_b, rot_a, pt, count, batch, ws,
                                   hs(s));
}

size_t fhe_rotate_sum_multi_workspace(const fhe_ctx* c, uint32_t count, uint32_t batch) {
  return c ? rotate_sum_multi_workspace_bytes(c, count, batch) : 0;
}

int fhe_rotate_sum_multi(const fhe_ctx* c, uint64_t* out, const uint64_t* const* cts,
                         const uint32_t* galois_elts, const uint64_t* const* rot_b,
                         const uint64_t* const* rot_a, uint32_t count, uint32_t batch, void* ws,
                         fhe_stream_t s) {
  int rc = check_window(c, 0, c ? c->L : 0, c ? c->L : 0, "fhe_rotate_sum_multi");
  if (rc) return rc;
  if (count == 0 || count > kRotSumMax) {
    set_error("fhe_rotate_sum_multi: count must be 1..16");
    return kInvalid;
  }
  if (!galois_elts || !cts || ((!rot_b || !rot_a) && std::any_of(galois_elts, galois_elts + count,
                                                                  [](uint32_t g) { return g != 1; }))) {
    set_error("fhe_rotate_sum_multi: null Galois element, ciphertext or key array");
    return kInvalid;
  }
  const uint64_t span = (uint64_t)batch * 2 * c->L * c->n;
  for (uint32_t r = 0; r < count; ++r) {
    if (!cts[r] || (galois_elts[r] != 1 && (!rot_b[r] || !rot_a[r]))) {
      set_error("fhe_rotate_sum_multi: null ciphertext or key pointer for term " +
                std::to_string(r));
      return kInvalid;
    }
    if (spans_overlap(out, span, cts[r], span)) {
      set_error("fhe_rotate_sum_multi: out must not overlap an input ciphertext (term " +
                std::to_string(r) + ")");
      return kInvalid;
    }
  }
  if ((rc = ensure_ws(c, rotate_sum_multi_workspace_bytes(c, count, batch), &ws, hs(s)))) return rc;
  return launch_rotate_sum_multi(c, out, cts, galois_elts, rot_b, rot_a, count, batch, ws, hs(s));
}

size_t fhe_linear_transform_workspace(const fhe_ctx* c, uint32_t n2, uint32_t batch) {
  return c ? linear_transform_workspace_bytes(c, n2, batch) : 0;
}

int fhe_linear_transform(const fhe_ctx* c, uint64_t* out, const uint64_t* in, uint32_t n1,
                         uint32_t n2, const uint32_t* baby_elts, const uint64_t* const* baby_b,
                         const uint64_t* const* baby_a, const uint32_t* giant_elts,
                         const uint64_t* const* giant_b, const uint64_t* const* giant_a,
                         const uint64_t* const* pt, uint32_t batch, void* ws, fhe_stream_t s) {
  int rc = check_window(c, 0, c ? c->L : 0, c ? c->L : 0, "fhe_linear_transform");
  if (rc) return rc;
  if (n1 == 0 || n1 > kRotSumMax || n2 == 0 || n2 > kRotSumMax) {
    set_error("fhe_linear_transform: n1 and n2 must be 1..16");
    return kInvalid;
  }
  if (!baby_elts || !giant_elts || !pt) {
    set_error("fhe_linear_transform: null Galois element or plaintext array");
    return kInvalid;
  }
  auto keyed = [](const uint32_t* e, uint32_t k, const uint64_t* const* b, const uint64_t* const* a) {
    for (uint32_t r = 0; r < k; ++r)
      if (e[r] != 1 && (!b || !a || !b[r] || !a[r])) return false;
    return true;
  };
  if (!keyed(baby_elts, n1, baby_b, baby_a) || !keyed(giant_elts, n2, giant_b, giant_a)) {
    set_error("fhe_linear_transform: a rotated baby or giant step without its key");
    return kInvalid;
  }
  for (uint64_t r = 0; r < (uint64_t)n1 * n2; ++r)
    if (!pt[r]) {
      set_error("fhe_linear_transform: null plaintext pointer " + std::to_string(r));
      return kInvalid;
    }
  const uint64_t span = (uint64_t)batch * 2 * c->L * c->n;
  if (spans_overlap(out, span, in, span)) {
    set_error("fhe_linear_transform: out must not overlap in");
    return kInvalid;
  }
  if ((rc = ensure_ws(c, linear_transform_workspace_bytes(c, n2, batch), &ws, hs(s)))) return rc;
  return launch_linear_transform(c, out, in, n1, n2, baby_elts, baby_b, baby_a, giant_elts, giant_b,
                                 giant_a, pt, batch, ws, hs(s));
}

size_t fhe_mul_relin_workspace(const fhe_ctx* c, uint32_t batch) {
  return c ? mul_relin_workspace_bytes(c, batch) : 0;
}

int fhe_mul_relin(const fhe_ctx* c, uint64_t* out, const uint64_t* a, const uint64_t* b,
                  const uint64_t* evk_b, const uint64_t* evk_a, uint32_t batch, int rescale,
                  void* ws, fhe_stream_t s) {
  int rc = check_window(c, 0, c ? c->L : 0, c ? c->L : 0, "fhe_mul_relin");
  if (rc) return rc;
  if ((rc = ensure_ws(c, mul_relin_workspace_bytes(c, ks_pass_batch(c, batch)), &ws, hs(s)))) return rc;
  return launch_mul_relin(c, out, a, b, evk_b, evk_a, batch, rescale != 0, ws, hs(s));
}

}  // extern "C"
