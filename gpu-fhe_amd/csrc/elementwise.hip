// Coefficient-wise modular add / sub / mul: the reference's vec_add / vec_sub / vec_mul
// (/root/reference/arithmetic.py:3-13; vec_mul in the NTT domain = poly_mul_pointwise).
//
// Two entry families:
//  * context kernels: canonical residues in [0, q_l) for the context's limb moduli, layout
//    [polys][nlimbs][N]; kU 16-byte non-temporal loads per operand per lane (HBM-bound, 24 B/elem);
//  * generic kernels for the reference-shaped Python API: any u64 (or signed i64) inputs, any
//    modulus 2 <= q < 2^64, one modulus per row (scalar MOD or a (L, 1) MOD column); results
//    equal Python's exact `(a op b) % MOD` (the object-dtype semantics).
#include "internal.hpp"

namespace fhe {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ u64 op_canon(int op, u64 a, u64 b, const ModParams& m) {
  if (op == kAdd) return csub(a + b, m.q);
  if (op == kSub) return a >= b ? a - b : a + (m.q - b);
  return mulmod_barrett(a, b, m);
}

// One poly-limb row per blockIdx.y (its ModParams uniform, no per-element limb division), kU
// 16-byte pairs per lane per operand.  Rows beyond the grid's y extent loop.  kU = 1 measured best
// (bench --workload vec, same-box: 1 / 2 / 4 / 8 -> 2.32 / 2.28 / 2.17 / 2.00 e11 coeff-op/s):
// more, shorter workgroups keep more loads in flight than more loads per lane.
// Every operand word is touched once, so loads and stores are non-temporal (streamed past the
// caches) and workgroups are 2 waves: same-box, 3 repetitions, 2.41-2.47 e11 coeff-op/s with cached
// accesses at 256 threads -> 2.69-2.74 e11 (+11 %; non-temporal stores alone +1 %, loads alone
// +3 %, both at 512 / 256 threads 2.65-2.70 e11; profiles/r05_vec_nontemporal_ab*.txt).
constexpr int kU = 1;
constexpr int kVecThreads = 128;
typedef u64 vu64x2 __attribute__((ext_vector_type(2)));
template <int OP>
__global__ __launch_bounds__(kVecThreads) void k_vec_ctx(u64* __restrict__ out,
                                                      const u64* __restrict__ a,
                                                      const u64* __restrict__ b, u32 row_pairs,
                                                      u32 rows, u32 nlimbs, u32 limb0,
                                                      const ModParams* __restrict__ mods) {
  const u32 p0 = blockIdx.x * (kVecThreads * kU) + threadIdx.x;
  for (u32 row = blockIdx.y; row < rows; row += gridDim.y) {
    const ModParams m = mods[limb0 + row % nlimbs];
    const u64 base = (u64)row * row_pairs;
    const vu64x2* pa = reinterpret_cast<const vu64x2*>(a) + base;
    const vu64x2* pb = reinterpret_cast<const vu64x2*>(b) + base;
    vu64x2* po = reinterpret_cast<vu64x2*>(out) + base;
    vu64x2 x[kU], y[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const u32 i = p0 + u * kVecThreads;
      if (i < row_pairs) {
        x[u] = __builtin_nontemporal_load(pa + i);
        y[u] = __builtin_nontemporal_load(pb + i);
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const u32 i = p0 + u * kVecThreads;
      if (i < row_pairs) {
        const vu64x2 r = {op_canon(OP, x[u].x, y[u].x, m), op_canon(OP, x[u].y, y[u].y, m)};
        __builtin_nontemporal_store(r, po + i);
      }
    }
  }
}

__device__ __forceinline__ u64 to_residue(u64 x, int signed_in, const ModParams& m) {
  if (signed_in && (int64_t)x < 0) {
    // x = -(|x|): |x| mod q, negated
    const u64 r = reduce_u64((u64)0 - x, m);
    return r == 0 ? 0 : m.q - r;
  }
  return reduce_u64(x, m);
}

// The generic kernel's moduli: up to kArgMods records travel in the kernel arguments (the
// reference's scalar MOD or an (L, 1) column: no device allocation, no copy, no synchronisation,
// so the call is graph-capturable); longer columns come from a device array.
template <int OP>
__global__ __launch_bounds__(kThreads) void k_vec_mod(u64* __restrict__ out,
                                                      const u64* __restrict__ a,
                                                      const u64* __restrict__ b, u64 rows,
                                                      u64 cols, const ModParams* __restrict__ mods,
                                                      ModArgs inl, u64 mod_stride, int signed_in) {
  const u64 total = rows * cols;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const u64 k = (i / cols) * mod_stride;
    const ModParams m = mods ? mods[k] : inl.m[k];
    const u64 x = to_residue(a[i], signed_in, m), y = to_residue(b[i], signed_in, m);
    u64 r;
    if (OP == kAdd) r = x >= m.q - y ? x - (m.q - y) : x + y;
    else if (OP == kSub) r = x >= y ? x - y : x + (m.q - y);
    else r = mulmod_any(x, y, m);
    out[i] = r;
  }
}

inline u32 grid_for(u64 work) {
  const u64 blocks = (work + kThreads - 1) / kThreads;
  return (u32)(blocks < 256 * 16 ? (blocks ? blocks : 1) : 256 * 16);
}

}  // namespace

int launch_vec_ctx(const fhe_ctx* c, int op, u64* out, const u64* a, const u64* b, u32 polys,
                   u32 limb0, u32 nlimbs, hipStream_t s) {
  const u64 rows64 = (u64)polys * nlimbs;
  if (rows64 == 0) return kOk;
  if (rows64 > 0xffffffffull) {
    set_error("vec: too many poly-limb rows");
    return kInvalid;
  }
  const u32 rows = (u32)rows64, row_pairs = (u32)(c->n / 2);  // N >= 2^10: whole pairs per row
  constexpr u32 kT = kVecThreads;
  const dim3 g((row_pairs + kT * kU - 1) / (kT * kU), rows < 65535 ? rows : 65535);
  switch (op) {
    case kAdd: k_vec_ctx<kAdd><<<g, kT, 0, s>>>(out, a, b, row_pairs, rows, nlimbs, limb0, c->d_mods); break;
    case kSub: k_vec_ctx<kSub><<<g, kT, 0, s>>>(out, a, b, row_pairs, rows, nlimbs, limb0, c->d_mods); break;
    case kMul: k_vec_ctx<kMul><<<g, kT, 0, s>>>(out, a, b, row_pairs, rows, nlimbs, limb0, c->d_mods); break;
    default: set_error("bad vec op"); return kInvalid;
  }
  FHE_HIP_CHECK(hipGetLastError());
  prof_mark(s, op == kAdd ? "vec_add" : op == kSub ? "vec_sub" : "vec_mul");
  return kOk;
}

int launch_vec_mod(int op, u64* out, const u64* a, const u64* b, u64 rows, u64 cols,
                   const ModParams* d_mods, const ModArgs& inl, u64 mod_stride, int signed_in,
                   hipStream_t s) {
  const u64 total = rows * cols;
  if (total == 0) return kOk;
  const u32 g = grid_for(total);
  switch (op) {
    case kAdd: k_vec_mod<kAdd><<<g, kThreads, 0, s>>>(out, a, b, rows, cols, d_mods, inl, mod_stride, signed_in); break;
    case kSub: k_vec_mod<kSub><<<g, kThreads, 0, s>>>(out, a, b, rows, cols, d_mods, inl, mod_stride, signed_in); break;
    case kMul: k_vec_mod<kMul><<<g, kThreads, 0, s>>>(out, a, b, rows, cols, d_mods, inl, mod_stride, signed_in); break;
    default: set_error("bad vec op"); return kInvalid;
  }
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}

}  // namespace fhe
