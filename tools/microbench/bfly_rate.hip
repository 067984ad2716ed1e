// Microbenchmark: register-resident Harvey CT butterflies (64-bit Shoup) on gfx950.
// Variants of the modular multiply / butterfly formulation, measured in butterflies per second
// and lane-cycles per butterfly (256 CUs x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T lane-cycles/s).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint64_t u64;
typedef uint32_t u32;
typedef unsigned __int128 u128;

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ u64 csub(u64 x, u64 m) { return x >= m ? x - m : x; }
__device__ __forceinline__ u64 mad64(u32 a, u32 b, u64 c) { return (u64)a * b + c; }

// V0: exact mulhi through __int128 (what ntt.hip uses)
__device__ __forceinline__ u64 shoup0(u64 x, u64 w, u64 ws, u64 q) {
  u64 qh = (u64)(((u128)x * ws) >> 64);
  return x * w - qh * q;
}
// V1: approximate quotient (3 partial products), corrected by one conditional subtract of 2q
__device__ __forceinline__ u64 shoup1(u64 x, u64 w, u64 ws, u64 q) {
  u32 x0 = (u32)x, x1 = x >> 32, s0 = (u32)ws, s1 = ws >> 32;
  u64 qh = mad64(x1, s1, (u64)__umulhi(x1, s0) + __umulhi(x0, s1));
  return csub(x * w - qh * q, 2 * q);
}
// V2: exact, hand-ordered partial products
__device__ __forceinline__ u64 shoup2(u64 x, u64 w, u64 ws, u64 q) {
  u32 x0 = (u32)x, x1 = x >> 32, s0 = (u32)ws, s1 = ws >> 32;
  u64 t = mad64(x1, s0, __umulhi(x0, s0));
  u64 v = mad64(x0, s1, (u32)t);
  u64 qh = mad64(x1, s1, (t >> 32) + (v >> 32));
  u32 w0 = (u32)w, w1 = w >> 32, q0 = (u32)q, q1 = q >> 32, h0 = (u32)qh, h1 = qh >> 32;
  u64 a = mad64(x0, w0, 0), b = mad64(h0, q0, 0);
  u32 hi = (u32)(a >> 32) + x1 * w0 + x0 * w1 - (u32)(b >> 32) - h1 * q0 - h0 * q1;
  u32 lo = (u32)a - (u32)b;
  return ((u64)hi << 32) | lo;  // borrow from the low word folded below
}

// V3: exact quotient; remainder via mad64 chains with -q (no carry chains, no compares)
__device__ __forceinline__ u64 shoup3(u64 y, u64 w, u64 ws, u64 nq) {
  const u32 y0 = (u32)y, y1 = y >> 32, s0 = (u32)ws, s1 = ws >> 32;
  const u32 w0 = (u32)w, w1 = w >> 32, n0 = (u32)nq, n1 = nq >> 32;
  const u64 a = mad64(y1, s0, __umulhi(y0, s0));
  const u64 b = mad64(y0, s1, (u32)a);
  const u64 h = mad64(y1, s1, a >> 32) + (b >> 32);
  const u32 h0 = (u32)h, h1 = h >> 32;
  const u64 t = mad64(h0, n0, mad64(y0, w0, 0));
  u64 c = mad64(y1, w0, t >> 32);
  c = mad64(y0, w1, c);
  c = mad64(h1, n0, c);
  c = mad64(h0, n1, c);
  return ((u64)(u32)c << 32) | (u32)t;
}
// v_mad_u64_u32 forced through inline asm (the compiler rewrites low-half-only mads into
// mul_lo + add chains, which cost more on gfx950)
__device__ __forceinline__ u64 mad64x(u32 a, u32 b, u64 c) {
  u64 r, sc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(sc) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ u32 bfi32(u32 m, u32 a, u32 b) {
  u32 r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ u32 sra31(u32 x) {
  u32 r;
  asm("v_ashrrev_i32 %0, 31, %1" : "=v"(r) : "v"(x));
  return r;
}
// V4: V3 with the mads pinned, and an asm sign-mask conditional subtraction
__device__ __forceinline__ u64 shoup4(u64 y, u64 w, u64 ws, u64 nq) {
  const u32 y0 = (u32)y, y1 = y >> 32, s0 = (u32)ws, s1 = ws >> 32;
  const u32 w0 = (u32)w, w1 = w >> 32, n0 = (u32)nq, n1 = nq >> 32;
  const u64 a = mad64x(y1, s0, __umulhi(y0, s0));
  const u64 b = mad64x(y0, s1, (u32)a);
  const u64 h = mad64x(y1, s1, a >> 32) + (b >> 32);
  const u32 h0 = (u32)h, h1 = h >> 32;
  const u64 t = mad64x(h0, n0, mad64x(y0, w0, 0));
  u64 c = mad64x(y1, w0, t >> 32);
  c = mad64x(y0, w1, c);
  c = mad64x(h1, n0, c);
  c = mad64x(h0, n1, c);
  return ((u64)(u32)c << 32) | (u32)t;
}
__device__ __forceinline__ u64 csub4(u64 x, u64 nm) {
  const u64 d = x + nm;
  const u32 m = sra31((u32)(d >> 32));
  return ((u64)bfi32(m, (u32)(x >> 32), (u32)(d >> 32)) << 32) | bfi32(m, (u32)x, (u32)d);
}
// x >= m ? x - m : x for x, m < 2^63 given nm = -m: sign-mask select, no compare
__device__ __forceinline__ u64 csub_mask(u64 x, u64 nm) {
  const u64 d = x + nm;
  const u64 msk = (u64)((int64_t)d >> 63);
  return (x & msk) | (d & ~msk);
}

// V5: plain C++ shaped for the compiler: T = x w + h (-q) (one 64-bit add, no borrow),
// u - 2q via add of -2q and a sign test
__device__ __forceinline__ u64 shoup5(u64 x, u64 w, u64 ws, u64 nq) {
  const u64 h = (u64)(((u128)x * ws) >> 64);
  return x * w + h * nq;
}
__device__ __forceinline__ u64 csub5(u64 x, u64 nm) {
  const u64 d = x + nm;
  return (int64_t)d < 0 ? x : d;
}

// V6: plain C++ with empty-asm value barriers that stop the compiler from shrinking the mad chain
// or turning mask selects back into compares (no inline instructions, so no hazard padding)
#define OPQ(x) asm("" : "+v"(x))
__device__ __forceinline__ u64 shoup6(u64 y, u64 w, u64 ws, u64 nq) {
  const u32 y0 = (u32)y, y1 = y >> 32, s0 = (u32)ws, s1 = ws >> 32;
  const u32 w0 = (u32)w, w1 = w >> 32, n0 = (u32)nq, n1 = nq >> 32;
  u64 a = mad64(y1, s0, __umulhi(y0, s0));
  u64 b = mad64(y0, s1, (u32)a);
  u64 h = mad64(y1, s1, a >> 32) + (b >> 32);
  const u32 h0 = (u32)h, h1 = h >> 32;
  u64 t = mad64(y0, w0, 0);
  t = mad64(h0, n0, t);
  OPQ(t);
  u64 c = mad64(y1, w0, t >> 32);
  OPQ(c);
  c = mad64(y0, w1, c);
  OPQ(c);
  c = mad64(h1, n0, c);
  OPQ(c);
  c = mad64(h0, n1, c);
  OPQ(c);
  return ((u64)(u32)c << 32) | (u32)t;
}
__device__ __forceinline__ u64 csub6(u64 x, u64 nm) {
  const u64 d = x + nm;
  u32 m = (u32)((int32_t)(d >> 32) >> 31);
  OPQ(m);
  const u32 lo = ((u32)x & m) | ((u32)d & ~m), hi = ((u32)(x >> 32) & m) | ((u32)(d >> 32) & ~m);
  return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 subp6(u64 u, u64 v, u64 kp1) {
  u64 nv = ~v;
  OPQ(nv);
  return (u + kp1) + nv;
}

template <int V>
__device__ __forceinline__ u64 mulw(u64 x, u64 w, u64 ws, u64 q) {
  if (V == 0) return shoup0(x, w, ws, q);
  if (V == 1) return shoup1(x, w, ws, q);
  return shoup0(x, w, ws, q);
}

template <int V, bool LANE_TW>
__global__ __launch_bounds__(256) void k_bfly(u64* out, const u64* tw, u64 q, int iters) {
  u64 x[16];
  for (int j = 0; j < 16; ++j) x[j] = (threadIdx.x * 977u + j * 131u) % q;
  const u64 q2 = 2 * q;
  u64 w[15], ws[15];
  for (int i = 0; i < 15; ++i) {
    const int k = LANE_TW ? (i * 64 + (threadIdx.x & 63)) : i;
    w[i] = tw[2 * k];
    ws[i] = tw[2 * k + 1];
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int b = 3; b >= 0; --b) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (j & (1 << b)) continue;
        const int jj = j | (1 << b);
        const int ti = ((1 << (3 - b)) - 1) + (j >> (b + 1));
        if (V == 6) {
          const u64 u = csub6(x[j], 0 - q2);
          const u64 v = shoup6(x[jj], w[ti], ws[ti], 0 - q);
          x[j] = u + v;
          x[jj] = subp6(u, v, q2 + 1);
        } else if (V == 5) {
          const u64 u = csub5(x[j], 0 - q2);
          const u64 v = shoup5(x[jj], w[ti], ws[ti], 0 - q);
          x[j] = u + v;
          x[jj] = u - v + q2;
        } else if (V == 4) {
          const u64 u = csub4(x[j], 0 - q2);
          const u64 v = shoup4(x[jj], w[ti], ws[ti], 0 - q);
          x[j] = u + v;
          x[jj] = (u + q2) - v;
        } else if (V == 3) {
          const u64 u = csub_mask(x[j], 0 - q2);
          const u64 v = shoup3(x[jj], w[ti], ws[ti], 0 - q);
          x[j] = u + v;
          x[jj] = (u + q2) - v;
        } else {
          const u64 u = csub(x[j], q2);
          const u64 v = mulw<V>(x[jj], w[ti], ws[ti], q);
          x[j] = u + v;
          x[jj] = u - v + q2;
        }
      }
    }
  }
  u64 r = 0;
  for (int j = 0; j < 16; ++j) r ^= x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

static size_t g_shmem = 0;  // dynamic LDS per workgroup: limits workgroups (waves) per CU

template <class K>
static int run(const char* name, K kern, u64* d, const u64* tw, u64 q) {
  const int iters = 256;
  dim3 grid(256 * 16), block(256);
  kern<<<grid, block, g_shmem>>>(d, tw, q, 2);
  CHK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  CHK(hipEventRecord(a));
  kern<<<grid, block, g_shmem>>>(d, tw, q, iters);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double bf = (double)grid.x * block.x * iters * 32;
  const double rate = bf / (ms * 1e-3);
  printf("%-22s %8.3f ms  %7.1f G bfly/s  %6.1f lane-cycles/bfly\n", name, ms, rate / 1e9,
         78.6432e12 / rate);
  return 0;
}

int main() {
  const u64 q = 0xffffffffffc0001ull;
  u64 *d, *tw;
  CHK(hipMalloc(&d, 256 * 16 * 256 * 8));
  CHK(hipMalloc(&tw, 2 * 15 * 64 * 8));
  u64 htw[2 * 15 * 64];
  for (int k = 0; k < 15 * 64; ++k) {
    u64 w = (0x123456789abcdefull * (k + 1)) % q;
    htw[2 * k] = w;
    htw[2 * k + 1] = (u64)(((u128)w << 64) / q);
  }
  CHK(hipMemcpy(tw, htw, sizeof(htw), hipMemcpyHostToDevice));
  for (size_t sh : {(size_t)34816, (size_t)20000}) {  // 4 and 8 workgroups (waves/SIMD) per CU
    g_shmem = sh;
    printf("-- dynamic LDS %zu B per workgroup\n", sh);
    run("v0 exact, lane tw", k_bfly<0, true>, d, tw, q);
    run("v6 c++ barriers, lane tw", k_bfly<6, true>, d, tw, q);
  }
  g_shmem = 0;
  printf("-- no LDS limit\n");
  run("v0 exact, sgpr tw", k_bfly<0, false>, d, tw, q);
  run("v0 exact, lane tw", k_bfly<0, true>, d, tw, q);
  run("v1 approx, sgpr tw", k_bfly<1, false>, d, tw, q);
  run("v1 approx, lane tw", k_bfly<1, true>, d, tw, q);
  run("v3 madchain, sgpr tw", k_bfly<3, false>, d, tw, q);
  run("v3 madchain, lane tw", k_bfly<3, true>, d, tw, q);
  run("v4 asm mads, sgpr tw", k_bfly<4, false>, d, tw, q);
  run("v4 asm mads, lane tw", k_bfly<4, true>, d, tw, q);
  run("v5 c++ shaped, sgpr tw", k_bfly<5, false>, d, tw, q);
  run("v5 c++ shaped, lane tw", k_bfly<5, true>, d, tw, q);
  run("v6 c++ barriers, sgpr tw", k_bfly<6, false>, d, tw, q);
  run("v6 c++ barriers, lane tw", k_bfly<6, true>, d, tw, q);
  return 0;
}
