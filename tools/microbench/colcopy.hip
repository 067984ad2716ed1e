// HBM rate of the column pass's access pattern (dev microbenchmark, not libfhecore): a copy of
// [polys][R1 = 256][R2 = 256] u64 planes where a workgroup of T threads moves a tile of W whole
// columns (lanes over columns, rows R2 words apart), each thread E = 256 W / T elements of one
// column, against a plain contiguous copy.  Out of place (HomMult's column forward) and in place
// (the standalone NTT's second pass).  usage: colcopy
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned long long u64;

// XG: the tiles of one plane go to one XCD back to back (workgroups are dealt to the 8 XCDs
// round-robin: XCD x takes planes p = x mod 8, all their tiles in order), instead of being spread
// over all 8 XCDs.
template <int W, int T, bool NT, bool XG = false>
__global__ __launch_bounds__(T) void k_colcopy(const u64* __restrict__ src, u64* dst, int tiles) {
  constexpr int R = 256, E = R * W / T, STEP = T / W;
  const int col = threadIdx.x % W, t = threadIdx.x / W;
  int tile = blockIdx.x % tiles, p = blockIdx.x / tiles;
  if (XG) {
    const int x = blockIdx.x % 8, k = blockIdx.x / 8;
    tile = k % tiles;
    p = (k / tiles) * 8 + x;
  }
  const u64 base = (u64)p * R * R + (u64)tile * W + col;
  u64 x[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const u64* a = src + base + (u64)(t + j * STEP) * R;
    x[j] = NT ? __builtin_nontemporal_load(a) : *a;
  }
#pragma unroll
  for (int j = 0; j < E; ++j) dst[base + (u64)(t + j * STEP) * R] = x[j] + 1;
}

// TPW tiles per workgroup, one after another (XCD-grouped as above): fewer, longer workgroups.
template <int TPW>
__global__ __launch_bounds__(256) void k_colcopy_loop(const u64* __restrict__ src, u64* dst) {
  constexpr int R = 256, W = 16, E = 16, STEP = 16, tiles = R / W;
  const int col = threadIdx.x % W, t = threadIdx.x / W;
  const int x = blockIdx.x % 8, k = blockIdx.x / 8;
#pragma unroll 1
  for (int i = 0; i < TPW; ++i) {
    const int kk = k * TPW + i;
    const int tile = kk % tiles, p = (kk / tiles) * 8 + x;
    const u64 base = (u64)p * R * R + (u64)tile * W + col;
    u64 v[E];
#pragma unroll
    for (int j = 0; j < E; ++j) v[j] = src[base + (u64)(t + j * STEP) * R];
#pragma unroll
    for (int j = 0; j < E; ++j) dst[base + (u64)(t + j * STEP) * R] = v[j] + 1;
  }
}

__global__ void k_linear(const ulonglong2* __restrict__ s, ulonglong2* d, u64 n2) {
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n2; i += (u64)gridDim.x * blockDim.x) {
    ulonglong2 v = s[i];
    v.x += 1;
    d[i] = v;
  }
}

static hipEvent_t ea, eb;
template <class F>
float timeit(F f) {
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(ea);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(eb);
  hipEventSynchronize(eb);
  float ms;
  hipEventElapsedTime(&ms, ea, eb);
  return ms / 20;
}

int main() {
  const int polys = 2048;
  const size_t words = (size_t)polys * 256 * 256;
  u64 *s, *d;
  if (hipMalloc(&s, words * 8) || hipMalloc(&d, words * 8)) return 1;
  hipMemset(s, 1, words * 8);
  hipMemset(d, 0, words * 8);
  hipEventCreate(&ea);
  hipEventCreate(&eb);
  const double bytes = 2.0 * words * 8;
#define RUN(W, T, NT, DST, tag) RUNX(W, T, NT, false, DST, tag)
#define RUNX(W, T, NT, XG, DST, tag)                                                                 \
  printf("%-28s %6.0f GB/s\n", tag,                                                            \
         bytes / timeit([&] { k_colcopy<W, T, NT, XG><<<polys * (256 / W), T>>>(s, DST, 256 / W); }) / 1e6);
  RUN(16, 256, false, d, "W=16 T=256 (shipped)")
  RUN(16, 256, true, d, "W=16 T=256 NT loads")
  RUN(16, 256, false, s, "W=16 T=256 in place")
  RUN(32, 256, false, d, "W=32 T=256 (E=32)")
  RUN(32, 512, false, d, "W=32 T=512")
  RUN(64, 256, false, d, "W=64 T=256 (E=64)")
  RUN(64, 1024, false, d, "W=64 T=1024")
  RUN(8, 256, false, d, "W=8 T=256 (E=8)")
  RUNX(16, 256, false, true, d, "W=16 T=256 XCD-grouped")
  RUNX(16, 256, true, true, d, "W=16 T=256 XCD-grouped NT")
  RUNX(32, 512, false, true, d, "W=32 T=512 XCD-grouped")
  RUNX(32, 256, false, true, d, "W=32 T=256 XCD-grouped")
  RUN(16, 256, false, d, "W=16 T=256 (shipped) again")
  printf("%-28s %6.0f GB/s\n", "XCD-grouped, 2 tiles/WG",
         bytes / timeit([&] { k_colcopy_loop<2><<<polys * 16 / 2, 256>>>(s, d); }) / 1e6);
  printf("%-28s %6.0f GB/s\n", "XCD-grouped, 4 tiles/WG",
         bytes / timeit([&] { k_colcopy_loop<4><<<polys * 16 / 4, 256>>>(s, d); }) / 1e6);
  printf("%-28s %6.0f GB/s\n", "XCD-grouped, 16 tiles/WG",
         bytes / timeit([&] { k_colcopy_loop<16><<<polys * 16 / 16, 256>>>(s, d); }) / 1e6);
  printf("%-28s %6.0f GB/s\n", "linear copy",
         bytes / timeit([&] { k_linear<<<8192, 256>>>((ulonglong2*)s, (ulonglong2*)d, words / 2); }) / 1e6);
  return 0;
}
