// Memory-pattern microbenchmark for the XA decimation stage (gfx950): one wave per frame
// walking its frame in 16-KB tiles (16 x 16 B per lane, next tile prefetched in registers)
// and writing 8 KB per tile, 2 waves per SIMD (LDS-limited), F = 4096 frames of 2.4 MB.
//   mode 0: input and output frame-major (today's layout)
//   mode 1: input frame-major, output tile-major (all waves' tile tau adjacent)
//   mode 2: input and output tile-major
//   mode 3: plain grid-stride copy of the same bytes (reference rate)
//   mode 4: mode 0 with the XA stage's store shapes: 6 x 16 B + 4 x 8 B per lane and tile
//   mode 5: mode 0 with the next tile's loads issued in the XA groups (8, then 4, then 4)
// usage: stream_pattern [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int kF = 4096, kTiles = 146;      // 146 x 16 KB = 2.39 MB per frame
constexpr int kTileV = 1024, kOutV = 512;   // v4f per tile in / out (16 KB / 8 KB)

template <int MODE>
__global__ __launch_bounds__(256) void walk(const v4f *__restrict__ in, v4f *__restrict__ out, float a) {
  __shared__ float pad[78 * 256];  // 78 KB: 2 workgroups (8 waves) per CU, as the XA stage
  const int lane = threadIdx.x & 63, f = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (a == 123.f) pad[threadIdx.x] = 0.f;
  auto in_at = [&](int tau, int q) -> const v4f * {
    const long t = MODE == 2 ? (long)tau * kF + f : (long)f * kTiles + tau;
    return in + t * kTileV + q * 64 + lane;
  };
  auto out_at = [&](int tau, int q) -> v4f * {
    const long t = MODE >= 1 ? (long)tau * kF + f : (long)f * kTiles + tau;
    return out + t * kOutV + q * 64 + lane;
  };
  v4f pf[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) pf[q] = __builtin_nontemporal_load(in_at(0, q));
  for (int tau = 0; tau < kTiles; ++tau) {
    v4f cur[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) cur[q] = pf[q];
    const int g0 = MODE == 5 ? 8 : 16;
    if (tau + 1 < kTiles) {
#pragma unroll
      for (int q = 0; q < g0; ++q) pf[q] = __builtin_nontemporal_load(in_at(tau + 1, q));
    }
    // some dependent work per tile so the wave does not race ahead
    v4f acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = cur[2 * q] * a + cur[2 * q + 1];
#pragma unroll
    for (int r = 0; r < 64; ++r) {
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = acc[q] * a + acc[(q + 1) & 7];
      if (MODE == 5 && tau + 1 < kTiles && (r == 20 || r == 40)) {
#pragma unroll
        for (int q = 0; q < 4; ++q) pf[(r == 20 ? 8 : 12) + q] = __builtin_nontemporal_load(in_at(tau + 1, (r == 20 ? 8 : 12) + q));
      }
    }
    if (MODE == 4) {
#pragma unroll
      for (int q = 0; q < 6; ++q) __builtin_nontemporal_store(acc[q], out_at(tau, q));
      typedef float v2f_ __attribute__((ext_vector_type(2)));
      const long t = (long)f * kTiles + tau;
      v2f_ *o2 = (v2f_ *)(out + t * kOutV + 6 * 64);  // the tile's last 2 KB as 4 x 8 B per lane
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_nontemporal_store(v2f_{acc[6 + (q >> 1)].x, acc[7 - (q >> 1)].y}, o2 + 64 * q + lane);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) __builtin_nontemporal_store(acc[q], out_at(tau, q));
    }
  }
}

__global__ __launch_bounds__(256) void copy(const v4f *__restrict__ in, v4f *__restrict__ out, long n_in) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n_in / 2; i += stride) {
    const v4f a = __builtin_nontemporal_load(in + 2 * i), b = __builtin_nontemporal_load(in + 2 * i + 1);
    __builtin_nontemporal_store(a + b, out + i);
  }
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  const size_t n_in = (size_t)kF * kTiles * kTileV, n_out = (size_t)kF * kTiles * kOutV;
  v4f *in, *out;
  if (hipMalloc(&in, n_in * 16) != hipSuccess || hipMalloc(&out, n_out * 16) != hipSuccess) return 1;
  (void)hipMemset(in, 0, n_in * 16);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double bytes = (double)(n_in + n_out) * 16;
  for (int mode = 0; mode < 6; ++mode) {
    float best = 1e9f;
    for (int r = 0; r < reps; ++r) {
      (void)hipEventRecord(e0);
      if (mode == 0) walk<0><<<kF / 4, 256>>>(in, out, 0.999f);
      if (mode == 1) walk<1><<<kF / 4, 256>>>(in, out, 0.999f);
      if (mode == 2) walk<2><<<kF / 4, 256>>>(in, out, 0.999f);
      if (mode == 3) copy<<<256 * 8, 256>>>(in, out, (long)n_in);
      if (mode == 4) walk<4><<<kF / 4, 256>>>(in, out, 0.999f);
      if (mode == 5) walk<5><<<kF / 4, 256>>>(in, out, 0.999f);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      if (hipGetLastError() != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) {
        printf("mode %d: launch failed\n", mode);
        return 1;
      }
      if (r > 0 && ms < best) best = ms;
    }
    printf("mode %d: %.3f ms  %.2f TB/s (read %.2f GB + write %.2f GB)\n", mode, best, bytes / best / 1e9,
           n_in * 16 / 1e9, n_out * 16 / 1e9);
  }
  return 0;
}
