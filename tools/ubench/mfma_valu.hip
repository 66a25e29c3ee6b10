// Does an f32 MFMA stream run beside a packed-f32 VALU stream on gfx950?  (Design input for
// moving the PC walk's input-rate FIRs to v_mfma_f32_16x16x4_f32)
// Cycles per iteration (s_memtime, median over waves), one workgroup per CU:
//   A: VALU only       8 independent v_pk_fma_f32 per iteration
//   B: MFMA only       1 v_mfma_f32_16x16x4_f32 per iteration (4 accumulators in turn)
//   C: both, one wave  1 MFMA + NV pk_fma per iteration, interleaved in the same wave
//   D: both, two waves per SIMD: waves 0-3 run B's stream, waves 4-7 A's
// usage: mfma_valu
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int kIter = 4096;

__device__ __forceinline__ unsigned long long now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int NV>
__device__ __forceinline__ void valu_iter(v2f (&a)[8], v2f m) {
#pragma unroll
  for (int i = 0; i < NV; ++i) a[i & 7] = __builtin_elementwise_fma(a[i & 7], m, m);
}

template <int MODE, int NV>
__global__ __launch_bounds__(512) void k(float *out, unsigned long long *cyc, float s) {
  const int t = threadIdx.x, w = t >> 6;
  v2f a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = v2f{s * i, s + i};
  const v2f m = v2f{0.999f, 0.999f};
  v4f c[4] = {};
  const float fa = s * t, fb = s + t;
  const bool do_mfma = MODE == 1 || MODE == 2 || (MODE == 3 && w < 4);
  const bool do_valu = MODE == 0 || MODE == 2 || (MODE == 3 && w >= 4);
  __syncthreads();
  const unsigned long long t0 = now();
  if (do_mfma && do_valu) {
    for (int it = 0; it < kIter; ++it) {
      c[it & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, c[it & 3], 0, 0, 0);
      valu_iter<NV>(a, m);
    }
  } else if (do_mfma) {
    for (int it = 0; it < kIter; ++it) c[it & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, c[it & 3], 0, 0, 0);
  } else {
    for (int it = 0; it < kIter; ++it) valu_iter<NV>(a, m);
  }
  const unsigned long long t1 = now();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) r += a[i].x + a[i].y;
#pragma unroll
  for (int i = 0; i < 4; ++i) r += c[i].x + c[i].y + c[i].z + c[i].w;
  out[blockIdx.x * 512 + t] = r;
  if ((t & 63) == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

template <int MODE, int NV>
void run(const char *name, int threads) {
  const int blocks = 256;
  float *out;
  unsigned long long *cyc;
  hipMalloc(&out, blocks * 512 * 4);
  hipMalloc(&cyc, blocks * 8 * 8);
  hipMemset(cyc, 0, blocks * 8 * 8);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((k<MODE, NV>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 1e-3f);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 8);
  hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> v;
  for (int b = 0; b < blocks; ++b)
    for (int w = 0; w < threads / 64; ++w) v.push_back((double)h[b * 8 + w] / kIter);
  std::sort(v.begin(), v.end());
  printf("%-34s waves/WG %d  cycles/iter median %.1f  (min %.1f max %.1f)\n", name, threads / 64, v[v.size() / 2], v.front(), v.back());
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<0, 8>("A VALU only (8 pk_fma)", 256);
  run<0, 8>("A VALU only (8 pk_fma), 2 w/SIMD", 512);
  run<1, 0>("B MFMA only", 256);
  run<1, 0>("B MFMA only, 2 w/SIMD", 512);
  run<2, 4>("C 1 MFMA + 4 pk_fma, one wave", 256);
  run<2, 8>("C 1 MFMA + 8 pk_fma, one wave", 256);
  run<2, 16>("C 1 MFMA + 16 pk_fma, one wave", 256);
  run<2, 8>("C 1 MFMA + 8 pk_fma, 2 w/SIMD", 512);
  run<3, 8>("D MFMA waves 0-3 | 8 pk_fma 4-7", 512);
  run<3, 16>("D MFMA waves 0-3 | 16 pk_fma 4-7", 512);
  return 0;
}
