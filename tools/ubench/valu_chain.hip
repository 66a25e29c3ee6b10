// Dependent-chain throughput of v_pk_fma_f32 and v_fma_f32 on gfx950: NC independent chains of
// FMAs per wave (each FMA depends on the previous one of its chain), one or two waves per
// SIMD.  Cycles per instruction (s_memtime, median over waves).  Design input for the PC walk's
// recurrences (one or two chains per lane block) and FIRs (4-9 accumulators).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int kIter = 2048;

template <int NC, bool PK>
__global__ __launch_bounds__(512) void k(float *out, unsigned long long *cyc, float s) {
  const int t = threadIdx.x;
  v2f a[NC];
  float b[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) a[i] = v2f{s * i, s + i}, b[i] = s * i + t;
  const v2f m = v2f{0.999f, 0.999f};
  unsigned long long t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      if constexpr (PK) a[i] = __builtin_elementwise_fma(a[i], m, m);
      else b[i] = __builtin_fmaf(b[i], 0.999f, 0.5f);
    }
  }
  unsigned long long t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) r += a[i].x + a[i].y + b[i];
  out[blockIdx.x * 512 + t] = r;
  if ((t & 63) == 0) cyc[blockIdx.x * 8 + (t >> 6)] = t1 - t0;
}

template <int NC, bool PK>
void run(int threads) {
  const int blocks = 256;
  float *out;
  unsigned long long *cyc;
  (void)hipMalloc(&out, blocks * 512 * 4);
  (void)hipMalloc(&cyc, blocks * 8 * 8);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((k<NC, PK>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 1e-3f);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 8);
  (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> v;
  for (int b = 0; b < blocks; ++b)
    for (int w = 0; w < threads / 64; ++w) v.push_back((double)h[b * 8 + w] / (kIter * NC));
  std::sort(v.begin(), v.end());
  printf("%-10s chains %2d  waves/SIMD %d  cycles per instruction per wave %.2f\n", PK ? "pk_fma" : "fma", NC,
         threads / 256, v[v.size() / 2]);
  (void)hipFree(out);
  (void)hipFree(cyc);
}

template <bool PK>
void all() {
  for (int th : {256, 512}) {
    run<1, PK>(th);
    run<2, PK>(th);
    run<4, PK>(th);
    run<8, PK>(th);
    run<16, PK>(th);
  }
}

int main() {
  all<true>();
  all<false>();
  return 0;
}
