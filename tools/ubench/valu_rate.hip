// VALU issue-rate microbenchmark (gfx950): packed vs scalar f32 FMA, independent chains,
// and a dependent packed chain; many waves so the SIMDs are saturated.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));

template <int CH>
__global__ __launch_bounds__(256) void pk_indep(v2f *out, int iters, float a) {
  v2f acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = v2f{(float)threadIdx.x + c, (float)c};
  const v2f m = v2f{a, a * 0.5f};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = __builtin_elementwise_fma(acc[c], m, m);
    }
  }
  v2f s = acc[0];
#pragma unroll
  for (int c = 1; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CH>
__global__ __launch_bounds__(256) void f_indep(float *out, int iters, float a) {
  float acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = (float)threadIdx.x + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = __builtin_fmaf(acc[c], a, a);
    }
  }
  float s = acc[0];
#pragma unroll
  for (int c = 1; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static float timeit(K k, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  k(blocks, iters);  // warm
  hipEventRecord(e0);
  k(blocks, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  void *buf; hipMalloc(&buf, 64 << 20);
  const int iters = 4096;
  for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: blocks of 4 waves, one block per CU x wps
    int blocks = 256 * wps;
    auto run_pk8 = [&](int b, int it) { pk_indep<8><<<b, 256>>>((v2f *)buf, it, 0.999f); };
    auto run_pk1 = [&](int b, int it) { pk_indep<1><<<b, 256>>>((v2f *)buf, it, 0.999f); };
    auto run_f8 = [&](int b, int it) { f_indep<8><<<b, 256>>>((float *)buf, it, 0.999f); };
    auto run_f1 = [&](int b, int it) { f_indep<1><<<b, 256>>>((float *)buf, it, 0.999f); };
    double waves = blocks * 4.0;
    double instr8 = (double)iters * 16 * 8, instr1 = (double)iters * 16;
    float t;
    t = timeit(run_pk8, blocks, iters);
    printf("waves/SIMD %d  pk_fma x8 chains: %.3f ms  -> %.2f cyc/instr/SIMD  (%.1f TFLOP/s)\n", wps, t,
           t * 1e-3 * 2.4e9 / (waves / 1024 * instr8), waves * 64 * instr8 * 4 / (t * 1e-3) / 1e12);
    t = timeit(run_pk1, blocks, iters);
    printf("waves/SIMD %d  pk_fma x1 chain : %.3f ms  -> %.2f cyc/instr/SIMD\n", wps, t,
           t * 1e-3 * 2.4e9 / (waves / 1024 * instr1));
    t = timeit(run_f8, blocks, iters);
    printf("waves/SIMD %d  fma    x8 chains: %.3f ms  -> %.2f cyc/instr/SIMD  (%.1f TFLOP/s)\n", wps, t,
           t * 1e-3 * 2.4e9 / (waves / 1024 * instr8), waves * 64 * instr8 * 2 / (t * 1e-3) / 1e12);
    t = timeit(run_f1, blocks, iters);
    printf("waves/SIMD %d  fma    x1 chain : %.3f ms  -> %.2f cyc/instr/SIMD\n", wps, t,
           t * 1e-3 * 2.4e9 / (waves / 1024 * instr1));
  }
  return 0;
}
