// Microbenchmark for DESIGN §8 item 4 (a band-limited Welch for N = 65536 without the Z round
// trip): can R workgroups that each read the same 1 MB frame share those reads in L2?
// Workgroups are sized like that kernel (256 threads, 64 KB of LDS: two per CU); each reads its
// frame with 16-B loads, folds it into a sum (so the loads cannot be dropped) and writes one value.
//   A  one workgroup per frame, one read                       (the HBM floor: F x 1 MB)
//   B  R workgroups per frame on one XCD, in step              (blockIdx -> frame XCD-aware)
//   C  R workgroups per frame, consecutive blockIdx            (spread over the 8 XCDs)
//   D  one workgroup per frame reading it R times in turn      (re-reads from L2 / the MALL)
// ms per launch (HIP events, median of 7 after 2 warm-ups) and the frame bytes per ms.
// build: hipcc --offload-arch=gfx950 -O3 -o l2share_bench tools/l2share_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float v4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kLdsBytes = 64 * 1024;

template <int MODE>
__global__ void __launch_bounds__(kThreads) read_frames(const v4 *__restrict__ x, long long frame_v4, int frames,
                                                        int R, float *__restrict__ out) {
  extern __shared__ v4 lds[];  // held only to set the occupancy (two workgroups per CU)
  const int t = threadIdx.x;
  const int b = blockIdx.x;
  int f, r;
  if (MODE == 1) {  // B: blocks b, b + 8, b + 16, ... share an XCD; R consecutive ones per frame
    const int xcd = b & 7, k = b >> 3;
    r = k % R;
    f = xcd + 8 * (k / R);
  } else if (MODE == 2) {  // C: frame b / R, its R readers on R different XCDs
    f = b / R;
    r = b % R;
  } else {
    f = b;
    r = 0;
  }
  if (f >= frames) return;
  const v4 *p = x + (long long)f * frame_v4;
  v4 acc = {0.f, 0.f, 0.f, 0.f};
  const int reps = MODE == 3 ? R : 1;
  for (int rep = 0; rep < reps; ++rep) {
#pragma unroll 8
    for (long long i = t; i < frame_v4; i += kThreads) acc += p[i] * (float)(rep + r + 1);
  }
  if (t == 0) lds[0] = acc;
  __syncthreads();
  const float s = acc.x + acc.y + acc.z + acc.w + lds[0].x * 0.f;
  if (t < 64) out[(long long)b * 64 + t] = s;
}

#define CHECK(e)                                                                      \
  do {                                                                                \
    hipError_t err_ = (e);                                                            \
    if (err_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(err_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

template <int MODE>
static float time_mode(const v4 *x, long long frame_v4, int frames, int R, float *out, int grid) {
  CHECK(hipFuncSetAttribute((const void *)read_frames<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int it = 0; it < 9; ++it) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(read_frames<MODE>, dim3(grid), dim3(kThreads), kLdsBytes, 0, x, frame_v4, frames, R, out);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 2) ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
  const int frames = argc > 1 ? std::atoi(argv[1]) : 2048;
  const long long frame_bytes = argc > 2 ? std::atoll(argv[2]) : (1 << 20);
  const int R = argc > 3 ? std::atoi(argv[3]) : 8;
  if (frames <= 0 || frames % 8 != 0 || frame_bytes % (16 * kThreads) != 0 || R <= 0 || R > 64) {
    std::fprintf(stderr, "usage: l2share_bench [frames (multiple of 8)] [frame bytes (multiple of 4096)] [R <= 64]\n");
    return 2;
  }
  const long long frame_v4 = frame_bytes / 16;
  v4 *x = nullptr;
  float *out = nullptr;
  CHECK(hipMalloc(&x, (size_t)frames * frame_bytes));
  CHECK(hipMalloc(&out, (size_t)frames * R * 64 * sizeof(float)));
  CHECK(hipMemset(x, 0, (size_t)frames * frame_bytes));
  CHECK(hipMemset(out, 0, (size_t)frames * R * 64 * sizeof(float)));
  const double gb = (double)frames * frame_bytes / 1e9;
  const float a = time_mode<0>(x, frame_v4, frames, R, out, frames);
  const float b = time_mode<1>(x, frame_v4, frames, R, out, frames * R);
  const float c = time_mode<2>(x, frame_v4, frames, R, out, frames * R);
  const float d = time_mode<3>(x, frame_v4, frames, R, out, frames);
  std::printf("{\"frames\": %d, \"frame_bytes\": %lld, \"R\": %d, \"frame_GB\": %.3f,\n", frames, frame_bytes, R, gb);
  std::printf(" \"ms\": {\"A_once\": %.4f, \"B_R_readers_one_xcd\": %.4f, \"C_R_readers_spread\": %.4f, \"D_R_passes_one_wg\": %.4f},\n",
              a, b, c, d);
  std::printf(" \"frame_GB_per_s\": {\"A\": %.1f, \"B\": %.1f, \"C\": %.1f, \"D\": %.1f},\n", gb / a * 1e3, gb / b * 1e3,
              gb / c * 1e3, gb / d * 1e3);
  std::printf(" \"vs_A\": {\"B\": %.3f, \"C\": %.3f, \"D\": %.3f}}\n", b / a, c / a, d / a);
  CHECK(hipFree(x));
  CHECK(hipFree(out));
  return 0;
}
