// zfft_kernels.hip -- CDNA4 (gfx950) kernels of the Zoom-FFT hot path.
//
// Reference path (alfille/pypanadapter, pypanadapter_spectrum.py):
//   S:2093-2094  LO mix  x * sqrt(2) exp(-2 pi i f n / fs)        -> fused into iir_forward<MIX>
//   S:2096-2098  log2(zoom) x scipy.signal.decimate(x, 2)          -> iir_forward + iir_backward
//                (cheby1(8,.05,.4) SOS, sosfiltfilt: odd pad 27, zi init, fwd + bwd, [::2])
//   S:2111       scipy.signal.welch(x, fs, window, nperseg=N, nfft=N)
//   S:2114-2119  fftshift + centre crop W + 20*log10              -> welch_rows (one kernel)
//   S:1638-1664  Waterfall.image_update (row write, np.roll, grid/tick stamps)
//                                                                  -> waterfall_push / _read
//
// Decimator design: every stage pass is a sequential IIR recurrence, so
// parallelism comes from cutting each frame's padded signal into blocks of S samples, one
// block per lane.  A block that does not touch the frame edge starts W samples early
// from a zero state (max pole radius 0.9351: W = 192 brings the state error below fp32
// rounding, tools/sim_blocked.py); blocks at the frame edges run scipy's exact
// initial conditions (zi * ext[0] forward, zi * y[-1] backward).  I and Q share the real
// coefficients, so each lane carries them as one packed float2 (v_pk_fma_f32).
#include <type_traits>

#include "zfft_internal.h"

namespace zfft {

typedef float v2f __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2f splat(float a) { return v2f{a, a}; }
__device__ __forceinline__ v2f vfma(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ v2f cmul(v2f a, v2f b) {
  return v2f{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}

struct IirState {
  v2f z0[4], z1[4];
};

__device__ __forceinline__ void state_zero(IirState &s) {
#pragma unroll
  for (int k = 0; k < 4; ++k) s.z0[k] = s.z1[k] = splat(0.f);
}

__device__ __forceinline__ void state_steady(IirState &s, const Sos32 &c, v2f u0) {
  // sosfilt_zi(sos) * x0 (sosfiltfilt, _signaltools.py:4817-4824)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    s.z0[k] = c.zi[k][0] * u0;
    s.z1[k] = c.zi[k][1] * u0;
  }
}

// One sample through the 4-section transposed-direct-form-II cascade (scipy _sosfilt).
// Sections 1..3 have the exact numerator [1, 2, 1]; the gain sits in section 0.
__device__ __forceinline__ v2f cascade(v2f u, IirState &s, const Sos32 &c) {
  v2f y = vfma(splat(c.b0), u, s.z0[0]);
  s.z0[0] = vfma(splat(-c.a1[0]), y, vfma(splat(c.b1), u, s.z1[0]));
  s.z1[0] = vfma(splat(-c.a2[0]), y, splat(c.b2) * u);
  u = y;
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    y = u + s.z0[k];
    s.z0[k] = vfma(splat(-c.a1[k]), y, vfma(splat(2.f), u, s.z1[k]));
    s.z1[k] = vfma(splat(-c.a2[k]), y, u);
    u = y;
  }
  return u;
}

// ------------------------------------------------------------------ forward pass
// yf[j], j in [0, n+54): sosfilt over the odd-extended stage input, state zi*ext[0].
template <bool MIX>
__global__ __launch_bounds__(256) void iir_forward_kernel(const v2f *__restrict__ in,
                                                          int64_t in_stride,
                                                          const v2f *__restrict__ lo,
                                                          v2f *__restrict__ yf, int64_t yf_stride,
                                                          StageGeom g, int frames, Sos32 c) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)frames * g.nblk) return;
  const int f = (int)(gid / g.nblk);
  const int b = (int)(gid - (int64_t)f * g.nblk);
  const int n = g.n, e = n + 2 * kPad;
  const v2f *__restrict__ x = in + (int64_t)f * in_stride;
  v2f *__restrict__ y = yf + (int64_t)f * yf_stride;

  auto X = [&](int i) -> v2f {
    v2f v = x[i];
    if constexpr (MIX) v = cmul(v, lo[i]);
    return v;
  };

  const int j0 = b * g.block;
  const int j1 = min(j0 + g.block, e);
  IirState s;
  int js;
  if (j0 - g.warmup <= 0) {
    js = 0;
    state_steady(s, c, 2.f * X(0) - X(kPad));  // ext[0]
  } else {
    js = j0 - g.warmup;
    state_zero(s);
  }

  auto run = [&](int ja, int jb, auto store_tag) {
    constexpr bool STORE = decltype(store_tag)::value;
    int j = ja;
    if (j < kPad && j < jb) {  // left odd extension: 2 x[0] - x[27 - j]
      const v2f x0 = X(0);
      const int je = min(jb, kPad);
      for (; j < je; ++j) {
        v2f o = cascade(2.f * x0 - X(kPad - j), s, c);
        if constexpr (STORE) y[j] = o;
      }
    }
    const int je = min(jb, n + kPad);
#pragma unroll 4
    for (; j < je; ++j) {
      v2f o = cascade(X(j - kPad), s, c);
      if constexpr (STORE) y[j] = o;
    }
    if (j < jb) {  // right odd extension: 2 x[n-1] - x[2n + 25 - j]
      const v2f xl = X(n - 1);
      for (; j < jb; ++j) {
        v2f o = cascade(2.f * xl - X(2 * n + kPad - 2 - j), s, c);
        if constexpr (STORE) y[j] = o;
      }
    }
  };
  run(js, j0, std::false_type{});
  run(j0, j1, std::true_type{});
}

// ------------------------------------------------------------------ backward pass
// sosfilt over reversed yf with state zi*yf[e-1]; keep j = 27 + 2m, m in [0, ceil(n/2)).
__global__ __launch_bounds__(256) void iir_backward_kernel(const v2f *__restrict__ yf,
                                                           int64_t yf_stride,
                                                           v2f *__restrict__ out,
                                                           int64_t out_stride, StageGeom g,
                                                           int frames, Sos32 c) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)frames * g.nblk) return;
  const int f = (int)(gid / g.nblk);
  const int b = (int)(gid - (int64_t)f * g.nblk);
  const int n = g.n, e = n + 2 * kPad;
  const v2f *__restrict__ y = yf + (int64_t)f * yf_stride;
  v2f *__restrict__ o = out + (int64_t)f * out_stride;

  const int j0 = b * g.block;
  const int j1 = min(j0 + g.block, e);
  const int jlo = max(j0, kPad);          // below kPad: left pad, no outputs -> skipped
  if (jlo >= j1) return;
  IirState s;
  int j;
  if (j1 + g.warmup >= e) {
    j = e - 1;
    state_steady(s, c, y[e - 1]);
  } else {
    j = j1 - 1 + g.warmup;
    state_zero(s);
  }
  const int jhi = min(j1, n + kPad) - 1;  // last j with an output candidate
#pragma unroll 4
  for (; j > jhi; --j) cascade(y[j], s, c);  // warm-up + right pad
  if (j >= jlo && ((j - kPad) & 1)) {       // odd m: no output
    cascade(y[j], s, c);
    --j;
  }
#pragma unroll 2
  for (; j - 1 >= jlo; j -= 2) {
    o[(j - kPad) >> 1] = cascade(y[j], s, c);
    cascade(y[j - 1], s, c);
  }
  if (j >= jlo) o[(j - kPad) >> 1] = cascade(y[j], s, c);
}

__global__ __launch_bounds__(256) void mix_kernel(const v2f *__restrict__ in,
                                                  const v2f *__restrict__ lo,
                                                  v2f *__restrict__ out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = cmul(in[i], lo[i]);
}

// ------------------------------------------------------------------ Welch row
__device__ __forceinline__ v2f wave_sum(v2f v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    v.x += __shfl_xor(v.x, m, 64);
    v.y += __shfl_xor(v.y, m, 64);
  }
  return v;
}

// Stockham autosort FFT (radix-4 passes, one leading radix-2 pass when log2 N is odd),
// natural-order in and out, in LDS with register staging (one buffer).
// Pass: v_r = a[j + r N/R] * w^{r k}, k = j mod Ns; DFT_R; a[(j-k) R + k + r Ns] = V_r.
__device__ void fft_lds(v2f *sh, int N, int log2n, const v2f *__restrict__ tw, int tid, int T) {
  int Ns = 1;
  if (log2n & 1) {
    const int nb = N >> 1;
    v2f a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = tid + i * T;
      if (j < nb) { a[i] = sh[j]; b[i] = sh[j + nb]; }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = tid + i * T;
      if (j < nb) {
        sh[2 * j] = a[i] + b[i];
        sh[2 * j + 1] = a[i] - b[i];
      }
    }
    __syncthreads();
    Ns = 2;
  }
  const int q = N >> 2;
  for (; Ns < N; Ns <<= 2) {
    v2f v[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = tid + i * T;
      if (j < q) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[i][r] = sh[j + r * q];
      }
    }
    __syncthreads();
    const int tstride = N / (4 * Ns);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = tid + i * T;
      if (j < q) {
        const int k = j & (Ns - 1);
        v2f v0 = v[i][0], v1 = v[i][1], v2 = v[i][2], v3 = v[i][3];
        if (Ns > 1) {
          const int t = k * tstride;
          v1 = cmul(v1, tw[t]);
          v2 = cmul(v2, tw[2 * t]);
          v3 = cmul(v3, tw[3 * t]);
        }
        const v2f a0 = v0 + v2, a1 = v0 - v2, a2 = v1 + v3, d = v1 - v3;
        const v2f a3 = v2f{d.y, -d.x};  // -i * (v1 - v3)
        const int idx = ((j - k) << 2) + k;
        sh[idx] = a0 + a2;
        sh[idx + Ns] = a1 + a3;
        sh[idx + 2 * Ns] = a0 - a2;
        sh[idx + 3 * Ns] = a1 - a3;
      }
    }
    __syncthreads();
  }
}

// One workgroup per frame: for each Welch segment, constant detrend + window + N-point
// FFT in LDS, |X|^2 accumulated in registers for the W cropped bins only; then density
// scale, fftshift crop and 20*log10 (S:2111-2119).
__global__ __launch_bounds__(1024) void welch_rows_kernel(const v2f *__restrict__ x,
                                                          int64_t x_stride,
                                                          const float *__restrict__ win,
                                                          const v2f *__restrict__ tw,
                                                          WelchGeom g, float *__restrict__ rows,
                                                          int64_t row_stride) {
  extern __shared__ v2f sh[];
  v2f *red = sh + g.n_fft;
  const int T = blockDim.x, tid = threadIdx.x, N = g.n_fft;
  const v2f *__restrict__ xf = x + (int64_t)blockIdx.x * x_stride;
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  for (int s = 0; s < g.nseg; ++s) {
    const v2f *__restrict__ seg = xf + (int64_t)s * g.step;
    v2f sum = splat(0.f);
    for (int n = tid; n < N; n += T) {
      const v2f v = n < g.nperseg ? seg[n] : splat(0.f);
      sh[n] = v;
      sum += v;
    }
    sum = wave_sum(sum);
    if ((tid & 63) == 0) red[tid >> 6] = sum;
    __syncthreads();
    if (tid < 64) {
      v2f t = tid < (T >> 6) ? red[tid] : splat(0.f);
      t = wave_sum(t);
      if (tid == 0) red[16] = t;
    }
    __syncthreads();
    const v2f mean = red[16] * (1.f / (float)g.nperseg);
    for (int n = tid; n < g.nperseg; n += T) sh[n] = (sh[n] - mean) * win[n];
    __syncthreads();
    fft_lds(sh, N, g.log2n, tw, tid, T);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int j = tid + i * T;
      if (j < g.n_win) {
        const v2f v = sh[(j - (g.n_win >> 1)) & (N - 1)];
        acc[i] = fmaf(v.x, v.x, fmaf(v.y, v.y, acc[i]));
      }
    }
    __syncthreads();
  }
  float *__restrict__ row = rows + (int64_t)blockIdx.x * row_stride;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int j = tid + i * T;
    if (j < g.n_win) row[j] = 20.f * log10f(acc[i] * g.scale);
  }
}

// ------------------------------------------------------------------ waterfall ring
// img[i] == ring[(i + off) mod H]; np.roll(img, -scroll, 0) is off += scroll.
__global__ void waterfall_init_kernel(float *ring, int H, int W) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)H * W) return;
  const int xcol = (int)(i % W);
  ring[i] = (xcol == 0 || xcol == W - 1) ? 0.f : -500.f;  // init_image, S:1631-1635
}

__device__ __forceinline__ int pmod(int64_t a, int m) {
  int r = (int)(a % m);
  return r < 0 ? r + m : r;
}

// Applies pushes [max(0,count-H), count) in order (earlier ones are fully overwritten:
// with a constant scroll every slot and every stamp is rewritten within H pushes).
__global__ __launch_bounds__(1024) void waterfall_push_kernel(float *ring, int H, int W,
                                                              const float *__restrict__ rows,
                                                              int64_t row_stride, int count,
                                                              int64_t off0, int scroll) {
  const int T = blockDim.x, tid = threadIdx.x;
  const int first = count > H ? count - H : 0;
  int o = pmod(off0 + (int64_t)first * scroll, H);
  const int tick = W / 10;
  const int nt = (W - 1 + tick - 1) / tick;  // len(range(0, W-1, W//10))
  const int nrows = scroll > 0 ? 10 : 8;     // img[5:15] or img[-10:-2]
  for (int r = first; r < count; ++r) {
    const float *__restrict__ src = rows + (int64_t)r * row_stride;
    const int slot = pmod(H - 1 + o, H);     // img[-1:] = psd
    for (int xcol = tid; xcol < W; xcol += T) {
      float v = src[xcol];
      if (xcol == 0 || xcol == (W >> 1) || xcol == W - 1) v = 0.f;  // grid, S:1646-1648
      ring[(int64_t)slot * W + xcol] = v;
    }
    o = pmod(o + scroll, H);
    __syncthreads();
    for (int idx = tid; idx < nt * nrows; idx += T) {  // tick stamps, S:1655-1662
      const int i = idx % nt, yy = idx / nt;
      if (i == 5 || i == 10) continue;
      const int yrow = scroll > 0 ? 5 + yy : H - 10 + yy;
      ring[(int64_t)pmod(yrow + o, H) * W + i * tick] = 0.f;
    }
    __syncthreads();
  }
}

__global__ void waterfall_read_kernel(const float *__restrict__ ring, int H, int W, int off,
                                      float *__restrict__ img) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)H * W) return;
  const int r = (int)(i / W), xcol = (int)(i % W);
  img[i] = ring[(int64_t)((r + off) % H) * W + xcol];
}

// ------------------------------------------------------------------ launchers
static inline unsigned nblocks(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

hipError_t launch_iir_forward(const float2 *in, int64_t in_stride, const float2 *lo, bool mix,
                              float2 *yf, int64_t yf_stride, const StageGeom &g, int frames,
                              hipStream_t st) {
  const int64_t lanes = (int64_t)frames * g.nblk;
  const Sos32 c = sos32();
  if (mix)
    hipLaunchKernelGGL(iir_forward_kernel<true>, dim3(nblocks(lanes, 256)), dim3(256), 0, st,
                       (const v2f *)in, in_stride, (const v2f *)lo, (v2f *)yf, yf_stride, g,
                       frames, c);
  else
    hipLaunchKernelGGL(iir_forward_kernel<false>, dim3(nblocks(lanes, 256)), dim3(256), 0, st,
                       (const v2f *)in, in_stride, (const v2f *)lo, (v2f *)yf, yf_stride, g,
                       frames, c);
  return hipGetLastError();
}

hipError_t launch_iir_backward(const float2 *yf, int64_t yf_stride, float2 *out,
                               int64_t out_stride, const StageGeom &g, int frames,
                               hipStream_t st) {
  const int64_t lanes = (int64_t)frames * g.nblk;
  hipLaunchKernelGGL(iir_backward_kernel, dim3(nblocks(lanes, 256)), dim3(256), 0, st,
                     (const v2f *)yf, yf_stride, (v2f *)out, out_stride, g, frames, sos32());
  return hipGetLastError();
}

hipError_t launch_mix(const float2 *in, const float2 *lo, float2 *out, int64_t n,
                      hipStream_t st) {
  hipLaunchKernelGGL(mix_kernel, dim3(nblocks(n, 256)), dim3(256), 0, st, (const v2f *)in,
                     (const v2f *)lo, (v2f *)out, n);
  return hipGetLastError();
}

hipError_t launch_welch_rows(const float2 *x, int64_t x_stride, const float *win,
                             const float2 *tw, const WelchGeom &g, float *rows,
                             int64_t row_stride, int frames, hipStream_t st) {
  const int T = g.n_fft / 16 > 64 ? g.n_fft / 16 : 64;  // <= 4 radix-4 butterflies per thread
  const size_t lds = (size_t)(g.n_fft + 32) * sizeof(v2f);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)welch_rows_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (kMaxLdsFft + 32) * (int)sizeof(v2f));
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(welch_rows_kernel, dim3(frames), dim3(T), lds, st, (const v2f *)x, x_stride,
                     win, (const v2f *)tw, g, rows, row_stride);
  return hipGetLastError();
}

hipError_t launch_waterfall_init(float *ring, int H, int W, hipStream_t st) {
  hipLaunchKernelGGL(waterfall_init_kernel, dim3(nblocks((int64_t)H * W, 256)), dim3(256), 0, st,
                     ring, H, W);
  return hipGetLastError();
}

hipError_t launch_waterfall_push(float *ring, int H, int W, const float *rows,
                                 int64_t row_stride, int count, int64_t off0, int scroll,
                                 hipStream_t st) {
  const int T = W >= 1024 ? 1024 : (W >= 256 ? 256 : 64);
  hipLaunchKernelGGL(waterfall_push_kernel, dim3(1), dim3(T), 0, st, ring, H, W, rows, row_stride,
                     count, off0, scroll);
  return hipGetLastError();
}

hipError_t launch_waterfall_read(const float *ring, int H, int W, int64_t off, float *img,
                                 hipStream_t st) {
  hipLaunchKernelGGL(waterfall_read_kernel, dim3(nblocks((int64_t)H * W, 256)), dim3(256), 0, st,
                     ring, H, W, (int)(off % H), img);
  return hipGetLastError();
}

}  // namespace zfft
