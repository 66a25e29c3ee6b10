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

// ------------------------------------------------------------------ work mapping
// Lanes <-> frames: a wave owns one block of one 64-frame group, so every lane runs the
// same (wave-uniform) sample index j and all loads/stores of an interleaved buffer are
// one contiguous 512 B row.  Frame-group-interleaved ("FGI") layout of a per-frame
// sequence of length len: element (f, j) at ((f / 64) * len + j) * 64 + f % 64.
// Block partition (per stage, in padded "ext" coordinates j in [0, e), e = n + 54):
//   block 0 = [0, 27 + S), block b >= 1 = [27 + b S, 27 + (b+1) S), last ends at e.
struct WaveCtx {
  int lane, b, fg, j0, j1;
  bool valid;
};

__device__ __forceinline__ WaveCtx wave_ctx(const StageGeom &g) {
  WaveCtx w;
  w.lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  w.valid = wid < g.ngroups * g.nblk;
  w.b = wid % g.nblk;
  w.fg = wid / g.nblk;
  const int e = g.n + 2 * kPad;
  w.j0 = w.b == 0 ? 0 : kPad + w.b * g.block;
  w.j1 = min(kPad + (w.b + 1) * g.block, e);
  return w;
}

__device__ __forceinline__ int64_t fgi(int fg, int64_t len, int64_t j) {
  return ((int64_t)fg * len + j) << 6;
}

constexpr int kU = 8;  // samples per prefetch group (register double buffer)

// Run the cascade over j in [ja, jb) reading src(j) (interleaved row pointer p, stride 64),
// with a two-group register pipeline: the loads of group g+1 are in flight while group g
// is computed.  emit(j, y) is called for every step when STORE.
template <bool STORE, class Src, class Emit>
__device__ __forceinline__ void pipelined_run(int ja, int jb, Src src, IirState &s,
                                              const Sos32 &c, Emit emit) {
  const int cnt = jb - ja;
  const int full = cnt > 0 ? cnt / kU : 0;
  int j = ja;
  if (full > 0) {
    v2f A[kU], B[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) A[u] = src(j + u);
    int gi = 0;
    while (true) {
      if (gi + 1 < full) {
#pragma unroll
        for (int u = 0; u < kU; ++u) B[u] = src(j + kU + u);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const v2f o = cascade(A[u], s, c);
        if constexpr (STORE) emit(j + u, o);
      }
      j += kU;
      if (++gi >= full) break;
      if (gi + 1 < full) {
#pragma unroll
        for (int u = 0; u < kU; ++u) A[u] = src(j + kU + u);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const v2f o = cascade(B[u], s, c);
        if constexpr (STORE) emit(j + u, o);
      }
      j += kU;
      if (++gi >= full) break;
    }
  }
  for (; j < jb; ++j) {
    const v2f o = cascade(src(j), s, c);
    if constexpr (STORE) emit(j, o);
  }
}

// ------------------------------------------------------------------ forward pass, stage >= 1
// yf(j) = sosfilt over ext(j), ext = odd extension of the FGI stage input, state zi*ext[0].
__global__ __launch_bounds__(256) void iir_forward_fgi_kernel(const v2f *__restrict__ in,
                                                              v2f *__restrict__ yf, StageGeom g,
                                                              Sos32 c) {
  const WaveCtx w = wave_ctx(g);
  if (!w.valid) return;
  const int n = g.n, e = n + 2 * kPad;
  const v2f *__restrict__ x = in + fgi(w.fg, n, 0) + w.lane;
  v2f *__restrict__ y = yf + fgi(w.fg, e, 0) + w.lane;
  auto X = [&](int i) -> v2f { return x[(int64_t)i << 6]; };
  auto ext = [&](int j) -> v2f {  // wave-uniform branch on j
    if (j < kPad) return 2.f * X(0) - X(kPad - j);
    if (j < n + kPad) return X(j - kPad);
    return 2.f * X(n - 1) - X(2 * n + kPad - 2 - j);
  };
  IirState s;
  int js;
  if (w.j0 - g.warmup <= 0) {
    js = 0;
    state_steady(s, c, ext(0));
  } else {
    js = w.j0 - g.warmup;
    state_zero(s);
  }
  auto emit = [&](int j, v2f o) { y[(int64_t)j << 6] = o; };
  auto run = [&](int ja, int jb, auto store_tag) {
    constexpr bool STORE = decltype(store_tag)::value;
    int a = ja;
    for (; a < min(jb, kPad); ++a) {  // left odd extension
      const v2f o = cascade(ext(a), s, c);
      if constexpr (STORE) emit(a, o);
    }
    const int ib = min(jb, n + kPad);
    if (a < ib) {
      pipelined_run<STORE>(a, ib, [&](int j) { return X(j - kPad); }, s, c, emit);
      a = ib;
    }
    for (; a < jb; ++a) {  // right odd extension
      const v2f o = cascade(ext(a), s, c);
      if constexpr (STORE) emit(a, o);
    }
  };
  run(js, w.j0, std::false_type{});
  run(w.j0, w.j1, std::true_type{});
}

// ------------------------------------------------------------------ forward pass, stage 0
// Input: the caller's frames in natural layout (frame-major complex64), mixed with the LO
// table on load.  Lanes are frames, so a direct per-lane load would touch 64 cache lines per
// instruction; instead each wave stages a 64-frame x 16-sample tile through LDS, loaded
// with 16 lanes per 128 B frame segment, and the next tile's loads are in flight while the
// current one is filtered.
constexpr int kTile = 16;
constexpr int kTileStride = kTile + 2;  // float2 units: 144 B rows, 16 B aligned, conflict-free

__global__ __launch_bounds__(256) void iir_forward_mix_kernel(const v2f *__restrict__ in,
                                                              int64_t L, int frames,
                                                              const v2f *__restrict__ lo,
                                                              v2f *__restrict__ yf, StageGeom g,
                                                              Sos32 c) {
  __shared__ __attribute__((aligned(16))) v2f tile_all[4][64 * kTileStride];
  const WaveCtx w = wave_ctx(g);
  if (!w.valid) return;
  const int n = g.n, e = n + 2 * kPad;  // n == L
  v2f *tile = tile_all[threadIdx.x >> 6];
  v2f *__restrict__ y = yf + fgi(w.fg, e, 0) + w.lane;
  const int f0 = w.fg * 64;
  // loader geometry: element (row r = 4q + lane/16, col k = lane%16)
  const int lrow = w.lane >> 4, lcol = w.lane & 15;

  auto xm = [&](int f, int i) -> v2f {  // mixed sample of frame f at index i (natural layout)
    return cmul(in[(int64_t)f * L + i], lo[i]);
  };
  auto ext_slow = [&](int f, int j) -> v2f {
    if (f >= frames || j < 0 || j >= e) return splat(0.f);
    if (j < kPad) return 2.f * xm(f, 0) - xm(f, kPad - j);
    if (j < n + kPad) return xm(f, j - kPad);
    return 2.f * xm(f, n - 1) - xm(f, 2 * n + kPad - 2 - j);
  };

  v2f pf[16];  // this lane's share of the next tile
  auto load_tile = [&](int jc) {
    const int j = jc + lcol;
    const bool fast = jc >= kPad && jc + kTile <= n + kPad && f0 + 64 <= frames;  // uniform
    if (fast) {
      const v2f l = lo[j - kPad];
      const v2f *p = in + (int64_t)(f0 + lrow) * L + (j - kPad);
#pragma unroll
      for (int q = 0; q < 16; ++q) pf[q] = cmul(p[(int64_t)q * 4 * L], l);
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) pf[q] = ext_slow(f0 + 4 * q + lrow, j);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int q = 0; q < 16; ++q) tile[(4 * q + lrow) * kTileStride + lcol] = pf[q];
  };

  IirState s;
  int js;
  if (w.j0 - g.warmup <= 0) {
    js = 0;
    state_steady(s, c, ext_slow(f0 + w.lane, 0));
  } else {
    js = w.j0 - g.warmup;
    state_zero(s);
  }
  load_tile(js);
  for (int jc = js; jc < w.j1; jc += kTile) {
    store_tile();                       // tile jc (its loads were issued one tile ago)
    __builtin_amdgcn_wave_barrier();
    if (jc + kTile < w.j1) load_tile(jc + kTile);  // in flight during the filter below
    const v2f *row = tile + w.lane * kTileStride;
    const int steps = min(kTile, w.j1 - jc);
    if (steps == kTile && jc >= w.j0) {
#pragma unroll
      for (int k = 0; k < kTile; ++k) y[(int64_t)(jc + k) << 6] = cascade(row[k], s, c);
    } else {
      for (int k = 0; k < steps; ++k) {
        const v2f o = cascade(row[k], s, c);
        if (jc + k >= w.j0) y[(int64_t)(jc + k) << 6] = o;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------ backward pass
// sosfilt over reversed yf with state zi*yf[e-1]; keep j = 27 + 2m -> out(m), FGI layout.
__global__ __launch_bounds__(256) void iir_backward_kernel(const v2f *__restrict__ yf,
                                                           v2f *__restrict__ out, StageGeom g,
                                                           Sos32 c) {
  const WaveCtx w = wave_ctx(g);
  if (!w.valid) return;
  const int n = g.n, e = n + 2 * kPad, m_len = (n + 1) >> 1;
  const v2f *__restrict__ y = yf + fgi(w.fg, e, 0) + w.lane;
  v2f *__restrict__ o = out + fgi(w.fg, m_len, 0) + w.lane;
  const int jlo = max(w.j0, kPad);  // below kPad: left pad, no outputs -> skipped
  if (jlo >= w.j1) return;
  const int jhi = min(w.j1, n + kPad);  // outputs for j in [jlo, jhi)
  IirState s;
  int jt;  // exclusive top of the descending run
  if (w.j1 + g.warmup >= e) {
    jt = e;
    state_steady(s, c, y[(int64_t)(e - 1) << 6]);
  } else {
    jt = w.j1 + g.warmup;
    state_zero(s);
  }
  // descending index d = jt - 1 - j; run over j in (jhi, jt) without output, then [jlo, jhi)
  auto Y = [&](int j) -> v2f { return y[(int64_t)j << 6]; };
  auto emit = [&](int d, v2f v) {
    const int j = jt - 1 - d;
    if (!((j - kPad) & 1)) o[(int64_t)((j - kPad) >> 1) << 6] = v;
  };
  pipelined_run<false>(0, jt - jhi, [&](int d) { return Y(jt - 1 - d); }, s, c, emit);
  pipelined_run<true>(jt - jhi, jt - jlo, [&](int d) { return Y(jt - 1 - d); }, s, c, emit);
}

// out[f][i] = in FGI (f, i): for zoomfft's host API
__global__ __launch_bounds__(256) void deinterleave_kernel(const v2f *__restrict__ in,
                                                           int64_t len, int frames,
                                                           v2f *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len * frames) return;
  const int f = (int)(i / len);
  const int64_t j = i - (int64_t)f * len;
  out[i] = in[fgi(f >> 6, len, j) + (f & 63)];
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
// Input either the FGI output of the last decimation stage (stride 64 between samples of a
// frame) or, at zoom 1, the caller's natural-layout frames.  Frames sharing FGI cache lines
// (16 consecutive frames per 128 B) are kept on one XCD: blocks b and b + 8 share an XCD.
template <bool FGI>
__global__ __launch_bounds__(1024) void welch_rows_kernel(const v2f *__restrict__ x,
                                                          int64_t len,
                                                          const float *__restrict__ win,
                                                          const v2f *__restrict__ tw,
                                                          WelchGeom g, float *__restrict__ rows,
                                                          int frames) {
  extern __shared__ v2f sh[];
  v2f *red = sh + g.n_fft;
  const int T = blockDim.x, tid = threadIdx.x, N = g.n_fft;
  int f = blockIdx.x;
  if ((frames & 7) == 0) f = (blockIdx.x & 7) * (frames >> 3) + (blockIdx.x >> 3);
  const int64_t sstride = FGI ? 64 : 1;
  const v2f *__restrict__ xf = FGI ? x + fgi(f >> 6, len, 0) + (f & 63) : x + (int64_t)f * len;
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  for (int s = 0; s < g.nseg; ++s) {
    const v2f *__restrict__ seg = xf + (int64_t)s * g.step * sstride;
    v2f sum = splat(0.f);
    for (int n = tid; n < N; n += T) {
      const v2f v = n < g.nperseg ? seg[n * sstride] : splat(0.f);
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
  float *__restrict__ row = rows + (int64_t)f * g.n_win;
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

static inline unsigned wave_blocks(const StageGeom &g) {
  return (unsigned)(((int64_t)g.ngroups * g.nblk + 3) / 4);
}

hipError_t launch_iir_forward_mix(const float2 *in, int64_t L, int frames, const float2 *lo,
                                  float2 *yf, const StageGeom &g, hipStream_t st) {
  hipLaunchKernelGGL(iir_forward_mix_kernel, dim3(wave_blocks(g)), dim3(256), 0, st,
                     (const v2f *)in, L, frames, (const v2f *)lo, (v2f *)yf, g, sos32());
  return hipGetLastError();
}

hipError_t launch_iir_forward_fgi(const float2 *in, float2 *yf, const StageGeom &g,
                                  hipStream_t st) {
  hipLaunchKernelGGL(iir_forward_fgi_kernel, dim3(wave_blocks(g)), dim3(256), 0, st,
                     (const v2f *)in, (v2f *)yf, g, sos32());
  return hipGetLastError();
}

hipError_t launch_iir_backward(const float2 *yf, float2 *out, const StageGeom &g,
                               hipStream_t st) {
  hipLaunchKernelGGL(iir_backward_kernel, dim3(wave_blocks(g)), dim3(256), 0, st,
                     (const v2f *)yf, (v2f *)out, g, sos32());
  return hipGetLastError();
}

hipError_t launch_deinterleave(const float2 *in, int64_t len, int frames, float2 *out,
                               hipStream_t st) {
  hipLaunchKernelGGL(deinterleave_kernel, dim3(nblocks(len * frames, 256)), dim3(256), 0, st,
                     (const v2f *)in, len, frames, (v2f *)out);
  return hipGetLastError();
}

hipError_t launch_mix(const float2 *in, const float2 *lo, float2 *out, int64_t n,
                      hipStream_t st) {
  hipLaunchKernelGGL(mix_kernel, dim3(nblocks(n, 256)), dim3(256), 0, st, (const v2f *)in,
                     (const v2f *)lo, (v2f *)out, n);
  return hipGetLastError();
}

hipError_t launch_welch_rows(const float2 *x, bool fgi_layout, int64_t len, const float *win,
                             const float2 *tw, const WelchGeom &g, float *rows, int frames,
                             hipStream_t st) {
  const int T = g.n_fft / 16 > 64 ? g.n_fft / 16 : 64;  // <= 4 radix-4 butterflies per thread
  const size_t lds = (size_t)(g.n_fft + 32) * sizeof(v2f);
  static bool attr_set = false;
  if (!attr_set) {
    for (const void *fn : {(const void *)welch_rows_kernel<true>, (const void *)welch_rows_kernel<false>}) {
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (kMaxLdsFft + 32) * (int)sizeof(v2f));
      if (e != hipSuccess) return e;
    }
    attr_set = true;
  }
  if (fgi_layout)
    hipLaunchKernelGGL(welch_rows_kernel<true>, dim3(frames), dim3(T), lds, st, (const v2f *)x, len,
                       win, (const v2f *)tw, g, rows, frames);
  else
    hipLaunchKernelGGL(welch_rows_kernel<false>, dim3(frames), dim3(T), lds, st, (const v2f *)x,
                       len, win, (const v2f *)tw, g, rows, frames);
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
