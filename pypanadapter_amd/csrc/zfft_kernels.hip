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
#include <algorithm>
#include <type_traits>

#include "zfft_device.h"
#include "zfft_fft.h"

namespace zfft {

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

template <int DT, bool MULTI_LO>
__global__ __launch_bounds__(256) void iir_forward_mix_kernel(InDesc in, int frames,
                                                              const v2f *__restrict__ lo,
                                                              v2f *__restrict__ yf, StageGeom g,
                                                              Sos32 c) {
  __shared__ __attribute__((aligned(16))) v2f tile_all[4][64 * kTileStride];
  const WaveCtx w = wave_ctx(g);
  if (!w.valid) return;
  const int n = g.n, e = n + 2 * kPad;
  v2f *tile = tile_all[threadIdx.x >> 6];
  v2f *__restrict__ y = yf + fgi(w.fg, e, 0) + w.lane;
  // Frame groups at or above g.split (a multiple of 64, 0 = none) are a second set of
  // windows starting g.alt_off samples into the same frames (edge windows, one launch).
  const bool second = g.split > 0 && w.fg * 64 >= g.split;
  const int64_t o = second ? g.alt_off : 0;  // window start in the frame
  const v2f *__restrict__ lob = lo + o;
  const int f0 = w.fg * 64 - (second ? g.split : 0);  // frame index of row 0 in its set
  // loader geometry: element (row r = 4q + lane/16, col k = lane%16)
  const int lrow = w.lane >> 4, lcol = w.lane & 15;

  auto xm = [&](int f, int i) -> v2f {  // mixed sample i of the window of frame f
    return cmul2(load_in_t<DT>(in, f, o + i), (MULTI_LO ? lo_row(lo, in, f) + o : lob)[i]);
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
    if (fast && MULTI_LO) {  // config 4: each frame (row) has its own LO row
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int f = f0 + lrow + 4 * q;
        pf[q] = cmul2(load_in_t<DT>(in, f, o + j - kPad), lo_row(lo, in, f)[o + j - kPad]);
      }
    } else if (fast) {
      const v2f l = lob[j - kPad];
#pragma unroll
      for (int q = 0; q < 16; ++q) pf[q] = cmul2(load_in_t<DT>(in, f0 + lrow + 4 * q, o + j - kPad), l);
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
// sosfilt over reversed yf with state zi*yf[e-1]; keep j = 27 + 2m -> out(m).  Output in
// FGI layout for the next stage, or (last stage, NATURAL) frame-major for the Welch kernel:
// then a store instruction scatters 8 B to 64 frames, but it is 1/2 the rate of the loads
// and L2 merges the lines before they leave the XCD.
template <bool NATURAL>
__global__ __launch_bounds__(256) void iir_backward_kernel(const v2f *__restrict__ yf,
                                                           v2f *__restrict__ out, StageGeom g,
                                                           int frames, Sos32 c) {
  const WaveCtx w = wave_ctx(g);
  if (!w.valid) return;
  const int n = g.n, e = n + 2 * kPad, m_len = (n + 1) >> 1;
  const v2f *__restrict__ y = yf + fgi(w.fg, e, 0) + w.lane;
  const int f = w.fg * 64 + w.lane;
  v2f *__restrict__ o = NATURAL ? out + (int64_t)min(f, frames - 1) * m_len
                                : out + fgi(w.fg, m_len, 0) + w.lane;
  const int64_t ostride = NATURAL ? 1 : 64;
  const bool store_ok = !NATURAL || f < frames;
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
    if (!((j - kPad) & 1) && store_ok) o[(int64_t)((j - kPad) >> 1) * ostride] = v;
  };
  pipelined_run<false>(0, jt - jhi, [&](int d) { return Y(jt - 1 - d); }, s, c, emit);
  pipelined_run<true>(jt - jhi, jt - jlo, [&](int d) { return Y(jt - 1 - d); }, s, c, emit);
}

// ------------------------------------------------------------------ fused interior passes
// The interior of each zero-phase stage is LTI, so its forward (C) and backward (A) passes
// commute; ordering them C0 A0 | A1 C1 | C2 A2 | A3 C3 ... makes neighbouring passes of
// consecutive stages run in the same direction, and this kernel runs such a pair in one
// sweep: pass 1 over the input at rate n_k, every other output of it (the ↓2 sample) feeds
// pass 2 at rate n_{k+1}; only pass 2's output reaches memory.  Without pass 2 (TWO =
// false) the decimated pass-1 output is stored (last stage, NAT = frame-major for Welch,
// written through an LDS transpose).  Frame edges are not reproduced here (different
// order, no odd padding): the host overwrites the edge outputs with an exact computation.
// Blocks partition the output index m; pass 1 starts w1 input samples (pass 2: w2 mid
// samples) outside the block with a zero state, or at the sequence end with zi * x.
template <bool DESC, bool TWO, bool NAT>
__global__ __launch_bounds__(256) void fused_pass_kernel(const v2f *__restrict__ in,
                                                         v2f *__restrict__ out, FusedGeom g,
                                                         int frames, Sos32 c) {
  __shared__ __attribute__((aligned(16))) v2f tile_all[NAT ? 4 : 1][NAT ? 64 * kTileStride : 1];
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= g.ngroups * g.nblk) return;
  const int b = wid % g.nblk, fg = wid / g.nblk;
  const v2f *__restrict__ x = in + fgi(fg, g.in_len, 0) + lane;
  auto IN = [&](int j) -> v2f { return x[(int64_t)j << 6]; };
  const int nk = g.in_len - 2 * g.in_off;
  const int m0 = b * g.block, m1 = min(m0 + g.block, g.n_mid);
  v2f *__restrict__ o = out + fgi(fg, g.n_mid, 0) + lane;  // FGI output (TWO or !NAT)
  v2f *tile = tile_all[NAT ? (threadIdx.x >> 6) : 0];
  const int f0 = fg * 64;

  IirState s1, s2;
  bool p2_pending = false;
  int j_first, count, mlo, mhi;  // input steps j_first + dir*q, q < count; emit m in [mlo, mhi]
  if constexpr (DESC) {
    const int mt = TWO ? min(m1 + g.w2, g.n_mid) : m1;  // pass-2 exclusive top
    const int J1 = g.in_off + 2 * (mt - 1) + 1;
    if (J1 + g.w1 >= g.in_len - 1) {
      j_first = g.in_len - 1;
      state_steady(s1, c, IN(j_first));
    } else {
      j_first = J1 + g.w1;
      state_zero(s1);
    }
    count = j_first - (g.in_off + 2 * m0) + 1;
    mlo = m0;
    mhi = mt - 1;
    if (TWO) {
      if (mt == g.n_mid) p2_pending = true;
      else state_zero(s2);
    }
  } else {
    const int ms = TWO ? max(0, m0 - g.w2) : m0;
    if (2 * ms - g.w1 <= 0) {
      j_first = g.in_off;
      state_steady(s1, c, IN(j_first));
    } else {
      j_first = g.in_off + 2 * ms - g.w1;
      state_zero(s1);
    }
    count = g.in_off + 2 * (m1 - 1) - j_first + 1;
    mlo = ms;
    mhi = m1 - 1;
    if (TWO) {
      if (ms == 0) p2_pending = true;
      else state_zero(s2);
    }
  }
  (void)nk;

  auto flush = [&](int mbase) {  // NAT: tile columns [mbase, mbase+16) -> frame rows
    const int lrow = lane >> 4, lcol = lane & 15;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = 4 * q + lrow, m = mbase + lcol;
      if (f0 + r < frames && m >= m0 && m < m1)
        out[(int64_t)(f0 + r) * g.n_mid + m] = tile[r * kTileStride + lcol];
    }
  };

  auto step = [&](int q, v2f u) {
    const v2f y1 = cascade(u, s1, c);
    const int j = DESC ? j_first - q : j_first + q;
    const int jr = j - g.in_off;
    if ((jr & 1) == 0) {  // wave-uniform
      const int m = jr >> 1;
      if (m >= mlo && m <= mhi) {
        if constexpr (TWO) {
          if (p2_pending) {
            state_steady(s2, c, y1);
            p2_pending = false;
          }
          const v2f y2 = cascade(y1, s2, c);
          if (m >= m0 && m < m1) o[(int64_t)m << 6] = y2;
        } else if constexpr (NAT) {
          tile[lane * kTileStride + (m & 15)] = y1;
          const bool last = DESC ? ((m & 15) == 0 || m == m0) : ((m & 15) == 15 || m == m1 - 1);
          if (last) {
            __builtin_amdgcn_wave_barrier();
            flush(m & ~15);
            __builtin_amdgcn_wave_barrier();
          }
        } else {
          o[(int64_t)m << 6] = y1;
        }
      }
    }
  };

  // register-pipelined input stream (two groups of kU in flight)
  const int full = count / kU;
  int q = 0;
  if (full > 0) {
    v2f A[kU], B[kU];
    auto load = [&](v2f *dst, int q0) {
#pragma unroll
      for (int u = 0; u < kU; ++u) dst[u] = IN(DESC ? j_first - (q0 + u) : j_first + (q0 + u));
    };
    load(A, 0);
    int gi = 0;
    while (true) {
      if (gi + 1 < full) load(B, q + kU);
#pragma unroll
      for (int u = 0; u < kU; ++u) step(q + u, A[u]);
      q += kU;
      if (++gi >= full) break;
      if (gi + 1 < full) load(A, q + kU);
#pragma unroll
      for (int u = 0; u < kU; ++u) step(q + u, B[u]);
      q += kU;
      if (++gi >= full) break;
    }
  }
  for (; q < count; ++q) step(q, IN(DESC ? j_first - q : j_first + q));
}

// The caller's frames as complex64, mixed with the LO when lo != nullptr (zoom 1 paths and
// zoomfft(x, 1), S:2093-2094).
template <int DT>
__global__ __launch_bounds__(256) void ingest_kernel(InDesc in, const v2f *__restrict__ lo,
                                                     v2f *__restrict__ out, int64_t total) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= total) return;
  const int64_t f = k / in.len, i = k - f * in.len;
  const v2f v = load_in_t<DT>(in, f, i);
  out[k] = lo ? cmul2(v, lo_row(lo, in, f)[i]) : v;
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

// Row slot of bin k (-1: cropped) and its one-sided factor.  Two-sided: fftshift + crop,
// row[j] = P[(j - W/2) mod N].  One-sided (WelchGeom::onesided): position
// (k + M/2) mod M of the fftshift of the M = N/2+1 bins, minus the slice start row_a.
__device__ __forceinline__ int welch_slot(const WelchGeom &g, int k, float &mult) {
  mult = 1.f;
  if (!g.onesided) {
    const int j = (k + (g.n_win >> 1)) & (g.n_fft - 1);
    return j < (g.n_win & ~1) ? j : -1;  // odd W: the reference's slice has W - 1 entries
  }
  const int h = g.n_fft >> 1, M = h + 1;
  if (k > h) return -1;
  if (k != 0 && k != h) mult = 2.f;
  const int j = (k + M / 2) % M - g.row_a;
  return (j >= 0 && j < g.row_len) ? j : -1;
}

// ---- in-register DFTs (forward, exp(-2 pi i k n / R)) ----
// Complex products here are cmul2 (two VOP3P instructions; the plain form compiles to four
// and a nop) and the -i rotations fold into the operand selects of one add (add/sub_negi).
// LDS index with one pad slot per 16 (breaks the power-of-two strides of the passes)
__device__ __forceinline__ int lp(int i) { return i + (i >> 4); }

// One Stockham DIT pass of radix R over N points.  Thread t holds 16 values: butterflies
// u = 0 .. 16/R-1 at j = t + u*N/16, inputs v[u + (16/R) r] = a[j + r N/R].
// Twiddle v_r *= W_N^(r k N/(R Ns)), k = j mod Ns; outputs a[(j-k) R + k + r Ns].
template <int R>
__device__ __forceinline__ void stockham_pass(v2f *v, int t, int N, int Ns,
                                              const v2f *__restrict__ tw) {
  constexpr int B = 16 / R;
#pragma unroll
  for (int u = 0; u < B; ++u) {
    const int j = t + u * (N >> 4);
    const int k = j & (Ns - 1);
    v2f w[R];
#pragma unroll
    for (int r = 0; r < R; ++r) w[r] = v[u + B * r];
    if (Ns > 1) {
      const int ts = k * (N / (R * Ns));
      if constexpr (R == 16) {  // W^(r ts) from the four table powers W^ts, W^2ts, W^4ts, W^8ts
        const v2f bp[4] = {tw[ts], tw[2 * ts], tw[4 * ts], tw[8 * ts]};
        apply_powers(w, bp);
      } else {
#pragma unroll
        for (int r = 1; r < R; ++r) w[r] = cmul2(w[r], tw[r * ts]);
      }
    }
    dft<R>(w);
#pragma unroll
    for (int r = 0; r < R; ++r) v[u + B * r] = w[r];
  }
}

template <int R>
__device__ __forceinline__ void stockham_store(const v2f *v, v2f *sh, int t, int N, int Ns) {
  constexpr int B = 16 / R;
#pragma unroll
  for (int u = 0; u < B; ++u) {
    const int j = t + u * (N >> 4);
    const int k = j & (Ns - 1);
    const int base = (j - k) * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) sh[lp(base + r * Ns)] = v[u + B * r];
  }
}

template <int R>
__device__ __forceinline__ int stockham_out_index(int t, int N, int Ns, int i) {
  constexpr int B = 16 / R;
  const int u = i % B, r = i / B;
  const int j = t + u * (N >> 4);
  const int k = j & (Ns - 1);
  return (j - k) * R + k + r * Ns;
}

// One workgroup (N/16 threads) per frame.  Per Welch segment (S:2111 -> scipy welch):
// the 16 samples a thread loads are exactly its first-pass butterfly inputs, so the
// constant detrend and the window are applied in registers before the first radix-R0
// pass; then radix-16 Stockham passes through LDS; the last pass accumulates |X|^2 in
// registers for every bin the thread owns.  The next segment's loads are issued before
// the current FFT (register prefetch).  Finally: density scale, fftshift crop, 20 log10.
template <int R0, bool PF, int MAXT>  // PF: register prefetch of the next segment
__global__ __launch_bounds__(MAXT, 1) void welch_rows_kernel(const v2f *__restrict__ x, int64_t len,
                                                          const float *__restrict__ win,
                                                          const v2f *__restrict__ tw,
                                                          WelchGeom g, float *__restrict__ rows,
                                                          int frames) {
  extern __shared__ v2f sh[];
  const int N = g.n_fft, T = blockDim.x, t = threadIdx.x;
  const int T16 = N >> 4;          // threads doing butterflies
  const bool act = t < T16;
  v2f *red = sh + lp(N);
  int f = blockIdx.x;
  if ((frames & 7) == 0 && frames >= 64)  // spread consecutive frames over the 8 XCDs evenly
    f = (blockIdx.x & 7) * (frames >> 3) + (blockIdx.x >> 3);
  const v2f *__restrict__ xf = x + (int64_t)f * len;

  auto load_seg = [&](v2f *dst, int s) {
    const v2f *__restrict__ seg = xf + (int64_t)s * g.step;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = t + i * T16;
      dst[i] = (act && n < g.nperseg) ? seg[n] : splat(0.f);
    }
  };
  v2f pf[16];
  if constexpr (PF) load_seg(pf, 0);
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  for (int s = 0; s < g.nseg; ++s) {
    v2f v[16];
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = pf[i];
      if (s + 1 < g.nseg) load_seg(pf, s + 1);  // in flight during this segment's FFT
    } else {
      load_seg(v, s);
    }
    v2f sum = splat(0.f);
#pragma unroll
    for (int i = 0; i < 16; ++i) sum += v[i];
    // constant detrend: block mean over the nperseg samples
    sum = wave_sum(sum);
    if ((t & 63) == 0) red[t >> 6] = sum;
    __syncthreads();
    if (t < 64) {
      v2f q = t < ((T + 63) >> 6) ? red[t] : splat(0.f);
      q = wave_sum(q);
      if (t == 0) red[16] = q;
    }
    __syncthreads();
    const v2f mean = red[16] * (1.f / (float)g.nperseg);
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // zero-pad slots (n >= nperseg) get window 0
      const int n = t + i * T16;
      v[i] = (v[i] - mean) * ((act && n < g.nperseg) ? win[n] : 0.f);
    }

    int Ns = 1;
    if (act) {
      stockham_pass<R0>(v, t, N, 1, tw);
      if (N > R0) stockham_store<R0>(v, sh, t, N, 1);
    }
    Ns = R0;
    while (Ns < N) {
      __syncthreads();
      if (act) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = sh[lp(t + r * T16)];
        stockham_pass<16>(v, t, N, Ns, tw);
      }
      if (Ns * 16 < N) {
        __syncthreads();
        if (act) stockham_store<16>(v, sh, t, N, Ns);
      }
      Ns *= 16;
    }
    if (act) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = fmaf(v[i].x, v[i].x, fmaf(v[i].y, v[i].y, acc[i]));
    }
    __syncthreads();  // LDS reads of this segment done before the next one writes
  }
  // bins owned by this thread: output positions of the last pass
  if (!act) return;
  float *__restrict__ row = rows + (int64_t)f * g.n_win;
  const int lastNs = N == R0 ? 1 : N / 16;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int k = N == R0 ? stockham_out_index<R0>(t, N, 1, i) : stockham_out_index<16>(t, N, lastNs, i);
    float mult;
    const int j = welch_slot(g, k, mult);
    if (j >= 0) row[j] = 20.f * log10f(acc[i] * g.scale * mult);
  }
}

// ------------------------------------------------------------------ Welch row, in-place DIF
// N = 16^P R0 (R0 in {1, 2, 4, 8}), 1024 <= N <= 16384: T = N/16 threads per frame, 16
// values each, FPB = 256/T frames per workgroup when T < 256 (a frame is then one wave).
// Gentleman-Sande in-place decimation in frequency: radix-16 stage s (span M = N/16^(s-1),
// stride M/16) gives thread t the block b = t / (M/16) and offset j = t % (M/16); it forms
// the DFT16 of the slots b M + j + (M/16) m and writes X_k W_M^(j k) back to the slots it
// read (k in place of m).  The last stage (radix RL = R0, or 16 when R0 = 1) takes the
// thread's 16 consecutive slots as 16/RL blocks of RL.  Slot Q = sum_s d_s N/16^s (+ d_(P+1))
// then holds bin k = sum_s d_s 16^(s-1) (+ 16^P d_(P+1)): the digits reversed.
// Stage 1 is the thread's own loads x[t + T m] (coalesced), so the window and the
// constant-detrend mean apply in registers first.  A stage writes back only the slots it
// read, so it needs no barrier between its reads and writes: one barrier after each
// stage's stores and one before the next segment's first stores -- 3 per segment at
// N = 4096 against the Stockham kernel's 6, and only wave barriers when a frame is one wave.
// The mean of segment s+1 is reduced from its prefetched registers during segment s
// (posted before segment s's last barrier, by segment parity); the twiddles are rebuilt
// per segment from four powers per stage (w, w^2, w^4, w^8; at most three products deep).
// PRUNE (W <= 2N/RL): the fftshift crop keeps only last-stage outputs 0 and RL-1, so the
// last stage forms just those two per block.
// Register plans (measured on MI355X):
#ifndef ZFFT_DIF_BUF
#define ZFFT_DIF_BUF 1  // segment and window loads through buffer resources (0: global loads)
#endif
#ifndef ZFFT_DIF_PP
#define ZFFT_DIF_PP 1   // two prefetch arrays used in turn, N < 16384 (0: one, copied into v
#endif                  // each segment): cfg2 Welch 0.486 -> 0.46 ms (profiles/r03_ab/r03dpp)
#ifndef ZFFT_DIF_PF4K
#define ZFFT_DIF_PF4K 16
#endif
#ifndef ZFFT_DIF_WAVES4K
#define ZFFT_DIF_WAVES4K 3
#endif
constexpr int kDifPf = ZFFT_DIF_PF4K;  // values per thread prefetched a segment ahead (N = 4096)
constexpr int kDifPfSmall = 8;         // the same for N <= 2048
constexpr int kDifWaves = ZFFT_DIF_WAVES4K;  // waves per SIMD the registers are cut for (PRUNE, N = 4096)
constexpr int kDifWavesSmall = 3;      // the same for N <= 2048 (full form)
constexpr int kDifWavesSmallPrune = 4; // N <= 2048, PRUNE: 4 waves/SIMD (cfg1: 4096 one-wave
                                       // frames fill the GPU's 4096 slots in one round)
constexpr int kDifPfSmallPrune = 4;    // prefetch of that form (fits 128 VGPRs)
#ifndef ZFFT_DIF_PF16K
#define ZFFT_DIF_PF16K 4
#endif
constexpr int kDifPf16k = ZFFT_DIF_PF16K;  // N = 16384 (PRUNE; the full form: none): one
                                            // 1024-thread frame, 4 waves/SIMD (128 VGPRs)
__host__ __device__ constexpr int dif_slot(int i) { return i + (i >> 4); }  // conflict-free strides 1, 16, 17

template <int N>
struct Dif {
  static constexpr int LOG2N = N == 1024 ? 10 : N == 2048 ? 11 : N == 4096 ? 12 : N == 8192 ? 13 : 14;
  static constexpr int T = N / 16;                   // threads per frame
  static constexpr int P = LOG2N / 4;                // radix-16 stages
  static constexpr int R0 = N >> (4 * P);            // 1, 2, 4 or 8
  static constexpr int RL = R0 > 1 ? R0 : 16;        // radix of the last stage
  static constexpr int PM = R0 > 1 ? P : P - 1;      // radix-16 stages before the last stage
  static constexpr int FPB = T >= 256 ? 1 : 256 / T; // frames per workgroup
  static constexpr int NT = T * FPB;                 // threads per workgroup
  static constexpr int NW = (T + 63) / 64;           // waves per frame
  static constexpr int SLOTS = dif_slot(N - 1) + 1;  // LDS image per frame (v2f)
  static constexpr int PF = N <= 2048 ? kDifPfSmall : N == 16384 ? 0 : kDifPf;
  static constexpr int PF_PRUNE = N <= 2048 ? kDifPfSmallPrune : N == 16384 ? kDifPf16k : kDifPf;
  // waves per SIMD the registers are cut for
  static constexpr int WAVES_PRUNE = N <= 2048 ? kDifWavesSmallPrune : N == 4096 ? kDifWaves : 2;
  static constexpr int WAVES_FULL = N <= 2048 ? kDifWavesSmall : 2;
};

// bin of slot q after the last stage (digits reversed)
template <int N>
__device__ __forceinline__ int dif_bin(int q) {
  using D = Dif<N>;
  int k = 0;
#pragma unroll
  for (int s = 1; s <= D::P; ++s) k += ((q >> (D::LOG2N - 4 * s)) & 15) << (4 * (s - 1));
  if constexpr (D::R0 > 1) k += (q & (D::R0 - 1)) << (4 * D::P);
  return k;
}

template <int N, bool PRUNE, bool HALF>
__global__ __launch_bounds__(Dif<N>::NT, PRUNE ? Dif<N>::WAVES_PRUNE : Dif<N>::WAVES_FULL)
void welch_dif_kernel(const v2f *__restrict__ x, int64_t len, const float *__restrict__ win,
                      const v2f *__restrict__ tw, WelchGeom g, float *__restrict__ rows, int frames) {
  using D = Dif<N>;
  constexpr int T = D::T, PF = PRUNE ? D::PF_PRUNE : D::PF;
  extern __shared__ v2f dyn_sh[];
  __shared__ v2f red[D::FPB][2][D::NW];  // wave partial sums of the segment mean, by parity
  const int fl = D::FPB == 1 ? 0 : (int)threadIdx.x / T;  // frame within the workgroup
  int blk = blockIdx.x;
  const int nblk = (int)gridDim.x;
  if ((nblk & 7) == 0 && nblk >= 64)  // spread consecutive frames over the 8 XCDs evenly
    blk = (blockIdx.x & 7) * (nblk >> 3) + (blockIdx.x >> 3);
  // a workgroup's spare frame slots (frames % FPB) recompute the last frame, unwritten
  const int f = min(blk * D::FPB + fl, frames - 1);
  const bool owner = blk * D::FPB + fl < frames;
  v2f *img = dyn_sh + fl * D::SLOTS;
#if !ZFFT_DIF_BUF
  const v2f *__restrict__ xf = x + (int64_t)f * len;
#endif
  auto sync = [&]() {
    if constexpr (D::NW > 1) __syncthreads();
    else __builtin_amdgcn_wave_barrier();
  };
  // twiddle bases of stages 1 and 2 held (stage s: W_N^(j 16^(s-1) m), j = t % (N/16^s),
  // m = 1, 2, 4, 8); later stages re-read theirs per segment
  auto base_of = [&](int s, int tt, int i) {
    const int j = tt & ((N >> (4 * s)) - 1);
    return tw[(j << (4 * (s - 1) + i)) & (N - 1)];
  };
  v2f b1[4], b2[4];
  {
    const int t = threadIdx.x % T;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      b1[i] = base_of(1, t, i);
      b2[i] = D::PM >= 2 ? base_of(2, t, i) : splat(0.f);
    }
  }
#if ZFFT_DIF_BUF
  // segment loads through a buffer resource per segment (a wave holds one frame, T >= 64:
  // the frame base is wave-uniform): the lane offset t*8 is one VGPR for the whole kernel and
  // the per-value offset T*r*8 an immediate or SGPR -- no 64-bit address arithmetic per load
  const v2f *xw = x + (int64_t)__builtin_amdgcn_readfirstlane(f) * len;
  auto seg_rsrc = [&](int s) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)(xw + (int64_t)s * g.step), (short)0, N * 8, 0x00020000);
  };
  auto ldx = [&](__amdgpu_buffer_rsrc_t rs, int tt, int r) -> v2f {
    const auto u = __builtin_amdgcn_raw_buffer_load_b64(rs, (uint32_t)(tt * 8), (uint32_t)(T * r * 8), 0);
    v2f v;
    __builtin_memcpy(&v, &u, 8);
    return v;
  };
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void *)win, (short)0, N * 4, 0x00020000);
  auto ldw = [&](int tt, int r) -> float {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wrs, (uint32_t)(tt * 4), (uint32_t)(T * r * 4), 0));
  };
#define DIF_X(s, tt, r) ldx(seg_rsrc(s), tt, r)
#define DIF_W(tt, r) ldw(tt, r)
#else
#define DIF_X(s, tt, r) xf[(int64_t)(s) * g.step + (tt) + T * (r)]
#define DIF_W(tt, r) win[(tt) + T * (r)]
#endif
  auto load_seg = [&](v2f *dst, int s, int t) {
#pragma unroll
    for (int r = 0; r < PF; ++r) dst[r] = DIF_X(s, t, r);
  };
  // partial sums of segment s: the prefetched values plus the rest read again
  auto post_sum = [&](const v2f *v, int slot, int s, int t) {
    v2f sum = splat(0.f);
#pragma unroll
    for (int r = 0; r < PF; ++r) sum += v[r];
#pragma unroll
    for (int r = PF; r < 16; ++r) sum += DIF_X(s, t, r);
    sum = wave_sum(sum);
    if ((t & 63) == 0) red[fl][slot][t >> 6] = sum;
  };
  constexpr int PFN = PF > 0 ? PF : 1;
  v2f pfa[PFN], pfb[PFN];  // ping-pong prefetch: segment s's values arrive in one, s+1's in
                           // the other (a single array was copied into v every segment)
  // this workgroup's segments [s0, s1): all of them, or part blockIdx.y of g.split
  const int per = (g.nseg + g.split - 1) / g.split;
  const int s0 = (int)blockIdx.y * per, s1 = min(g.nseg, s0 + per);
  load_seg(pfa, s0, threadIdx.x % T);
  post_sum(pfa, s0 & 1, s0, threadIdx.x % T);
  sync();
  constexpr int NACC = PRUNE ? 2 * (16 / D::RL) : 16;
  float acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = 0.f;

  auto seg_step = [&](const int s, v2f (&pf)[PFN], v2f (&pn)[PFN]) {
    // opaque per-segment copies: twiddle powers and LDS addresses are rebuilt in the loop
    // rather than hoisted out of it (dozens of registers held across the loop)
    int t = D::FPB == 1 ? (int)threadIdx.x : (int)threadIdx.x % T;
    asm volatile("" : "+v"(t));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      asm volatile("" : "+v"(b1[i]));
      asm volatile("" : "+v"(b2[i]));
    }
    v2f v[16];
    {  // values [0, PF) were prefetched a segment ahead, the rest load now
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = r < PF ? pf[r] : DIF_X(s, t, r);
    }
    // the window values requested before the next segment's prefetch: the wait for them (the
    // vector-memory counter completes in order) then leaves the prefetch in flight (requested
    // after it, every segment drained its own prefetch right away)
    float wv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) wv[r] = DIF_W(t, r);
    __builtin_amdgcn_sched_barrier(0);
    const bool more = s + 1 < s1;
    // (addresses from the loop-invariant thread id: computed once, outside the loop)
    // In flight during this segment's transform.  Issued on every segment (the last re-reads
    // its own values, cached): with the loads under a branch the compiler's wait tracking
    // merged the paths and drained them at the window's wait, so no segment's prefetch stayed
    // in flight (round 6, the walk's finding).
    const int sn = more ? s + 1 : s;
    if constexpr (HALF) {
      // 50 % overlap (scipy's default noverlap): segment s+1's values [0, 8) are this
      // segment's raw [8, 16) -- only [8, PF) are loaded
      const int tt = (int)threadIdx.x % T;
#pragma unroll
      for (int r = 0; r < PF; ++r) pn[r] = r < 8 ? v[r + 8] : DIF_X(sn, tt, r);
    } else {
      load_seg(pn, sn, (int)threadIdx.x % T);
    }
    {
      v2f sum = splat(0.f);
#pragma unroll
      for (int w = 0; w < D::NW; ++w) sum += red[fl][s & 1][w];
      const v2f mean = sum * (1.f / (float)N);
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = (v[r] - mean) * wv[r];
    }
    // stage 1: DFT16 over the thread's own samples, twiddle, store at t + T k
    dft<16>(v);
    apply_powers(v, b1);
#pragma unroll
    for (int k = 0; k < 16; ++k) img[dif_slot(T * k + t)] = v[k];
    sync();
    // middle radix-16 stages 2 .. PM
#pragma unroll
    for (int st = 2; st <= D::PM; ++st) {
      const int S16 = N >> (4 * st), M = S16 * 16;
      const int base = (t / S16) * M + (t & (S16 - 1));
#pragma unroll
      for (int m = 0; m < 16; ++m) v[m] = img[dif_slot(base + S16 * m)];
      dft<16>(v);
      if (st == 2) {
        apply_powers(v, b2);
      } else {
        v2f bs[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) bs[i] = base_of(st, t, i);
        apply_powers(v, bs);
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) img[dif_slot(base + S16 * k)] = v[k];
      if (st == D::PM && more) post_sum(pn, (s + 1) & 1, s + 1, t);  // next mean, read after 2 syncs
      sync();
    }
    if (D::PM < 2 && more) {  // (no middle stage: post before the last barrier instead)
      post_sum(pn, (s + 1) & 1, s + 1, t);
      sync();
    }
    // last stage: the thread's 16 consecutive slots as 16/RL blocks of RL
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = img[dif_slot(16 * t + m)];
    constexpr int RL = D::RL;
#pragma unroll
    for (int u = 0; u < 16 / RL; ++u) {
      v2f *blkv = v + RL * u;
      if constexpr (PRUNE) {  // outputs 0 and RL-1: X_(RL-1) = sum_m v_m W_RL^(-m)
        v2f a0 = splat(0.f), a1 = splat(0.f);
#pragma unroll
        for (int m = 0; m < RL; ++m) {
          a0 += blkv[m];
          a1 += m == 0 ? blkv[0] : cmul2(blkv[m], w16((16 - (16 / RL) * m) & 15));
        }
        acc[2 * u] = fmaf(a0.x, a0.x, fmaf(a0.y, a0.y, acc[2 * u]));
        acc[2 * u + 1] = fmaf(a1.x, a1.x, fmaf(a1.y, a1.y, acc[2 * u + 1]));
      } else {
        dft<RL>(blkv);
#pragma unroll
        for (int m = 0; m < RL; ++m) acc[RL * u + m] = fmaf(blkv[m].x, blkv[m].x, fmaf(blkv[m].y, blkv[m].y, acc[RL * u + m]));
      }
    }
    sync();  // last-stage reads done before the next segment's stage-1 stores
    };
  if constexpr (ZFFT_DIF_PP && N != 16384) {  // N = 16384 (4-value prefetch): one array
    for (int s = s0; s < s1; s += 2) {         // measured faster (0.69 vs 0.78 ms at cfg3)
      seg_step(s, pfa, pfb);
      if (s + 1 < s1) seg_step(s + 1, pfb, pfa);
    }
  } else {
    (void)pfb;
    for (int s = s0; s < s1; ++s) seg_step(s, pfa, pfa);
  }
  const int t = threadIdx.x % T;
  if (!owner) return;
  float *__restrict__ row = g.split > 1 ? g.parts + ((int64_t)f * g.split + blockIdx.y) * g.n_win
                                        : rows + (int64_t)f * g.n_win;
#pragma unroll
  for (int i = 0; i < NACC; ++i) {
    const int q = PRUNE ? 16 * t + D::RL * (i >> 1) + ((i & 1) ? D::RL - 1 : 0) : 16 * t + i;
    const int k = dif_bin<N>(q);
    float mult;
    const int j = welch_slot(g, k, mult);
    if (j >= 0) row[j] = g.split > 1 ? acc[i] * g.scale * mult : 20.f * log10f(acc[i] * g.scale * mult);
  }
}

// The split form's second launch: row j = 20 log10 of the parts' sum, in part order.
__global__ void __launch_bounds__(256) welch_parts_kernel(const float *__restrict__ parts, WelchGeom g,
                                                          float *__restrict__ rows) {
  const int f = blockIdx.y;
  const int n = g.onesided ? g.row_len : (g.n_win & ~1);
  for (int j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256) {
    const float *pp = parts + (int64_t)f * g.split * g.n_win + j;
    float sum = 0.f;
    for (int q = 0; q < g.split; ++q) sum += pp[(int64_t)q * g.n_win];
    rows[(int64_t)f * g.n_win + j] = 20.f * log10f(sum);
  }
}

#undef DIF_X
#undef DIF_W

constexpr int kDifMinSplit = 1024;
template <int N>
static hipError_t welch_dif_launch(const float2 *x, int64_t len, const float *win, const float2 *tw,
                                   const WelchGeom &g, float *rows, int frames, hipStream_t st) {
  using D = Dif<N>;
  const size_t lds = (size_t)D::FPB * D::SLOTS * sizeof(v2f);
  const bool prune = !g.onesided && g.n_win <= 2 * N / D::RL;
  const bool half = 2 * g.step == N;
  const void *const ks[2][2] = {{(const void *)welch_dif_kernel<N, false, false>, (const void *)welch_dif_kernel<N, false, true>},
                                {(const void *)welch_dif_kernel<N, true, false>, (const void *)welch_dif_kernel<N, true, true>}};
  static bool attr_set[2][2] = {};
  if (lds > 48 * 1024 && !attr_set[prune][half]) {
    hipError_t e = hipFuncSetAttribute(ks[prune][half], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr_set[prune][half] = true;
  }
  const dim3 grid((unsigned)((frames + D::FPB - 1) / D::FPB), (unsigned)g.split), block(D::NT);
#define WELCH_DIF_GO(P, H)                                                                          \
  hipLaunchKernelGGL((welch_dif_kernel<N, P, H>), grid, block, lds, st, (const v2f *)x, len, win, \
                     (const v2f *)tw, g, rows, frames)
  if (prune) {
    if (half) WELCH_DIF_GO(true, true);
    else WELCH_DIF_GO(true, false);
  } else {
    if (half) WELCH_DIF_GO(false, true);
    else WELCH_DIF_GO(false, false);
  }
#undef WELCH_DIF_GO
  if (g.split > 1) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int n = g.onesided ? g.row_len : (g.n_win & ~1);
    hipLaunchKernelGGL(welch_parts_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)frames), dim3(256), 0,
                       st, (const float *)g.parts, g, rows);
  }
  return hipGetLastError();
}

int welch_dif_split(int n_fft, int nseg, int frames) {
  if (n_fft < kDifMinSplit || n_fft > 16384 || nseg < 4) return 1;
  const int fpb = n_fft / 16 >= 256 ? 1 : 256 / (n_fft / 16);
  const int blocks = (frames + fpb - 1) / fpb;
  const int target = 768 * 256 / std::max(256, n_fft / 16);  // workgroups that fill the chip
  if (blocks >= target / 2) return 1;
  const int want = std::min((target + blocks - 1) / blocks, nseg / 2);
  const int per = (nseg + want - 1) / want;
  return (nseg + per - 1) / per;  // every part non-empty
}

// ------------------------------------------------------------------ Welch row, four-step
// N = N1 * N2 (N2 = 256) for segments too long for one workgroup's LDS (N = 32768 is in
// the reference UI's range S:1397, N = 65536 is BASELINE cfg5).  With n = n1 + N1 n2 and
// k = k2 + N2 k1:  X[k] = sum_n1 W_N1^(n1 k1) W_N^(n1 k2) sum_n2 x[n] W_N2^(n2 k2).
//   welch4_means: the constant-detrend mean of every segment (one workgroup per segment)
//   welch4_cols : ZFFT_W4_CPW (32) columns n1 per workgroup (256 B of every row n2 ->
//                 coalesced loads); window applied on load (the mean's partial sums taken
//                 beside it), length-256 FFT, twiddle W_N^(n1 k2), stored as Z[k2][n1]
//                 (rows of N1 contiguous samples)
//   welch4_rows : 16 rows k2 per workgroup, length-N1 FFT per segment (the next segment's
//                 row prefetched), mean·FFT(w) subtracted, |X|^2 summed over the segments in
//                 registers, then scale, fftshift crop and 20 log10.
// tws = [W_256^m, m < 256] ++ [W_N1^m, m < N1].
__global__ __launch_bounds__(256) void welch4_means_kernel(const v2f *__restrict__ x, int64_t len,
                                                           WelchGeom g, v2f *__restrict__ means) {
  __shared__ v2f red[4];
  const int fs = blockIdx.x;  // frame * nseg + segment
  const int f = fs / g.nseg, s = fs % g.nseg;
  const v2f *__restrict__ seg = x + (int64_t)f * len + (int64_t)s * g.step;
  v2f sum = splat(0.f);
  for (int n = threadIdx.x; n < g.nperseg; n += 256) sum += seg[n];
  sum = wave_sum(sum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0)
    means[fs] = ((red[0] + red[1]) + (red[2] + red[3])) * (1.f / (float)g.nperseg);
}

constexpr int kN2 = 256;
constexpr int kColStride = 256 + 16 + 2;  // lp(256) + 2: 16 B aligned, spreads the columns
// with 64 columns across a wave's lanes (one t) an odd column stride puts the 32 lanes of
// each half-wave on distinct bank pairs
template <int CPW> constexpr int col_stride() { return CPW >= 32 ? 256 + 16 + 1 : kColStride; }

// CPW columns per workgroup, 16 threads per column (16 * CPW threads): a wave holds 64
// consecutive columns of one row set, so every load and store instruction moves 512
// contiguous bytes of a row (CPW = 64; N1 < 64 uses CPW = 16)
template <int CPW>
__global__ __launch_bounds__(16 * CPW) void welch4_cols_kernel(const v2f *__restrict__ x, int64_t len,
                                                               const float *__restrict__ win,
                                                               const v2f *__restrict__ tw,
                                                               const v2f *__restrict__ tws, WelchGeom g,
                                                               v2f *__restrict__ means,
                                                               v2f *__restrict__ z) {
  extern __shared__ __attribute__((aligned(16))) v2f shc[];  // CPW columns of kColStride
  constexpr int NT = 16 * CPW, NWV = NT / 64;
  const int N = g.n_fft, N1 = N / kN2, groups = N1 / CPW;
  const int fs = blockIdx.x / groups, cg = blockIdx.x % groups;
  const int f = fs / g.nseg, s = fs % g.nseg;
  const int c = threadIdx.x % CPW, t = threadIdx.x / CPW;
  const int n1 = cg * CPW + c;
  const v2f *__restrict__ seg = x + (int64_t)f * len + (int64_t)s * g.step;
  v2f v[16];
  if (g.fused_mean) {  // the mean comes off after the transform (welch4_rows_kernel)
    v2f sum = splat(0.f);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = n1 + N1 * (t + 16 * i);
      const v2f xv = seg[n];
      sum += xv;
      v[i] = xv * win[n];
    }
    __shared__ v2f red[NWV];
    sum = wave_sum(sum);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
      v2f tot = splat(0.f);
      for (int w = 0; w < NWV; ++w) tot += red[w];
      means[(int64_t)fs * groups + cg] = tot;
    }
  } else {
    const v2f mean = means[fs];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = n1 + N1 * (t + 16 * i);
      v[i] = n < g.nperseg ? (seg[n] - mean) * win[n] : splat(0.f);  // short branch: zero pad
    }
  }
  v2f *col = shc + c * col_stride<CPW>();
  stockham_pass<16>(v, t, kN2, 1, tws);
  stockham_store<16>(v, col, t, kN2, 1);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = col[lp(t + r * 16)];
  stockham_pass<16>(v, t, kN2, 16, tws);
  // output i is k2 = t + 16 i (stockham_out_index<16>(t, 256, 16, i)): its twiddle
  // W_N^(n1 k2) = W_N^(n1 t) b^i with b = W_N^(16 n1), the powers of b formed from b, b^2,
  // b^4, b^8 (at most three products deep) instead of 16 gathers from the length-N table
  {
    const v2f a = tw[n1 * t];
    v2f bp[4];
    bp[0] = tw[16 * n1];
    bp[1] = cmul2(bp[0], bp[0]);
    bp[2] = cmul2(bp[1], bp[1]);
    bp[3] = cmul2(bp[2], bp[2]);
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = cmul2(v[i], a);
    apply_powers(v, bp);
  }
  v2f *__restrict__ zs = z + (int64_t)fs * N;
#pragma unroll
  for (int i = 0; i < 16; ++i) zs[(int64_t)(t + 16 * i) * N1 + n1] = v[i];
}

// columns per workgroup of the column pass (the row pass reads that many partial sums):
// cfg5 column pass 1.22 / 1.05 / 1.52 ms at 16 / 32 / 64 (profiles/r03_ab/r03tu)
#ifndef ZFFT_W4_CPW
#define ZFFT_W4_CPW 32
#endif
__host__ __device__ inline int welch4_cpw(int N1) { return N1 >= ZFFT_W4_CPW ? ZFFT_W4_CPW : 16; }

template <int R0>
__device__ __forceinline__ int welch4_k1(int t, int N1, int i) {
  return N1 == R0 ? stockham_out_index<R0>(t, N1, 1, i) : stockham_out_index<16>(t, N1, R0, i);
}

// Row pass at 2 waves/SIMD (216 VGPRs): capping registers for 4 or 5 waves/SIMD measured
// 1.39 / 2.04 ms against 0.81 ms at cfg5 (profiles/r03_ab/r03tu); the next segment's
// prefetch took it from 1.03 ms
#ifndef ZFFT_W4_RWPE
#define ZFFT_W4_RWPE 2
#endif
// PRUNE (two-sided rows with n_win <= N/8, every zoom >= 8; N1 > R0): the crop keeps bins
// |k| < N/16, i.e. only the last radix-16 pass's outputs 0 and 15 (k1 = t + Ns r, r = 0, 15:
// the top digit is resolved last), so that pass forms just those two sums and the thread
// keeps 2 accumulators and 2 FFT(window) values instead of 16 (the FFT(window) gathers were
// half the pass's time at cfg5)
template <int R0, bool PRUNE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ZFFT_W4_RWPE))) void welch4_rows_kernel(const v2f *__restrict__ z,
                                                          const v2f *__restrict__ tws,
                                                          const v2f *__restrict__ winf,
                                                          const v2f *__restrict__ means,
                                                          WelchGeom g, float *__restrict__ rows) {
  extern __shared__ v2f shr[];
  constexpr int NO = PRUNE ? 2 : 16;  // outputs kept per thread: i = 0, 15 when pruned
  auto out_i = [](int o) { return PRUNE ? 15 * o : o; };
  const int N = g.n_fft, N1 = N / kN2, T16 = N1 / 16;
  const int f = blockIdx.x / (kN2 / 16), kg = blockIdx.x % (kN2 / 16);
  const int c = threadIdx.x / T16, t = threadIdx.x % T16;
  const int k2 = kg * 16 + c;
  const v2f *__restrict__ tw1 = tws + kN2;
  v2f *row_sh = shr + c * (lp(N1) + 2);
  float acc[NO];
#pragma unroll
  for (int i = 0; i < NO; ++i) acc[i] = 0.f;
  v2f wf[NO];  // FFT(window) at this thread's bins (fused mean)
  if (g.fused_mean) {
#pragma unroll
    for (int i = 0; i < NO; ++i) wf[i] = winf[k2 + kN2 * welch4_k1<R0>(t, N1, out_i(i))];
  }
  const int groups = N1 / welch4_cpw(N1);
  const v2f *__restrict__ zr = z + (int64_t)f * g.nseg * N + (int64_t)k2 * N1 + t;
  v2f vn[16];  // the next segment's row, loaded while this one is transformed
#pragma unroll
  for (int i = 0; i < 16; ++i) vn[i] = zr[i * T16];
  for (int s = 0; s < g.nseg; ++s) {
    v2f v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = vn[i];
    if (s + 1 < g.nseg) {
#pragma unroll
      for (int i = 0; i < 16; ++i) vn[i] = zr[(int64_t)(s + 1) * N + i * T16];
    }
    stockham_pass<R0>(v, t, N1, 1, tw1);
    if (N1 > R0) {
      stockham_store<R0>(v, row_sh, t, N1, 1);
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = row_sh[lp(t + r * T16)];
      if constexpr (PRUNE) {  // the last pass's twiddles (stockham_pass<16>, Ns = R0), then
                              // X_0 = sum v_m and X_15 = sum v_m W16^(-m)
        const int ts = (t & (R0 - 1)) * (N1 / (16 * R0));
        const v2f bp[4] = {tw1[ts], tw1[2 * ts], tw1[4 * ts], tw1[8 * ts]};
        apply_powers(v, bp);
        v2f a0 = v[0], a1 = v[0];
#pragma unroll
        for (int m = 1; m < 16; ++m) {
          a0 += v[m];
          a1 += cmul2(v[m], w16(16 - m));
        }
        v[0] = a0;
        v[1] = a1;
      } else {
        stockham_pass<16>(v, t, N1, R0, tw1);
      }
      __syncthreads();  // reads done before the next segment's store
    }
    if (g.fused_mean) {  // X = FFT(x w) - mean FFT(w): the column groups' partial sums
      const v2f *__restrict__ ps = means + ((int64_t)f * g.nseg + s) * groups;
      v2f sum = splat(0.f);
      for (int q = 0; q < groups; ++q) sum += ps[q];
      const v2f mean = sum * (1.f / (float)g.nperseg);
#pragma unroll
      for (int i = 0; i < NO; ++i) v[i] -= cmul(mean, wf[i]);
    }
#pragma unroll
    for (int i = 0; i < NO; ++i) acc[i] = fmaf(v[i].x, v[i].x, fmaf(v[i].y, v[i].y, acc[i]));
  }
  float *__restrict__ row = rows + (int64_t)f * g.n_win;
#pragma unroll
  for (int i = 0; i < NO; ++i) {
    const int k1 = welch4_k1<R0>(t, N1, out_i(i));
    const int k = k2 + kN2 * k1;
    float mult;
    const int j = welch_slot(g, k, mult);
    if (j >= 0) row[j] = 20.f * log10f(acc[i] * g.scale * mult);
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

// Applies pushes [first, count), first = max(0, count - H), as the reference's sequence of
// image_update calls would (earlier pushes are fully overwritten: every slot and stamp is
// rewritten within H pushes), in parallel for scroll = +-1 (the reference's two scroll
// directions, S:2074-2077; the plan admits no other), in two launches.  Push r (first <= r < count) writes slot
// s_r = (H - 1 + off0 + r scroll) mod H -- distinct slots, since count - first <= H -- so
// every row lands at once (waterfall_rows_kernel).  Its tick stamps then hit slots
// q = (y + off0 + (r + 1) scroll) mod H; a stamp survives iff no later push rewrote q, i.e.
// q has no writer in the batch or its writer r' <= r (waterfall_stamps_kernel).
__global__ __launch_bounds__(256) void waterfall_rows_kernel(float *ring, int H, int W,
                                                             const float *__restrict__ rows,
                                                             int64_t row_stride, int first,
                                                             int64_t off0, int scroll) {
  const int xcol = blockIdx.x * 256 + threadIdx.x;
  if (xcol >= W) return;
  const int r = first + (int)blockIdx.y;
  const int slot = pmod(H - 1 + off0 + (int64_t)r * scroll, H);
  float v = rows[(int64_t)r * row_stride + xcol];
  if (xcol == 0 || xcol == (W >> 1) || xcol == W - 1) v = 0.f;  // grid, S:1646-1648
  ring[(int64_t)slot * W + xcol] = v;
}

__global__ __launch_bounds__(256) void waterfall_stamps_kernel(float *ring, int H, int W, int first,
                                                               int count, int64_t off0, int scroll) {
  const int tick = W / 10;
  const int nt = (W - 1 + tick - 1) / tick;  // len(range(0, W-1, W//10))
  const int nrows = scroll > 0 ? 10 : 8;     // img[5:15] or img[-10:-2]
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)(count - first) * nrows * nt) return;
  const int i = (int)(idx % nt), yy = (int)((idx / nt) % nrows);
  const int r = first + (int)(idx / ((int64_t)nt * nrows));
  if (i == 5 || i == 10) return;  // S:1655-1662
  const int yrow = scroll > 0 ? 5 + yy : H - 10 + yy;
  const int q = pmod(yrow + off0 + (int64_t)(r + 1) * scroll, H);
  // the push writing slot q: (H - 1 + off0 + w scroll) = q (mod H), w in [first, first + H)
  const int w = first + pmod((int64_t)scroll * (q + 1 - off0) - first, H);
  if (w < count && w > r) return;  // rewritten by a later push
  ring[(int64_t)q * W + i * tick] = 0.f;
}

// Waterfall rendering: pyqtgraph makeARGB of the ring image, pixel order as
// waterfall_read.  idx = clip((v - lo) * scale, 0, 255) truncated (rescaleData then
// astype(uint8)), computed in fp64 as numpy does on the float64 image; NaN -> alpha 0.
__global__ void waterfall_render_kernel(const float *__restrict__ ring, int H, int W, int off,
                                        const uchar4 *__restrict__ lut, double lo, double scale,
                                        uchar4 *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)H * W) return;
  const int r = (int)(i / W), xcol = (int)(i % W);
  const float v = ring[(int64_t)((r + off) % H) * W + xcol];
  double t = ((double)v - lo) * scale;
  t = t < 0.0 ? 0.0 : (t > 255.0 ? 255.0 : t);
  uchar4 c = lut[v == v ? (int)t : 0];
  if (v != v) c.w = 0;
  out[i] = c;
}

// Autolevel order statistics of the ring pixels below 0: keys are the float bits made
// order-preserving (negative floats: all bits flipped), counted in 65536 bins of the top 16
// bits, then -- inside the bins that hold the wanted ranks -- of the low 16 bits.
__device__ __forceinline__ uint32_t neg_key(float v) { return ~__float_as_uint(v); }
__global__ void autolevel_hist_hi_kernel(const float *__restrict__ ring, int64_t n,
                                         unsigned *__restrict__ hist) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = ring[i];
    if (v < 0.f) atomicAdd(&hist[neg_key(v) >> 16], 1u);
  }
}
__global__ void autolevel_hist_lo_kernel(const float *__restrict__ ring, int64_t n,
                                         const unsigned *__restrict__ bins, int nbins,
                                         unsigned *__restrict__ hist) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = ring[i];
    if (!(v < 0.f)) continue;
    const uint32_t k = neg_key(v);
    for (int b = 0; b < nbins; ++b)
      if ((k >> 16) == bins[b]) atomicAdd(&hist[b * 65536 + (k & 0xFFFF)], 1u);
  }
}

__global__ void waterfall_read_kernel(const float *__restrict__ ring, int H, int W, int off,
                                      float *__restrict__ img) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)H * W) return;
  const int r = (int)(i / W), xcol = (int)(i % W);
  img[i] = ring[(int64_t)((r + off) % H) * W + xcol];
}

// Per-line display in one launch: push one row (or none) and emit the
// image -- RGBA8 (MODE 0, as waterfall_render_kernel) or float64 (MODE 1, img_array's dtype).
// Image row r is ring slot s = (r + off1) mod H after the push (off1 = off0 + scroll).  The
// row lands in slot (H - 1 + off0) mod H with its grid zeros (waterfall_rows_kernel, r = 0),
// and this push's tick stamps hit slots (yrow + off1) mod H, i.e. image rows yrow
// (waterfall_stamps_kernel with count 1: no later push rewrites them).  Pixels and slots are
// a bijection, so the thread of a changed slot writes it back to the ring unraced.
template <int MODE>
__global__ void waterfall_push_emit_kernel(float *__restrict__ ring, int H, int W, int off0, int scroll,
                                           const float *__restrict__ row, const uchar4 *__restrict__ lut,
                                           double lo, double scale, void *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)H * W) return;
  const int r = (int)(i / W), xcol = (int)(i % W);
  const int off1 = row ? pmod((int64_t)off0 + scroll, H) : off0;
  const int64_t at = (int64_t)((r + off1) % H) * W + xcol;
  float v;
  if (row) {
    bool dirty = false;
    if ((r + off1) % H == pmod((int64_t)H - 1 + off0, H)) {
      v = row[xcol];
      if (xcol == 0 || xcol == (W >> 1) || xcol == W - 1) v = 0.f;  // grid, S:1646-1648
      dirty = true;
    } else {
      v = ring[at];
    }
    const int tick = W / 10;
    if (tick > 0 && xcol % tick == 0) {  // S:1650-1662
      const int it = xcol / tick, nt = (W - 1 + tick - 1) / tick;
      const int y0 = scroll > 0 ? 5 : H - 10, nrows = scroll > 0 ? 10 : 8;
      if (it < nt && it != 5 && it != 10 && pmod((int64_t)r - y0, H) < nrows) {
        v = 0.f;
        dirty = true;
      }
    }
    if (dirty) ring[at] = v;
  } else {
    v = ring[at];
  }
  if constexpr (MODE == 0) {
    double t = ((double)v - lo) * scale;
    t = t < 0.0 ? 0.0 : (t > 255.0 ? 255.0 : t);
    uchar4 c = lut[v == v ? (int)t : 0];
    if (v != v) c.w = 0;
    ((uchar4 *)out)[i] = c;
  } else {
    ((double *)out)[i] = (double)v;
  }
}

// ------------------------------------------------------------------ launchers
static inline unsigned nblocks(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

static inline int ilog2_dev(int v) {
  int r = 0;
  while ((1 << (r + 1)) <= v) ++r;
  return r;
}

static inline unsigned wave_blocks(const StageGeom &g) {
  return (unsigned)(((int64_t)g.ngroups * g.nblk + 3) / 4);
}

hipError_t launch_iir_forward_mix(const InDesc &in, int frames, const float2 *lo, float2 *yf,
                                  const StageGeom &g, hipStream_t st) {
  const dim3 grid(wave_blocks(g)), block(256);
  const v2f *l = (const v2f *)lo;
  v2f *y = (v2f *)yf;
  if (in.lo_n > 1) {
    if (in.dtype == kInC64)
      hipLaunchKernelGGL((iir_forward_mix_kernel<kInC64, true>), grid, block, 0, st, in, frames, l, y, g, sos32());
    else if (in.dtype == kInC32H)
      hipLaunchKernelGGL((iir_forward_mix_kernel<kInC32H, true>), grid, block, 0, st, in, frames, l, y, g, sos32());
    else if (in.dtype == kInF32R)
      hipLaunchKernelGGL((iir_forward_mix_kernel<kInF32R, true>), grid, block, 0, st, in, frames, l, y, g, sos32());
    else
      hipLaunchKernelGGL((iir_forward_mix_kernel<kInCU8, true>), grid, block, 0, st, in, frames, l, y, g, sos32());
  } else if (in.dtype == kInC64)
    hipLaunchKernelGGL((iir_forward_mix_kernel<kInC64, false>), grid, block, 0, st, in, frames, l, y, g, sos32());
  else if (in.dtype == kInC32H)
    hipLaunchKernelGGL((iir_forward_mix_kernel<kInC32H, false>), grid, block, 0, st, in, frames, l, y, g, sos32());
  else if (in.dtype == kInF32R)
    hipLaunchKernelGGL((iir_forward_mix_kernel<kInF32R, false>), grid, block, 0, st, in, frames, l, y, g, sos32());
  else
    hipLaunchKernelGGL((iir_forward_mix_kernel<kInCU8, false>), grid, block, 0, st, in, frames, l, y, g, sos32());
  return hipGetLastError();
}

hipError_t launch_iir_forward_fgi(const float2 *in, float2 *yf, const StageGeom &g,
                                  hipStream_t st) {
  hipLaunchKernelGGL(iir_forward_fgi_kernel, dim3(wave_blocks(g)), dim3(256), 0, st,
                     (const v2f *)in, (v2f *)yf, g, sos32());
  return hipGetLastError();
}

hipError_t launch_iir_backward(const float2 *yf, float2 *out, bool natural, int frames,
                               const StageGeom &g, hipStream_t st) {
  if (natural)
    hipLaunchKernelGGL(iir_backward_kernel<true>, dim3(wave_blocks(g)), dim3(256), 0, st,
                       (const v2f *)yf, (v2f *)out, g, frames, sos32());
  else
    hipLaunchKernelGGL(iir_backward_kernel<false>, dim3(wave_blocks(g)), dim3(256), 0, st,
                       (const v2f *)yf, (v2f *)out, g, frames, sos32());
  return hipGetLastError();
}

hipError_t launch_fused_pass(const float2 *in, float2 *out, bool desc, bool two, bool nat,
                             const FusedGeom &g, int frames, hipStream_t st) {
  const unsigned blocks = (unsigned)(((int64_t)g.ngroups * g.nblk + 3) / 4);
  const v2f *i = (const v2f *)in;
  v2f *o = (v2f *)out;
  const Sos32 c = sos32();
  if (desc && two)
    hipLaunchKernelGGL((fused_pass_kernel<true, true, false>), dim3(blocks), dim3(256), 0, st, i, o, g, frames, c);
  else if (!desc && two)
    hipLaunchKernelGGL((fused_pass_kernel<false, true, false>), dim3(blocks), dim3(256), 0, st, i, o, g, frames, c);
  else if (desc && nat)
    hipLaunchKernelGGL((fused_pass_kernel<true, false, true>), dim3(blocks), dim3(256), 0, st, i, o, g, frames, c);
  else if (!desc && nat)
    hipLaunchKernelGGL((fused_pass_kernel<false, false, true>), dim3(blocks), dim3(256), 0, st, i, o, g, frames, c);
  else if (desc)
    hipLaunchKernelGGL((fused_pass_kernel<true, false, false>), dim3(blocks), dim3(256), 0, st, i, o, g, frames, c);
  else
    hipLaunchKernelGGL((fused_pass_kernel<false, false, false>), dim3(blocks), dim3(256), 0, st, i, o, g, frames, c);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void fill_c64_kernel(v2f *__restrict__ out, int64_t n, v2f v) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] = v;
}
hipError_t launch_fill_c64(float2 *out, int64_t n, float re, float im, hipStream_t st) {
  hipLaunchKernelGGL(fill_c64_kernel, dim3(nblocks(n, 256)), dim3(256), 0, st, (v2f *)out, n, v2f{re, im});
  return hipGetLastError();
}

hipError_t launch_ingest(const InDesc &in, const float2 *lo, float2 *out, int frames,
                         hipStream_t st) {
  const int64_t total = (int64_t)frames * in.len;
  const dim3 grid(nblocks(total, 256)), block(256);
  const v2f *l = (const v2f *)lo;
  v2f *o = (v2f *)out;
  if (in.dtype == kInC64)
    hipLaunchKernelGGL(ingest_kernel<kInC64>, grid, block, 0, st, in, l, o, total);
  else if (in.dtype == kInC32H)
    hipLaunchKernelGGL(ingest_kernel<kInC32H>, grid, block, 0, st, in, l, o, total);
  else if (in.dtype == kInF32R)
    hipLaunchKernelGGL(ingest_kernel<kInF32R>, grid, block, 0, st, in, l, o, total);
  else
    hipLaunchKernelGGL(ingest_kernel<kInCU8>, grid, block, 0, st, in, l, o, total);
  return hipGetLastError();
}

template <int R0, bool PF, int MAXT>
static hipError_t welch_launch_t(const float2 *x, int64_t len, const float *win,
                                 const float2 *tw, const WelchGeom &g, float *rows, int frames,
                                 hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)welch_rows_kernel<R0, PF, MAXT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (kMaxLdsFft + kMaxLdsFft / 16 + 32) * (int)sizeof(v2f));
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int T = g.n_fft / 16 > 64 ? g.n_fft / 16 : 64;
  const size_t lds = (size_t)(g.n_fft + g.n_fft / 16 + 32) * sizeof(v2f);
  hipLaunchKernelGGL((welch_rows_kernel<R0, PF, MAXT>), dim3(frames), dim3(T), lds, st, (const v2f *)x,
                     len, win, (const v2f *)tw, g, rows, frames);
  return hipGetLastError();
}

// the in-place DIF kernel covers 1024 <= N <= 16384 (N = 16384: one 1024-thread frame per
// workgroup, 139 KB of LDS, a 4-value prefetch to stay within 128 VGPRs)
#ifndef ZFFT_DIF_MAX
#define ZFFT_DIF_MAX 16384
#endif
constexpr int kDifMin = 1024, kDifMax = ZFFT_DIF_MAX;
template <int R0>
static hipError_t welch_launch(const float2 *x, int64_t len, const float *win, const float2 *tw,
                               const WelchGeom &g, float *rows, int frames, hipStream_t st) {
  if (g.nperseg == g.n_fft && g.n_fft >= kDifMin && g.n_fft <= kDifMax) {
    switch (g.n_fft) {
      case 1024: return welch_dif_launch<1024>(x, len, win, tw, g, rows, frames, st);
      case 2048: return welch_dif_launch<2048>(x, len, win, tw, g, rows, frames, st);
      case 4096: return welch_dif_launch<4096>(x, len, win, tw, g, rows, frames, st);
      case 8192: return welch_dif_launch<8192>(x, len, win, tw, g, rows, frames, st);
      case 16384: return welch_dif_launch<16384>(x, len, win, tw, g, rows, frames, st);
      default: break;
    }
  }
  // threads = N/16 (>= 64): N <= 4096 -> <= 256 threads, room for the prefetch registers
  if (g.n_fft <= 4096) return welch_launch_t<R0, true, 256>(x, len, win, tw, g, rows, frames, st);
  if (g.n_fft <= 8192) return welch_launch_t<R0, false, 512>(x, len, win, tw, g, rows, frames, st);
  return welch_launch_t<R0, false, 1024>(x, len, win, tw, g, rows, frames, st);
}

// x: natural layout, frame f at x + f*len (the caller's frames at zoom 1, otherwise the
// last decimation stage's output).  N = R0 * 16^p.
hipError_t launch_welch_rows(const float2 *x, int64_t len, const float *win, const float2 *tw,
                             const WelchGeom &g, float *rows, int frames, hipStream_t st) {
  switch (g.log2n % 4) {
    case 0: return welch_launch<16>(x, len, win, tw, g, rows, frames, st);
    case 1: return welch_launch<2>(x, len, win, tw, g, rows, frames, st);
    case 2: return welch_launch<4>(x, len, win, tw, g, rows, frames, st);
    default: return welch_launch<8>(x, len, win, tw, g, rows, frames, st);
  }
}

template <int CPW>
static hipError_t welch4_cols_launch(const void *x, int64_t len, const float *win, const void *tw,
                                     const void *tws, const WelchGeom &g, void *means, void *z,
                                     int64_t segs, int N1, hipStream_t st) {
  const size_t lds = (size_t)CPW * col_stride<CPW>() * sizeof(v2f);
  static bool attr = false;
  if (!attr && lds > 65536) {
    const hipError_t e = hipFuncSetAttribute((const void *)welch4_cols_kernel<CPW>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  attr = true;
  hipLaunchKernelGGL(welch4_cols_kernel<CPW>, dim3(segs * (N1 / CPW)), dim3(16 * CPW), lds, st,
                     (const v2f *)x, len, win, (const v2f *)tw, (const v2f *)tws, g, (v2f *)means,
                     (v2f *)z);
  return hipGetLastError();
}

hipError_t launch_welch4(const float2 *x, int64_t len, const float *win, const float2 *tw,
                         const float2 *tws, const float2 *winf, const WelchGeom &g, float2 *means,
                         float2 *z, float *rows, int frames, hipStream_t st) {
  const int N1 = g.n_fft / kN2;
  if (N1 < 16 || N1 > 256 || g.n_fft != N1 * kN2) return hipErrorInvalidValue;
  if (g.fused_mean && !winf) return hipErrorInvalidValue;
  const unsigned segs = (unsigned)frames * (unsigned)g.nseg;
  hipError_t e = hipSuccess;
  if (!g.fused_mean) {
    hipLaunchKernelGGL(welch4_means_kernel, dim3(segs), dim3(256), 0, st, (const v2f *)x, len, g,
                       (v2f *)means);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const int cpw = welch4_cpw(N1);
  if (cpw == 64)
    e = welch4_cols_launch<64>(x, len, win, tw, tws, g, means, z, segs, N1, st);
  else if (cpw == 32)
    e = welch4_cols_launch<32>(x, len, win, tw, tws, g, means, z, segs, N1, st);
  else
    e = welch4_cols_launch<16>(x, len, win, tw, tws, g, means, z, segs, N1, st);
  if (e != hipSuccess) return e;
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t lds = (size_t)16 * (N1 + N1 / 16 + 2) * sizeof(v2f);
  const dim3 grid((unsigned)frames * (kN2 / 16)), block(N1);
  const v2f *zc = (const v2f *)z, *tc = (const v2f *)tws, *wc = (const v2f *)winf, *mc = (const v2f *)means;
#ifndef ZFFT_W4_PRUNE
#define ZFFT_W4_PRUNE 1
#endif
  const bool prune = ZFFT_W4_PRUNE && !g.onesided && N1 > 16 && (int64_t)g.n_win * 8 <= g.n_fft;
#define W4_ROWS(R)                                                                                    \
  do {                                                                                                \
    if (prune)                                                                                        \
      hipLaunchKernelGGL((welch4_rows_kernel<R, true>), grid, block, lds, st, zc, tc, wc, mc, g, rows);  \
    else                                                                                              \
      hipLaunchKernelGGL((welch4_rows_kernel<R, false>), grid, block, lds, st, zc, tc, wc, mc, g, rows); \
  } while (0)
  switch (ilog2_dev(N1) % 4) {
    case 0: W4_ROWS(16); break;
    case 1: W4_ROWS(2); break;
    case 2: W4_ROWS(4); break;
    default: W4_ROWS(8); break;
  }
#undef W4_ROWS
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
  if (count <= 0) return hipSuccess;
  if (scroll == 1 || scroll == -1) {  // ring rows, then the stamps that survive
    const int first = count > H ? count - H : 0;
    hipLaunchKernelGGL(waterfall_rows_kernel, dim3((unsigned)((W + 255) / 256), (unsigned)(count - first)),
                       dim3(256), 0, st, ring, H, W, rows, row_stride, first, off0, scroll);
    const int tick = W / 10, nt = (W - 1 + tick - 1) / tick, nrows = scroll > 0 ? 10 : 8;
    hipLaunchKernelGGL(waterfall_stamps_kernel, dim3(nblocks((int64_t)(count - first) * nrows * nt, 256)),
                       dim3(256), 0, st, ring, H, W, first, count, off0, scroll);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;  // (zfft_plan validates scroll)
}

hipError_t launch_waterfall_read(const float *ring, int H, int W, int64_t off, float *img,
                                 hipStream_t st) {
  hipLaunchKernelGGL(waterfall_read_kernel, dim3(nblocks((int64_t)H * W, 256)), dim3(256), 0, st,
                     ring, H, W, (int)(off % H), img);
  return hipGetLastError();
}

hipError_t launch_waterfall_render(const float *ring, int H, int W, int64_t off, const void *lut,
                                   double lo, double scale, void *out, hipStream_t st) {
  const int64_t total = (int64_t)H * W;
  hipLaunchKernelGGL(waterfall_render_kernel, dim3(nblocks(total, 256)), dim3(256), 0, st, ring, H,
                     W, (int)off, (const uchar4 *)lut, lo, scale, (uchar4 *)out);
  return hipGetLastError();
}

hipError_t launch_waterfall_push_emit(float *ring, int H, int W, int64_t off0, int scroll,
                                      const float *row, const void *lut, double lo, double scale,
                                      void *out, bool f64, hipStream_t st) {
  const dim3 g(nblocks((int64_t)H * W, 256));
  if (f64)
    hipLaunchKernelGGL(waterfall_push_emit_kernel<1>, g, dim3(256), 0, st, ring, H, W, (int)(off0 % H), scroll,
                       row, (const uchar4 *)lut, lo, scale, out);
  else
    hipLaunchKernelGGL(waterfall_push_emit_kernel<0>, g, dim3(256), 0, st, ring, H, W, (int)(off0 % H), scroll,
                       row, (const uchar4 *)lut, lo, scale, out);
  return hipGetLastError();
}

hipError_t launch_autolevel_hist_hi(const float *ring, int64_t n, unsigned *hist, hipStream_t st) {
  const unsigned blocks = (unsigned)std::min<int64_t>(nblocks(n, 256), 4096);
  hipLaunchKernelGGL(autolevel_hist_hi_kernel, dim3(blocks), dim3(256), 0, st, ring, n, hist);
  return hipGetLastError();
}

hipError_t launch_autolevel_hist_lo(const float *ring, int64_t n, const unsigned *bins, int nbins,
                                    unsigned *hist, hipStream_t st) {
  const unsigned blocks = (unsigned)std::min<int64_t>(nblocks(n, 256), 4096);
  hipLaunchKernelGGL(autolevel_hist_lo_kernel, dim3(blocks), dim3(256), 0, st, ring, n, bins, nbins,
                     hist);
  return hipGetLastError();
}

}  // namespace zfft
