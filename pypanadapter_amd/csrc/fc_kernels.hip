// fc_kernels.hip -- "FC", the fast-convolution form of the zoom-8 decimator on gfx950 (host
// tables: fc_build_table in pc_tables.cpp; design model: tools/fc_model.py).
//
// The interior of three scipy.signal.decimate(x, 2) (pypanadapter_spectrum.py:2096-2098) is the
// zero-phase LTI filter G = prod_k |H(z^(2^k))|^2 on the zero-extended frame followed by [::8]
// (DESIGN §3.5).  Its input-rate impulse response g falls below 1.0e-6 of sum |g| beyond
// |k| = kFcK = 768 (1.4e-8 beyond 1024; tools/fc_model.py); truncated there it is applied by
// overlap-save FFT convolution, one 8192-sample window per block:
//   block b: window w[n] = x[6656 b - 768 + n], n < 8192 (zero outside the frame)
//   residues a_r[m] = w[8m + r]: eight 1024-point DFTs A_r (radix 16, 16, 4; decimation in
//            frequency, in lock step: the residues share every twiddle)
//   Yf[k] = sum_r A_r[k] C[k][r],  C[k][r] = W_8192^(rk) sum_q G[k + 1024 q] W_8^(rq) / 8192
//            -- the [::8] is an alias sum in frequency, here fused with the filter
//   y[j] = IDFT_1024(Yf)[j] (five radix-4 stages), outputs m = 832 b + j - 96, j in [96, 928)
// The LO mix moves into the filter: (x lo) * g at 8m equals lo[8m] (x * g') with
// g'[k] = g[k] e^(2 pi i f_lo k / fs) (lo[n] = sqrt 2 e^(-2 pi i f_lo n / fs) is an exact
// exponential), so C holds the modulated filter's spectrum (one table per LO row) and each output
// takes lo[8m] once, as the composite lo[6656 b] lo[8 (j - 96)] / sqrt 2.
// Frame ends: the walk's maps (pc_edge_v beside this kernel on the side stream, pc_edge_u after
// the join: exact minus the zero-extended model), which g's truncation changes by < 2e-8.
//
// Work per input sample: ~30 VALU lane-instructions (the walk: 74); LDS: two
// exchanges of the 8192-point window plus five small ones of the 1024-point inverse per block.
#include <algorithm>

#include "zfft_device.h"
#include "zfft_fft.h"
#include "zfft_pairs.h"

// Diagnostic builds only (ZFFT_DIAG=1, never set by build.py), timing knockouts with wrong
// results by design: FC_KO 1 the input loads (window values from registers), 2 the filter-table
// loads, 4 the output stores (profiles/r06fc/r06fc4: 2.84 ms -> 1.85 / 2.61 / 2.54, all three
// 1.56 at K = 1024).  Measured and removed: the filter table requested before the prefetch
// (2.98 ms, spills) and the prefetch requested after the table (2.80, r06fc5).
#ifndef ZFFT_DIAG
#define ZFFT_DIAG 0
#endif
#if !ZFFT_DIAG && defined(FC_KO)
#error "FC_KO is a diagnostic knob: build with -DZFFT_DIAG"
#endif
#ifndef FC_KO
#define FC_KO 0
#endif
#ifndef FC_WSYNC
#define FC_WSYNC 1  // A/B knob: 0 = a workgroup barrier between the wave-local inverse stages
#endif
#ifndef FC_HOLD
#define FC_HOLD (-1)  // diagnostic override of fc_hold for every non-cu8 instantiation
#endif


namespace zfft {
namespace fc {

typedef v2f __attribute__((address_space(3))) *LP;
typedef v4f __attribute__((address_space(3))) *LP4;

// Block geometry per zoom (zfft_internal.h): Z residues of an M = 8192 / Z point DFT; a block
// advances 512 S samples and makes P = 512 S / Z outputs; K = (8192 - 512 S) / 2.
template <int Z> struct Geo;
template <> struct Geo<8> { static constexpr int S = kFcStep, K = kFcK, P = kFcP; };
template <> struct Geo<4> { static constexpr int S = kFc4Step, K = kFc4K, P = kFc4P; };
constexpr int kN = kFcN;
// LDS: the window as [pos][residue] with 2 pad slots per 32 (conflict-free b128 reads in all
// three forward passes, tools/fc_model.py layout check); the inverse M points, 1 pad per 16 --
// its own array at zoom 8 (1024 points), inside the window's at zoom 4 (2048: two arrays would
// not fit two workgroups per CU)
constexpr int kBigSlots = kN + 2 * (kN / 32);
constexpr int kSmallSlots8 = 1024 + 1024 / 16;
__device__ __forceinline__ int ps(int i) { return i + (i >> 4); }

// acc + a b (complex) in two VOP3P instructions (cmul2 with the accumulator as the addend)
__device__ __forceinline__ v2f cmac2(v2f acc, v2f a, v2f b) {
  v2f t, r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(t) : "v"(a), "v"(b), "v"(acc));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
__device__ __forceinline__ v2f conj(v2f a) { return v2f{a.x, -a.y}; }
// sum_a v_a W_R^(-ab): the forward radix R with outputs b and R - b exchanged
template <int R>
__device__ __forceinline__ void idft(v2f *v) {
  dft<R>(v);
#pragma unroll
  for (int b = 1; b < R / 2; ++b) {
    const v2f s = v[b];
    v[b] = v[R - b];
    v[R - b] = s;
  }
}
// v[b] *= w^b, b = 1 .. R-1 (R = 4, 8)
template <int R>
__device__ __forceinline__ void pow_tw(v2f *v, v2f w);
template <>
__device__ __forceinline__ void pow_tw<4>(v2f *v, v2f w) {
  const v2f w2 = cmul2(w, w);
  v[1] = cmul2(v[1], w);
  v[2] = cmul2(v[2], w2);
  v[3] = cmul2(v[3], cmul2(w2, w));
}
template <>
__device__ __forceinline__ void pow_tw<8>(v2f *v, v2f w) {  // each power from at most 3 products
  const v2f w2 = cmul2(w, w), w4 = cmul2(w2, w2), w3 = cmul2(w2, w);
  v[1] = cmul2(v[1], w);
  v[2] = cmul2(v[2], w2);
  v[3] = cmul2(v[3], w3);
  v[4] = cmul2(v[4], w4);
  v[5] = cmul2(v[5], cmul2(w4, w));
  v[6] = cmul2(v[6], cmul2(w4, w2));
  v[7] = cmul2(v[7], cmul2(w4, w3));
}

// Loads through buffer resources: one lane offset VGPR and constant SGPR offsets per load (64-bit
// addresses per load, hoisted out of the block loop, spilled 60-100 VGPRs), and a load past the
// resource's end returns 0 (the window's samples outside the frame).
constexpr int kBufFlags = 0x00020000;
template <int DT>
constexpr int ebytes() { return DT == kInC64 ? 8 : DT == kInCU8 ? 2 : 4; }
template <int DT>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const InDesc &in, int64_t f) {
  constexpr int eb = ebytes<DT>();
  return __builtin_amdgcn_make_buffer_rsrc((void *)((const char *)in.p + f * in.stride * eb), (short)0,
                                           (int)(in.len * eb), kBufFlags);
}
// sample n of the frame, 0 outside it (the load returns raw 0 there, which is -1 - 1i for cu8:
// the value is selected after the conversion)
template <int DT, int FLIP>
__device__ __forceinline__ v2f load_sample(__amdgpu_buffer_rsrc_t rs, int64_t L, int64_t n) {
  constexpr int eb = ebytes<DT>();
  const int64_t k = FLIP ? L - 1 - n : n;
  const bool in = n >= 0 && n < L;
  const uint32_t vo = in ? (uint32_t)(k * eb) : 0x80000000u;
  if constexpr (DT == kInC64) {
    return __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(rs, vo, 0, 0));
  } else if constexpr (DT == kInC32H) {
    const h2 h = __builtin_bit_cast(h2, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, 0, 0));
    return v2f{(float)h.x, (float)h.y};
  } else if constexpr (DT == kInF32R) {
    return v2f{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, 0, 0)), 0.f};
  } else {
    const u8x2 u = __builtin_bit_cast(u8x2, __builtin_amdgcn_raw_buffer_load_b16(rs, vo, 0, 0));
    const v2f v{((float)u.x - 127.5f) * (1.f / 127.5f), ((float)u.y - 127.5f) * (1.f / 127.5f)};
    return in ? v : splat(0.f);
  }
}
// the raw pair (n, n + 1), n = s + 2t + 512 j, of a window inside the frame: voffset from
// pair_vo (per block), soffset the constant 512 eb j (mirrored for FLIP)
template <int DT, int FLIP>
__device__ __forceinline__ uint32_t pair_vo(int64_t L, int64_t s, int t) {
  constexpr int eb = ebytes<DT>();
  return (uint32_t)((FLIP ? L - 2 - s - 7680 - 2 * t : s + 2 * t) * eb);
}
template <int DT, int FLIP>
__device__ __forceinline__ typename RawP<DT>::T load_pair_b(__amdgpu_buffer_rsrc_t rs, uint32_t vo, int j) {
  constexpr int eb = ebytes<DT>();
  const int so = 512 * eb * (FLIP ? 15 - j : j);
  typedef typename RawP<DT>::T T;
  constexpr int aux = 2;  // non-temporal: the window is streamed once (-1 % per step, r06fc6)
  if constexpr (DT == kInC64) return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, aux));
  else if constexpr (DT == kInCU8) return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, aux));
  else return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, aux));
}
// Between two inverse stages whose LDS slots stay inside one wave: a wave's LDS operations
// complete in issue order, so ordering the compiler's view (wavefront-scope fences around a
// wave barrier) is all it takes -- no s_barrier
__device__ __forceinline__ void stage_sync() {
  if (FC_WSYNC) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// How many of a thread's 16 C pairs stay in registers for the whole kernel instead of being
// re-read from L2 every block: as many as each instantiation holds without spilling at 2 WG/CU
// (cu8 has no room; against none, complex64 8 at zoom 8: fc_decim 2.62 -> 2.55 ms at cfg2,
// r06fc10; 6 at zoom 4 and 14 for complex32 beat 4 and 12 by 1.1 / 0.6 % per step, r06fc13)
constexpr int fc_hold(int Z, int DT) {
  return DT == kInCU8 ? 0 : DT == kInC64 ? (Z == 8 ? 8 : 6) : 14;
}

// One workgroup walks blocks [bpc * blockIdx.x, +bpc) of frame blockIdx.y.  tab: W_M^k (k < M),
// then per LO row (row_stride apart) C as v4f pairs [(Z / 2) k3 + r / 2][t] (r, r + 1) for thread t
// of pass C.  Needs frames of >= kFcN samples and < 2^31 bytes (launch_fc_decim).
template <int Z, int DT, int FLIP>
__global__ void __launch_bounds__(256, 2) fc_decim_kernel(InDesc in, const v2f *lo, const v2f *tab,
                                                         int64_t row_stride, v2f *out, int64_t nd,
                                                         int bpc) {
  constexpr int M = kN / Z;             // per-residue transform: 1024 (zoom 8), 2048 (zoom 4)
  constexpr int R1 = M / 256;           // radix of the last forward / first inverse stage
  constexpr int S = Geo<Z>::S, K = Geo<Z>::K, P = Geo<Z>::P;
  constexpr int KEEP = 16 - S;          // a thread's pairs carried into the next window
  constexpr int J0 = K / Z;             // first valid inverse output
  constexpr int NB = M / 1024;          // inverse butterflies per thread in stages 2..5
  constexpr bool ALIAS = Z == 4;        // the inverse array inside the window's
  static_assert(K == (kN - 512 * S) / 2 && P * Z == 512 * S && K % Z == 0 && KEEP >= 1, "FC block geometry");
  static_assert(J0 + P <= M && J0 < 256 * NB, "FC outputs");
  __shared__ v4f big4[kBigSlots / 2];
  __shared__ v2f small_[ALIAS ? 2 : kSmallSlots8];
  const LP bl = (LP)big4;
  const LP sl = ALIAS ? bl : (LP)small_;
  const int t = threadIdx.x;
  const int64_t f = blockIdx.y, L = in.len;
  const int nb = (int)((nd + P - 1) / P);
  const int b0 = (int)blockIdx.x * bpc, b1 = min(nb, b0 + bpc);
  if (b0 >= b1) return;
  const v2f *lor = lo_row(lo, in, f);
  const int row = in.lo_n <= 1 ? 0 : (int)((((int64_t)in.lo_first + f) / in.lo_per) % in.lo_n);
  const v2f *tw = tab;
  const __amdgpu_buffer_rsrc_t crs =
      __builtin_amdgcn_make_buffer_rsrc((void *)(tab + M + row * row_stride), (short)0, kFcRow * 8, kBufFlags);
  const __amdgpu_buffer_rsrc_t xrs = frame_rsrc<DT>(in, f);
  // pass A: residues of thread t's pairs 2t + 512 i are (2t mod Z, +1), at m = j0 + (M / 16) i;
  // pass B: k1 = t >> 4, j1 = the digit below i2 of the (M / 16)-point remainder
  const int j0 = t >> (Z == 8 ? 2 : 1), j1 = Z == 8 ? (t >> 2) & 3 : (t >> 1) & 7;
  v2f bA[4], bB[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    bA[s] = tw[(j0 << s) & (M - 1)];
    bB[s] = tw[((16 * j1) << s) & (M - 1)];
  }
  // pass C: k1 = t >> 4, k2 = t & 15 -> kp = k1 + 16 k2
  const int kp = (t >> 4) + 16 * (t & 15);
  // the first HOLD of its 16 C pairs held for the whole kernel (the rest read per block)
  constexpr int HOLD = FC_HOLD >= 0 ? (DT == kInCU8 ? 0 : FC_HOLD) : fc_hold(Z, DT);
  v4f ch[HOLD > 0 ? HOLD : 1];
#pragma unroll
  for (int i = 0; i < HOLD; ++i)
    ch[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(crs, (uint32_t)(16 * t), 4096 * i, 0));
  // inverse twiddle bases, conjugated: stage 1 W_M^kp, 2 W_256^(t & 63), 3 W_64^(t & 15),
  // 4 W_16^(t & 3) (the digits below each stage's)
  const v2f ib0 = conj(tw[kp]), ib1 = conj(tw[(M / 256) * (t & 63)]), ib2 = conj(tw[(M / 64) * (t & 15)]),
            ib3 = conj(tw[(M / 16) * (t & 3)]);
  // outputs: butterfly u = t + 256 h of stage 5 gives j = u + (M / 4) b4, valid for j in
  // [J0, J0 + P), at output jm = j - J0 of the block; their lo[Z jm] (0 where invalid / past
  // the frame)
  v2f lj[NB][4];
#pragma unroll
  for (int h = 0; h < NB; ++h)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int jm = t + 256 * h + (M / 4) * q - J0;
      lj[h][q] = jm >= 0 && jm < P && jm < nd ? lor[Z * jm] : splat(0.f);
    }
  // LDS bases (v2f slots; the pads folded into the constant strides)
  const int aA = 2 * t + 2 * (t >> 4);                 // pb(512 k + 2t) = aA + 544 k
  const int aB = 2 * (t & 15) + 544 * (t >> 4);        // pb(base + 32 i) = aB + 34 i
  const int aC = 544 * (t >> 4) + 34 * (t & 15);       // pair p of pass C: aC + 2 p
  const int a1 = ps(kp);                               // ps(kp + 256 q) = a1 + 272 q
  // stages 2..4 (butterfly t + 256 h at +1088 h), stage 5
  const int a2 = ps((t & 63) + 256 * (t >> 6));                                      // + 68 a
  const int a3 = ps((t & 15) + 64 * ((t >> 4) & 3) + 256 * (t >> 6));               // + 17 a
  const int a4 = ps((t & 3) + 16 * ((t >> 2) & 3) + 64 * ((t >> 4) & 3) + 256 * (t >> 6));  // + 4 a
  auto a5 = [&](int h) {  // u = b0 + R1 (b1 + 4 b2 + 16 b3) reads (a0 + 4 b3 + 16 b2 + 64 b1 + 256 b0)
    const int u = t + 256 * h, r = u / R1;
    return ps(4 * ((r >> 4) & 3) + 16 * ((r >> 2) & 3) + 64 * (r & 3) + 256 * (u % R1));
  };

  auto wstart = [&](int b) -> int64_t { return (int64_t)(512 * S) * b - K; };
  auto inside = [&](int b) { const int64_t s = wstart(b); return s >= 0 && s + kN <= L; };
  typename RawP<DT>::T pf[S];  // the next window's pairs KEEP .. 15
  v2f ka[KEEP], kb[KEEP];      // this window's pairs S .. 15 = the next window's 0 .. KEEP-1
  bool carried = false;        // ka, kb and pf hold this block's window
  // the next window's new pairs, issued on every block from a window start clamped into the
  // frame (values unused when the next window is not inside it): one unconditional call site,
  // so the wait before their use counts only what was issued after them
  auto issue_pf = [&](int b) {
    carried = b + 1 < b1 && inside(b + 1);
    int64_t sn = wstart(b + 1);
    sn = sn < 0 ? 0 : (sn > L - kN ? L - kN : sn);
    const uint32_t vo = pair_vo<DT, FLIP>(L, sn, t);
#pragma unroll
    for (int i = 0; i < S; ++i)
      if (!(FC_KO & 1)) pf[i] = load_pair_b<DT, FLIP>(xrs, vo, KEEP + i);
  };
  for (int b = b0; b < b1; ++b) {
    v2f xa[16], xb[16];
    // this block's lo[Z m0], requested before the prefetch: its wait at the outputs then
    // leaves the prefetch in flight (the vector-memory counter completes in order)
    const int64_t m0 = (int64_t)P * b;
    const v2f lob = lor[Z * m0];
    {
      const int64_t s = wstart(b);
      if (FC_KO & 1) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          xa[i] = v2f{(float)(t + i), 1.f};
          xb[i] = v2f{1.f, (float)(t - i)};
        }
      } else if (carried) {
#pragma unroll
        for (int i = 0; i < KEEP; ++i) {
          xa[i] = ka[i];
          xb[i] = kb[i];
        }
#pragma unroll
        for (int i = 0; i < S; ++i) cvt_pair<DT, FLIP>(pf[i], xa[KEEP + i], xb[KEEP + i]);
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int64_t n = s + 2 * t + 512 * i;
          xa[i] = load_sample<DT, FLIP>(xrs, L, n);
          xb[i] = load_sample<DT, FLIP>(xrs, L, n + 1);
        }
      }
#pragma unroll
      for (int i = 0; i < KEEP; ++i) {
        ka[i] = xa[S + i];
        kb[i] = xb[S + i];
      }
      issue_pf(b);
    }
    // pass A: DFT16 over i -> k1, twiddle W_M^(j0 k1), to LDS at ((M / 16) k1 + j0, r)
    dft<16>(xa);
    dft<16>(xb);
    apply_powers2(xa, xb, bA);
#pragma unroll
    for (int k = 0; k < 16; ++k) *(LP4)(bl + aA + 544 * k) = cat(xa[k], xb[k]);
    __syncthreads();
    // pass B: ((M / 16) k1 + j1 + (M / 256) i2) -> DFT16 over i2 -> k2, twiddle
    // W_(M / 16)^(j1 k2), in place
    {
      v2f ya[16], yb[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const v4f w = *(LP4)(bl + aB + 34 * i);
        ya[i] = lo2(w);
        yb[i] = hi2(w);
      }
      dft<16>(ya);
      dft<16>(yb);
      apply_powers2(ya, yb, bB);
#pragma unroll
      for (int k = 0; k < 16; ++k) *(LP4)(bl + aB + 34 * k) = cat(ya[k], yb[k]);
    }
    __syncthreads();
    // pass C: ((M / 16) k1 + R1 k2 + j1, r) for all j1 < R1, r < Z -> DFT_R1 over j1 -> k3;
    // Yf = sum_r A_r C; inverse stage 1 (radix R1 over k3 -> b0, twiddle W_M^(-b0 kp)) to
    // (kp + 256 b0)
    {
      v4f cr[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        cr[i] = (FC_KO & 2) ? v4f{1.f, 0.5f, 0.25f, 1.f}
                : i < HOLD  ? ch[i < HOLD ? i : 0]
                            : __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(crs, (uint32_t)(16 * t), 4096 * i, 0));
      // one residue pair at a time: its R1 values, DFT each, accumulated into Yf (the whole
      // window's 32 values and C's 32 at once spilled)
      v2f yf[R1];
#pragma unroll
      for (int k = 0; k < R1; ++k) yf[k] = splat(0.f);
#pragma unroll
      for (int rp = 0; rp < Z / 2; ++rp) {
        v2f ea[R1], eb[R1];
#pragma unroll
        for (int j = 0; j < R1; ++j) {
          const v4f w = *(LP4)(bl + aC + 2 * (Z / 2 * j + rp));
          ea[j] = lo2(w);
          eb[j] = hi2(w);
        }
        dft<R1>(ea);
        dft<R1>(eb);
#pragma unroll
        for (int k = 0; k < R1; ++k) {
          const v4f c = cr[Z / 2 * k + rp];
          yf[k] = cmac2(cmac2(yf[k], ea[k], lo2(c)), eb[k], hi2(c));
        }
      }
      idft<R1>(yf);
      pow_tw<R1>(yf, ib0);
      if (ALIAS) __syncthreads();  // every pass-C read done before the inverse array overwrites
#pragma unroll
      for (int q = 0; q < R1; ++q) sl[a1 + 272 * q] = yf[q];
    }
    __syncthreads();
    // inverse stages 2..4: radix 4 over the digit at stride S, twiddle W_(4S)^(-b k_low)
    auto istage = [&](int a0, int st, v2f w) {
#pragma unroll
      for (int h = 0; h < NB; ++h) {
        v2f v[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) v[a] = sl[a0 + 1088 * h + st * a];
        idft<4>(v);
        pow_tw<4>(v, w);
#pragma unroll
        for (int a = 0; a < 4; ++a) sl[a0 + 1088 * h + st * a] = v[a];
      }
    };
    // stages 2..4 read and write only the slots of their wave's b0 (t >> 6, + 4 h): the
    // exchanges between them are wave-local, stage 5 reads every wave's
    istage(a2, 68, ib1);
    stage_sync();
    istage(a3, 17, ib2);
    stage_sync();
    istage(a4, 4, ib3);
    __syncthreads();  // (stage 5 inside the wave, outputs R1 apart: 3.11 -> 3.31 ms, r06fc12)
    // stage 5: radix 4 over a0 -> b4; outputs j = u + (M / 4) b4
    {
      v2f *o = out + f * nd + m0;
#pragma unroll
      for (int h = 0; h < NB; ++h) {
        const int i5 = a5(h);
        v2f v[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) v[a] = sl[i5 + a];
        idft<4>(v);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int jm = t + 256 * h + (M / 4) * q - J0;
          if (jm >= 0 && jm < P && m0 + jm < nd && !(FC_KO & 4))
            __builtin_nontemporal_store(cmul2(v[q], cmul2(lob, lj[h][q])), o + jm);
        }
      }
    }
    if (ALIAS) __syncthreads();  // stage-5 reads done before the next window's pass-A stores
  }
}

}  // namespace fc

hipError_t launch_fc_decim(const InDesc &in, const float2 *lo, const float2 *tab, int64_t row_stride,
                           float2 *out, int64_t nd, int frames, int zoom, hipStream_t st) {
  if (in.len < kFcN || in.len * (int64_t)in_elem_bytes(in.dtype) >= ((int64_t)1 << 31) ||
      (zoom != 8 && zoom != 4))
    return hipErrorInvalidValue;
  const int P = zoom == 8 ? kFcP : kFc4P;
  const int nb = (int)((nd + P - 1) / P);
  // about two rounds of the chip's 512 resident workgroups: whole frames from 1024 frames per
  // call, below that each frame split into runs of blocks (a run's first window loads in full)
  const int chunks = std::max(1, std::min(nb, (1024 + frames - 1) / frames));
  const int bpc = (nb + chunks - 1) / chunks;
  const dim3 grid((unsigned)((nb + bpc - 1) / bpc), (unsigned)frames);
  const v2f *l = (const v2f *)lo, *tb = (const v2f *)tab;
  v2f *o = (v2f *)out;
#define FC_GO(Z, DT, FL) \
  hipLaunchKernelGGL((fc::fc_decim_kernel<Z, DT, FL>), grid, dim3(256), 0, st, in, l, tb, row_stride, o, nd, bpc)
#define FC_DT(Z, FL)                           \
  do {                                         \
    if (in.dtype == kInC64) FC_GO(Z, kInC64, FL);        \
    else if (in.dtype == kInC32H) FC_GO(Z, kInC32H, FL); \
    else if (in.dtype == kInCU8) FC_GO(Z, kInCU8, FL);   \
    else FC_GO(Z, kInF32R, FL);                          \
  } while (0)
  if (zoom == 8) {
    if (in.flip) FC_DT(8, 1);
    else FC_DT(8, 0);
  } else {
    if (in.flip) FC_DT(4, 1);
    else FC_DT(4, 0);
  }
#undef FC_DT
#undef FC_GO
  return hipGetLastError();
}

}  // namespace zfft
