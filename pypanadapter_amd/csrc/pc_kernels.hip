// pc_kernels.hip -- "PC" (polyphase cascade) decimator for zoom 8 on gfx950 (tables:
// pc_tables.cpp; design model: tools/pc_model.py).
//
// Three x scipy.signal.decimate(x, 2) (pypanadapter_spectrum.py:2096-2098) as, exactly,
//   K1  y1 = (g0 * x)|2,  y2 = (g1 * y1)|2          two FIRs (33, 49 taps): no recurrence at the
//                                                   input rate, independent tiles
//   K2  z2 = S(v) S(1/v) y2                         two sections at rate 1/4 (zero phase)
//       u3 = (g2 * z2)|2                            FIR (57 taps)
//       out = A(w) A(1/w) u3                        10 sections at the output rate
//   K3  out += U (V^T x_edge)                       frame-start / frame-end maps (rank ~10)
// on the frame extended by zeros.  Recurrences run over lane blocks: every lane runs its
// block from a zero state, the exit states are combined by a Kogge-Stone scan over lanes
// (depth from the block decay, pc_own_levels / pc_ap_levels), and each output gets the
// entering state's response ct[t] . s (t < its decay length).  K2 tiles carry warm-up halos
// (own rate 276 / 438 samples, output rate 64) instead of state across tiles, so every tile and
// every K1 tile is independent.
// Intermediates: only y2 (rate 1/4, 8 B per 4 input samples) goes through device memory.
#include "zfft_device.h"
#include "zfft_pairs.h"

// Diagnostic builds only (ZFFT_DIAG=1, never set by build.py): PC_KO timing knockouts with
// wrong results by design -- 1 own-rate sections, 2 FIR gamma, 4 output-rate sections,
// 8 K1's LO mix (and its table loads); KW only: 16 the two input-rate FIRs, 32 the input loads,
// 64 the FIR sub-tile's barriers after the input and after FIR beta, 128 the two around the y1
// hand-over (timing of the barriers alone: the LDS data races by design).
#ifndef ZFFT_DIAG
#define ZFFT_DIAG 0
#endif
#if ZFFT_DIAG && defined(PC_KO)
constexpr int kKo = PC_KO;
#else
constexpr int kKo = 0;
#endif
// PC_STAMPS=1 (diagnostic builds only): per-phase s_memtime sums of every walk wave, read back
// with zfft_debug_pc_stamps (tools/pc_stamps.py); no stamp exists otherwise.
#if !ZFFT_DIAG && defined(PC_STAMPS)
#error "PC_STAMPS is a diagnostic knob: build with -DZFFT_DIAG"
#endif
#ifndef PC_STAMPS
#define PC_STAMPS 0
#endif
// PC_DPPSHIFT = largest lane shift of the recurrence scans done as a chain of whole-wave DPP
// shifts (wave_shr/shl:1, a few cycles each) instead of one ds_bpermute (an LDS round trip):
// 4 -- shifts 1, 2, 4 by DPP, 8 and 16 by ds_bpermute (walk 1.5-3 % faster than 1 in three
// same-box A/Bs, profiles/r05a, r05b, r05d; 16: no better).  A/B knobs (diagnostic builds only):
// PC_DPPSHIFT, PC_PRIO = s_setprio level of the walk's recurrence phases (own-rate and
// output-rate sections), the FIR phases running at 0 (default 0: no setprio; 2: within noise).
#if !ZFFT_DIAG && (defined(PC_DPPSHIFT) || defined(PC_PRIO))
#error "PC_DPPSHIFT / PC_PRIO are diagnostic knobs: build with -DZFFT_DIAG"
#endif
#ifndef PC_DPPSHIFT
#define PC_DPPSHIFT 4
#endif
#ifndef PC_PRIO
#define PC_PRIO 0
#endif
#if !ZFFT_DIAG && defined(PC_ASMFMA)
#error "PC_ASMFMA is a diagnostic knob: build with -DZFFT_DIAG"
#endif
#ifndef PC_ASMFMA
#define PC_ASMFMA 0  // walk FIRs: taps as aligned SGPR pairs selected by op_sel (no s_mov)
#endif
// PC_OCC3 (diagnostic builds only, timing-only: the LDS regions race by design): the walk at
// three workgroups per CU -- the own-rate span aliases the input tile (LDS 81 -> 45 KB) and the
// kernel is compiled for 3 waves per SIMD (<= 168 VGPRs, spilling what does not fit)
#if !ZFFT_DIAG && defined(PC_OCC3)
#error "PC_OCC3 is a diagnostic knob: build with -DZFFT_DIAG"
#endif
#ifndef PC_OCC3
#define PC_OCC3 0
#endif
// PC_CENSUS (diagnostic builds only, listing only, wrong at frame edges): every walk sub-tile
// takes the interior path, so the edge code is dead and the assembly is the steady-state tile
// that tools/isa_census.py counts
#if !ZFFT_DIAG && defined(PC_CENSUS)
#error "PC_CENSUS is a diagnostic knob: build with -DZFFT_DIAG"
#endif
#ifndef PC_CENSUS
#define PC_CENSUS 0
#endif


namespace zfft {
namespace pc {

[[maybe_unused]] constexpr int kPcStampSegs = 10;
#if PC_STAMPS
__device__ unsigned long long g_pc_stamps[kPcStampSegs + 1];
#define PC_STAMP(i)                                                                   \
  {                                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                                \
    unsigned long long t_;                                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
    __builtin_amdgcn_sched_barrier(0);                                                \
    st_acc[i] += t_ - t_prev;                                                         \
    t_prev = t_;                                                                      \
  }
#else
#define PC_STAMP(i)
#endif

typedef v2f __attribute__((address_space(3))) *LP;
typedef v4f __attribute__((address_space(3))) *LP4;
typedef const PcTab __attribute__((address_space(4))) *CT;
typedef const PcTab4 __attribute__((address_space(4))) *CT4;
typedef const PcTab2 __attribute__((address_space(4))) *CT2;
typedef const PcSec __attribute__((address_space(4))) &CS;

__device__ __forceinline__ v2f shup(v2f v, int d) {
  return v2f{__shfl_up(v.x, d, 64), __shfl_up(v.y, d, 64)};
}
__device__ __forceinline__ v2f shdn(v2f v, int d) {
  return v2f{__shfl_down(v.x, d, 64), __shfl_down(v.y, d, 64)};
}
__device__ __forceinline__ v2f shxor(v2f v, int d) {
  return v2f{__shfl_xor(v.x, d, 64), __shfl_xor(v.y, d, 64)};
}
// An opaque copy of the table pointer per phase: the scalar loads of a phase's coefficients
// are not hoisted out of it (hoisted, all 12 sections' tables would sit in SGPRs and spill).
template <class P>
__device__ __forceinline__ P fresh(P p) {
  asm volatile("" : "+s"(p));
  return p;
}
// acc += g[u] x0 (+ g[u + 1] x1): one FIR tap pair (u even) as an aligned SGPR pair, the tap
// picked by op_sel -- the compiler's own form copies the odd tap into an even SGPR first
typedef unsigned long long u64s;
template <class TP>
__device__ __forceinline__ u64s tap_pair(TP taps, int u) {
  return *(const u64s __attribute__((address_space(4))) *)(taps + u);
}
__device__ __forceinline__ void fma_tap_lo(v2f &acc, u64s g, v2f x) {
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc) : "s"(g), "v"(x));
}
__device__ __forceinline__ void fma_tap_hi(v2f &acc, u64s g, v2f x) {
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "s"(g), "v"(x));
}
// acc + c[1] b + c[0] a (inner product first, as vfma(c0, a, vfma(c1, b, acc))), c an aligned
// coefficient pair of the section tables
template <class PP>
__device__ __forceinline__ v2f fma2(PP c, v2f a, v2f b, v2f acc) {
  if constexpr (PC_ASMFMA) {
    const u64s g = tap_pair(c, 0);
    fma_tap_hi(acc, g, b);
    fma_tap_lo(acc, g, a);
    return acc;
  } else {
    return vfma(splat(c[0]), a, vfma(splat(c[1]), b, acc));
  }
}
template <int G, class TP>
__device__ __forceinline__ void fir_pair(v2f &acc, TP taps, int u, v2f x0, v2f x1) {
  if constexpr (PC_ASMFMA) {
    if (u >= 0 && u < G) {
      const u64s g = tap_pair(taps, u);
      fma_tap_lo(acc, g, x0);
      if (u + 1 < G) fma_tap_hi(acc, g, x1);
    }
  } else {
    if (u >= 0 && u < G) acc = vfma(splat(taps[u]), x0, acc);
    if (u + 1 >= 0 && u + 1 < G) acc = vfma(splat(taps[u + 1]), x1, acc);
  }
}
// cmul2 with a wave-uniform first factor held in an SGPR pair (VOP3P takes it as a source:
// no v_mov of the pair into VGPRs first)
__device__ __forceinline__ v2f cmul2s(v2f a, v2f b) {
  v2f t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "s"(a), "v"(b));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "=v"(r) : "s"(a), "v"(b), "v"(t));
  return r;
}
// lane k's v of a wave, for a wave-uniform k (v_readlane: an SGPR pair, no memory round trip)
__device__ __forceinline__ v2f lane_val(v2f v, int k) {
  return v2f{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), k)),
             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), k))};
}

// ---------------------------------------------------------------------------------- K1

constexpr int kXRow = 18;  // input tile: rows of 16 samples padded to 18 (b128 reads conflict-free)
constexpr int kYRow = 10;  // y1: rows of 8 padded to 10
constexpr int kXRows = kPcK1In / 16;
__device__ __forceinline__ int xidx(int s) { return (s >> 4) * kXRow + (s & 15); }

// One tile: y2 for q in [q_s, q_s + 992), q_s = -16 + 992 tile, from the mixed input
// x[4 q_s - 64, + 4128) (zero outside the frame):
//   y1[m] = sum_t g0[t + 16] x[2m - t],  m in [2 q_s - 24, + 2048)   (8 per thread)
//   y2[q] = sum_t g1[t + 24] y1[2q - t]                            (4 per thread)
template <int ZOOM> struct PcTabOf { typedef CT T; };
template <> struct PcTabOf<4> { typedef CT4 T; };
template <> struct PcTabOf<2> { typedef CT2 T; };
// ZOOM = 4: FIR alpha only, y1 [m_s, m_s + 2048), m_s = kPc4Q0 + 2048 tile, from the mixed
// input x[2 m_s - 16, + 4128) -- the same input tile and thread map -- written to y2 (= y1 here)
template <int DT, int FLIP, int ZOOM>
__global__ void __launch_bounds__(256) pc_fir_kernel(InDesc in, const v2f *lo, v2f *y2,
                                                     int64_t y2s, typename PcTabOf<ZOOM>::T tab) {
  __shared__ v4f lds4[kXRows * kXRow / 2];
  const LP xl = (LP)lds4;
  const int t = threadIdx.x;
  const int tile = blockIdx.x;
  const int64_t f = blockIdx.y, L = in.len;
  const int64_t xs = ZOOM == 4 ? 2 * ((int64_t)kPc4Q0 + (int64_t)kPc4K1M * tile) - 16
                               : 4 * ((int64_t)kPcQ0 + (int64_t)kPcK1Q * tile) - 64;
  const v2f *lor = lo_row(lo, in, f);
  if (xs >= 0 && xs + kPcK1In <= L) {
    // LO factor lo[n0 + 2t + j] = lo[n0] lo[2t + j] / sqrt 2 (the table is an exact
    // exponential): one uniform entry per 512 samples instead of a table stream beside the
    // input (which cost 13 % of the kernel, profiles/r04c); the nine entries lo[xs + 512 k]
    // are loaded by lanes k = 0..8 together with the input, and read back with v_readlane
    // (issued one by one at their use, each load's round trip was exposed)
    const v4f lane_lo = *(const v4f *)(lor + 2 * t) * (float)M_SQRT1_2;
    const v2f lo_k = lor[xs + 512 * min(t & 63, 8)];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int s = 2 * t + 512 * i;
      if (i == 8 && t >= (kPcK1In - 4096) / 2) break;
      v2f a, b;
      load_pair<DT, FLIP>(in, f, xs + s, a, b);
      if constexpr (kKo & 8) {
        *(LP4)(xl + xidx(s)) = cat(a, b);
      } else {
        const v2f c = lane_val(lo_k, i);  // lo[xs + 512 i]
        *(LP4)(xl + xidx(s)) = cat(cmul2(a, cmul2(c, lo2(lane_lo))), cmul2(b, cmul2(c, hi2(lane_lo))));
      }
    }
  } else {
    for (int s = t; s < kPcK1In; s += 256) {
      const int64_t n = xs + s;
      v2f v = splat(0.f);
      if (n >= 0 && n < L) v = cmul2(load_in_t<DT, FLIP>(in, f, n), lor[n]);
      xl[xidx(s)] = v;
    }
  }
  __syncthreads();
  v2f acc[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) acc[r] = splat(0.f);
  {
    const LP xb = xl + t * kXRow;  // local sample 16 t; outputs i = 8t + r read [16t + 2r, + 32]
#pragma unroll
    for (int p = 0; p < 24; ++p) {
      const int j = 2 * p;
      const v4f w = *(LP4)(xb + (j >> 4) * kXRow + (j & 15));
      const v2f x0 = lo2(w), x1 = hi2(w);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int u = j - 2 * r;
        if (u >= 0 && u < kPcG0) acc[r] = vfma(splat(tab->g0[u]), x0, acc[r]);
        if (u + 1 >= 0 && u + 1 < kPcG0) acc[r] = vfma(splat(tab->g0[u + 1]), x1, acc[r]);
      }
    }
  }
  if constexpr (ZOOM == 4) {
    v2f *o = y2 + f * y2s + (int64_t)kPc4K1M * tile + 8 * t;
#pragma unroll
    for (int q = 0; q < 4; ++q) *(v4f *)(o + 2 * q) = cat(acc[2 * q], acc[2 * q + 1]);
    return;
  }
  __syncthreads();
  const LP yl = xl;
#pragma unroll
  for (int q = 0; q < 4; ++q) *(LP4)(yl + t * kYRow + 2 * q) = cat(acc[2 * q], acc[2 * q + 1]);
  __syncthreads();
  if constexpr (ZOOM == 8) if (t < kPcK1Q / 4) {
    v2f b[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) b[r] = splat(0.f);
    const LP yb = yl + t * kYRow;  // y1 local 8t; outputs k = 4t + r read [2k, 2k + 48]
#pragma unroll
    for (int p = 0; p < 28; ++p) {
      const int j = 2 * p;
      const v4f w = *(LP4)(yb + (j >> 3) * kYRow + (j & 7));
      const v2f x0 = lo2(w), x1 = hi2(w);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int u = j - 2 * r;
        if (u >= 0 && u < kPcG1) b[r] = vfma(splat(tab->g1[u]), x0, b[r]);
        if (u + 1 >= 0 && u + 1 < kPcG1) b[r] = vfma(splat(tab->g1[u + 1]), x1, b[r]);
      }
    }
    v2f *o = y2 + f * y2s + (int64_t)kPcK1Q * tile + 4 * t;
    *(v4f *)o = cat(b[0], b[1]);
    *(v4f *)(o + 2) = cat(b[2], b[3]);
  }
}

// ---------------------------------------------------------------------------------- K2

// Whole-wave DPP shift by one lane toward higher (UP, wave_shr:1) or lower lanes
// (wave_shl:1); the lane without a source reads 0.
template <bool UP>
__device__ __forceinline__ v2f wshift(v2f v) {
  constexpr int ctrl = UP ? 0x138 : 0x130;
  return v2f{__int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v.x), ctrl, 0xF, 0xF, true)),
             __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v.y), ctrl, 0xF, 0xF, true))};
}
// Shift by SH >= 2 lanes (0 where there is no source) through ds_bpermute: the LDS crossbar
// instead of SH dependent DPP moves on the VALU.
template <bool UP, int SH>
__device__ __forceinline__ v2f shiftk(v2f v, int lane) {
  if constexpr (SH <= PC_DPPSHIFT) {  // SH dependent DPP moves (diagnostic A/B form)
#pragma unroll
    for (int i = 0; i < SH; ++i) v = wshift<UP>(v);
    return v;
  } else {
    const v2f r = UP ? v2f{__shfl_up(v.x, SH, 64), __shfl_up(v.y, SH, 64)}
                     : v2f{__shfl_down(v.x, SH, 64), __shfl_down(v.y, SH, 64)};
    return (UP ? lane < SH : lane >= 64 - SH) ? splat(0.f) : r;
  }
}
__device__ __forceinline__ void walk_prio(bool recurrence) {
  if constexpr (PC_PRIO > 0) {
    if (recurrence) __builtin_amdgcn_s_setprio(PC_PRIO);
    else __builtin_amdgcn_s_setprio(0);
  }
}

// One all-pole section over this lane's block v[0..B) in time order (UP) or reversed (!UP),
// the wave's lane blocks adjacent in time: zero-state run, Kogge-Stone over lanes on DPP
// shifts (levels d: + A^(B 2^d) times the state 2^d lanes back), the entering state's
// response ct[t] for t < DCUT.  XW: the block's 4 waves continue each other (one
// cross-wave step through scr: 4 waves x 2 states); otherwise lane 0 (UP) / 63 enters
// from a zero state.
template <int B, int LEV, int DCUT, bool UP, bool XW, bool OWN, int SI, class TP>
__device__ __forceinline__ void sec_block(v2f (&v)[B], TP tab0, LP scr, int lane, int wave) {
  const TP tab = fresh(tab0);
  CS S = OWN ? tab->own[SI] : tab->ap[SI];
  const v2f na1 = splat(-S.a1), na2 = splat(-S.a2);
  v2f y1 = splat(0.f), y2 = splat(0.f);
#pragma unroll
  for (int c = 0; c < B; ++c) {
    const int k = UP ? c : B - 1 - c;
    const v2f y = vfma(na1, y1, vfma(na2, y2, v[k]));
    y2 = y1;
    y1 = y;
    v[k] = y;
  }
  v2f e0 = y1, e1 = y2;  // exit state from a zero entering state
#pragma unroll
  for (int d = 0; d < LEV; ++d) {
    v2f p0, p1;
    if (d == 0) p0 = wshift<UP>(e0), p1 = wshift<UP>(e1);
    else if (d == 1) p0 = shiftk<UP, 2>(e0, lane), p1 = shiftk<UP, 2>(e1, lane);
    else if (d == 2) p0 = shiftk<UP, 4>(e0, lane), p1 = shiftk<UP, 4>(e1, lane);
    else p0 = shiftk<UP, 8>(e0, lane), p1 = shiftk<UP, 8>(e1, lane);
    const v2f n0 = fma2(&S.pw[d][0], p0, p1, e0);
    e1 = fma2(&S.pw[d][2], p0, p1, e1);
    e0 = n0;
  }
  v2f s0 = splat(0.f), s1 = splat(0.f);  // state entering this wave's first block
  if constexpr (XW) {
    if (lane == (UP ? 63 : 0)) {
      scr[2 * wave] = e0;
      scr[2 * wave + 1] = e1;
    }
    __syncthreads();
    const int src = UP ? wave - 1 : wave + 1;
    if (src >= 0 && src < 4) {
      s0 = scr[2 * src];
      s1 = scr[2 * src + 1];
      const int dist = UP ? lane : 63 - lane;  // blocks between this one and the source's
      const float __attribute__((address_space(4))) *x = &tab->own_x[OWN ? SI : 0][dist][0];
      const v2f n0 = vfma(splat(x[0]), s0, vfma(splat(x[1]), s1, e0));
      e1 = vfma(splat(x[2]), s0, vfma(splat(x[3]), s1, e1));
      e0 = n0;
    }
  }
  // the lane without a source reads 0 from the shift (bound_ctrl), which is the zero
  // entering state of a block that does not continue another wave
  v2f i0 = wshift<UP>(e0), i1 = wshift<UP>(e1);
  if (XW && lane == (UP ? 0 : 63)) {
    i0 = s0;
    i1 = s1;
  }
#pragma unroll
  for (int c = 0; c < DCUT; ++c) {
    const int k = UP ? c : B - 1 - c;
    v[k] = fma2(&S.ct[c][0], i0, i1, v[k]);
  }
}

template <int S, bool UP>
__device__ __forceinline__ void ap_cascade(v2f (&a)[kPcApBlk], CT tab, int lane) {
  sec_block<kPcApBlk, pc_ap_levels(S), pc_ap_dcut(S), UP, false, false, S>(a, tab, nullptr, lane, 0);
  if constexpr (S + 1 < kPcAp) ap_cascade<S + 1, UP>(a, tab, lane);
}
// zoom 4's output-rate cascade (PcTab4::ap, 6 sections): sec_block's arithmetic on its tables
template <int B, int LEV, int DCUT, bool UP>
__device__ __forceinline__ void sec_run(v2f (&v)[B], CS S, int lane) {
  const v2f na1 = splat(-S.a1), na2 = splat(-S.a2);
  v2f y1 = splat(0.f), y2 = splat(0.f);
#pragma unroll
  for (int c = 0; c < B; ++c) {
    const int k = UP ? c : B - 1 - c;
    const v2f y = vfma(na1, y1, vfma(na2, y2, v[k]));
    y2 = y1;
    y1 = y;
    v[k] = y;
  }
  v2f e0 = y1, e1 = y2;
#pragma unroll
  for (int d = 0; d < LEV; ++d) {
    v2f p0, p1;
    if (d == 0) p0 = wshift<UP>(e0), p1 = wshift<UP>(e1);
    else if (d == 1) p0 = shiftk<UP, 2>(e0, lane), p1 = shiftk<UP, 2>(e1, lane);
    else if (d == 2) p0 = shiftk<UP, 4>(e0, lane), p1 = shiftk<UP, 4>(e1, lane);
    else p0 = shiftk<UP, 8>(e0, lane), p1 = shiftk<UP, 8>(e1, lane);
    const v2f n0 = fma2(&S.pw[d][0], p0, p1, e0);
    e1 = fma2(&S.pw[d][2], p0, p1, e1);
    e0 = n0;
  }
  const v2f i0 = wshift<UP>(e0), i1 = wshift<UP>(e1);  // 0 on the first lane (bound_ctrl)
#pragma unroll
  for (int c = 0; c < DCUT; ++c) {
    const int k = UP ? c : B - 1 - c;
    v[k] = fma2(&S.ct[c][0], i0, i1, v[k]);
  }
}
template <int S, bool UP>
__device__ __forceinline__ void ap_cascade(v2f (&a)[kPcApBlk], CT4 tab0, int lane) {
  const CT4 tab = fresh(tab0);
  sec_run<kPcApBlk, pc4_ap_levels(S), pc4_ap_dcut(S), UP>(a, tab->ap[S], lane);
  if constexpr (S + 1 < kPc4Ap) ap_cascade<S + 1, UP>(a, tab, lane);
}
// zoom 2's (PcTab2::ap, 4 sections)
template <int S, bool UP>
__device__ __forceinline__ void ap_cascade(v2f (&a)[kPcApBlk], CT2 tab0, int lane) {
  const CT2 tab = fresh(tab0);
  sec_run<kPcApBlk, pc2_ap_levels(S), pc2_ap_dcut(S), UP>(a, tab->ap[S], lane);
  if constexpr (S + 1 < kPc2Ap) ap_cascade<S + 1, UP>(a, tab, lane);
}

constexpr int kU3 = 256 * 9;                   // FIR gamma outputs per tile (9 per thread)
constexpr int kU3Base = 128;                    // u3 index k <-> output m0 - 128 + k
constexpr int kApWave = 64 * kPcApBlk;          // output-rate samples per wave (512 + halos)
constexpr int kOutOff = kU3;                    // final outputs staged after u3
static_assert(kOutOff + kPcK2M <= kPcK2Span, "K2 LDS layout");
static_assert(kApWave == kPcK2M / 4 + 2 * kPcApHalo, "one wave per quarter tile with its halos");
static_assert(kU3Base - kPcApHalo + 3 * (kPcK2M / 4) + kApWave <= kU3, "u3 covers the waves");

// One tile: outputs [m0, m0 + 2048), m0 = 2048 tile, from y2 over [2 m0 - 560, + 5376).
// ZOOM = 4: the same on y1 (stored from kPc4Q0) with zoom 4's FIR g1 and output-rate sections.
// ZOOM = 2: XA's factorisation -- the own-rate signal is the mixed input itself (span sample
// s = input sample 2 m0 - 560 + s, zero outside the frame), D's 4 sections causal only, the
// 25-tap FIR M (z^-8 .. z^16), D2's 4 sections anticausal only.
template <int ZOOM, int DT = kInC64, int FLIP = 0>
__global__ void __launch_bounds__(256) pc_tail_kernel(const v2f *y2, int64_t y2s, int64_t y2n,
                                                      v2f *out, int64_t n3, typename PcTabOf<ZOOM>::T tab,
                                                      InDesc in, const v2f *lo) {
  __shared__ v4f sp4[kPcK2Span / 2];
  __shared__ v4f scr4[4 * 4];
  const LP sp = (LP)sp4;
  const LP scr = (LP)scr4;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t f = blockIdx.y, m0 = (int64_t)kPcK2M * blockIdx.x;
  if constexpr (ZOOM == 2) {
    const int64_t n0 = 2 * m0 - kPcK2Left, L = in.len;
    const v2f *lor = lo_row(lo, in, f);
    for (int s = 2 * t; s < kPcK2Span; s += 512) {
      const int64_t n = n0 + s;
      v2f a = splat(0.f), b = splat(0.f);
      if (n >= 0 && n + 2 <= L) {
        load_pair<DT, FLIP>(in, f, n, a, b);
        a = cmul2(a, lor[n]);
        b = cmul2(b, lor[n + 1]);
      } else {
        if (n >= 0 && n < L) a = cmul2(load_in_t<DT, FLIP>(in, f, n), lor[n]);
        if (n + 1 >= 0 && n + 1 < L) b = cmul2(load_in_t<DT, FLIP>(in, f, n + 1), lor[n + 1]);
      }
      *(LP4)(sp + s) = cat(a, b);
    }
  } else {
    const int64_t g0 = 2 * m0 - kPcK2Left - (ZOOM == 4 ? kPc4Q0 : kPcQ0);  // y2 entry of span sample 0
    const v2f *yb = y2 + f * y2s;
    for (int s = 2 * t; s < kPcK2Span; s += 512) {
      const int64_t g = g0 + s;  // even: a pair is wholly inside or outside [0, y2n)
      v4f w = v4f{0.f, 0.f, 0.f, 0.f};
      if (g >= 0 && g < y2n) w = *(const v4f *)(yb + g);
      *(LP4)(sp + s) = w;
    }
  }
  __syncthreads();
  v2f v[kPcOwnBlk];
#pragma unroll
  for (int k = 0; k < kPcOwnBlk; ++k) v[k] = sp[kPcOwnBlk * t + k];
  // own-rate sections, causal then anticausal (warm-up: the span's first / last 330); zoom 2:
  // D's four, causal only (XA's forward pass, warm-up: the span's first 296)
  if constexpr (ZOOM == 2) {
    sec_block<kPcOwnBlk, pc2_own_levels(0), kPcOwnBlk, true, true, true, 0>(v, tab, scr, lane, wave);
    sec_block<kPcOwnBlk, pc2_own_levels(1), kPcOwnBlk, true, true, true, 1>(v, tab, scr + 8, lane, wave);
    sec_block<kPcOwnBlk, pc2_own_levels(2), kPcOwnBlk, true, true, true, 2>(v, tab, scr + 16, lane, wave);
    sec_block<kPcOwnBlk, pc2_own_levels(3), kPcOwnBlk, true, true, true, 3>(v, tab, scr + 24, lane, wave);
  } else if constexpr (!(kKo & 1)) {
    sec_block<kPcOwnBlk, pc_own_levels(0), kPcOwnBlk, true, true, true, 0>(v, tab, scr, lane, wave);
    sec_block<kPcOwnBlk, pc_own_levels(1), kPcOwnBlk, true, true, true, 1>(v, tab, scr + 8, lane, wave);
    sec_block<kPcOwnBlk, pc_own_levels(0), kPcOwnBlk, false, true, true, 0>(v, tab, scr + 16, lane, wave);
    sec_block<kPcOwnBlk, pc_own_levels(1), kPcOwnBlk, false, true, true, 1>(v, tab, scr + 24, lane, wave);
  }
  __syncthreads();  // every thread has its block in registers
#pragma unroll
  for (int k = 0; k < kPcOwnBlk; ++k) sp[kPcOwnBlk * t + k] = v[k];
  __syncthreads();
  // FIR gamma: u3 index k = 9t + r (output m0 - 128 + k) from z2 local [2k + 276, 2k + 332]
  v2f u[9];
#pragma unroll
  for (int r = 0; r < 9; ++r) u[r] = splat(0.f);
  if constexpr (kKo & 2) {
#pragma unroll
    for (int r = 0; r < 9; ++r) u[r] = sp[18 * t + 2 * r + 304];
  } else {
    // zoom 8: g2 (57 taps) on z2; zoom 4: g1 (41 taps) on z1; zoom 2: g (25 taps) on z
    constexpr int G = ZOOM == 2 ? kPc2G : ZOOM == 4 ? kPc4G1 : kPcG2;
    const auto taps = [&]() {
      if constexpr (ZOOM == 8) return tab->g2;
      else if constexpr (ZOOM == 4) return tab->g1;
      else return tab->g;
    };
    // tap u multiplies z[2 m + u - C]: centred (C = (G - 1) / 2), or M's z^-8 .. z^16 at zoom 2
    constexpr int C = ZOOM == 2 ? -kPc2M0 : (G - 1) / 2;
    const LP zb = sp + 18 * t + (kPcK2Left - 2 * kU3Base) - C;
#pragma unroll
    for (int p = 0; p < (G + 17) / 2; ++p) {
      const int j = 2 * p;
      const v4f w = *(LP4)(zb + j);
      const v2f x0 = lo2(w), x1 = hi2(w);
#pragma unroll
      for (int r = 0; r < 9; ++r) fir_pair<G>(u[r], taps(), j - 2 * r, x0, x1);
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 9; ++r) sp[9 * t + r] = u[r];
  __syncthreads();
  // output-rate sections: wave q takes outputs [512 q, + 512) with 64-sample halos, u3
  // index k = 64 + 512 q + 10 lane + i; zoom 2: anticausal only (XA's backward pass at half
  // rate), so no lower halo and a 128-sample upper one (.874^128 = 3.2e-8)
  {
    v2f a[kPcApBlk];
    const int k0 = kU3Base - (ZOOM == 2 ? 0 : kPcApHalo) + (kPcK2M / 4) * wave + kPcApBlk * lane;
#pragma unroll
    for (int i = 0; i < kPcApBlk; ++i) a[i] = sp[k0 + i];
    if constexpr (ZOOM == 2) {
      ap_cascade<0, false>(a, tab, lane);
    } else if constexpr (!(kKo & 4)) {
      ap_cascade<0, true>(a, tab, lane);
      ap_cascade<0, false>(a, tab, lane);
    }
    __syncthreads();  // every wave has read its (overlapping) u3 range
#pragma unroll
    for (int i = 0; i < kPcApBlk; ++i) {
      const int k = k0 + i - kU3Base;  // output index within the tile
      const int q = k - (kPcK2M / 4) * wave;
      if (q >= 0 && q < kPcK2M / 4) sp[kOutOff + k] = a[i];
    }
  }
  __syncthreads();
  v2f *ob = out + f * n3;
  for (int s = t; s < kPcK2M; s += 256)
    if (m0 + s < n3) ob[m0 + s] = sp[kOutOff + s];
}

// ---------------------------------------------------------------------------------- KW

// sec_block for KW: own-rate section SI (causal: table wf, B = 16; anticausal: wb, B = 20)
// over the 4 waves' lane blocks, the waves continuing each other; the first wave in time
// order enters with (c0, c1): the state carried from the previous tile (causal) or 0.
template <int B, int LEV, bool UP, int SI, class TP>
__device__ __forceinline__ void wsec(v2f (&v)[B], TP tab0, LP scr, int lane, int wave, v2f c0, v2f c1) {
  const TP tab = fresh(tab0);
  CS S = UP ? tab->wf[SI] : tab->wb[SI];
  // this lane's cross-wave factors A^(B (dist + 1)), loaded first: the run hides their latency
  const int dist = UP ? lane : 63 - lane;
  typedef float v4u __attribute__((ext_vector_type(4), aligned(4)));
  const v4f xw = *(const v4u __attribute__((address_space(4))) *)(UP ? &tab->wf_x[SI][dist][0] : &tab->wb_x[SI][dist][0]);
  const v2f na1 = splat(-S.a1), na2 = splat(-S.a2);
  v2f y1 = splat(0.f), y2 = splat(0.f);
#pragma unroll
  for (int c = 0; c < B; ++c) {
    const int k = UP ? c : B - 1 - c;
    const v2f y = vfma(na1, y1, vfma(na2, y2, v[k]));
    y2 = y1;
    y1 = y;
    v[k] = y;
  }
  v2f e0 = y1, e1 = y2;
#pragma unroll
  for (int d = 0; d < LEV; ++d) {
    v2f p0, p1;
    if (d == 0) p0 = wshift<UP>(e0), p1 = wshift<UP>(e1);
    else if (d == 1) p0 = shiftk<UP, 2>(e0, lane), p1 = shiftk<UP, 2>(e1, lane);
    else if (d == 2) p0 = shiftk<UP, 4>(e0, lane), p1 = shiftk<UP, 4>(e1, lane);
    else if (d == 3) p0 = shiftk<UP, 8>(e0, lane), p1 = shiftk<UP, 8>(e1, lane);
    else p0 = shiftk<UP, 16>(e0, lane), p1 = shiftk<UP, 16>(e1, lane);
    const v2f n0 = fma2(&S.pw[d][0], p0, p1, e0);
    e1 = fma2(&S.pw[d][2], p0, p1, e1);
    e0 = n0;
  }
  if (lane == (UP ? 63 : 0)) {
    scr[2 * wave] = e0;
    scr[2 * wave + 1] = e1;
  }
  __syncthreads();
  const int src = UP ? wave - 1 : wave + 1;
  v2f s0 = c0, s1 = c1;
  if (src >= 0 && src < 4) {
    s0 = scr[2 * src];
    s1 = scr[2 * src + 1];
  }
  {
    const v2f n0 = vfma(splat(xw.x), s0, vfma(splat(xw.y), s1, e0));
    e1 = vfma(splat(xw.z), s0, vfma(splat(xw.w), s1, e1));
    e0 = n0;
  }
  v2f i0 = wshift<UP>(e0), i1 = wshift<UP>(e1);
  if (lane == (UP ? 0 : 63)) {
    i0 = s0;
    i1 = s1;
  }
#pragma unroll
  for (int c = 0; c < B; ++c) {
    const int k = UP ? c : B - 1 - c;
    v[k] = fma2(&S.ct[c][0], i0, i1, v[k]);
  }
}

constexpr int kWZ = 256 * kPcWb;  // own-rate samples held: span s in [256, 5376)
// Until the anticausal pass reads them, the own-rate samples sit in a padded layout, one
// 16-B pad after every 32 (i -> i + 2 (i / 32)): the causal pass's lane blocks of 16 are
// 128 B apart, 8-way conflicts on every ds_read_b128 / ds_write_b128 of the plain layout and
// none in this one.  The anticausal pass writes its outputs back in the plain layout, which
// FIR gamma reads.
constexpr int kWZP = kWZ + 2 * (kWZ / 32);
__device__ __forceinline__ int zp(int i) { return i + ((i >> 5) << 1); }
static_assert(kWZ == kPcK2Span - 256 && 256 * kPcWf == 4 * kPcWQ, "KW geometry");
static_assert(kOutOff + kPcK2M <= kXRows * kXRow, "KW: u3 + outputs fit the input tile's LDS");

// One workgroup per frame, tiles in order.  Tile tau: outputs [m0, m0 + 2048), m0 = -368 +
// 2048 tau, K2's span origin 2 m0 - 560 (span index s); its FIR part makes y2 for s in
// [1280, 5376) (= [4096 tau - 16, + 4096)), four sub-tiles of 1024 from 4128 input samples
// each (the y1 they share carried in LDS); the causal sections run on those 4096 with the
// state carried from the previous tile; the anticausal ones on s in [256, 5376) from a zero
// state at the top (s >= 4938 is warm-up only: 0.935^438 < 1e-12), whose lower 1024 are the
// previous tile's top causal outputs; then K2's FIR gamma and output-rate sections.
// ZOOM = 4 (PcTab4): the same walk one stage shorter -- per tile two sub-tiles of 2048 y1 (the
// same 4128-sample input tile and FIR alpha) written straight into the own-rate span (y1 is
// zoom 4's own-rate signal), then the own-rate sections, FIR g1 (41 taps, gamma's place) and
// 6 output-rate sections.
template <int ZOOM> struct WalkZ;
template <> struct WalkZ<8> {
  typedef CT Tab;
  static constexpr int SUB = 4, WM0 = kPcWM0, G = kPcG2;
  // sub-tile g's first input sample (y2 from 2 m0 + 720 + 1024 c, the y1 carry of 48 below it)
  static __device__ __forceinline__ int64_t xs_of(int g) { return 4 * (2 * (int64_t)WM0 + 720 + (int64_t)kPcWQ * g) + 32; }
};
template <> struct WalkZ<4> {
  typedef CT4 Tab;
  static constexpr int SUB = 2, WM0 = kPc4WM0, G = kPc4G1;
  // y1 local i <-> m = xs / 2 + 8 + i; sub-tile g makes y1 from 2 m0 + 720 + 2048 c
  static __device__ __forceinline__ int64_t xs_of(int g) { return 2 * (2 * (int64_t)WM0 + 720 + 2048 * (int64_t)g) - 16; }
};
template <int DT, int FLIP, int ZOOM>
__global__ void __launch_bounds__(256)
#if PC_OCC3
__attribute__((amdgpu_waves_per_eu(3)))
#endif
pc_walk_kernel(InDesc in, const v2f *lo, v2f *out, int64_t n3, typename WalkZ<ZOOM>::Tab tab) {
  using Z = WalkZ<ZOOM>;
#if PC_OCC3
  __shared__ v4f xl4[(kWZP > kXRows * kXRow ? kWZP : kXRows * kXRow) / 2];
  v4f __attribute__((address_space(3))) *z4 = (v4f __attribute__((address_space(3))) *)xl4;
#else
  __shared__ v4f xl4[kXRows * kXRow / 2];  // K1 input tile, then y1; then u3 + staged outputs
  __shared__ v4f z4[kWZP / 2];             // own-rate samples, span s in [256, 5376)
#endif
  __shared__ v4f scr4[16];                 // cross-wave states (4 section calls)
  __shared__ v4f car4[2];                  // causal sections' carried states
  __shared__ v4f y1c4[24];                 // the 48 y1 two sub-tiles share
  const LP xl = (LP)xl4, zl = (LP)z4, scr = (LP)scr4, car = (LP)car4;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t f = blockIdx.x, L = in.len;
  const v2f *lor = lo_row(lo, in, f);
  const v4f lane_lo = *(const v4f *)(lor + 2 * t) * (float)M_SQRT1_2;
  for (int i = t; i < kPcWQ; i += 256) zl[zp(i)] = splat(0.f);
  if (t < 24) y1c4[t] = v4f{0.f, 0.f, 0.f, 0.f};
  if (t < 2) car4[t] = v4f{0.f, 0.f, 0.f, 0.f};
  const int ntiles = (int)((n3 - Z::WM0 + kPcWM - 1) / kPcWM);
  // sub-tile g's first input sample; inside the frame ("fast") its pairs are prefetched into
  // registers one sub-tile ahead (the first of a tile during the previous tile's sections)
  auto xs_of = [&](int g) { return Z::xs_of(g); };
  auto fast = [&](int64_t xs) { return PC_CENSUS || (xs >= 0 && xs + kPcK1In <= L); };
  typename RawP<DT>::T pf[9];
  auto prefetch = [&](int g) {
    const int64_t xs = xs_of(g);
    if (g < Z::SUB * ntiles && fast(xs) && !(kKo & 32)) {
#pragma unroll
      for (int i = 0; i < 9; ++i)
        if (i < 8 || t < (kPcK1In - 4096) / 2) pf[i] = raw_pair<DT, FLIP>(in, f, xs + 2 * t + 512 * i);
    }
  };
  prefetch(0);
  // the LO table entries the fast sub-tiles of tile tau mix with, lo[xs_of(4 tau) + 512 k] for
  // k = 8 c + i in [0, 32] (sub-tile c, chunk i): lane k holds entry k, loaded a tile ahead and
  // read with v_readlane (a load per chunk at its use exposed the table's round trip in every
  // sub-tile); clamped into the frame, which only the unused entries of edge tiles need
  auto lo_chunks = [&](int tau_) -> v2f {
    const int64_t n = xs_of(Z::SUB * tau_) + 512 * (int64_t)min(lane, 8 * Z::SUB);
    return lor[n < 0 ? 0 : (n >= L ? L - 1 : n)];
  };
  v2f lo_nx = lo_chunks(0);
#if PC_STAMPS
  unsigned long long st_acc[kPcStampSegs] = {}, t_prev;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_prev)::"memory");
#endif
  for (int tau = 0; tau < ntiles; ++tau) {
    const int64_t m0 = Z::WM0 + (int64_t)kPcWM * tau;
    const v2f lo_cur = lo_nx;
    if (tau + 1 < ntiles) lo_nx = lo_chunks(tau + 1);
    // ---- FIRs: y2 for s in [1280, 5376), four sub-tiles
    walk_prio(false);
    for (int c = 0; c < Z::SUB; ++c) {
      const int64_t xs = xs_of(Z::SUB * tau + c);  // first input sample
      if (fast(xs)) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
          const int s = 2 * t + 512 * i;
          if (i == 8 && t >= (kPcK1In - 4096) / 2) break;
          v2f a, b;
          cvt_pair<DT, FLIP>(pf[i], a, b);
          const v2f cc = lane_val(lo_cur, 8 * c + i);  // lo[xs + 512 i]
          *(LP4)(xl + xidx(s)) = cat(cmul2(a, cmul2s(cc, lo2(lane_lo))), cmul2(b, cmul2s(cc, hi2(lane_lo))));
        }
      } else {
        for (int s = t; s < kPcK1In; s += 256) {
          const int64_t n = xs + s;
          v2f v = splat(0.f);
          if (n >= 0 && n < L) v = cmul2(load_in_t<DT, FLIP>(in, f, n), lor[n]);
          xl[xidx(s)] = v;
        }
      }
      // one call site for both paths: the loads land in the same registers on either, so the
      // compiler's wait tracking has no stale load to drain (two call sites made it put a
      // vmcnt(0) right behind the barrier, exposing every prefetch's round trip); the next
      // tile's first sub-tile is fetched after the own-rate sections' table loads instead
      if (c + 1 < Z::SUB) prefetch(Z::SUB * tau + c + 1);
      PC_STAMP(9);  // (stamp segment 9: the mix and x to LDS; segment 0 then the barrier wait)
      if constexpr (!(kKo & 64)) __syncthreads();
      PC_STAMP(0);
      v2f acc[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) acc[r] = splat(0.f);
      {
        const LP xb = xl + t * kXRow;
#pragma unroll
        for (int p = 0; p < ((kKo & 16) ? 1 : 24); ++p) {
          const int j = 2 * p;
          const v4f w = *(LP4)(xb + (j >> 4) * kXRow + (j & 15));
          const v2f x0 = lo2(w), x1 = hi2(w);
#pragma unroll
          for (int r = 0; r < 8; ++r) fir_pair<kPcG0>(acc[r], tab->g0, j - 2 * r, x0, x1);
        }
      }
      if constexpr (!(kKo & 128)) __syncthreads();
      PC_STAMP(1);
      if constexpr (ZOOM == 4) {  // y1 local 8 t + r -> span index 1280 + 2048 c + 8 t + r
        const LP zo = zl + zp(kPcWQ + 2048 * c + 8 * t);  // 8 never straddle a pad
#pragma unroll
        for (int q = 0; q < 4; ++q) *(LP4)(zo + 2 * q) = cat(acc[2 * q], acc[2 * q + 1]);
        continue;  // the next sub-tile's input overwrites xl: every alpha read is done
      } else {
      // y1 local i <-> 2 Q - 24 + i: [0, 48) carried, thread t's 8 at 48 + 8 t (row 6 + t)
      const LP yl = xl;
      if (t < 24) *(LP4)(yl + (t >> 2) * kYRow + 2 * (t & 3)) = y1c4[t];
#pragma unroll
      for (int q = 0; q < 4; ++q) *(LP4)(yl + (6 + t) * kYRow + 2 * q) = cat(acc[2 * q], acc[2 * q + 1]);
      if constexpr (!(kKo & 128)) __syncthreads();
      PC_STAMP(2);
      {
        v2f b[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) b[r] = splat(0.f);
        const LP yb = yl + t * kYRow;
#pragma unroll
        for (int p = 0; p < ((kKo & 16) ? 1 : 28); ++p) {
          const int j = 2 * p;
          const v4f w = *(LP4)(yb + (j >> 3) * kYRow + (j & 7));
          const v2f x0 = lo2(w), x1 = hi2(w);
#pragma unroll
          for (int r = 0; r < 4; ++r) fir_pair<kPcG1>(b[r], tab->g1, j - 2 * r, x0, x1);
        }
        const LP zo = zl + zp(kPcWQ * (1 + c) + 4 * t);
        *(LP4)zo = cat(b[0], b[1]);
        *(LP4)(zo + 2) = cat(b[2], b[3]);
        if (t < 24) y1c4[t] = *(LP4)(yl + (256 + (t >> 2)) * kYRow + 2 * (t & 3));  // i = 2048 + 2 t
      }
      if constexpr (!(kKo & 64)) __syncthreads();
      PC_STAMP(3);
      }
    }
    if constexpr (ZOOM == 4) __syncthreads();  // the span's new y1 are in
    // ---- own-rate sections, causal, on the new 4096 (carried states)
    walk_prio(true);
    {
      v2f v[kPcWf];
      const LP zb = zl + zp(kPcWQ + kPcWf * t);  // a block of 16 never straddles a pad
#pragma unroll
      for (int k = 0; k < kPcWf; ++k) v[k] = zb[k];
      if constexpr (!(kKo & 1)) {
        const v2f c0 = car[0], c1 = car[1], c2 = car[2], c3 = car[3];
        wsec<kPcWf, pc_wf_levels(0), true, 0>(v, tab, scr, lane, wave, c0, c1);
        if (t == 255) {
          car[0] = v[kPcWf - 1];
          car[1] = v[kPcWf - 2];
        }
        wsec<kPcWf, pc_wf_levels(1), true, 1>(v, tab, scr + 8, lane, wave, c2, c3);
        if (t == 255) {
          car[2] = v[kPcWf - 1];
          car[3] = v[kPcWf - 2];
        }
      }
#pragma unroll
      for (int k = 0; k < kPcWf; ++k) zb[k] = v[k];
    }
    __syncthreads();
    PC_STAMP(4);
    // the next tile's lower 1024 causal outputs (s in [4352, 5376) -> [256, 1280))
    v2f cz[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) cz[r] = zl[zp(4 * kPcWQ + 4 * t) + r];
    // ---- own-rate sections, anticausal, on s in [256, 5376)
    {
      v2f v[kPcWb];
#pragma unroll
      for (int k = 0; k < kPcWb; k += 2) {  // padded layout (pairs never straddle a pad)
        const v4f w = *(LP4)(zl + zp(kPcWb * t + k));
        v[k] = lo2(w);
        v[k + 1] = hi2(w);
      }
      const LP zb = zl + kPcWb * t;  // written back in the plain layout
      __syncthreads();  // cz and every block read before anything is written back
      if constexpr (!(kKo & 1)) {
        wsec<kPcWb, pc_wb_levels(0), false, 0>(v, tab, scr + 16, lane, wave, splat(0.f), splat(0.f));
        wsec<kPcWb, pc_wb_levels(1), false, 1>(v, tab, scr + 24, lane, wave, splat(0.f), splat(0.f));
      }
#pragma unroll
      for (int k = 0; k < kPcWb; ++k) zb[k] = v[k];
    }
    prefetch(Z::SUB * (tau + 1));  // overlaps FIR gamma, the output-rate sections and the stores
    __syncthreads();
    PC_STAMP(5);
    // ---- FIR gamma (K2's): u3 index k = 9 t + r (output m0 - 128 + k) from z s in [2k + 276, + 56]
    walk_prio(false);
    {
      v2f u[9];
#pragma unroll
      for (int r = 0; r < 9; ++r) u[r] = splat(0.f);
      // zoom 8: g2 (57 taps) on z2 at rate 1/4; zoom 4: g1 (41 taps) on z1 at rate 1/2
      constexpr int G = Z::G;
      const auto taps = [&]() {
        if constexpr (ZOOM == 8) return tab->g2;
        else return tab->g1;
      };
      const LP zb = zl + 18 * t + (kPcK2Left - 2 * kU3Base) - (G - 1) / 2 - 256;
#pragma unroll
      for (int p = 0; p < ((kKo & 2) ? 1 : (G + 17) / 2); ++p) {
        const int j = 2 * p;
        const v4f w = *(LP4)(zb + j);
        const v2f x0 = lo2(w), x1 = hi2(w);
#pragma unroll
        for (int r = 0; r < 9; ++r) fir_pair<G>(u[r], taps(), j - 2 * r, x0, x1);
      }
#pragma unroll
      for (int r = 0; r < 9; ++r) xl[9 * t + r] = u[r];
    }
    __syncthreads();
    PC_STAMP(6);
#pragma unroll
    for (int r = 0; r < 4; ++r) zl[zp(4 * t) + r] = cz[r];
    // ---- output-rate sections (K2's: wave q takes outputs [512 q, + 512) with halos)
    walk_prio(true);
    {
      v2f a[kPcApBlk];
      const int k0 = kU3Base - kPcApHalo + (kPcK2M / 4) * wave + kPcApBlk * lane;
#pragma unroll
      for (int i = 0; i < kPcApBlk; ++i) a[i] = xl[k0 + i];
      if constexpr (!(kKo & 4)) {
        ap_cascade<0, true>(a, tab, lane);
        ap_cascade<0, false>(a, tab, lane);
      }
      PC_STAMP(7);
#pragma unroll
      for (int i = 0; i < kPcApBlk; ++i) {
        const int k = k0 + i - kU3Base;
        const int q = k - (kPcK2M / 4) * wave;
        if (q >= 0 && q < kPcK2M / 4) xl[kOutOff + k] = a[i];
      }
    }
    __syncthreads();
    v2f *ob = out + f * n3;
    for (int s = t; s < kPcK2M; s += 256) {
      const int64_t m = m0 + s;
      if (m >= 0 && m < n3) ob[m] = xl[kOutOff + s];
    }
    __syncthreads();
    PC_STAMP(8);
  }
#if PC_STAMPS
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < kPcStampSegs; ++i) atomicAdd(&g_pc_stamps[i], st_acc[i]);
    atomicAdd(&g_pc_stamps[kPcStampSegs], (unsigned long long)ntiles);
  }
#endif
}

// ---------------------------------------------------------------------------------- K3

// out[m] += sum_k U[m][k] (sum_j V[j][k] x[j]): side 0 from the frame start, side 1 from
// its end (x[j] = mixed input L-1-j, out index n3-1-m).  One block per frame and side; V is
// uploaded transposed (r x J) so a wave's V loads are coalesced.
template <int DT, int FLIP>
__global__ void __launch_bounds__(256) pc_edge_kernel(InDesc in, const v2f *lo, v2f *out, int64_t n3,
                                                      const float *U0, const float *V0, int R0, int J0,
                                                      int r0, const float *U1, const float *V1, int R1,
                                                      int J1, int r1) {
  __shared__ v2f red[4][kPcEdgeRank];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t f = blockIdx.x, L = in.len;
  const int side = blockIdx.y;
  const float *U = side ? U1 : U0, *V = side ? V1 : V0;
  const int R = side ? R1 : R0, J = side ? J1 : J0, r = side ? r1 : r0;
  const v2f *lor = lo_row(lo, in, f);
  v2f acc[kPcEdgeRank];
#pragma unroll
  for (int k = 0; k < kPcEdgeRank; ++k) acc[k] = splat(0.f);
  for (int j = t; j < J; j += 256) {
    const int64_t n = side ? L - 1 - j : j;
    const v2f x = cmul2(load_in_t<DT, FLIP>(in, f, n), lor[n]);
#pragma unroll
    for (int k = 0; k < kPcEdgeRank; ++k)
      if (k < r) acc[k] = vfma(splat(V[(int64_t)k * J + j]), x, acc[k]);  // V stored r x J
  }
#pragma unroll
  for (int k = 0; k < kPcEdgeRank; ++k) {
    v2f a = acc[k];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) a += shxor(a, d);
    if (lane == 0) red[wave][k] = a;
  }
  __syncthreads();
  if (t < R) {
    v2f c = splat(0.f);
    for (int k = 0; k < r; ++k)
      c = vfma(splat(U[t * r + k]), red[0][k] + red[1][k] + red[2][k] + red[3][k], c);
    const int64_t m = side ? n3 - 1 - t : t;
    out[f * n3 + m] += c;
  }
}

// K3 split for the walk: KV makes v = V^T x for every frame end on a side
// stream while the walk runs -- one wave per (frame, side, 4 ranks), no LDS and few VGPRs, so its
// waves fit beside the walk's two workgroups per CU and use issue slots the walk leaves idle --
// and KU adds U v to the walk's output once both are done (a tiny launch).  Same sums as K3.
constexpr int kEdgeRanksPerWave = 4;
template <int DT, int FLIP>
__global__ void __launch_bounds__(64) pc_edge_v_kernel(InDesc in, const v2f *lo, v2f *vout,
                                                       const float *V0, int J0, int r0,
                                                       const float *V1, int J1, int r1) {
  const int lane = threadIdx.x;
  const int64_t f = blockIdx.x, L = in.len;
  const int side = blockIdx.y, k0 = kEdgeRanksPerWave * blockIdx.z;
  const float *V = side ? V1 : V0;
  const int J = side ? J1 : J0, r = side ? r1 : r0;
  if (k0 >= r) return;  // wave-uniform
  const v2f *lor = lo_row(lo, in, f);
  v2f acc[kEdgeRanksPerWave];
#pragma unroll
  for (int k = 0; k < kEdgeRanksPerWave; ++k) acc[k] = splat(0.f);
  for (int j = lane; j < J; j += 64) {
    const int64_t n = side ? L - 1 - j : j;
    const v2f x = cmul2(load_in_t<DT, FLIP>(in, f, n), lor[n]);
#pragma unroll
    for (int k = 0; k < kEdgeRanksPerWave; ++k)
      if (k0 + k < r) acc[k] = vfma(splat(V[(int64_t)(k0 + k) * J + j]), x, acc[k]);
  }
#pragma unroll
  for (int k = 0; k < kEdgeRanksPerWave; ++k) {
    v2f a = acc[k];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) a += shxor(a, d);
    if (lane == 0 && k0 + k < r) vout[(f * 2 + side) * kPcEdgeRank + k0 + k] = a;
  }
}
// out[m] += sum_k U[m][k] v[k] at both ends: one block per frame, thread t < R0 the start's
// output t, thread 192 + t < 192 + R1 the end's output n3 - 1 - t
__global__ void __launch_bounds__(384) pc_edge_u_kernel(const v2f *vin, v2f *out, int64_t n3,
                                                        const float *U0, int R0, int r0,
                                                        const float *U1, int R1, int r1) {
  const int side = threadIdx.x >= kPcEdgeR, t = threadIdx.x - (side ? kPcEdgeR : 0);
  const int R = side ? R1 : R0, r = side ? r1 : r0;
  if (t >= R) return;
  const int64_t f = blockIdx.x;
  const float *U = side ? U1 : U0;
  const v2f *v = vin + (f * 2 + side) * kPcEdgeRank;
  v2f c = splat(0.f);
  for (int k = 0; k < r; ++k) c = vfma(splat(U[t * r + k]), v[k], c);
  const int64_t m = side ? n3 - 1 - t : t;
  out[f * n3 + m] += c;
}

}  // namespace pc

// Debug hook (not part of zfft.h): copies and clears the walk's stamp sums of a PC_STAMPS build
// (segment cycles summed over waves, then the tile count summed over workgroups); -1 otherwise.
extern "C" int zfft_debug_pc_stamps(unsigned long long *out) {
#if PC_STAMPS
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pc::g_pc_stamps), sizeof(pc::g_pc_stamps)) != hipSuccess) return -2;
  unsigned long long z[pc::kPcStampSegs + 1] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(pc::g_pc_stamps), z, sizeof(z)) == hipSuccess ? 0 : -2;
#else
  (void)out;
  return -1;
#endif
}

#define PC_LAUNCH2(KERNEL, DT, fl, ...)                                                         \
  do {                                                                                           \
    if (fl) hipLaunchKernelGGL((KERNEL<DT, 1>), __VA_ARGS__);                                    \
    else hipLaunchKernelGGL((KERNEL<DT, 0>), __VA_ARGS__);                                       \
  } while (0)
#define PC_DISPATCH(KERNEL, in, ...)                                                             \
  do {                                                                                           \
    const bool fl = (in).flip != 0;                                                              \
    switch ((in).dtype) {                                                                        \
      case kInC64: PC_LAUNCH2(KERNEL, kInC64, fl, __VA_ARGS__); break;                           \
      case kInC32H: PC_LAUNCH2(KERNEL, kInC32H, fl, __VA_ARGS__); break;                         \
      case kInCU8: PC_LAUNCH2(KERNEL, kInCU8, fl, __VA_ARGS__); break;                           \
      default: PC_LAUNCH2(KERNEL, kInF32R, fl, __VA_ARGS__); break;                              \
    }                                                                                            \
  } while (0)

#define PC_LAUNCH2Z(KERNEL, DT, fl, Z, ...)                                                     \
  do {                                                                                           \
    if (fl) hipLaunchKernelGGL((KERNEL<DT, 1, Z>), __VA_ARGS__);                                 \
    else hipLaunchKernelGGL((KERNEL<DT, 0, Z>), __VA_ARGS__);                                    \
  } while (0)
#define PC_DISPATCH_Z(KERNEL, Z, in, ...)                                                        \
  do {                                                                                           \
    const bool fl = (in).flip != 0;                                                              \
    switch ((in).dtype) {                                                                        \
      case kInC64: PC_LAUNCH2Z(KERNEL, kInC64, fl, Z, __VA_ARGS__); break;                       \
      case kInC32H: PC_LAUNCH2Z(KERNEL, kInC32H, fl, Z, __VA_ARGS__); break;                     \
      case kInCU8: PC_LAUNCH2Z(KERNEL, kInCU8, fl, Z, __VA_ARGS__); break;                       \
      default: PC_LAUNCH2Z(KERNEL, kInF32R, fl, Z, __VA_ARGS__); break;                          \
    }                                                                                            \
  } while (0)

hipError_t launch_pc_fir(const InDesc &in, const float2 *lo, float2 *y2, int64_t y2_stride,
                         int frames, const PcTab *tab, hipStream_t st) {
  const int ntiles = (int)((pc_y2_len(in.len) + kPcK1Q - 1) / kPcK1Q);
  const dim3 grid(ntiles, frames);
  const pc::CT ct = (pc::CT)tab;
  PC_DISPATCH_Z(pc::pc_fir_kernel, 8, in, grid, dim3(256), 0, st, in, (const v2f *)lo, (v2f *)y2,
                y2_stride, ct);
  return hipGetLastError();
}

hipError_t launch_pc_tail(const float2 *y2, int64_t y2_stride, float2 *out, int64_t n3,
                          int frames, const PcTab *tab, hipStream_t st) {
  const dim3 grid((unsigned)((n3 + kPcK2M - 1) / kPcK2M), frames);
  hipLaunchKernelGGL((pc::pc_tail_kernel<8>), grid, dim3(256), 0, st, (const v2f *)y2, y2_stride,
                     y2_stride, (v2f *)out, n3, (pc::CT)tab, InDesc{}, (const v2f *)nullptr);
  return hipGetLastError();
}

hipError_t launch_pc4_fir(const InDesc &in, const float2 *lo, float2 *y1, int64_t y1_stride,
                          int frames, const PcTab4 *tab, hipStream_t st) {
  const dim3 grid((unsigned)((pc4_y1_len(in.len) + kPc4K1M - 1) / kPc4K1M), frames);
  PC_DISPATCH_Z(pc::pc_fir_kernel, 4, in, grid, dim3(256), 0, st, in, (const v2f *)lo, (v2f *)y1,
                y1_stride, (pc::CT4)tab);
  return hipGetLastError();
}

hipError_t launch_pc4_tail(const float2 *y1, int64_t y1_stride, int64_t y1n, float2 *out, int64_t n2,
                           int frames, const PcTab4 *tab, hipStream_t st) {
  const dim3 grid((unsigned)((n2 + kPcK2M - 1) / kPcK2M), frames);
  hipLaunchKernelGGL((pc::pc_tail_kernel<4>), grid, dim3(256), 0, st, (const v2f *)y1, y1_stride, y1n,
                     (v2f *)out, n2, (pc::CT4)tab, InDesc{}, (const v2f *)nullptr);
  return hipGetLastError();
}

#define PC_LAUNCH_TAIL2(DT, fl, ...)                                                            \
  do {                                                                                           \
    if (fl) hipLaunchKernelGGL((pc::pc_tail_kernel<2, DT, 1>), __VA_ARGS__);                     \
    else hipLaunchKernelGGL((pc::pc_tail_kernel<2, DT, 0>), __VA_ARGS__);                        \
  } while (0)
hipError_t launch_pc2_tail(const InDesc &in, const float2 *lo, float2 *out, int64_t n1, int frames,
                           const PcTab2 *tab, hipStream_t st) {
  const dim3 grid((unsigned)((n1 + kPcK2M - 1) / kPcK2M), frames);
  const bool fl = in.flip != 0;
#define PC_TAIL2_ARGS grid, dim3(256), 0, st, (const v2f *)nullptr, (int64_t)0, (int64_t)0, (v2f *)out, n1, \
                      (pc::CT2)tab, in, (const v2f *)lo
  switch (in.dtype) {
    case kInC64: PC_LAUNCH_TAIL2(kInC64, fl, PC_TAIL2_ARGS); break;
    case kInC32H: PC_LAUNCH_TAIL2(kInC32H, fl, PC_TAIL2_ARGS); break;
    case kInCU8: PC_LAUNCH_TAIL2(kInCU8, fl, PC_TAIL2_ARGS); break;
    default: PC_LAUNCH_TAIL2(kInF32R, fl, PC_TAIL2_ARGS); break;
  }
#undef PC_TAIL2_ARGS
  return hipGetLastError();
}

hipError_t launch_pc_walk(const InDesc &in, const float2 *lo, float2 *out, int64_t n3, int frames,
                          const PcTab *tab, hipStream_t st) {
  PC_DISPATCH_Z(pc::pc_walk_kernel, 8, in, dim3((unsigned)frames), dim3(256), 0, st, in, (const v2f *)lo,
                (v2f *)out, n3, (pc::CT)tab);
  return hipGetLastError();
}

hipError_t launch_pc_walk4(const InDesc &in, const float2 *lo, float2 *out, int64_t n2, int frames,
                           const PcTab4 *tab, hipStream_t st) {
  PC_DISPATCH_Z(pc::pc_walk_kernel, 4, in, dim3((unsigned)frames), dim3(256), 0, st, in, (const v2f *)lo,
                (v2f *)out, n2, (pc::CT4)tab);
  return hipGetLastError();
}

hipError_t launch_pc_edge_v(const InDesc &in, const float2 *lo, float2 *v, int frames,
                            const float *const V[2], const int J[2], const int r[2], hipStream_t st) {
  const dim3 grid(frames, 2, (kPcEdgeRank + pc::kEdgeRanksPerWave - 1) / pc::kEdgeRanksPerWave);
  PC_DISPATCH(pc::pc_edge_v_kernel, in, grid, dim3(64), 0, st, in, (const v2f *)lo, (v2f *)v, V[0], J[0],
              r[0], V[1], J[1], r[1]);
  return hipGetLastError();
}

hipError_t launch_pc_edge_u(const float2 *v, float2 *out, int64_t n3, int frames, const float *const U[2],
                            const int R[2], const int r[2], hipStream_t st) {
  hipLaunchKernelGGL(pc::pc_edge_u_kernel, dim3(frames), dim3(2 * kPcEdgeR), 0, st, (const v2f *)v,
                     (v2f *)out, n3, U[0], R[0], r[0], U[1], R[1], r[1]);
  return hipGetLastError();
}

hipError_t launch_pc_edge(const InDesc &in, const float2 *lo, float2 *out, int64_t n3, int frames,
                          const float *const U[2], const float *const V[2], const int R[2],
                          const int J[2], const int r[2], hipStream_t st) {
  const dim3 grid(frames, 2);
  PC_DISPATCH(pc::pc_edge_kernel, in, grid, dim3(256), 0, st, in, (const v2f *)lo, (v2f *)out, n3,
              U[0], V[0], R[0], J[0], r[0], U[1], V[1], R[1], J[1], r[1]);
  return hipGetLastError();
}

}  // namespace zfft
