// xt_kernels.hip -- exact-tile ("XT") zero-phase decimation stage for gfx950.
//
// One stage of the reference's decimate(x, 2) (pypanadapter_spectrum.py:2096-2098 ->
// scipy sosfiltfilt: odd pad 27, zi initial conditions, forward + backward, [::2]) on one
// frame per wave, reading the stage input once and writing only the decimated output:
// no forward-pass intermediate ever reaches memory.
//
// A wave walks its frame in tiles of 1024 samples; lane i owns the 16-sample sub-block i.
//  forward (exact):  every lane runs the cascade from a zero state over its sub-block;
//                    its end state goes to the real modal basis of A (T^-1, block lower
//                    triangular), where a sub-block step is one complex multiply per
//                    mode; a Kogge-Stone scan over the lanes, per mode only as deep as its
//                    pole radius needs (.587 .682 .808 .935 -> 2 2 3 5 levels,
//                    |lambda|^(16*2^L) < 1e-9), gives each lane its entering state (the
//                    tile's entering state folded into lane 0), and the outputs are
//                    corrected by C A^t T m_in.
//  backward:         the same over the forward outputs in descending order, with the
//                    state entering the tile from above provisionally zero.  The state
//                    this leaves at the tile bottom is exact anyway (its dependence on the
//                    top state is lambda^1024 < 1e-29), and it is precisely the top state
//                    of the tile below, which was processed one step earlier: its kept
//                    outputs get C A^(15-t) T lambda^(16 (63-lane)) q, then are stored.
//  frame ends:       forward starts from zi * ext[0]; the last tile's backward starts from
//                    zi * y[e-1] with a constant y[e-1] tail above e-1 (the steady state
//                    is a fixed point of the recursion), exactly scipy's initial condition.
// Numerics: float32; tools/xt_modal_proto.py models the schedule (fp32 max relative error
// vs float64 sosfiltfilt 9.5e-7 on white noise; plain float32 sosfiltfilt 5.8e-7).
#include "zfft_device.h"

namespace zfft {

constexpr int kXtLdsStride = kXtB + 1;      // padded sub-block rows: conflict-free ds_read_b64

// Build knobs (A/B of register allocation vs. constant refetch; defaults are the shipped
// choice): XT_WAVES = waves per SIMD the kernel is compiled for; XT_CM_GROUP = output rows
// per refetch of the C A^t T table; XT_SCAN_FRESH = refetch the scan coefficients per level.
#ifndef XT_WAVES
#define XT_WAVES 4
#endif
#ifndef XT_CM_GROUP
#define XT_CM_GROUP 1
#endif
#ifndef XT_SCAN_FRESH
#define XT_SCAN_FRESH 1
#endif
constexpr int kLevels[4] = {2, 2, 3, kXtScan};

struct Modal {
  v2f r[8];  // a0 b0 a1 b1 a2 b2 a3 b3 (complex: I and Q of the frame share the real basis)
};

__device__ __forceinline__ v2f sget(const IirState &s, int r) {
  return (r & 1) ? s.z1[r >> 1] : s.z0[r >> 1];
}

__device__ __forceinline__ float uni(float a) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(a)));
}
__device__ __forceinline__ v2f uni2(v2f v) { return v2f{uni(v.x), uni(v.y)}; }
__device__ __forceinline__ v2f lane_of(v2f v, int src) {  // value of lane src, uniform
  return v2f{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), src)),
             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), src))};
}
__device__ __forceinline__ v2f shfl2(v2f v, int src) {
  return v2f{__shfl(v.x, src, 64), __shfl(v.y, src, 64)};
}

// The table pointer laundered through an opaque (volatile) asm: loads through the result
// stay scalar (K$ hits) but cannot be hoisted above it, so each phase of the tile loop
// re-reads the few constants it needs instead of the compiler keeping every table entry
// live across the loop in SGPRs (and spilling them).
// Constant address space (AS4): reads of uniform addresses are s_load (the table is never
// written by a kernel), and the pointer keeps that property through the asm.
typedef const XtModal __attribute__((address_space(4))) *CTab;
__device__ __forceinline__ CTab fresh(CTab p) {
  asm volatile("" : "+s"(p));
  return p;
}

// Whole-wave DPP shift by one lane (GFX9 wave_shr:1 / wave_shl:1): lane i takes lane i-1
// (SHR) or i+1 (SHL); the lane without a source keeps `old`.  One VALU op per dword,
// instead of an LDS-routed ds_bpermute plus a select.
constexpr int kWaveShr1 = 0x138, kWaveShl1 = 0x130;
template <int CTRL>
__device__ __forceinline__ v2f wave_shift(v2f old, v2f src) {
  return v2f{__int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old.x), __float_as_int(src.x),
                                                        CTRL, 0xF, 0xF, false)),
             __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old.y), __float_as_int(src.y),
                                                        CTRL, 0xF, 0xF, false))};
}

__device__ __forceinline__ Sos32 load_sos(CTab t) {  // field-wise: scalar loads from AS4
  Sos32 c;
  c.b0 = t->sos.b0;
  c.b1 = t->sos.b1;
  c.b2 = t->sos.b2;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    c.a1[k] = t->sos.a1[k];
    c.a2[k] = t->sos.a2[k];
    c.zi[k][0] = t->sos.zi[k][0];
    c.zi[k][1] = t->sos.zi[k][1];
  }
  return c;
}

// (a, b) <- [[c, s], [-s, c]] (a, b): one mode times lambda^p = c + i s
__device__ __forceinline__ void rot(v2f &a, v2f &b, float c, float s) {
  const v2f na = vfma(splat(c), a, splat(s) * b);
  b = vfma(splat(c), b, splat(-s) * a);
  a = na;
}

// m = T^-1 z; T^-1 is block lower triangular (mode j depends on sections <= j)
__device__ __forceinline__ void to_modal(CTab tab, const IirState &z,
                                         Modal &m) {
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    CTab tb = fresh(tab);
    v2f acc = splat(0.f);
#pragma unroll
    for (int q = 0; q < (r | 1) + 1; ++q) acc = vfma(splat(tb->ti[r][q]), sget(z, q), acc);
    m.r[r] = acc;
  }
}

__device__ __forceinline__ v2f dot_cm(CTab tab, int t, const Modal &m,
                                      v2f acc) {
#pragma unroll
  for (int r = 0; r < 8; ++r) acc = vfma(splat(tab->cm[t][r]), m.r[r], acc);
  return acc;
}

// inclusive scan over lanes: UP (lane i accumulates lanes j <= i) or down (j >= i),
// m_i = sum_j lambda^(16 |i-j|) m_j per mode
template <bool UP>
__device__ __forceinline__ void modal_scan(Modal &m, CTab tab, int lane) {
  // an opaque copy of the lane id: the per-level masks and shuffle addresses below are
  // recomputed here (a few VALU ops) rather than hoisted into the loop preheader, where
  // they would pin ~20 SGPR pairs and VGPRs for the whole kernel
  asm volatile("" : "+v"(lane));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int d = 0; d < kLevels[j]; ++d) {
      CTab tb = XT_SCAN_FRESH ? fresh(tab) : tab;
      float c = tb->scan[d][j][0], sn = tb->scan[d][j][1];
      v2f pa, pb;
      if (d == 0) {  // neighbour lane: DPP shift, zero at the open end
        constexpr int ctrl = UP ? kWaveShr1 : kWaveShl1;
        pa = wave_shift<ctrl>(splat(0.f), m.r[2 * j]);
        pb = wave_shift<ctrl>(splat(0.f), m.r[2 * j + 1]);
      } else {       // distance 2^d: ds_bpermute, lanes without a source get coefficient 0
        const int sh = 1 << d;
        const bool take = UP ? lane >= sh : lane + sh <= 63;
        const int src = (UP ? lane - sh : lane + sh) & 63;
        pa = shfl2(m.r[2 * j], src);
        pb = shfl2(m.r[2 * j + 1], src);
        c = take ? c : 0.f;
        sn = take ? sn : 0.f;
      }
      rot(pa, pb, c, sn);
      m.r[2 * j] += pa;
      m.r[2 * j + 1] += pb;
    }
  }
}

template <bool MIX, int DT, int FLIP>  // DT, FLIP: input format (stage 0 reads the caller's frames)
__global__ __launch_bounds__(256, XT_WAVES) void xt_stage_kernel(InDesc in, int n,
                                                       const v2f *__restrict__ lo,
                                                       v2f *__restrict__ out, int frames,
                                                       const XtModal *tab_g,
                                                       Sos32 c) {
  const CTab tab = (CTab)tab_g;
  __shared__ __attribute__((aligned(16))) v2f lds_all[4][64 * kXtLdsStride];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int f = blockIdx.x * 4 + wv;
  if (f >= frames) return;  // whole wave
  v2f *lds = lds_all[wv];
  const int e = n + 2 * kPad, n_out = (n + 1) >> 1;
  v2f *__restrict__ o = out + (int64_t)f * n_out;
  auto X = [&](int i) -> v2f {
    v2f v = load_in_t<DT, FLIP>(in, f, i);
    if constexpr (MIX) v = cmul(v, lo[i]);
    return v;
  };
  auto ext = [&](int j) -> v2f {
    if (j < kPad) return 2.f * X(0) - X(kPad - j);
    if (j < n + kPad) return X(j - kPad);
    if (j < e) return 2.f * X(n - 1) - X(2 * n + kPad - 2 - j);
    return splat(0.f);
  };
  const int nt = (e + kXtT - 1) / kXtT;

  // per-lane powers lambda^(16 (63 - lane)): the held tile's lanes from its top state
  float lgc[4], lgs[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    lgc[j] = tab->lag[63 - lane][j][0];
    lgs[j] = tab->lag[63 - lane][j][1];
  }
  Modal m_in;  // modal state entering the current tile (forward), wave-uniform
  {
    const v2f x0 = uni2(ext(0));
#pragma unroll
    for (int r = 0; r < 8; ++r) m_in.r[r] = uni2(tab->zim[r] * x0);
  }
  v2f held[kXtHeld];  // previous tile's kept backward outputs, awaiting the lag correction

  auto store_kept = [&](int tile, const v2f *val) {  // decimated outputs -> frame row
#pragma unroll
    for (int k = 0; k < kXtHeld; ++k) lds[lane * (kXtHeld + 1) + k] = val[k];
    __builtin_amdgcn_wave_barrier();
    const int m0 = tile * (kXtT / 2) - (kPad - 1) / 2;  // m of (lane 0, k 0): j = 1024 tile + 1
#pragma unroll
    for (int q = 0; q < kXtHeld; ++q) {
      const int idx = lane + 64 * q;
      const int m = m0 + idx;
      const v2f v = lds[(idx / kXtHeld) * (kXtHeld + 1) + (idx % kXtHeld)];
      if (m >= 0 && m < n_out) o[m] = v;
    }
    __builtin_amdgcn_wave_barrier();
  };

  for (int tau = 0; tau < nt; ++tau) {
    const int base = tau * kXtT;
    // ---- tile -> LDS (coalesced: 64 consecutive samples per load instruction) ----
    const bool fast = base >= kPad && base + kXtT <= n + kPad;  // wave-uniform
    // sample s = lane + 64 q -> row s/16 = lane/16 + 4 q, column lane%16
    v2f *st = lds + (lane >> 4) * kXtLdsStride + (lane & 15);
    v2f lo0 = splat(0.f);
    if (fast) {
      // raw samples only: all 16 loads in flight at once (no per-load mixing in between);
      // the LO is applied after the transpose, per lane on consecutive samples
      if constexpr (MIX) lo0 = lo[base - kPad + kXtB * lane];
      v2f raw[kXtB];
#pragma unroll
      for (int q = 0; q < kXtB; ++q) raw[q] = load_in_t<DT, FLIP>(in, f, base - kPad + lane + 64 * q);
#pragma unroll
      for (int q = 0; q < kXtB; ++q) st[4 * kXtLdsStride * q] = raw[q];
    } else {  // frame edges: odd extension of the mixed signal, built sample by sample
#pragma unroll
      for (int q = 0; q < kXtB; ++q) st[4 * kXtLdsStride * q] = ext(base + lane + 64 * q);
    }
    __builtin_amdgcn_wave_barrier();
    v2f y[kXtB];
    const v2f *row = lds + lane * kXtLdsStride;
#pragma unroll
    for (int t = 0; t < kXtB; ++t) y[t] = row[t];
    __builtin_amdgcn_wave_barrier();
    if constexpr (MIX) {
      if (fast) {  // lo[i0 + t] = lo[i0] exp(-2 pi i f_lo t / fs), the w^t from the plan
        const CTab tb = fresh(tab);
#pragma unroll
        for (int t = 0; t < kXtB; ++t)
          y[t] = cmul2(y[t], cmul2(lo0, v2f{tb->wt[t][0], tb->wt[t][1]}));
      }
    }

    // ---- forward pass ----
    Modal m;
    {
      const Sos32 cs = load_sos(fresh(tab));
      IirState v;
      state_zero(v);
#pragma unroll
      for (int t = 0; t < kXtB; ++t) y[t] = cascade(y[t], v, cs);
      to_modal(tab, v, m);
    }
    {  // lane 0 also carries lambda^16 m_in (the tile's entering state)
      CTab tb = fresh(tab);
      Modal u = m_in;
#pragma unroll
      for (int j = 0; j < 4; ++j) rot(u.r[2 * j], u.r[2 * j + 1], tb->p16[j][0], tb->p16[j][1]);
      if (lane == 0) {  // exec-masked: 8 packed adds, no selects
#pragma unroll
        for (int r = 0; r < 8; ++r) m.r[r] += u.r[r];
      }
    }
    modal_scan<true>(m, tab, lane);
    {
      Modal me;  // state entering this lane's sub-block
#pragma unroll
      for (int r = 0; r < 8; ++r) me.r[r] = wave_shift<kWaveShr1>(m_in.r[r], m.r[r]);
#pragma unroll
      for (int r = 0; r < 8; ++r) m_in.r[r] = lane_of(m.r[r], 63);  // next tile's entering state
#pragma unroll
      for (int t0 = 0; t0 < kXtB; t0 += XT_CM_GROUP) {
        const CTab tb = fresh(tab);
#pragma unroll
        for (int t = t0; t < t0 + XT_CM_GROUP; ++t) y[t] = dot_cm(tb, t, me, y[t]);
      }
    }

    // ---- backward pass ----
    const bool last = tau == nt - 1;
    v2f ylast = splat(0.f);
    if (last) {  // steady state zi * y[e-1] above the frame end, constant tail
      const int pl = e - 1 - base;
      v2f *w = lds + lane * kXtLdsStride;
#pragma unroll
      for (int t = 0; t < kXtB; ++t) w[t] = y[t];
      __builtin_amdgcn_wave_barrier();
      ylast = uni2(lds[(pl >> 4) * kXtLdsStride + (pl & 15)]);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int t = 0; t < kXtB; ++t)
        if (base + lane * kXtB + t >= e) y[t] = ylast;
    }
    v2f kept[kXtHeld];
    {
      const Sos32 cs = load_sos(fresh(tab));
      IirState v;
      state_zero(v);
#pragma unroll
      for (int t = kXtB - 1; t >= 0; --t) {
        const v2f yb = cascade(y[t], v, cs);
        if (t & 1) kept[t >> 1] = yb;  // j = base + 16 lane + t odd <=> (j - 27) even
      }
      to_modal(tab, v, m);
    }
    Modal qtop;  // state entering the tile from above: exact steady state on the last tile
#pragma unroll
    for (int r = 0; r < 8; ++r) qtop.r[r] = last ? fresh(tab)->zim[r] * ylast : splat(0.f);
    if (last) {
      CTab tb = fresh(tab);
      Modal u = qtop;
#pragma unroll
      for (int j = 0; j < 4; ++j) rot(u.r[2 * j], u.r[2 * j + 1], tb->p16[j][0], tb->p16[j][1]);
      if (lane == 63) {
#pragma unroll
        for (int r = 0; r < 8; ++r) m.r[r] += u.r[r];
      }
    }
    modal_scan<false>(m, tab, lane);
    {
      Modal qe;  // state entering this lane's sub-block from above
#pragma unroll
      for (int r = 0; r < 8; ++r) qe.r[r] = wave_shift<kWaveShl1>(qtop.r[r], m.r[r]);
#pragma unroll
      for (int k0 = 0; k0 < kXtHeld; k0 += XT_CM_GROUP) {
        const CTab tb = fresh(tab);
#pragma unroll
        for (int k = k0; k < k0 + XT_CM_GROUP && k < kXtHeld; ++k)
          kept[k] = dot_cm(tb, kXtB - 2 - 2 * k, qe, kept[k]);
      }
    }
    // ---- the tile below is now complete: its top state is this tile's bottom state ----
    if (tau > 0) {
      Modal q;
#pragma unroll
      for (int r = 0; r < 8; ++r) q.r[r] = lane_of(m.r[r], 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) rot(q.r[2 * j], q.r[2 * j + 1], lgc[j], lgs[j]);
#pragma unroll
      for (int k0 = 0; k0 < kXtHeld; k0 += XT_CM_GROUP) {
        const CTab tb = fresh(tab);
#pragma unroll
        for (int k = k0; k < k0 + XT_CM_GROUP && k < kXtHeld; ++k)
          held[k] = dot_cm(tb, kXtB - 2 - 2 * k, q, held[k]);
      }
      store_kept(tau - 1, held);
    }
#pragma unroll
    for (int k = 0; k < kXtHeld; ++k) held[k] = kept[k];
  }
  store_kept(nt - 1, held);  // the last tile's top state was exact
}

template <bool MIX, int DT, int FLIP>
static void xt_launch(const InDesc &in, int n, const float2 *lo, float2 *out, int frames,
                      const XtModal *tab, hipStream_t st) {
  hipLaunchKernelGGL((xt_stage_kernel<MIX, DT, FLIP>), dim3((unsigned)((frames + 3) / 4)), dim3(256),
                     0, st, in, n, (const v2f *)lo, (v2f *)out, frames, tab, sos32());
}

hipError_t launch_xt_stage(const InDesc &in, int n, const float2 *lo, bool mix, float2 *out,
                           int frames, const XtModal *tab, hipStream_t st) {
  if (!mix) {
    if (in.dtype != kInC64 || in.flip) return hipErrorInvalidValue;  // stages >= 1: internal
    xt_launch<false, kInC64, 0>(in, n, lo, out, frames, tab, st);
  } else if (in.dtype == kInC64) {
    if (in.flip) xt_launch<true, kInC64, 1>(in, n, lo, out, frames, tab, st);
    else xt_launch<true, kInC64, 0>(in, n, lo, out, frames, tab, st);
  } else if (in.dtype == kInC32H) {
    if (in.flip) xt_launch<true, kInC32H, 1>(in, n, lo, out, frames, tab, st);
    else xt_launch<true, kInC32H, 0>(in, n, lo, out, frames, tab, st);
  } else if (in.dtype == kInF32R) {
    if (in.flip) xt_launch<true, kInF32R, 1>(in, n, lo, out, frames, tab, st);
    else xt_launch<true, kInF32R, 0>(in, n, lo, out, frames, tab, st);
  } else {
    if (in.flip) xt_launch<true, kInCU8, 1>(in, n, lo, out, frames, tab, st);
    else xt_launch<true, kInCU8, 0>(in, n, lo, out, frames, tab, st);
  }
  return hipGetLastError();
}

}  // namespace zfft
