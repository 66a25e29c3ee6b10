// xt_kernels.hip -- exact-tile ("XT") zero-phase decimation stage for gfx950.
//
// One stage of the reference's decimate(x, 2) (pypanadapter_spectrum.py:2096-2098 ->
// scipy sosfiltfilt: odd pad 27, zi initial conditions, forward + backward, [::2]) on one
// frame per wave, reading the stage input once and writing only the decimated output:
// no forward-pass intermediate ever reaches memory.
//
// A wave walks its frame in tiles of 1024 samples; lane i owns the 16-sample sub-block i.
//  forward (exact):  every lane runs the cascade from a zero state over its sub-block;
//                    a Kogge-Stone scan over the 64 lane end-states with the matrices
//                    (A^16)^(2^d) gives each lane its true entering state (the tile's
//                    entering state folded into lane 0), and the outputs are corrected
//                    by C A^t s_in.  The scan stops at d = 4: (A^16)^32 = A^512 ~ 1e-15.
//  backward:         the same over the forward outputs in descending order, with the
//                    state entering the tile from above provisionally zero.  The state
//                    this leaves at the tile bottom is exact anyway (its dependence on
//                    the unknown top state is A^1024 ~ 1e-30), and it is precisely the
//                    top state of the tile below, which was processed one step earlier:
//                    its kept outputs get the correction D[lane][k] . q (table), then
//                    are stored.  One tile of lag.
//  frame ends:       forward starts from zi * ext[0]; the last tile's backward starts from
//                    zi * y[e-1] with a constant y[e-1] tail above e-1 (the steady state
//                    is a fixed point of the recursion), exactly scipy's initial condition.
// Numerics: float32, max relative error vs float64 sosfiltfilt ~7.6e-7 on white noise,
// the same as a sequential float32 sosfiltfilt (6.2e-7): /tmp-free reproduction in
// tools/xt_proto.py.
#include "zfft_device.h"

namespace zfft {

constexpr int kXtLdsStride = kXtB + 1;  // padded sub-block rows: conflict-free ds_read_b64

__device__ __forceinline__ v2f sget(const IirState &s, int r) {
  return (r & 1) ? s.z1[r >> 1] : s.z0[r >> 1];
}
__device__ __forceinline__ void sset(IirState &s, int r, v2f v) {
  if (r & 1) s.z1[r >> 1] = v;
  else s.z0[r >> 1] = v;
}

__device__ __forceinline__ v2f shfl2(v2f v, int src) {
  return v2f{__shfl(v.x, src, 64), __shfl(v.y, src, 64)};
}

// a wave-uniform value into scalar registers (every lane holds the same state)
__device__ __forceinline__ float uni(float a) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(a)));
}
__device__ __forceinline__ v2f uni2(v2f v) { return v2f{uni(v.x), uni(v.y)}; }

// uniform state = state of lane `src` (broadcast, kept in SGPRs)
__device__ __forceinline__ void bcast_state(const IirState &v, int src, IirState &out) {
#pragma unroll
  for (int r = 0; r < 8; ++r) sset(out, r, uni2(shfl2(sget(v, r), src)));
}

// Compiler-only barrier: the table constants below are re-read (scalar loads, K$ hits)
// after it instead of being hoisted out of the tile loop into ~900 SGPRs.
__device__ __forceinline__ void refetch_tables() { asm volatile("" ::: "memory"); }

// out = M s (8x8 real matrix, row-major, uniform) applied to both channels
__device__ __forceinline__ void matvec(const float *__restrict__ M, const IirState &s,
                                       IirState &out) {
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    refetch_tables();
    v2f acc = splat(0.f);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc = vfma(splat(M[r * 8 + q]), sget(s, q), acc);
    sset(out, r, acc);
  }
}

// inclusive Kogge-Stone scan of lane states in the direction UP (lane i accumulates lanes
// j <= i) or down (j >= i): v_i = sum_j (A^16)^|i-j| z_j.
template <bool UP>
__device__ __forceinline__ void state_scan(IirState &v, const XtTables *__restrict__ tab, int lane) {
#pragma unroll 1
  for (int d = 0; d < kXtScan; ++d) {
    const int sh = 1 << d;
    const int src = UP ? lane - sh : lane + sh;
    const bool take = UP ? lane >= sh : lane + sh <= 63;
    IirState w;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const v2f t = shfl2(sget(v, r), src & 63);
      sset(w, r, take ? t : splat(0.f));
    }
    const float *__restrict__ M = &tab->M[d][0][0];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      refetch_tables();  // one row of constants live at a time
      v2f acc = sget(v, r);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc = vfma(splat(M[r * 8 + q]), sget(w, q), acc);
      sset(v, r, acc);
    }
  }
}

template <bool MIX, int DT>  // DT: input format (stage 0 reads the caller's frames)
__global__ __launch_bounds__(256) void xt_stage_kernel(InDesc in, int n,
                                                       const v2f *__restrict__ lo,
                                                       v2f *__restrict__ out, int frames,
                                                       const XtTables *__restrict__ tab,
                                                       Sos32 c) {
  __shared__ __attribute__((aligned(16))) v2f lds_all[4][64 * kXtLdsStride];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int f = blockIdx.x * 4 + wv;
  if (f >= frames) return;  // whole wave
  v2f *lds = lds_all[wv];
  const int e = n + 2 * kPad, n_out = (n + 1) >> 1;
  v2f *__restrict__ o = out + (int64_t)f * n_out;
  auto X = [&](int i) -> v2f {
    v2f v = load_in_t<DT>(in, f, i);
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

  IirState s_in;  // state entering the current tile (forward), wave-uniform (SGPRs)
  state_steady(s_in, c, uni2(ext(0)));
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
#pragma unroll
    for (int q = 0; q < kXtB; ++q) {
      const int s = lane + 64 * q;
      lds[(s >> 4) * kXtLdsStride + (s & 15)] = fast ? X(base + s - kPad) : ext(base + s);
    }
    __builtin_amdgcn_wave_barrier();
    v2f y[kXtB];
#pragma unroll
    for (int t = 0; t < kXtB; ++t) y[t] = lds[lane * kXtLdsStride + t];
    __builtin_amdgcn_wave_barrier();

    // ---- forward pass ----
    IirState v;
    state_zero(v);
#pragma unroll
    for (int t = 0; t < kXtB; ++t) y[t] = cascade(y[t], v, c);
    {
      refetch_tables();
      IirState u;
      matvec(&tab->M[0][0][0], s_in, u);  // lane 0 also carries (A^16) s_in
#pragma unroll
      for (int r = 0; r < 8; ++r) sset(v, r, sget(v, r) + (lane == 0 ? sget(u, r) : splat(0.f)));
    }
    state_scan<true>(v, tab, lane);
    IirState se;  // state entering this lane's sub-block
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const v2f up = shfl2(sget(v, r), (lane + 63) & 63);
      sset(se, r, lane == 0 ? sget(s_in, r) : up);
    }
    bcast_state(v, 63, s_in);  // next tile's entering state
#pragma unroll
    for (int t = 0; t < kXtB; ++t) {
      refetch_tables();
      v2f acc = y[t];
#pragma unroll
      for (int r = 0; r < 8; ++r) acc = vfma(splat(tab->Ct[t][r]), sget(se, r), acc);
      y[t] = acc;
    }

    // ---- backward pass ----
    const bool last = tau == nt - 1;
    IirState qtop;
    state_zero(qtop);
    if (last) {  // steady state zi * y[e-1] above the frame end, constant tail
      const int pl = e - 1 - base;
      v2f cand = y[0];
#pragma unroll
      for (int t = 1; t < kXtB; ++t)
        if (t == (pl & 15)) cand = y[t];
      const v2f ylast = uni2(shfl2(cand, pl >> 4));
#pragma unroll
      for (int t = 0; t < kXtB; ++t)
        if (base + lane * kXtB + t >= e) y[t] = ylast;
      state_steady(qtop, c, ylast);
    }
    state_zero(v);
    v2f kept[kXtHeld];
#pragma unroll
    for (int t = kXtB - 1; t >= 0; --t) {
      const v2f yb = cascade(y[t], v, c);
      if (t & 1) kept[t >> 1] = yb;  // j = base + 16 lane + t odd <=> (j - 27) even
    }
    if (last) {
      refetch_tables();
      IirState u;
      matvec(&tab->M[0][0][0], qtop, u);
#pragma unroll
      for (int r = 0; r < 8; ++r) sset(v, r, sget(v, r) + (lane == 63 ? sget(u, r) : splat(0.f)));
    }
    state_scan<false>(v, tab, lane);
    IirState qe;  // state entering this lane's sub-block from above
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const v2f dn = shfl2(sget(v, r), (lane + 1) & 63);
      sset(qe, r, lane == 63 ? sget(qtop, r) : dn);
    }
#pragma unroll
    for (int k = 0; k < kXtHeld; ++k) {
      refetch_tables();
      v2f acc = kept[k];
#pragma unroll
      for (int r = 0; r < 8; ++r) acc = vfma(splat(tab->Ct[kXtB - 2 - 2 * k][r]), sget(qe, r), acc);
      kept[k] = acc;
    }
    // ---- the tile below is now complete: its top state is this tile's bottom state ----
    if (tau > 0) {
      IirState qb;
      bcast_state(v, 0, qb);
#pragma unroll
      for (int k = 0; k < kXtHeld; ++k) {
        v2f acc = held[k];
#pragma unroll
        for (int r = 0; r < 8; ++r) acc = vfma(splat(tab->D[lane][k][r]), sget(qb, r), acc);
        held[k] = acc;
      }
      store_kept(tau - 1, held);
    }
#pragma unroll
    for (int k = 0; k < kXtHeld; ++k) held[k] = kept[k];
  }
  store_kept(nt - 1, held);  // the last tile's top state was exact
}

hipError_t launch_xt_stage(const InDesc &in, int n, const float2 *lo, bool mix, float2 *out,
                           int frames, const XtTables *tab, hipStream_t st) {
  const dim3 grid((unsigned)((frames + 3) / 4)), block(256);
  const v2f *l = (const v2f *)lo;
  v2f *o = (v2f *)out;
  if (!mix)
    hipLaunchKernelGGL((xt_stage_kernel<false, kInC64>), grid, block, 0, st, in, n, l, o, frames, tab, sos32());
  else if (in.dtype == kInC64)
    hipLaunchKernelGGL((xt_stage_kernel<true, kInC64>), grid, block, 0, st, in, n, l, o, frames, tab, sos32());
  else if (in.dtype == kInC32H)
    hipLaunchKernelGGL((xt_stage_kernel<true, kInC32H>), grid, block, 0, st, in, n, l, o, frames, tab, sos32());
  else
    hipLaunchKernelGGL((xt_stage_kernel<true, kInCU8>), grid, block, 0, st, in, n, l, o, frames, tab, sos32());
  return hipGetLastError();
}

}  // namespace zfft
