// zfft_device.h -- device helpers shared by the HIP kernel files (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include "zfft_internal.h"

namespace zfft {

typedef float v2f __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2f splat(float a) { return v2f{a, a}; }
__device__ __forceinline__ v2f vfma(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ v2f cmul(v2f a, v2f b) {
  return v2f{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}

// a * b in two VOP3P instructions: t = (a.x b.x, a.x b.y); (a.y (-b.y), a.y b.x) + t
__device__ __forceinline__ v2f cmul2(v2f a, v2f b) {
  v2f t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef unsigned char u8x2 __attribute__((ext_vector_type(2)));

// Sample index i of frame f of the caller's input as complex64 (InDesc, zfft_internal.h).
// FLIP: -1 = read d.flip at run time, 0 / 1 = known at compile time (immediate offsets).
template <int DT, int FLIP = -1>
__device__ __forceinline__ v2f load_in_t(const InDesc &d, int64_t f, int64_t i) {
  const bool flip = FLIP < 0 ? d.flip != 0 : FLIP != 0;
  const int64_t k = f * d.stride + (flip ? d.len - 1 - i : i);
  if constexpr (DT == kInC64) {
    return ((const v2f *)d.p)[k];
  } else if constexpr (DT == kInC32H) {
    const h2 h = ((const h2 *)d.p)[k];
    return v2f{(float)h.x, (float)h.y};
  } else if constexpr (DT == kInF32R) {
    return v2f{((const float *)d.p)[k], 0.f};
  } else {
    const u8x2 b = ((const u8x2 *)d.p)[k];
    return v2f{((float)b.x - 127.5f) * (1.f / 127.5f), ((float)b.y - 127.5f) * (1.f / 127.5f)};
  }
}

// The LO table row of frame f of a call (InDesc lo_* fields; row 0 for a single f_lo).
__device__ __forceinline__ const v2f *lo_row(const v2f *lo, const InDesc &d, int64_t f) {
  if (d.lo_n <= 1) return lo;
  return lo + (int64_t)((((int64_t)d.lo_first + f) / d.lo_per) % d.lo_n) * d.lo_stride;
}

__device__ __forceinline__ v2f load_in(const InDesc &d, int64_t f, int64_t i) {
  if (d.dtype == kInC64) return load_in_t<kInC64>(d, f, i);
  if (d.dtype == kInC32H) return load_in_t<kInC32H>(d, f, i);
  if (d.dtype == kInF32R) return load_in_t<kInF32R>(d, f, i);
  return load_in_t<kInCU8>(d, f, i);
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

}  // namespace zfft
