// zfft_pairs.h -- two consecutive input samples per lane: the raw load of a pair in the caller's
// storage type and its conversion to complex64 (used by the PC walk and tiles, pc_kernels.hip, and
// the fast-convolution decimator, fc_kernels.hip).  Not part of the C-ABI.
#pragma once

#include "zfft_device.h"

namespace zfft {

typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v2f lo2(v4f w) { return v2f{w.x, w.y}; }
__device__ __forceinline__ v2f hi2(v4f w) { return v2f{w.z, w.w}; }
__device__ __forceinline__ v4f cat(v2f a, v2f b) { return v4f{a.x, a.y, b.x, b.y}; }

// x[n], x[n+1] of frame f (both inside the frame): the raw load (issued early by KW's
// prefetch) and its conversion to complex64
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef unsigned char u8x4 __attribute__((ext_vector_type(4)));
// T: the pair as a value; U: the same type aligned only to one element, the alignment the
// address has (the first sample of a pair is any sample: odd L, flip).  The U loads still
// compile to one global_load_dwordx4 / dwordx2 / dword / short: gfx950 global loads need no
// natural alignment (unaligned access mode), and the type says so instead of relying on it.
template <int DT> struct RawP;
template <> struct RawP<kInC64> {
  typedef v4f T;
  typedef float U __attribute__((ext_vector_type(4), aligned(8)));
};
template <> struct RawP<kInC32H> {
  typedef h4 T;
  typedef _Float16 U __attribute__((ext_vector_type(4), aligned(4)));
};
template <> struct RawP<kInF32R> {
  typedef v2f T;
  typedef float U __attribute__((ext_vector_type(2), aligned(4)));
};
template <> struct RawP<kInCU8> {
  typedef u8x4 T;
  typedef unsigned char U __attribute__((ext_vector_type(4), aligned(2)));
};
template <int DT, int FLIP>
__device__ __forceinline__ typename RawP<DT>::T raw_pair(const InDesc &in, int64_t f, int64_t n) {
  typedef const typename RawP<DT>::U *UP;
  const int64_t k = f * in.stride + (FLIP ? in.len - 2 - n : n);  // first raw element
  if constexpr (DT == kInC64) return *(UP)((const v2f *)in.p + k);
  else if constexpr (DT == kInC32H) return *(UP)((const h2 *)in.p + k);
  else if constexpr (DT == kInF32R) return *(UP)((const float *)in.p + k);
  else return *(UP)((const u8x2 *)in.p + k);
}
template <int DT, int FLIP>
__device__ __forceinline__ void cvt_pair(typename RawP<DT>::T w, v2f &a, v2f &b) {
  v2f p, q;
  if constexpr (DT == kInC64) {
    p = lo2(w);
    q = hi2(w);
  } else if constexpr (DT == kInC32H) {
    p = v2f{(float)w.x, (float)w.y};
    q = v2f{(float)w.z, (float)w.w};
  } else if constexpr (DT == kInF32R) {
    p = v2f{w.x, 0.f};
    q = v2f{w.y, 0.f};
  } else {
    const float s = 1.f / 127.5f;
    p = v2f{((float)w.x - 127.5f) * s, ((float)w.y - 127.5f) * s};
    q = v2f{((float)w.z - 127.5f) * s, ((float)w.w - 127.5f) * s};
  }
  a = FLIP ? q : p;
  b = FLIP ? p : q;
}
template <int DT, int FLIP>
__device__ __forceinline__ void load_pair(const InDesc &in, int64_t f, int64_t n, v2f &a, v2f &b) {
  cvt_pair<DT, FLIP>(raw_pair<DT, FLIP>(in, f, n), a, b);
}

}  // namespace zfft
