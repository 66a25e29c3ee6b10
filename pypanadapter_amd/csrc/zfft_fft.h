// zfft_fft.h -- radix-2/4/8/16 butterflies and twiddle powers on packed complex64 (v2f),
// shared by the Welch transforms (zfft_kernels.hip) and the fast-convolution decimator
// (fc_kernels.hip).  Not part of the C-ABI.
#pragma once

#include "zfft_device.h"

namespace zfft {

// a + (-i) d = (a.x + d.y, a.y - d.x) and a - (-i) d = (a.x - d.y, a.y + d.x): one VOP3P add
// each, the swap and sign in the operand selects (the plain form costs moves)
__device__ __forceinline__ v2f add_negi(v2f a, v2f d) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(d));
  return r;
}
__device__ __forceinline__ v2f sub_negi(v2f a, v2f d) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(d));
  return r;
}

template <int R>
__device__ __forceinline__ void dft(v2f *v);

template <>
__device__ __forceinline__ void dft<2>(v2f *v) {
  const v2f a = v[0], b = v[1];
  v[0] = a + b;
  v[1] = a - b;
}

template <>
__device__ __forceinline__ void dft<4>(v2f *v) {
  const v2f a0 = v[0] + v[2], a1 = v[0] - v[2], a2 = v[1] + v[3], d = v[1] - v[3];
  v[0] = a0 + a2;
  v[1] = add_negi(a1, d);  // a1 + (-i) d
  v[2] = a0 - a2;
  v[3] = sub_negi(a1, d);
}

// W_16^m for m = 0..15 as compile-time constants
__device__ __forceinline__ v2f w16(int m) {
  constexpr float c1 = 0.92387953251128674f, s1 = 0.38268343236508977f, h = 0.70710678118654752f;
  const float cs[16][2] = {{1.f, 0.f},  {c1, -s1},  {h, -h},    {s1, -c1}, {0.f, -1.f}, {-s1, -c1},
                           {-h, -h},    {-c1, -s1}, {-1.f, 0.f}, {-c1, s1}, {-h, h},     {-s1, c1},
                           {0.f, 1.f},  {s1, c1},   {h, h},      {c1, s1}};
  return v2f{cs[m & 15][0], cs[m & 15][1]};
}

// n = n2 + 2*n1 (n1 < 4): inner DFT4 over n1, twiddle W8^(n2 k1), outer DFT2 -> X[k1 + 4 k2]
template <>
__device__ __forceinline__ void dft<8>(v2f *v) {
  v2f a[2][4];
#pragma unroll
  for (int n2 = 0; n2 < 2; ++n2) {
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1) a[n2][n1] = v[n2 + 2 * n1];
    dft<4>(a[n2]);
  }
#pragma unroll
  for (int k1 = 1; k1 < 4; ++k1) a[1][k1] = cmul2(a[1][k1], w16(2 * k1));
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    v[k1] = a[0][k1] + a[1][k1];
    v[k1 + 4] = a[0][k1] - a[1][k1];
  }
}

// n = n2 + 4*n1: inner DFT4 over n1, twiddle W16^(n2 k1), outer DFT4 over n2 -> X[k1 + 4 k2]
template <>
__device__ __forceinline__ void dft<16>(v2f *v) {
  v2f a[4][4];
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) {
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1) a[n2][n1] = v[n2 + 4 * n1];
    dft<4>(a[n2]);
  }
#pragma unroll
  for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
    for (int k1 = 1; k1 < 4; ++k1) a[n2][k1] = cmul2(a[n2][k1], w16(n2 * k1));
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    v2f b[4] = {a[0][k1], a[1][k1], a[2][k1], a[3][k1]};
    dft<4>(b);
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) v[k1 + 4 * k2] = b[k2];
  }
}

// v[r] *= b^r, r = 1..15, from bp = {b, b^2, b^4, b^8}: each power applied as soon as it
// is formed (at most eight of them live)
__device__ __forceinline__ void apply_powers(v2f *v, const v2f *bp) {
  v[1] = cmul2(v[1], bp[0]);
  v[2] = cmul2(v[2], bp[1]);
  v[4] = cmul2(v[4], bp[2]);
  v[8] = cmul2(v[8], bp[3]);
  const v2f w3 = cmul2(bp[0], bp[1]), w5 = cmul2(bp[0], bp[2]), w6 = cmul2(bp[1], bp[2]);
  const v2f w7 = cmul2(w3, bp[2]);
  v[3] = cmul2(v[3], w3);
  v[5] = cmul2(v[5], w5);
  v[6] = cmul2(v[6], w6);
  v[7] = cmul2(v[7], w7);
  v[9] = cmul2(v[9], cmul2(bp[0], bp[3]));
  v[10] = cmul2(v[10], cmul2(bp[1], bp[3]));
  v[11] = cmul2(v[11], cmul2(w3, bp[3]));
  v[12] = cmul2(v[12], cmul2(bp[2], bp[3]));
  v[13] = cmul2(v[13], cmul2(w5, bp[3]));
  v[14] = cmul2(v[14], cmul2(w6, bp[3]));
  v[15] = cmul2(v[15], cmul2(w7, bp[3]));
}

// apply_powers on two vectors sharing the base (the FC decimator's residue pairs): each power
// formed once and applied to both
__device__ __forceinline__ void apply_powers2(v2f *v, v2f *u, const v2f *bp) {
  auto ap = [&](int i, v2f w) {
    v[i] = cmul2(v[i], w);
    u[i] = cmul2(u[i], w);
  };
  ap(1, bp[0]);
  ap(2, bp[1]);
  ap(4, bp[2]);
  ap(8, bp[3]);
  const v2f w3 = cmul2(bp[0], bp[1]), w5 = cmul2(bp[0], bp[2]), w6 = cmul2(bp[1], bp[2]);
  const v2f w7 = cmul2(w3, bp[2]);
  ap(3, w3);
  ap(5, w5);
  ap(6, w6);
  ap(7, w7);
  ap(9, cmul2(bp[0], bp[3]));
  ap(10, cmul2(bp[1], bp[3]));
  ap(11, cmul2(w3, bp[3]));
  ap(12, cmul2(bp[2], bp[3]));
  ap(13, cmul2(w5, bp[3]));
  ap(14, cmul2(w6, bp[3]));
  ap(15, cmul2(w7, bp[3]));
}

}  // namespace zfft
