// xa_kernels.hip -- "XA" zero-phase decimation stage for gfx950 (design model:
// tools/xa_proto.py; tables: zfft_plan.cpp xa_build_tables).
//
// One stage of the reference's decimate(x, 2) (pypanadapter_spectrum.py:2096-2098 ->
// scipy sosfiltfilt: odd pad 27, steady-state initial conditions, forward + backward,
// [::2]) on one frame per wave, reading the stage input once and writing only the
// decimated output.  The cascade H = N(z)/D(z) is factored (exactly, edges included) as
//
//   v = ext / D(z)                         forward all-pole cascade, input rate
//   h_j = sum_t M_t v[j-8+t], j odd        25-tap FIR M = N(z) N(1/z) D(-1/z), kept j only
//   g = h / D2(1/w)                        backward all-pole cascade, output rate
//
// so a stage costs 8 + 12.5 + 4 packed multiply-adds per input sample, against 2 x 17 for
// two DF2T passes.  A wave walks its frame in tiles of 64 lanes x B = 32 samples (lane i
// owns the sub-block of B consecutive samples, K = B/2 kept outputs), loaded a tile ahead
// as pairs of consecutive samples per lane and transposed to lane rows through LDS:
//  forward:   every lane runs the all-pole cascade once, from a zero state, over its B
//             samples, streaming v into the FIR; its end state goes to the real modal
//             basis (T^-1, block lower triangular, one rotation-scaling 2x2 block per pole
//             pair), a Kogge-Stone scan over lanes -- per mode only as deep as its radius
//             needs (xa_levels) -- gives each lane its exact entering state, whose
//             zero-input response through the FIR is added from precomputed tables (gown,
//             gnb) instead of a second pass.  The tile's entering state is folded into lane 0.
//  FIR:       lane i evaluates h at the K odd positions of [B i - 16, B i + B - 16) from
//             v[B i - 24, B i + B): its own v and the last 24 v of lane i-1, whose share
//             lane i-1 accumulates itself and hands over with one DPP shift (lane 0 takes
//             the previous tile's lane-63 share from LDS).
//  backward:  one pass on the K h values of each lane, descending, from a zero state, the
//             scan down, and the entering state's response from the lag rows; the state
//             entering the tile from above is provisionally zero, the state it leaves at
//             the tile bottom is exact regardless (its dependence on the top state is
//             |lambda^2|^(32 B) < 1e-29) and is the top state of the tile below, processed
//             one step earlier: that tile's top kXaLag outputs get C A2^d T q, then all
//             its outputs are stored.
//  frame end: the forward pre-history is the steady state of constant ext[0]
//             (sosfilt_zi * ext[0]); the backward post-history is the steady state of
//             constant f[e-1], f = N v formed explicitly for the last 16 positions, whose
//             h use the unmerged form N(1/z) D(-1/z) on f clamped at e-1.
// B = 32 keeps a tile in 256 VGPRs (2 waves/SIMD).  B = 64 would halve the per-tile scan
// and basis-change work per sample, but its fully unrolled tile is 112 KB of code against
// the 64 KB instruction cache two CUs share (B = 32: 32 KB): measured 6.6x slower on
// MI355X, so only B = 32 is instantiated.
// Numerics: float32, max relative error ~8e-6 of the decimated IQ vs float64 sosfiltfilt
// (plain float32 sosfiltfilt: ~1e-6); end-to-end rows within 1e-5 dB (tools/xa_proto.py).
#include <cstddef>
#include <type_traits>

#include "zfft_device.h"

// Diagnostic knobs exist only in a -DZFFT_DIAG build (tools/build_variants.py; build.py never
// sets it): XA_STAMPS = per-phase s_memtime sums (tools/xa_stamps.py), XA_EXP = timing-only
// knockouts with wrong results (tools/ab.sh): 1 scans, 2 state corrections, 4 LO products,
// 8 next-tile loads, 16 output stores, 32 forward pass, 64 frame-end tiles as fast tiles.
// The production variants measured against the alternatives are DESIGN.md §3.1's.
#if defined(ZFFT_DIAG) && ZFFT_DIAG
#ifndef XA_STAMPS
#define XA_STAMPS 0
#endif
#ifndef XA_EXP
#define XA_EXP 0
#endif
#else
#if defined(XA_STAMPS) || defined(XA_EXP)
#error "XA_STAMPS / XA_EXP are diagnostic knobs: build with -DZFFT_DIAG"
#endif
#define XA_STAMPS 0
#define XA_EXP 0
#endif

namespace zfft {
namespace xa {

// Tiles go in and out through LDS transposes with both halves (32 lanes' rows each) held at
// once: one LDS round trip per direction and tile (two halves in turn: 4 % slower at cfg2).
// 4-wave workgroups: 2 of them (78 KB of LDS each) fill a CU at 2 waves per SIMD.
constexpr int kHalfRows = 32;           // rows of one transpose half (32 lanes' sub-blocks)
constexpr int kWaves = 4;               // waves (frames) per workgroup
constexpr int kLagChunks = kXaLag / 64; // held output chunks of a tile

template <int B>
struct Geo {
  static constexpr int K = B / 2;            // kept outputs per lane and tile
  static constexpr int T = 64 * B;           // tile (input samples)
  static constexpr int kRow = B + 2;         // LDS row stride (v2f): ds_read_b128 rows conflict-free
  // output-transpose rows (v2f): b128 writes conflict-free; the pair and single reads see
  // 2-way conflicts on a few lanes (~30 LDS cycles per tile).  No padding makes all three
  // conflict-free; an XOR swizzle of the 16-B slots by row does (SQ_LDS_BANK_CONFLICT
  // 29.1 M -> 0.4 M per stage-0 dispatch) but costs 12 VALU instructions per tile for the
  // per-slot write addresses, and measured 0.7 % slower (profiles/r03_ab/r03w)
  static constexpr int kHeldRow = K + 2;
  static constexpr int kOutChunks = K;       // 64-output chunks per tile
  static constexpr int kRowsPerChunk = 64 / B > 0 ? 64 / B : 1;  // input rows one 64-sample chunk fills
  // LDS per wave: the tile transpose (both halves) + FIR carry (12 used) + frame-end v
  // carry (the 64 v before the last tile)
  // (the output transpose, 64 rows of kHeldRow, reuses the input transpose's space)
  static constexpr int kIn = 2 * kHalfRows * kRow;
  static constexpr int kMain = kIn > 64 * kHeldRow ? kIn : 64 * kHeldRow;
  static constexpr int kBuf = kMain + 16 + 64;
  static constexpr int kWavesPerSimd = B == 32 ? 2 : 1;  // the register budget is cut for
};

typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
// LDS pointers keep their address space (a generic pointer turns every LDS access into a
// flat access, which waits on vector memory too)
typedef v2f __attribute__((address_space(3))) *LP;
typedef v4f __attribute__((address_space(3))) *LP4;
// Filter tables: scalar (K$) reads of the constant table; the far-field `lag` rows are
// per-lane reads from an LDS copy.
typedef const XaTab __attribute__((address_space(4))) *CT;
// an opaque copy per phase: reads are not hoisted out of the tile loop (which would pin
// the whole table in SGPRs and spill), each phase re-reads the few it needs
__device__ __forceinline__ CT fresh(CT p) {
  asm volatile("" : "+s"(p));
  return p;
}

// Raw input element of each in_dtype: tile loads are issued one tile ahead and converted
// only when consumed, so no conversion (and no wait) sits behind the load.
template <int DT> struct Raw;
template <> struct Raw<kInC64> { typedef v2f T; };
template <> struct Raw<kInC32H> { typedef h2 T; };
template <> struct Raw<kInCU8> { typedef u8x2 T; };
template <> struct Raw<kInF32R> { typedef float T; };
template <int DT>
__device__ __forceinline__ v2f cvt_raw(typename Raw<DT>::T r) {  // as load_in_t (zfft_device.h)
  if constexpr (DT == kInC64) return r;
  else if constexpr (DT == kInC32H) return v2f{(float)r.x, (float)r.y};
  else if constexpr (DT == kInF32R) return v2f{r, 0.f};
  else return v2f{((float)r.x - 127.5f) * (1.f / 127.5f), ((float)r.y - 127.5f) * (1.f / 127.5f)};
}

// Two consecutive raw elements: the wide tile loads take a pair per lane (16 B for
// complex64: the gfx950 memory path moves 16-B lanes at a better rate than 8-B ones).
template <int DT> struct Pair {
  typename Raw<DT>::T a, b;
};

// one raw element (or pair) through a buffer resource (out-of-range offsets read 0)
constexpr int kLoadAux = 2;   // aux 2 = nt (streaming): tile loads and output stores
constexpr int kStoreAux = 2;
template <class T>
__device__ __forceinline__ T buf_load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  T v;
  if constexpr (sizeof(T) == 16) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kLoadAux);
    __builtin_memcpy(&v, &u, 16);
  } else if constexpr (sizeof(T) == 8) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kLoadAux);
    __builtin_memcpy(&v, &u, 8);
  } else if constexpr (sizeof(T) == 4) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kLoadAux);
    __builtin_memcpy(&v, &u, 4);
  } else {
    const auto u = __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, kLoadAux);
    __builtin_memcpy(&v, &u, 2);
  }
  return v;
}

__device__ __forceinline__ void st_out(v2f *p, v2f v) {  // one output (final, unmasked form)
  if constexpr (kStoreAux) __builtin_nontemporal_store(v, p);
  else *p = v;
}

struct Md {
  v2f r[8];  // a0 b0 a1 b1 a2 b2 a3 b3 per mode (I and Q share the real basis)
};

__device__ __forceinline__ float uni(float a) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(a)));
}
__device__ __forceinline__ v2f lane_of(v2f v, int src) {
  return v2f{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), src)),
             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), src))};
}
__device__ __forceinline__ v2f shfl2(v2f v, int src) {
  return v2f{__shfl(v.x, src, 64), __shfl(v.y, src, 64)};
}
// whole-wave DPP shift by one lane (wave_shr:1 / wave_shl:1); the lane without a source
// keeps `old`
constexpr int kShr1 = 0x138, kShl1 = 0x130;
template <int CTRL>
__device__ __forceinline__ v2f wave_shift(v2f old, v2f src) {
  return v2f{__int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old.x), __float_as_int(src.x),
                                                        CTRL, 0xF, 0xF, false)),
             __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old.y), __float_as_int(src.y),
                                                        CTRL, 0xF, 0xF, false))};
}

// (a, b) <- [[c, s], [-s, c]] (a, b): one mode times lambda^p = c + i s
__device__ __forceinline__ void rot(v2f &a, v2f &b, float c, float s) {
  const v2f na = vfma(splat(c), a, splat(s) * b);
  b = vfma(splat(c), b, splat(-s) * a);
  a = na;
}

// One sample through the all-pole cascade; s[2k] = y_k[t-1], s[2k+1] = y_k[t-2].
__device__ __forceinline__ v2f ap_step(v2f x, v2f s[8], const float a1[4], const float a2[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // the y[t-2] term first: one multiply-add of latency per step on the recurrence
    const v2f y = vfma(splat(-a1[k]), s[2 * k], vfma(splat(-a2[k]), s[2 * k + 1], x));
    s[2 * k + 1] = s[2 * k];
    s[2 * k] = y;
    x = y;
  }
  return x;
}

template <int PASS>  // 0 forward, 1 backward
__device__ __forceinline__ const XaPass __attribute__((address_space(4))) &pass_of(CT t) {
  if constexpr (PASS == 0) return t->f;
  else return t->b;
}

template <int PASS>
__device__ __forceinline__ void load_ap(CT tab, float a1[4], float a2[4]) {
  CT t = fresh(tab);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    a1[k] = pass_of<PASS>(t).a1[k];
    a2[k] = pass_of<PASS>(t).a2[k];
  }
}

// m = T^-1 s; T^-1 is block lower triangular (mode j depends on sections <= j)
template <int PASS>
__device__ __forceinline__ void to_modal(CT tab, const v2f s[8], Md &m) {
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    CT t = fresh(tab);
    v2f acc = splat(0.f);
#pragma unroll
    for (int q = 0; q < (r | 1) + 1; ++q) acc = vfma(splat(pass_of<PASS>(t).ti[r][q]), s[q], acc);
    m.r[r] = acc;
  }
}

// Inclusive weighted scan over lanes: UP (lane i sums lanes j <= i) or down (j >= i),
// m_i = sum_j lambda^(S |i-j|) m_j per mode, every term within the mode's reach exact.
// Modes 0, 1 run Kogge-Stone inside 16-lane rows on DPP row shifts, then add the adjacent
// row's end lane (its within-row inclusive sum) weighted by the lane's own distance to it
// (xw: c0 s0 c1 s1 for this lane-in-row): UP by DPP row_bcast:15, down by one ds_bpermute
// round; modes 2, 3 need one whole-wave DPP shift.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ v2f dpp0(v2f src) {  // lanes without a source (or row) get 0
  if constexpr (ROWMASK == 0xF)  // bound_ctrl: a lane without a source reads 0, no old value
    return v2f{__int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(src.x), CTRL, 0xF, 0xF, true)),
               __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(src.y), CTRL, 0xF, 0xF, true))};
  else
    return v2f{__int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(src.x), CTRL, ROWMASK, 0xF, false)),
               __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(src.y), CTRL, ROWMASK, 0xF, false))};
}
constexpr int kRowShr = 0x110, kRowShl = 0x100, kRowBcast15 = 0x142;
template <bool UP>
__device__ __forceinline__ v2f row_shift(v2f src, int d) {  // by 2^d lanes inside 16-lane rows
  switch (d) {
    case 0: return dpp0<(UP ? kRowShr : kRowShl) + 1, 0xF>(src);
    case 1: return dpp0<(UP ? kRowShr : kRowShl) + 2, 0xF>(src);
    case 2: return dpp0<(UP ? kRowShr : kRowShl) + 4, 0xF>(src);
    default: return dpp0<(UP ? kRowShr : kRowShl) + 8, 0xF>(src);
  }
}
template <int B, int PASS, bool UP>
__device__ __forceinline__ void modal_scan(Md &m, CT tab, int lane, v4f xw) {
  if (XA_EXP & 1) return;
  asm volatile("" : "+v"(lane));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int d = 0; d < xa_levels(B, j); ++d) {
      CT t = fresh(tab);
      const float c = pass_of<PASS>(t).scan[d][j][0], sn = pass_of<PASS>(t).scan[d][j][1];
      v2f pa, pb;
      if (j < kXaRowModes) {
        pa = row_shift<UP>(m.r[2 * j], d);
        pb = row_shift<UP>(m.r[2 * j + 1], d);
      } else {  // one level: a whole-wave shift by one lane
        constexpr int ctrl = UP ? kShr1 : kShl1;
        pa = dpp0<ctrl, 0xF>(m.r[2 * j]);
        pb = dpp0<ctrl, 0xF>(m.r[2 * j + 1]);
      }
      rot(pa, pb, c, sn);
      m.r[2 * j] += pa;
      m.r[2 * j + 1] += pb;
    }
  }
  v2f pa[kXaRowModes], pb[kXaRowModes];
#pragma unroll
  for (int j = 0; j < kXaRowModes; ++j) {
    if (UP) {  // rows 1..3 <- lane 15 of the row below
      pa[j] = dpp0<kRowBcast15, 0xE>(m.r[2 * j]);
      pb[j] = dpp0<kRowBcast15, 0xE>(m.r[2 * j + 1]);
    } else {   // rows 0..2 <- lane 0 of the row above
      const int src = ((lane | 15) + 1) & 63;
      pa[j] = shfl2(m.r[2 * j], src);
      pb[j] = shfl2(m.r[2 * j + 1], src);
    }
  }
  const bool take = UP || lane < 48;
#pragma unroll
  for (int j = 0; j < kXaRowModes; ++j) {
    const float c = take ? (j == 0 ? xw.x : xw.z) : 0.f, sn = take ? (j == 0 ? xw.y : xw.w) : 0.f;
    rot(pa[j], pb[j], c, sn);
    m.r[2 * j] += pa[j];
    m.r[2 * j + 1] += pb[j];
  }
}

// The table pointer, but only once v is computed: scalar reads through it cannot be
// hoisted above v (the scheduler would otherwise issue every row's reads at once and spill).
__device__ __forceinline__ CT after(CT p, v2f v) {
  asm volatile("" : "+s"(p) : "v"(v));
  return p;
}

// acc + sum_r row[r] m_r: one output's zero-input response to a modal state (row: 8 floats,
// read by scalar loads)
__device__ __forceinline__ v2f add_modal(v2f acc, const float __attribute__((address_space(4))) *row,
                                         const Md &m) {
  if (XA_EXP & 2) return acc + m.r[0];
#pragma unroll
  for (int r = 0; r < 8; ++r) acc = vfma(splat(row[r]), m.r[r], acc);
  return acc;
}

// the state entering a lane, rotated over one sub-block and folded into that lane's end
// state before the scan
template <int PASS>
__device__ __forceinline__ void fold_entering(Md &m, const Md &in, CT tab, bool here) {
  CT t = fresh(tab);
  Md u = in;
#pragma unroll
  for (int j = 0; j < 4; ++j) rot(u.r[2 * j], u.r[2 * j + 1], pass_of<PASS>(t).pS[j][0], pass_of<PASS>(t).pS[j][1]);
  if (here) {
#pragma unroll
    for (int r = 0; r < 8; ++r) m.r[r] += u.r[r];
  }
}

// Diagnostic build only (-DXA_STAMPS=1, tools/build_variants.py): per-phase s_memtime
// sums of every wave, read back with zfft_debug_xa_stamps; no stamp exists otherwise.
[[maybe_unused]] constexpr int kStampSegs = 10;
#if XA_STAMPS
__device__ unsigned long long g_xa_stamps[kStampSegs + 1];
#define XA_STAMP(i)                                                                   \
  {                                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                                \
    unsigned long long t_;                                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
    __builtin_amdgcn_sched_barrier(0);                                                \
    st_acc[i] += t_ - t_prev;                                                         \
    t_prev = t_;                                                                      \
  }
#else
#define XA_STAMP(i)
#endif

template <int B, bool MIX, int DT, int FLIP>
__global__ __launch_bounds__(64 * kWaves, Geo<B>::kWavesPerSimd) void xa_stage_kernel(
    InDesc in, int n, const v2f *__restrict__ lo, v2f *__restrict__ out, int frames, const XaTab *tab_g) {
  using G = Geo<B>;
  constexpr int K = G::K, T = G::T, kRow = G::kRow, kHeldRow = G::kHeldRow, kChunks = G::kOutChunks;
  __shared__ __attribute__((aligned(16))) v2f lds_all[kWaves][G::kBuf];
  const CT tab = (CT)tab_g;
  // lag rows, copied once as two planes (the rows' first and second 16 B): a lane per row
  // d reads 16 B at a 16-B stride, conflict-free per ds_read_b128 group (rows of 32 B, read
  // whole, put 16 lanes on 8 bank slots: 2-way)
  __shared__ __attribute__((aligned(16))) v4f lag_l[kXaLag * 2];
  for (int i = threadIdx.x; i < kXaLag * 2; i += 64 * kWaves)
    lag_l[(i & 1) * kXaLag + (i >> 1)] = ((const v4f *)tab_g->lag)[i];
  __shared__ v4f xw_l[2][16];  // cross-row scan weights (XaPass::xr), forward / backward
  if (threadIdx.x < 32) xw_l[threadIdx.x >> 4][threadIdx.x & 15] = ((const v4f *)((threadIdx.x >> 4) ? tab_g->b.xr : tab_g->f.xr))[threadIdx.x & 15];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // SGPR
  const int f = blockIdx.x * kWaves + wv;
  if (f >= frames) return;  // whole wave
  if constexpr (MIX) lo = lo_row(lo, in, f);  // this frame's LO (config 4: one per IF)
  const LP buf0 = (LP)lds_all[wv];           // half-tile transposes: 32 rows of kRow v2f
  LP buf = buf0;
  LP pcarry = buf + G::kMain;  // lane 63's FIR neighbour part, for next lane 0
  LP vcarry = pcarry + 16;                  // the 64 v before the last tile
  const int e = n + 2 * kPad, n_out = (n + 1) >> 1;
  const int nt = (e + 15) / T + 1;  // the last FIR/backward tile reaches e - 1
  v2f *__restrict__ o = out + (int64_t)f * n_out;
  const __amdgpu_buffer_rsrc_t orsrc =  // the frame's output row (wide stores)
      __builtin_amdgcn_make_buffer_rsrc((void *)o, (short)0, n_out * 8, 0x00020000);
  auto X = [&](int i) -> v2f {
    v2f v = load_in_t<DT, FLIP>(in, f, i);
    if constexpr (MIX) v = cmul(v, lo[i]);
    return v;
  };
  auto ext = [&](int j) -> v2f {  // scipy odd_ext by 27 (_arraytools.py:57); 0 beyond e
    if (j < kPad) return 2.f * X(0) - X(kPad - j);
    if (j < n + kPad) return X(j - kPad);
    if (j < e) return 2.f * X(n - 1) - X(2 * n + kPad - 2 - j);
    return splat(0.f);
  };

  const v2f x0 = v2f{uni(ext(0).x), uni(ext(0).y)};
  Md m_in;  // modal state entering the current tile (forward), wave-uniform
#pragma unroll
  for (int r = 0; r < 8; ++r) m_in.r[r] = tab->f.ss[r] * x0;
  {  // v pre-history (steady output for constant ext[0]): the FIR part lane -1 owes lane 0
    const v2f vs = tab->vss * x0;
    if (lane < 12) {
      CT tb = fresh(tab);
      v2f acc = splat(0.f);
      for (int t = 0; t < 25; ++t)  // taps on W[m], 1 <= m <= 23, of output k = lane
        if (2 * lane + t + 1 < 24) acc = vfma(splat(tb->m25[t]), vs, acc);
      pcarry[lane] = acc;
    }
    vcarry[lane] = vs;
  }
  __builtin_amdgcn_wave_barrier();

  auto m_of = [&](int tile, int idx) { return tile * (T / 2) - (kPad + 15) / 2 + idx; };
  // Tile outputs -> frame row through LDS transposes (64 consecutive outputs per store
  // instruction), one half tile at a time.  Chunks below the top kXaLag outputs are final
  // at once; the top chunks wait in registers for the next tile's exact top state q.
  v2f held[kLagChunks];
#pragma unroll
  for (int c = 0; c < kLagChunks; ++c) held[c] = splat(0.f);
  auto flush_tile = [&](int tile, const v2f *h, int ln) {
    const int m0 = m_of(tile, ln);
    v2f *__restrict__ od = o + m0;
    const bool inside = m_of(tile, 0) >= 0 && m_of(tile, T / 2) <= n_out;  // wave-uniform
    {  // every lane's K outputs into row ln, one LDS round trip
      {
        LP4 hw = (LP4)(buf + ln * kHeldRow);
#pragma unroll
        for (int k = 0; k < K / 2; ++k) hw[k] = v4f{h[2 * k].x, h[2 * k].y, h[2 * k + 1].x, h[2 * k + 1].y};
      }
      __builtin_amdgcn_wave_barrier();
      // output idx = 64 c + ln sits at row idx/K, column idx % K
      const LP hr = buf + (ln / K) * kHeldRow + (ln % K);
      v2f vc[kChunks];
      // wide: the final outputs 0 .. 128 nw - 1 as pairs (128 C + 2 ln + {0, 1}: row 8 C +
      // ln/8, cols 2 (ln%8) + {0, 1}; one b128 read, one 16-B store), the rest one per lane
      constexpr int nw = (kChunks - kLagChunks) / 2;
      v4f vw[nw > 0 ? nw : 1];
      if constexpr (nw > 0) {
        const LP4 hr2 = (LP4)(buf + (ln / 8) * kHeldRow + 2 * (ln % 8));
#pragma unroll
        for (int c = 0; c < nw; ++c) vw[c] = hr2[c * (8 * kHeldRow / 2)];
      }
#pragma unroll
      for (int c = 2 * nw; c < kChunks; ++c) vc[c] = hr[c * (64 / K) * kHeldRow];
      if (inside && (XA_EXP & 16)) {
        if (vw[0].x == 1.2345f && vc[kChunks - 1].x == 1.2345f) od[0] = vc[kChunks - 1];
      } else if (inside) {
#pragma unroll
        for (int c = 0; c < nw; ++c)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, vw[c]), orsrc,
                                                 (uint32_t)(m_of(tile, 128 * c + 2 * ln) * 8), 0, kStoreAux);
#pragma unroll
        for (int c = 2 * nw; c < kChunks - kLagChunks; ++c) st_out(od + 64 * c, vc[c]);
      } else {
#pragma unroll
        for (int c = 0; c < nw; ++c) {
          const int m = m_of(tile, 128 * c + 2 * ln);
          if (m >= 0 && m < n_out) o[m] = v2f{vw[c].x, vw[c].y};
          if (m + 1 >= 0 && m + 1 < n_out) o[m + 1] = v2f{vw[c].z, vw[c].w};
        }
#pragma unroll
        for (int c = 2 * nw; c < kChunks - kLagChunks; ++c)
          if (m0 + 64 * c >= 0 && m0 + 64 * c < n_out) od[64 * c] = vc[c];
      }
#pragma unroll
      for (int c = kChunks - kLagChunks; c < kChunks; ++c) held[c - (kChunks - kLagChunks)] = vc[c];
      __builtin_amdgcn_wave_barrier();
    }
  };
  auto finish_held = [&](int tile, const Md *q, const v4f *lg, int ln) {  // + C A2^d T q
    const int m0 = m_of(tile, (kChunks - kLagChunks) * 64 + ln);
#pragma unroll
    for (int c = 0; c < kLagChunks; ++c) {
      v2f v = held[c];
      if (q != nullptr) {
        const v4f l0 = lg[2 * c], l1 = lg[2 * c + 1];
        v = vfma(splat(l0.x), q->r[0], v);
        v = vfma(splat(l0.y), q->r[1], v);
        v = vfma(splat(l0.z), q->r[2], v);
        v = vfma(splat(l0.w), q->r[3], v);
        v = vfma(splat(l1.x), q->r[4], v);
        v = vfma(splat(l1.y), q->r[5], v);
        v = vfma(splat(l1.z), q->r[6], v);
        v = vfma(splat(l1.w), q->r[7], v);
      }
      held[c] = v;
    }
    // wave-uniform: every held output of the tile inside the frame -> unconditional stores
    const bool inside = m_of(tile, (kChunks - kLagChunks) * 64) >= 0 && m_of(tile, kChunks * 64) <= n_out;
    if (inside) {
#pragma unroll
      for (int c = 0; c < kLagChunks; ++c) st_out(o + m0 + 64 * c, held[c]);
    } else {
#pragma unroll
      for (int c = 0; c < kLagChunks; ++c) {
        const int m = m0 + 64 * c;
        if (m >= 0 && m < n_out) o[m] = held[c];
      }
    }
  };

  // coalesced tile loads: sample s = 64 q + lane of the tile -> row s/B, col s%B, in two
  // halves of 32 rows; a fast tile (inside [27, n + 27): no odd extension) is loaded during
  // the previous tile, through a range-checked buffer resource over the frame, for every
  // tile (out-of-range lanes read 0; an edge tile never reads them): the prefetch registers
  // are then dead between their use at the tile start and their reload
  typedef typename Raw<DT>::T RawT;
  const RawT *__restrict__ src = (const RawT *)in.p + (int64_t)f * in.stride;
  auto fast_tile = [&](int b) { return b >= kPad && ((XA_EXP & 64) || b + T <= n + kPad); };
  // chunk q = samples 128 q + 2 lane + {0, 1}: a pair per lane (16 B for complex64; one
  // element per lane measured 4.5 % slower at stage 0)
  constexpr int kPer = 2;           // elements per lane and chunk
  constexpr int kCh = B / kPer;     // input chunks per tile
  constexpr int kSpan = 64 * kPer;  // samples per chunk
  static_assert(B == 32, "the pair layout of the tile loads assumes 32-sample lane rows");
  typedef Pair<DT> LoadT;
  // lo[n0 + l] = lo[n0] lo[l] / sqrt(2): the chunk start times a per-lane factor (one per
  // element of the lane); lo has >= 2048 entries whenever a fast tile exists (L > 2048)
  v2f wl0 = splat(0.f), wl1 = splat(0.f);
  if constexpr (MIX) {
    wl0 = lo[min(kPer * lane, n - 1)] * 0.70710678118654752f;
    wl1 = lo[min(kPer * lane + 1, n - 1)] * 0.70710678118654752f;
  }
  v2f cqv = splat(0.f);  // lo[next tile start - 27 + kSpan (lane % kCh)], loaded a tile ahead
  LoadT pf[kCh];         // the next tile's input chunks
  bool next_fast = false;
  int next_i0 = 0;  // first input index of the next tile
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void *)src, (short)0, (int)(in.len * (int64_t)sizeof(RawT)), 0x00020000);
  uint32_t next_off = 0;  // byte offset of this lane's (first) element of the next tile's chunk 0
  // next-tile loads: group g = chunks [g kCh/8, (g+1) kCh/8), issued at 8 points of the tile
  auto issue_group = [&](int g) {
    if ((XA_EXP & 8) && next_i0 > 4 * T) return;
    if (MIX && g == 0 && next_fast) cqv = lo[next_i0 + kSpan * (lane % kCh)];
#pragma unroll
    for (int q = g * (kCh / 8); q < (g + 1) * (kCh / 8); ++q)
      pf[q] = buf_load<LoadT>(rsrc, next_off + (uint32_t)((FLIP ? -kSpan : kSpan) * q * (int)sizeof(RawT)));
  };

#if XA_STAMPS
  unsigned long long st_acc[kStampSegs] = {}, t_prev;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_prev)::"memory");
#endif
  for (int tau = 0; tau < nt; ++tau) {
    // an opaque copy of the ln id per tile: ln-derived addresses are recomputed
    // (a few VALU ops) instead of dozens of them being hoisted and held (or spilled)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    {  // opaque per-tile copy of the LDS base, for the same reason
      LP b = buf0;
      asm volatile("" : "+s"(b));
      buf = b;
      pcarry = buf + G::kMain;
      vcarry = pcarry + 16;
    }
    const int base = tau * T;
    const bool last = tau == nt - 1;
    v2f y[B];
    {
      const bool fast = fast_tile(base);  // wave-uniform
      LP st = buf + (ln / B) * kRow + (ln % B);
      // the fast and the edge path are separate blocks end to end: raw registers of the
      // fast path never live across the edge path's code (which would force their spill)
      auto read_all_rows = [&]() {  // every lane its row (half ln / 32), both halves at once
        __builtin_amdgcn_wave_barrier();
        const LP4 rp = (LP4)(buf + (ln >> 5) * (kHalfRows * kRow) + (ln & 31) * kRow);
#pragma unroll
        for (int t = 0; t < B / 2; ++t) {
          const v4f w = rp[t];
          y[2 * t] = v2f{w.x, w.y};
          y[2 * t + 1] = v2f{w.z, w.w};
        }
        __builtin_amdgcn_wave_barrier();
      };
      auto fast_chunk = [&](int q) -> v4f {
        // FLIP: the pair was read from descending addresses, so its halves swap
        v2f x0 = cvt_raw<DT>(FLIP ? pf[q].b : pf[q].a), x1 = cvt_raw<DT>(FLIP ? pf[q].a : pf[q].b);
        if constexpr (MIX && !(XA_EXP & 4)) {
          const v2f c = lane_of(cqv, q);  // lane q holds chunk q's start (LDS: 1 % slower)
          x0 = cmul2(x0, cmul2(c, wl0));
          x1 = cmul2(x1, cmul2(c, wl1));
        }
        return v4f{x0.x, x0.y, x1.x, x1.y};
      };
      if (fast) {
        // sample s at row s/B, col s%B; chunk q's pair of lane l is row 4q + l/16, cols
        // 2 (l%16) + {0, 1}: one b128; the 64 rows contiguous (both halves at once)
        const LP4 st2 = (LP4)(buf + (ln / 16) * kRow + 2 * (ln % 16));
#pragma unroll
        for (int q = 0; q < kCh; ++q) st2[q * (4 * kRow / 2)] = fast_chunk(q);
        read_all_rows();
      } else {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
#pragma unroll 4
          for (int qq = 0; qq < B / 2; ++qq)
            st[hf * kHalfRows * kRow + G::kRowsPerChunk * kRow * qq] = ext(base + ln + 64 * (hf * (B / 2) + qq));
        }
        read_all_rows();
      }
    }
    next_fast = tau + 1 < nt && fast_tile(base + T);  // wave-uniform
    next_i0 = base + T - kPad;
    {  // (FLIP: the pair's elements i0, i0 + 1 sit at len-1-i0 and len-2-i0)
      const int i0 = base + T - kPad + kPer * ln;
      next_off = (uint32_t)((FLIP ? in.len - kPer - i0 : (int64_t)i0) * (int64_t)sizeof(RawT));
    }
    // the next tile's loads: groups 0-3 now, 4-5 after the forward pass, 6-7 after the scan
    // (later issue points leave the register allocator room it does not use: spills; all
    // eight groups at the tile start measured no faster)
    issue_group(0);
    issue_group(1);
    issue_group(2);
    issue_group(3);
    XA_STAMP(0);

    // ---- forward all-pole cascade: one pass from a zero state streaming the FIR (v0 -> h
    //      and the neighbour share P); the modal scan over lanes then gives each lane its
    //      exact entering state, whose zero-input response C A^t T m enters h and P through
    //      the tables gown / gnb (the FIR of it, precomputed) instead of a second pass ----
    v2f h[K];
    Md me;  // state entering this ln's sub-block
    {
      v2f P[12];
#pragma unroll
      for (int k = 0; k < K; ++k) h[k] = splat(0.f);
#pragma unroll
      for (int k = 0; k < 12; ++k) P[k] = splat(0.f);
      {
        Md m;
        {
          float a1[4], a2[4];
          v2f s[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) s[r] = splat(0.f);
          // the pass + FIR constants as SGPRs (wide scalar loads): this phase holds the
          // most VGPRs of the tile
          const CT tbs = fresh(tab);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            a1[k] = tbs->f.a1[k];
            a2[k] = tbs->f.a2[k];
          }
          float m25s[25];
#pragma unroll
          for (int t = 0; t < 25; ++t) m25s[t] = tbs->m25[t];
          // frame end: the 64 v before the last tile (lanes 64 - 64/B .. 63 of the tile
          // before it) and the last tile's two lanes around e-25 .. e-1 go to LDS for
          // f = N v -- v0 after the pass (v overwrites y in place), the entering state's part
          // once it is known.  The neighbour share P is accumulated from the last 23 v after
          // the pass (accumulating it inside the pass measured no faster).
          {
            LP wrow = buf;
            bool wlane = false;
            if (tau >= nt - 2) {
              const int la = max(0, (e - 25 - base) / B);
              wlane = (!last && ln >= 64 - 64 / B) || (last && (ln == la || ln == la + 1));
              // (no null test on an LDS pointer: LDS address 0 is this workgroup's first row)
              wrow = last ? buf + (ln - la) * kRow : vcarry + (ln - (64 - 64 / B)) * B;
            }
#pragma unroll
            for (int t = 0; t < B; ++t) {
              if (XA_EXP & 32) {
                h[t / 2] += y[t];
                if (t >= 20) s[t & 7] += y[t];
                continue;
              }
              const v2f v = ap_step(y[t], s, a1, a2);
#pragma unroll
              for (int k = 0; k < K; ++k) {
                const int tap = 24 + t - 1 - 2 * k;
                if (tap >= 0 && tap < 25) h[k] = vfma(splat(m25s[tap]), v, h[k]);
              }
              y[t] = v;
            }
            // this lane's share of its right neighbour's outputs: W[m] = v[B - 24 + m],
            // 1 <= m < 24
#pragma unroll
            for (int t = B - 23; t < B; ++t) {
#pragma unroll
              for (int k = 0; k < 12; ++k) {
                const int tap = t - (B - 24) - 1 - 2 * k;
                if (tap >= 0 && tap < 25) P[k] = vfma(splat(m25s[tap]), y[t], P[k]);
              }
            }
            if (wlane) {
              LP4 wp = (LP4)wrow;
#pragma unroll
              for (int t = 0; t < B / 2; ++t) wp[t] = v4f{y[2 * t].x, y[2 * t].y, y[2 * t + 1].x, y[2 * t + 1].y};
            }
          }
          to_modal<0>(tab, s, m);
        }
        XA_STAMP(1);
        issue_group(4);
        issue_group(5);
        fold_entering<0>(m, m_in, tab, ln == 0);
        modal_scan<B, 0, true>(m, tab, ln, xw_l[0][ln & 15]);
#pragma unroll
        for (int r = 0; r < 8; ++r) me.r[r] = wave_shift<kShr1>(m_in.r[r], m.r[r]);
#pragma unroll
        for (int r = 0; r < 8; ++r) m_in.r[r] = lane_of(m.r[r], 63);  // next tile's entering state
      }
      XA_STAMP(2);
      issue_group(6);
      issue_group(7);
      // + the entering state's response through the FIR (own outputs, neighbour share);
      // row k's constants are read once output k-4 is done (at most 4 rows in flight)
      // (scalar reads; row k once output k-4 is done: LDS broadcast reads measured 6 % slower)
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const CT t = k >= 4 ? after(tab, h[k - 4]) : fresh(tab);
        h[k] = add_modal(h[k], t->gown[k], me);
      }
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        const CT t = after(tab, k >= 4 ? P[k - 4] : h[K - 4 + k]);
        P[k] = add_modal(P[k], t->gnb[k], me);
      }
      {  // neighbour shares: ln i takes ln i-1's P, ln 0 the previous tile's ln 63's
        const LP4 pc = (LP4)pcarry;
#pragma unroll
        for (int k2 = 0; k2 < 6; ++k2) {
          const v4f c4 = pc[k2];
          h[2 * k2] += wave_shift<kShr1>(v2f{c4.x, c4.y}, P[2 * k2]);
          h[2 * k2 + 1] += wave_shift<kShr1>(v2f{c4.z, c4.w}, P[2 * k2 + 1]);
        }
        __builtin_amdgcn_wave_barrier();
        if (ln == 63) {
          LP4 pw = (LP4)pcarry;
#pragma unroll
          for (int k2 = 0; k2 < 6; ++k2) pw[k2] = v4f{P[2 * k2].x, P[2 * k2].y, P[2 * k2 + 1].x, P[2 * k2 + 1].y};
        }
      }
    }
    XA_STAMP(3);
    const int la = max(0, (e - 25 - base) / B);
    if (tau >= nt - 2 && ((!last && ln >= 64 - 64 / B) || (last && (ln == la || ln == la + 1)))) {
      // v = v0 + C A^t T me on the rows stored after the pass
      LP wp = last ? buf + (ln - la) * kRow : vcarry + (ln - (64 - 64 / B)) * B;
#pragma unroll 4
      for (int t = 0; t < B; ++t) {
        CT tb = fresh(tab);
        v2f acc = wp[t];
#pragma unroll
        for (int r = 0; r < 8; ++r) acc = vfma(splat(tb->fcat[t][r]), me.r[r], acc);
        wp[t] = acc;
      }
    }
    __builtin_amdgcn_wave_barrier();
    v4f lg[2 * kLagChunks];
    XA_STAMP(4);
    v2f h_ss = splat(0.f);  // backward steady input (last tile only)
    if (last) {
      // f = N v explicitly for s in [e-16, e-1] (clamped at e-1 beyond), one value per
      // lane 0..15; h at the odd j in (e-17, e-1] in the unmerged form, one per lane 0..7
      auto v_at = [&](int p) -> v2f {
        const int r = p - base;
        return r < 0 ? vcarry[64 + r] : buf[(r / B - la) * kRow + (r % B)];
      };
      LP fbuf = buf + 2 * kRow, tbuf = buf + 3 * kRow;
      if (ln < 16) {
        CT tb = fresh(tab);
        v2f acc = splat(0.f);
        for (int i = 0; i < 9; ++i) acc = vfma(splat(tb->n9[i]), v_at(e - 16 + ln - i), acc);
        fbuf[ln] = acc;
      }
      __builtin_amdgcn_wave_barrier();
      const v2f fe = fbuf[15];
      h_ss = fe * fresh(tab)->mp_sum;
      const int j0 = (e - 16) | 1;  // first odd position above e-17
      if (ln < 8 && j0 + 2 * ln <= e - 1) {
        CT tb = fresh(tab);
        const int j = j0 + 2 * ln;
        v2f acc = splat(0.f);
        for (int t = 0; t < 17; ++t) {
          const int sidx = j + t - (e - 16);
          acc = vfma(splat(tb->mp17[t]), sidx < 16 ? fbuf[sidx] : fe, acc);
        }
        tbuf[ln] = acc;
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int j = base + B * ln - 15 + 2 * k;
        if (j > e - 1) h[k] = h_ss;
        else if (j > e - 17) h[k] = tbuf[(j - j0) >> 1];
      }
      __builtin_amdgcn_wave_barrier();
    }
    XA_STAMP(5);

    // ---- backward all-pole cascade on h, descending (ln 63 holds the tile top): one pass
    //      from a zero state, the scan down, then the entering state's zero-input response
    //      C A2^d T q (the first rows of the lag table) added to each output ----
    Md q_exit;
    {
      Md qe;
      {
        Md m;
        {
          float a1[4], a2[4];
          load_ap<1>(tab, a1, a2);
          v2f s[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) s[r] = splat(0.f);
#pragma unroll
          for (int k = K - 1; k >= 0; --k) h[k] = ap_step(h[k], s, a1, a2);
          to_modal<1>(tab, s, m);
        }
        XA_STAMP(6);
        Md qtop;  // state entering the tile from above: exact steady state on the last tile
        {
          CT tb = fresh(tab);
#pragma unroll
          for (int r = 0; r < 8; ++r) qtop.r[r] = last ? tb->b.ss[r] * h_ss : splat(0.f);
        }
        if (last) fold_entering<1>(m, qtop, tab, ln == 63);
        modal_scan<B, 1, false>(m, tab, ln, xw_l[1][ln & 15]);
#pragma unroll
        for (int r = 0; r < 8; ++r) qe.r[r] = wave_shift<kShl1>(qtop.r[r], m.r[r]);
#pragma unroll
        for (int r = 0; r < 8; ++r) q_exit.r[r] = lane_of(m.r[r], 0);
      }
#pragma unroll
      for (int k = K - 1; k >= 0; --k) {
        const CT t = k < K - 4 ? after(tab, h[k + 4]) : fresh(tab);
        h[k] = add_modal(h[k], t->lag[K - 1 - k], qe);
      }
    }
    XA_STAMP(7);
    // ---- the tile below is complete: its top state is this tile's bottom state ----
    if (tau > 0) {
#pragma unroll
      for (int c = 0; c < kLagChunks; ++c) {
        const int d = kXaLag - 1 - 64 * c - ln;
        lg[2 * c] = lag_l[d];
        lg[2 * c + 1] = lag_l[kXaLag + d];
      }
      finish_held(tau - 1, &q_exit, lg, ln);
    }
    XA_STAMP(8);
    flush_tile(tau, h, ln);
    XA_STAMP(9);
  }
  finish_held(nt - 1, nullptr, nullptr, lane);  // the last tile's top state was exact
#if XA_STAMPS
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < kStampSegs; ++i) atomicAdd(&g_xa_stamps[i], st_acc[i]);
    atomicAdd(&g_xa_stamps[kStampSegs], (unsigned long long)nt);
  }
#endif
}

template <int B, bool MIX, int DT, int FLIP>
static void xa_launch(const InDesc &in, int n, const float2 *lo, float2 *out, int frames,
                      const XaTab *tab, hipStream_t st) {
  hipLaunchKernelGGL((xa_stage_kernel<B, MIX, DT, FLIP>), dim3((unsigned)((frames + kWaves - 1) / kWaves)),
                     dim3(64 * kWaves), 0, st, in, n, (const v2f *)lo, (v2f *)out, frames, tab);
}

template <int B>
static hipError_t xa_dispatch(const InDesc &in, int n, const float2 *lo, bool mix, float2 *out,
                              int frames, const XaTab *tab, hipStream_t st) {
  if (!mix) {
    if (in.dtype != kInC64 || in.flip) return hipErrorInvalidValue;  // stages >= 1: internal
    xa_launch<B, false, kInC64, 0>(in, n, lo, out, frames, tab, st);
  } else if (in.dtype == kInC64) {
    if (in.flip) xa_launch<B, true, kInC64, 1>(in, n, lo, out, frames, tab, st);
    else xa_launch<B, true, kInC64, 0>(in, n, lo, out, frames, tab, st);
  } else if (in.dtype == kInC32H) {
    if (in.flip) xa_launch<B, true, kInC32H, 1>(in, n, lo, out, frames, tab, st);
    else xa_launch<B, true, kInC32H, 0>(in, n, lo, out, frames, tab, st);
  } else if (in.dtype == kInF32R) {
    if (in.flip) xa_launch<B, true, kInF32R, 1>(in, n, lo, out, frames, tab, st);
    else xa_launch<B, true, kInF32R, 0>(in, n, lo, out, frames, tab, st);
  } else {
    if (in.flip) xa_launch<B, true, kInCU8, 1>(in, n, lo, out, frames, tab, st);
    else xa_launch<B, true, kInCU8, 0>(in, n, lo, out, frames, tab, st);
  }
  return hipGetLastError();
}

}  // namespace xa

// Debug hook (not part of zfft.h): copies and clears the stamp sums of a XA_STAMPS build
// (segment cycles summed over waves, then the tile count); -1 in a normal build.
extern "C" int zfft_debug_xa_stamps(unsigned long long *out) {
#if XA_STAMPS
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(xa::g_xa_stamps), sizeof(xa::g_xa_stamps)) != hipSuccess) return -2;
  unsigned long long z[xa::kStampSegs + 1] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(xa::g_xa_stamps), z, sizeof(z)) == hipSuccess ? 0 : -2;
#else
  (void)out;
  return -1;
#endif
}

hipError_t launch_xa_stage(const InDesc &in, int n, const float2 *lo, bool mix, float2 *out,
                           int frames, const XaTab *tab, hipStream_t st) {
  return xa::xa_dispatch<kXaB>(in, n, lo, mix, out, frames, tab, st);
}

}  // namespace zfft
