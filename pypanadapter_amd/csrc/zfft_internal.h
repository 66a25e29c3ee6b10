// Internal declarations shared by the plan (zfft_plan.cpp) and the HIP kernels
// (zfft_kernels.hip).  Not part of the C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace zfft {

constexpr int kPad = 27;      // sosfiltfilt odd-extension length (3 * ntaps)
constexpr int kMaxLdsFft = 16384;

// float32 copy of the ↓2 Chebyshev-I SOS cascade (cheby1_q2.h); passed by value as a
// kernel argument so every coefficient lives in SGPRs.
struct Sos32 {
  float b0, b1, b2;  // section 0 numerator; sections 1..3 are exactly [1, 2, 1]
  float a1[4], a2[4];
  float zi[4][2];    // sosfilt_zi
};

Sos32 sos32();

// The caller's frames (the `chunk` of S:2102 / T:1516): sample i of frame f is element
// f * stride + (flip ? len - 1 - i : i) of p, in one of the zfft_config in_dtype formats:
//   0 complex64 (interleaved f32), 1 complex32 (interleaved f16, BASELINE cfg5),
//   2 RTL-SDR interleaved uint8 I,Q, value b/127.5 - 1 (pyrtlsdr packed_bytes_to_iq),
//   3 real float32 (AudioPan's pyaudio paFloat32 stream, S:712-713): I = x, Q = 0.
// flip fuses the sources' np.flip (S:541-543, 459-460) into the stage-0 loads.
enum InDtype { kInC64 = 0, kInC32H = 1, kInCU8 = 2, kInF32R = 3 };
// LO rows (config 4, batched multi-IF): the mixer table holds lo_n rows of lo_stride
// entries; frame f of a call uses row ((lo_first + f) / lo_per) % lo_n (lo_first: the call's
// first frame within a batched host call).  One row (the default) = the plan's f_lo.
struct InDesc {
  const void *p;
  int64_t stride, len;
  int dtype, flip;
  int64_t lo_stride = 0;
  int lo_n = 1, lo_per = 1, lo_first = 0;
};
inline size_t in_elem_bytes(int dtype) { return dtype == kInC64 ? 8 : (dtype == kInC32H || dtype == kInF32R) ? 4 : 2; }

// --- kernels (zfft_kernels.hip); all enqueue on `st`, return hipError_t of the launch ---
// Intermediates use the frame-group-interleaved (FGI) layout: element (f, j) of a
// per-frame sequence of length len lives at ((f/64)*len + j)*64 + f%64 (float2 units);
// buffers hold ngroups = ceil(frames/64) full groups.
struct StageGeom {
  int n;        // stage input length
  int nblk;     // blocks per frame: ceil((n + 27) / block)
  int block;    // S, samples per block (multiple of 16)
  int warmup;   // W, warm-up samples (multiple of 16)
  int ngroups;  // 64-frame groups
  int split = 0;         // stage 0 only: frame groups >= split read a second window set ...
  int64_t alt_off = 0;   // ... starting alt_off samples into each frame (edge windows)
};

hipError_t launch_iir_forward_mix(const InDesc &in, int frames, const float2 *lo,
                                  float2 *yf, const StageGeom &g, hipStream_t st);
hipError_t launch_iir_forward_fgi(const float2 *in, float2 *yf, const StageGeom &g,
                                  hipStream_t st);
hipError_t launch_iir_backward(const float2 *yf, float2 *out, bool natural, int frames,
                               const StageGeom &g, hipStream_t st);

// Fused interior pass pair (commuted stage order, zfft_kernels.hip fused_pass_kernel).
struct FusedGeom {
  int in_len;   // FGI input length (with pads when in_off > 0)
  int in_off;   // 27 when the input is in padded "ext" coordinates, else 0
  int n_mid;    // decimated length ceil((in_len - 2*in_off) / 2) = output length
  int block;    // S in output units (multiple of 16)
  int nblk;     // ceil(n_mid / S)
  int w1, w2;   // warm-up of pass 1 (input rate) and pass 2 (output rate)
  int ngroups;  // 64-frame groups
};

hipError_t launch_fused_pass(const float2 *in, float2 *out, bool desc, bool two, bool nat,
                             const FusedGeom &g, int frames, hipStream_t st);

// "XA" decimation stage (xa_kernels.hip; design model tools/xa_proto.py).  The cascade
// H = N(z)/D(z), N = b0 (1+z^-1)^8, is run as a forward all-pole cascade 1/D(z) at the
// input rate, a 25-tap FIR M = N(z) N(1/z) D(-1/z) evaluated only at the kept (odd)
// positions, and a backward all-pole cascade 1/D2(w), D2(z^2) = D(z) D(-z), at the output
// rate: 8 + 12.5 + 4 multiply-adds per input sample instead of 2 x 17 for two DF2T passes,
// with scipy's pad / steady-state edge rules carried over exactly.  One wave per frame,
// tiles of 64 lanes x B samples (B = 32 or 64), states scanned over lanes in the real modal
// basis of each all-pole cascade (sections slowest pole first, the lower-error fp32 order).
constexpr int kXaLag = 192;          // held-tile outputs corrected by the one-tile lag
constexpr int kXaB = 32;             // lane sub-block: samples per lane and tile
constexpr int kXaRowModes = 2;       // modes scanned inside 16-lane DPP rows (+ one cross-row step)
// Scan levels of mode j for lane sub-blocks of B forward samples (B/2 backward): mode j
// needs |lambda_j|^(S 2^levels) < 1e-9 (radii .935 .808 .682 .587, the backward poles
// squared at half the steps); checked when the tables are built.  Modes 0, 1 scan inside
// 16-lane rows (DPP row shifts, <= 4 levels) and then add the adjacent row's end lane;
// modes 2, 3 take one whole-wave shift (1 level).
__host__ __device__ constexpr int xa_levels(int B, int j) {
  return B == 32 ? (j == 0 ? 4 : j == 1 ? 2 : 1) : (j == 0 ? 3 : 1);
}
struct XaPass {                      // one all-pole cascade, DF-I state (y[t-1], y[t-2]) per section
  float a1[4], a2[4];                // y = x - a1 y[t-1] - a2 y[t-2], cascade order
  float ti[8][8];                    // T^-1: state -> real modal (block lower triangular)
  float t[8][8];                     // T: real modal -> state (block lower triangular)
  float ss[8];                       // modal steady state per unit constant input
  float pS[4][2];                    // lambda_j^S (one lane sub-block of S steps)
  float scan[4][4][2];               // lambda_j^(S 2^d), scan level d
  // modes 0, 1 cross the 16-lane DPP rows once: weight lambda_j^(S dist) of the adjacent
  // row's end lane for lane-in-row i (dist = i + 1 forward, 16 - i backward): c0 s0 c1 s1
  alignas(16) float xr[16][4];
};
struct XaTab {
  XaPass f, b;                       // forward (full rate, S = B), backward (S = B/2)
  float m25[25];                     // M on v[j-8 .. j+16]
  float mp17[17];                    // N(1/z) D(-1/z) on f[j .. j+16] (frame-end form)
  float n9[9];                       // N on v[s .. s-8] (f = N v, frame-end form)
  float mp_sum;                      // h per unit constant f (backward steady input)
  float vss;                         // forward cascade output per unit constant input
  float pad_[2];
  alignas(16) float lag[kXaLag][8];  // backward C A2^d T: held output d steps below the top
  // forward zero-input responses (the exact entering state's part, added after the zero-state
  // pass instead of a second pass): C A^t T for the B own samples, and their images through
  // the FIR -- on this lane's K outputs (gown) and on its share of the next lane's 12 (gnb)
  alignas(16) float fcat[kXaB][8];
  alignas(16) float gown[kXaB / 2][8];
  alignas(16) float gnb[12][8];
};

hipError_t launch_xa_stage(const InDesc &in, int n, const float2 *lo, bool mix,
                           float2 *out, int frames, const XaTab *tab, hipStream_t st);

// "PC" (polyphase cascade) decimator for zoom 8 (pc_kernels.hip, host tables pc_tables.cpp,
// design model tools/pc_model.py).  The interior of the three zero-phase stages is, exactly,
//   y1 = (g0 * x)|2, y2 = (g1 * y1)|2        FIRs (33, 49 taps): every all-pole factor of
//                                            stages 0-1 moved to the output rate (polyphase)
//   z2 = S(v) S(1/v) y2                      the two slowest sections of stage 2 at their own
//                                            rate (fp32 conditioning), zero-phase
//   u3 = (g2 * z2)|2                         FIR (57 taps)
//   out = A(w) A(1/w) u3                     10 sections at the output rate (radius <= .765)
// on the zero-extended frame; the frame ends (odd extension, sosfilt_zi states) add a
// low-rank linear map of the first / last input samples onto the first / last outputs.
// K1 = the two FIRs (independent tiles) -> y2 in device memory; K2 = the rest (independent
// tiles with warm-up halos); K3 = the edge maps.  KW ("walk") = K1 + K2 in one launch, one
// workgroup per frame walking its tiles in order: y2 stays in LDS, the causal own-rate
// sections carry their state from tile to tile (no warm-up halo), the anticausal ones warm
// up over the next tile's first 1024 own-rate samples (the output tile lags the FIR tile).
constexpr int kPcStages = 3;              // zoom 8 only
constexpr int kPcQ0 = -16;                // first y2 index of the model's support
constexpr int kPcK1Q = 992;               // y2 outputs per K1 tile
constexpr int kPcK1In = 4128;             // input samples per K1 tile (from 4 q_s - 64)
constexpr int kPcK2M = 2048;              // outputs per K2 tile
constexpr int kPcK2Span = 5376;           // y2 samples per K2 tile: 256 thread blocks of 21
constexpr int kPcK2Left = 560;            // span starts at 2 m0 - 560
constexpr int kPcOwnBlk = 21;             // own-rate samples per thread
constexpr int kPcApBlk = 10;              // output-rate samples per lane (each wave a quarter)
constexpr int kPcApHalo = 64;             // output-rate warm-up per wave (0.765^64 = 3.6e-8:
                                          // the model's fp64 error 5e-8, fp32 2.5e-6 as with 96)
constexpr int kPcG0 = 33, kPcG1 = 49, kPcG2 = 57;
constexpr int kPcOwn = 2, kPcAp = 10;
constexpr int kPcEdgeR = 192, kPcEdgeJ = 1536, kPcEdgeRank = 16;  // edge map capacities
// One second-order all-pole section y[t] = x[t] - a1 y[t-1] - a2 y[t-2] run over lane blocks
// of B samples: state s = (y[t-1], y[t-2]); pw[d] = A^(B 2^d) (row-major 2x2) for the lane
// scan; ct[t] = e0 A^(t+1): output t's response to the entering state.
constexpr int kPcCt = 24;                 // zero-input response rows (>= both block lengths)
struct PcSec {
  float a1, a2, pad_[2];
  float pw[5][4];
  float ct[kPcCt][2];
};
struct PcTab {
  float g0[36], g1[52], g2[60];     // zero-phase FIR taps (centred)
  PcSec own[kPcOwn];                // B = 21 (stage 2's sections 2, 3)
  float own_x[kPcOwn][64][4];       // A^(21 (i + 1)) for lane i (cross-wave scan step)
  PcSec ap[kPcAp];                  // B = 11, slowest first
  PcSec wf[kPcOwn], wb[kPcOwn];     // KW own-rate sections: causal B = 16, anticausal B = 20
  float wf_x[kPcOwn][64][4], wb_x[kPcOwn][64][4];  // A^(B (i + 1)) for those
};
constexpr int kPcWf = 16, kPcWb = 20;    // KW own-rate block lengths (4096 / 5120 samples)
constexpr int kPcWM = 2048;              // KW outputs per tile (= kPcK2M: K2's geometry)
constexpr int kPcWQ = 1024;              // KW y2 per FIR sub-tile (4 per tile)
constexpr int kPcWM0 = -368;             // KW first tile's m0: its FIR tile starts at kPcQ0
__host__ __device__ constexpr int pc_wf_levels(int s) { return s == 0 ? 3 : 5; }
__host__ __device__ constexpr int pc_wb_levels(int s) { return s == 0 ? 3 : 4; }
// Scan levels and correction lengths the kernels are compiled for (checked by the builder).
__host__ __device__ constexpr int pc_own_levels(int s) { return s == 0 ? 3 : 4; }
__host__ __device__ constexpr int pc_ap_levels(int s) {
  return s == 0 ? 3 : s <= 3 ? 2 : s <= 6 ? 1 : 0;
}
__host__ __device__ constexpr int pc_ap_dcut(int s) { return s < 8 ? kPcApBlk : s == 8 ? 8 : 6; }
// Zoom 4 (two stages): the same construction one stage shorter --
//   y1 = (g0 * x)|2                 FIR (33 taps; stage 0's poles moved to the output rate)
//   z1 = S(u) S(1/u) y1             stage 1's two slowest sections at their own rate (= wf, wb)
//   u2 = (g1 * z1)|2                FIR (41 taps: N D2(-u) D{0,1}(-u), zero phase)
//   out = A(w) A(1/w) u2            6 sections at the output rate (D4, D2{0,1}; radius <= .765)
// run by the walk only (pc_walk_kernel<ZOOM = 4>): per tile two FIR sub-tiles of 2048 y1 (the
// input tile of zoom 8's sub-tile) go straight into the own-rate span.
constexpr int kPc4G1 = 41, kPc4Ap = 6;
constexpr int kPc4WM0 = -364;            // first tile's m0: its FIR tile starts at y1 index -8
struct PcTab4 {
  float g0[36], g1[44];             // zero-phase FIR taps (centred)
  PcSec ap[kPc4Ap];                 // B = 11, slowest first
  PcSec wf[kPcOwn], wb[kPcOwn];     // own-rate sections (those of PcTab)
  float wf_x[kPcOwn][64][4], wb_x[kPcOwn][64][4];
  PcSec own[kPcOwn];                // the tiles' own-rate sections (B = 21, those of PcTab)
  float own_x[kPcOwn][64][4];
};
// Zoom 4 as tiles (path 4; few frames per call): K1 = FIR alpha only, y1 (the own-rate signal)
// through device memory from index kPc4Q0 in tiles of 2048; K2 = zoom 8's tail kernel on y1
// with zoom 4's FIR g1 and 6 output-rate sections.
constexpr int kPc4Q0 = -8;               // first y1 index of the model's support
constexpr int kPc4K1M = 2048;            // y1 per K1 tile
int64_t pc4_y1_len(int64_t L);           // y1 entries per frame (from kPc4Q0)
hipError_t launch_pc4_fir(const InDesc &in, const float2 *lo, float2 *y1, int64_t y1_stride,
                          int frames, const PcTab4 *tab, hipStream_t st);
hipError_t launch_pc4_tail(const float2 *y1, int64_t y1_stride, int64_t y1n, float2 *out, int64_t n2,
                           int frames, const PcTab4 *tab, hipStream_t st);
__host__ __device__ constexpr int pc4_ap_levels(int s) { return s == 0 ? 3 : s <= 2 ? 2 : s <= 4 ? 1 : 0; }
__host__ __device__ constexpr int pc4_ap_dcut(int) { return kPcApBlk; }
bool pc_build_tables4(PcTab4 &tab);
// Zoom 2 (one stage) as tiles (the tail kernel on the mixed input, path 4; few frames per call):
// XA's factorisation in the tail kernel's span geometry --
//   v = x / D(z)                    the stage's 4 sections, causal, at the input rate (B = 21)
//   u = (M * v)|2                   M = N(z) N(1/z) D(-1/z): 25 taps, z^-8 .. z^16
//   out = u / D2(1/w)               D2's 4 sections, anticausal, at rate 1/2 (radius <= .874)
// -- each pole once per direction.  The zero-phase form with the two slow sections both ways
// at the input rate (and the other poles at rate 1/2) missed the row gate on a band-edge tone
// (|damp| 1.9e-5); this one is XA's arithmetic.
constexpr int kPc2G = 25, kPc2Ap = 4, kPc2Own = 4;
constexpr int kPc2M0 = -8;                 // power of z of M's first tap
struct PcTab2 {
  float g[28];                      // M_(i + kPc2M0), i < 25
  PcSec own[kPc2Own];               // D's sections at the input rate, B = 21, slowest first
  float own_x[kPc2Own][64][4];      // A^(21 (i + 1)) for lane i (cross-wave step)
  PcSec ap[kPc2Ap];                 // D2's sections at rate 1/2, B = 10, slowest first
};
__host__ __device__ constexpr int pc2_own_levels(int s) { return 4 - s; }
__host__ __device__ constexpr int pc2_ap_levels(int s) { return 4 - s; }
__host__ __device__ constexpr int pc2_ap_dcut(int) { return kPcApBlk; }
bool pc_build_tables2(PcTab2 &tab);
hipError_t launch_pc2_tail(const InDesc &in, const float2 *lo, float2 *out, int64_t n1, int frames,
                           const PcTab2 *tab, hipStream_t st);
// Frame-end maps, out[m] += sum_k U[m][k] (sum_j V[j][k] x[j]) (left: m, j from the start;
// right: from the end), rank r.
struct PcEdge {
  int R = 0, J = 0, r = 0;
  std::vector<float> U, V;         // R x r, J x r (row-major)
};
bool pc_build_tables(PcTab &tab);
// side 0 = frame start, 1 = frame end (depends on L mod 8); _k: K stages (zoom 2^K, L mod 2^K)
bool pc_edge_map(int side, int lmod8, PcEdge &out);
bool pc_edge_map_k(int K, int side, int lmod, PcEdge &out);
int64_t pc_y2_len(int64_t L);      // y2 entries per frame (from kPcQ0)
hipError_t launch_pc_fir(const InDesc &in, const float2 *lo, float2 *y2, int64_t y2_stride,
                         int frames, const PcTab *tab, hipStream_t st);
hipError_t launch_pc_tail(const float2 *y2, int64_t y2_stride, float2 *out, int64_t n3,
                          int frames, const PcTab *tab, hipStream_t st);
hipError_t launch_pc_walk(const InDesc &in, const float2 *lo, float2 *out, int64_t n3, int frames,
                          const PcTab *tab, hipStream_t st);
hipError_t launch_pc_walk4(const InDesc &in, const float2 *lo, float2 *out, int64_t n2, int frames,
                           const PcTab4 *tab, hipStream_t st);
// both frame ends in one launch: [0] = start, [1] = end
// K3 split (the walk): v = V^T x per frame end into v[frames][2][kPcEdgeRank] (may run on a
// side stream beside the walk), then out += U v
hipError_t launch_pc_edge_v(const InDesc &in, const float2 *lo, float2 *v, int frames,
                            const float *const V[2], const int J[2], const int r[2], hipStream_t st);
hipError_t launch_pc_edge_u(const float2 *v, float2 *out, int64_t n3, int frames, const float *const U[2],
                            const int R[2], const int r[2], hipStream_t st);
hipError_t launch_pc_edge(const InDesc &in, const float2 *lo, float2 *out, int64_t n3, int frames,
                          const float *const U[2], const float *const V[2], const int R[2],
                          const int J[2], const int r[2], hipStream_t st);
// FC (fc_kernels.hip, path 6): the zoom-8 model G as a truncated FIR (|k| <= kFcK) applied by
// overlap-save FFT convolution in 8192-sample windows advancing 512 kFcStep samples (kFcP
// outputs); the ↓8 is an alias sum in frequency fused with the filter, the LO mix is the
// filter's modulation.  The table: W_1024^k (k < 1024), then kFcRow entries per LO row.
#ifndef FC_STEP
#define FC_STEP 13  // K = 768 (tail 1.0e-6 of sum |g|; 12 = K 1024, 1.4e-8: 5.5 % slower, r06fc6)
#endif
constexpr int kFcN = 8192, kFcStep = FC_STEP;
constexpr int kFcK = (kFcN - 512 * kFcStep) / 2;   // 768
constexpr int kFcP = 64 * kFcStep;                 // 832
// Zoom 4 (cfg1): four residues of 2048 points, the zoom-4 model truncated at |k| <= 512 (tail
// 1.4e-8 of sum |g|), windows advancing 7168 samples (1792 outputs).
constexpr int kFc4Step = 14;
constexpr int kFc4K = (kFcN - 512 * kFc4Step) / 2;  // 512
constexpr int kFc4P = 512 * kFc4Step / 4;          // 1792
constexpr int kFcRow = kFcN;  // C[k][r] per LO row, v4f pairs [(zoom / 2) k3 + r / 2][t] (r, r+1)
// C for zoom 8 or 4 and LO frequency ratio f_lo / fs into row (kFcRow entries); false if the
// model is unavailable
bool fc_build_row(int zoom, double lo_ratio, float2 *row);
void fc_build_twiddles(int M, float2 *tw);         // W_M^k, k < M (M = kFcN / zoom)
hipError_t launch_fc_decim(const InDesc &in, const float2 *lo, const float2 *tab, int64_t row_stride,
                           float2 *out, int64_t nd, int frames, int zoom, hipStream_t st);

struct WelchGeom {
  int n_fft, log2n;
  int n_win;
  int nperseg, step, nseg;
  float scale;  // 1 / (fs * sum(w^2) * nseg)
  // one-sided (real input at zoom 1, scipy's rfft branch): bins 0..N/2,
  // doubled except 0 and N/2, then the reference's fftshift of those N/2+1 bins and its
  // [N/2 - W/2, N/2 + W/2) slice -- row_len = that slice's length, from row_a
  int onesided = 0, row_a = 0, row_len = 0;
  // four-step only: the column pass leaves per-column-group partial sums of each segment and
  // the row pass subtracts mean * FFT(window) after the transform (nperseg == n_fft)
  int fused_mean = 0;
  // in-place DIF only: each frame's segments split over `split` workgroups (few frames per
  // call), their linear partial PSDs in parts[(f split + part) n_win + j], summed in part
  // order and converted to dB by a second launch (split 1: the row directly)
  int split = 1;
  float *parts = nullptr;
};
// DIF Welch split for a call of `frames` frames: enough workgroups for the chip (about 768 at
// N = 4096), at least two segments each; 1 for full batches.
int welch_dif_split(int n_fft, int nseg, int frames);

hipError_t launch_welch_rows(const float2 *x, int64_t len, const float *win, const float2 *tw,
                             const WelchGeom &g, float *rows, int frames, hipStream_t st);

// Four-step Welch for N = N1 * 256, 16 <= N1 <= 256: means (frames*nseg), z (frames*nseg*N)
// workspaces; tws = W_256^m (256) ++ W_N1^m (N1).
hipError_t launch_welch4(const float2 *x, int64_t len, const float *win, const float2 *tw,
                         const float2 *tws, const float2 *winf, const WelchGeom &g, float2 *means,
                         float2 *z, float *rows, int frames, hipStream_t st);

hipError_t launch_waterfall_init(float *ring, int H, int W, hipStream_t st);
hipError_t launch_waterfall_push(float *ring, int H, int W, const float *rows,
                                 int64_t row_stride, int count, int64_t off0, int scroll,
                                 hipStream_t st);
hipError_t launch_waterfall_read(const float *ring, int H, int W, int64_t off, float *img,
                                 hipStream_t st);
// waterfall rendering: RGBA8 pixels of the ring in read order
// one row (host-visible `row`, or null: none) pushed and the image emitted in one launch:
// RGBA8 through `lut` (f64 false) or float64 (f64 true) into `out` (H*W pixels)
hipError_t launch_waterfall_push_emit(float *ring, int H, int W, int64_t off0, int scroll,
                                      const float *row, const void *lut, double lo, double scale,
                                      void *out, bool f64, hipStream_t st);
hipError_t launch_waterfall_render(const float *ring, int H, int W, int64_t off, const void *lut,
                                   double lo, double scale, void *out, hipStream_t st);
// autolevel order statistics of the pixels < 0: top-16-bit key histogram (65536 bins), then
// the low-16-bit histograms inside nbins (<= 4) chosen top bins
hipError_t launch_autolevel_hist_hi(const float *ring, int64_t n, unsigned *hist, hipStream_t st);
hipError_t launch_autolevel_hist_lo(const float *ring, int64_t n, const unsigned *bins, int nbins,
                                    unsigned *hist, hipStream_t st);
// out[f][i] = in(f, i) (* lo[i] when lo) as complex64, natural layout, frames x len.
hipError_t launch_fill_c64(float2 *out, int64_t n, float re, float im, hipStream_t st);
hipError_t launch_ingest(const InDesc &in, const float2 *lo, float2 *out, int frames,
                         hipStream_t st);

// --- host helpers ---
void set_error(const std::string &msg);
bool window_kind_native(int kind);
bool make_window(int kind, const double *param, int M, std::vector<double> &out);

}  // namespace zfft
