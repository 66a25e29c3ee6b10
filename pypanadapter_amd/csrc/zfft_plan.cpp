// zfft_plan.cpp -- plan, workspace and C-ABI entry points of libzfft.so.
//
// One plan = one (N, zoom, W, window, fs, f_lo, scroll) configuration on one device, the
// analogue of the AppState fields the reference re-reads every frame
// (pypanadapter_spectrum.py:1492-1497, 2102-2119).  It owns the HIP stream, the LO /
// window / twiddle tables, a grow-only workspace and the waterfall ring.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "cheby1_q2.h"
#include "pc_edge_maps.h"
#include "zfft.h"
#include "zfft_internal.h"

namespace zfft {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }

Sos32 sos32() {
  static const Sos32 c = [] {
    Sos32 s{};
    s.b0 = (float)kDecimSos[0][0];
    s.b1 = (float)kDecimSos[0][1];
    s.b2 = (float)kDecimSos[0][2];
    for (int k = 0; k < 4; ++k) {
      s.a1[k] = (float)kDecimSos[k][4];
      s.a2[k] = (float)kDecimSos[k][5];
      s.zi[k][0] = (float)kDecimZi[k][0];
      s.zi[k][1] = (float)kDecimZi[k][1];
    }
    return s;
  }();
  return c;
}

namespace {

// ---- 8x8 helpers (fp64) for the modal bases of the XA cascades ----
using Mat8 = std::vector<double>;  // 8x8 row-major
Mat8 matmul8(const Mat8 &a, const Mat8 &b) {
  Mat8 c(64, 0.0);
  for (int i = 0; i < 8; ++i)
    for (int k = 0; k < 8; ++k)
      for (int j = 0; j < 8; ++j) c[i * 8 + j] += a[i * 8 + k] * b[k * 8 + j];
  return c;
}
using cd = std::complex<double>;

void mat_inverse8(const Mat8 &a, Mat8 &inv) {
  Mat8 m = a;
  inv.assign(64, 0.0);
  for (int i = 0; i < 8; ++i) inv[i * 8 + i] = 1.0;
  for (int c = 0; c < 8; ++c) {
    int piv = c;
    for (int r = c + 1; r < 8; ++r)
      if (std::fabs(m[r * 8 + c]) > std::fabs(m[piv * 8 + c])) piv = r;
    for (int k = 0; k < 8; ++k) {
      std::swap(m[c * 8 + k], m[piv * 8 + k]);
      std::swap(inv[c * 8 + k], inv[piv * 8 + k]);
    }
    const double d = m[c * 8 + c];
    for (int k = 0; k < 8; ++k) {
      m[c * 8 + k] /= d;
      inv[c * 8 + k] /= d;
    }
    for (int r = 0; r < 8; ++r) {
      if (r == c) continue;
      const double f = m[r * 8 + c];
      for (int k = 0; k < 8; ++k) {
        m[r * 8 + k] -= f * m[c * 8 + k];
        inv[r * 8 + k] -= f * inv[c * 8 + k];
      }
    }
  }
}

// ---- XA tables (xa_kernels.hip, tools/xa_proto.py): all-pole cascades in DF-I state
// (y_k[t-1], y_k[t-2]) per section, real modal bases, the 25-tap FIR and frame-end forms ----
struct ApD {
  double a1[4], a2[4];
};
void ap_step_d(const ApD &c, const double in[8], double u, double out[8], double *y) {
  double s[8];
  for (int i = 0; i < 8; ++i) s[i] = in[i];
  double x = u;
  for (int k = 0; k < 4; ++k) {
    const double yy = x - c.a1[k] * s[2 * k] - c.a2[k] * s[2 * k + 1];
    s[2 * k + 1] = s[2 * k];
    s[2 * k] = yy;
    x = yy;
  }
  for (int i = 0; i < 8; ++i) out[i] = s[i];
  *y = x;
}

// Real modal basis of a cascade state matrix A (block lower triangular: section k's state is
// driven by the outputs of sections < k).  Mode j = the pole pair of section j, lambda_j =
// sigma + i omega = (-a1 + i sqrt(4 a2 - a1^2)) / 2; its eigenvector v is zero on sections
// < j, the null vector of (A_jj - lambda) on section j and found by forward substitution
// below.  Columns (Re v, Im v) of T give T^-1 A T = diag([[sigma, omega], [-omega, sigma]]),
// so a power of A is a per-mode complex power.
void modal_basis(const Mat8 &A, const cd lam[4], Mat8 &T) {
  T.assign(64, 0.0);
  for (int j = 0; j < 4; ++j) {
    cd v[8] = {};
    const double p = A[(2 * j) * 8 + 2 * j], q = A[(2 * j) * 8 + 2 * j + 1];
    v[2 * j] = q;
    v[2 * j + 1] = lam[j] - p;
    for (int k = j + 1; k < 4; ++k) {
      cd r0 = 0, r1 = 0;
      for (int l = 2 * j; l < 2 * k; ++l) {
        r0 -= A[(2 * k) * 8 + l] * v[l];
        r1 -= A[(2 * k + 1) * 8 + l] * v[l];
      }
      const cd m00 = A[(2 * k) * 8 + 2 * k] - lam[j], m01 = A[(2 * k) * 8 + 2 * k + 1];
      const cd m10 = A[(2 * k + 1) * 8 + 2 * k], m11 = A[(2 * k + 1) * 8 + 2 * k + 1] - lam[j];
      const cd det = m00 * m11 - m01 * m10;
      v[2 * k] = (r0 * m11 - m01 * r1) / det;
      v[2 * k + 1] = (m00 * r1 - m10 * r0) / det;
    }
    double nrm = 0;
    int big = 0;
    for (int i = 0; i < 8; ++i) {
      nrm += std::norm(v[i]);
      if (std::abs(v[i]) > std::abs(v[big])) big = i;
    }
    const cd rot = std::conj(v[big]) / std::abs(v[big]) / std::sqrt(nrm);
    for (int i = 0; i < 8; ++i) {
      const cd w = v[i] * rot;
      T[i * 8 + 2 * j] = w.real();
      T[i * 8 + 2 * j + 1] = w.imag();
    }
  }
}

// One pass: fills P, the output table cm (steps rows) and, when lag != nullptr, the
// far-field rows C A^d T for d < n_lag.
bool xa_pass_tables(const ApD &c, int steps, bool up, XaPass &P, float (*lag)[8], int n_lag, int B,
                    double (*lag_d)[8] = nullptr) {
  Mat8 A(64);
  double C[8];
  for (int q = 0; q < 8; ++q) {
    double e[8] = {0}, s2[8], y;
    e[q] = 1.0;
    ap_step_d(c, e, 0.0, s2, &y);
    for (int r = 0; r < 8; ++r) A[r * 8 + q] = s2[r];
    C[q] = y;
  }
  cd lam[4];
  for (int j = 0; j < 4; ++j) lam[j] = cd(-0.5 * c.a1[j], std::sqrt(c.a2[j] - 0.25 * c.a1[j] * c.a1[j]));
  Mat8 T, Ti;
  modal_basis(A, lam, T);
  mat_inverse8(T, Ti);
  double st[8], x = 1.0;
  for (int k = 0; k < 4; ++k) {
    P.a1[k] = (float)c.a1[k];
    P.a2[k] = (float)c.a2[k];
    x /= 1.0 + c.a1[k] + c.a2[k];
    st[2 * k] = st[2 * k + 1] = x;
  }
  for (int r = 0; r < 8; ++r) {
    double acc = 0;
    for (int k = 0; k < 8; ++k) acc += Ti[r * 8 + k] * st[k];
    P.ss[r] = (float)acc;
    for (int k = 0; k < 8; ++k) {
      P.ti[r][k] = (float)Ti[r * 8 + k];
      P.t[r][k] = (float)T[r * 8 + k];
    }
  }
  for (int j = 0; j < 4; ++j) {
    // the kernel's truncated scan must reach fp32-negligible powers for every mode
    if (std::pow(std::abs(lam[j]), (double)(steps << xa_levels(B, j))) > 1e-9) return false;
    const cd w = std::pow(lam[j], steps);
    P.pS[j][0] = (float)w.real();
    P.pS[j][1] = (float)w.imag();
    for (int d = 0; d < 4; ++d) {
      const cd u = std::pow(lam[j], steps << d);
      P.scan[d][j][0] = (float)u.real();
      P.scan[d][j][1] = (float)u.imag();
    }
  }
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 4; ++j) P.xr[i][j] = 0.f;
  for (int j = 0; j < kXaRowModes; ++j) {
    if (xa_levels(B, j) > 4) return false;  // row shifts reach at most 8 lanes
    for (int i = 0; i < 16; ++i) {
      const cd u = std::pow(lam[j], steps * (up ? i + 1 : 16 - i));
      P.xr[i][2 * j] = (float)u.real();
      P.xr[i][2 * j + 1] = (float)u.imag();
    }
  }
  Mat8 AtT = T;  // A^t T
  for (int t = 0; lag && t < n_lag; ++t) {
    for (int q = 0; q < 8; ++q) {
      double acc = 0;
      for (int r = 0; r < 8; ++r) acc += C[r] * AtT[r * 8 + q];
      lag[t][q] = (float)acc;
      if (lag_d) lag_d[t][q] = acc;
    }
    AtT = matmul8(A, AtT);
  }
  return true;
}

bool xa_build_tables(XaTab &X, int B) {
  // sections slowest pole first (the lower-error fp32 order; any order is exact)
  ApD fw, bw;
  for (int k = 0; k < 4; ++k) {
    const double a1 = kDecimSos[3 - k][4], a2 = kDecimSos[3 - k][5];
    fw.a1[k] = a1;
    fw.a2[k] = a2;
    bw.a1[k] = 2.0 * a2 - a1 * a1;  // D(z) D(-z) = D2(z^2)
    bw.a2[k] = a2 * a2;
  }
  if (B != kXaB) return false;
  static double fcat[kXaB][8];
  if (!xa_pass_tables(fw, B, true, X.f, X.fcat, B, B, fcat) ||
      !xa_pass_tables(bw, B / 2, false, X.b, X.lag, kXaLag, B))
    return false;
  // N = b0 (1 + z^-1)^8 (sections 1..3 are exactly [1, 2, 1], section 0 is b0 [1, 2, 1])
  double n9[9], dneg[9] = {1.0}, mp[17] = {0}, m25[25] = {0};
  const double b0 = kDecimSos[0][0];
  for (int i = 0; i < 9; ++i) {
    double bin = 1.0;
    for (int r = 0; r < i; ++r) bin = bin * (8 - r) / (r + 1);
    n9[i] = b0 * bin;
  }
  int len = 1;
  for (int k = 0; k < 4; ++k) {  // D(-z) = prod (1 - a1 z^-1 + a2 z^-2)
    const double c1 = -kDecimSos[k][4], c2 = kDecimSos[k][5];
    double nx[9] = {0};
    for (int i = 0; i < len; ++i) {
      nx[i] += dneg[i];
      nx[i + 1] += c1 * dneg[i];
      nx[i + 2] += c2 * dneg[i];
    }
    len += 2;
    for (int i = 0; i < len; ++i) dneg[i] = nx[i];
  }
  for (int i = 0; i < 9; ++i)
    for (int k = 0; k < 9; ++k) mp[i + k] += n9[i] * dneg[k];   // taps on f[j + t]
  for (int t = 0; t < 17; ++t)
    for (int i = 0; i < 9; ++i) m25[t + i] += mp[t] * n9[8 - i];  // taps on v[j - 8 + u]
  double mps = 0, vss = 1.0;
  for (int t = 0; t < 17; ++t) {
    X.mp17[t] = (float)mp[t];
    mps += mp[t];
  }
  for (int u = 0; u < 25; ++u) X.m25[u] = (float)m25[u];
  // the zero-input responses through the FIR (xa_kernels.hip): output k of a lane takes
  // taps m25[24 + t - 1 - 2k] on its own v[t]; its share of the next lane's output k takes
  // m25[t - (B - 24) - 1 - 2k] on its v[t], t >= B - 23
  for (int k = 0; k < B / 2; ++k)
    for (int r = 0; r < 8; ++r) {
      double g = 0;
      for (int t = 0; t < B; ++t) {
        const int tap = 24 + t - 1 - 2 * k;
        if (tap >= 0 && tap < 25) g += m25[tap] * fcat[t][r];
      }
      X.gown[k][r] = (float)g;
    }
  for (int k = 0; k < 12; ++k)
    for (int r = 0; r < 8; ++r) {
      double g = 0;
      for (int t = B - 23; t < B; ++t) {
        const int tap = t - (B - 24) - 1 - 2 * k;
        if (tap >= 0 && tap < 25) g += m25[tap] * fcat[t][r];
      }
      X.gnb[k][r] = (float)g;
    }
  for (int i = 0; i < 9; ++i) X.n9[i] = (float)n9[i];
  for (int k = 0; k < 4; ++k) vss /= 1.0 + fw.a1[k] + fw.a2[k];
  X.mp_sum = (float)mps;
  X.vss = (float)vss;
  X.pad_[0] = X.pad_[1] = 0.f;
  return true;
}

// ---- waterfall colormaps (Waterfall.Colors / lookuptable, S:1580-1585, 1613-1623) ----
// pg.ColorMap(pos, color).getLookupTable(0.0, 1.0, 256): x = linspace(0, 1, 256), each
// channel np.interp(x, pos, color), truncated to uint8; the maps are opaque, so the LUT has
// no alpha channel and makeARGB draws alpha 255.  'Default' keeps the reference's stop
// value 2020 as a numpy < 2 uint8 array stored it (2020 mod 256 = 228).
struct ColorStops {
  const char *name;
  int n;
  double pos[6];
  int rgba[6][4];
};
const ColorStops kColormaps[] = {
    {"Default", 3, {0.0, 0.4, 1.0}, {{0, 0, 90, 255}, {200, 2020 % 256, 0, 255}, {255, 0, 0, 255}}},
    {"Matrix", 2, {0.0, 1.0}, {{0, 0, 0, 255}, {0, 255, 0, 255}}},
    {"Red Green", 3, {0.0, 0.5, 1.0}, {{0, 0, 0, 255}, {0, 255, 0, 255}, {255, 0, 0, 255}}},
    {"Tropical", 6, {0.0, 0.2, 0.4, 0.6, 0.8, 1.0},
     {{68, 40, 153, 255}, {222, 68, 252, 255}, {252, 38, 99, 255}, {252, 181, 38, 255},
      {86, 235, 49, 255}, {3, 71, 7, 255}}},
};

// np.interp(x, xp, fp) for increasing xp (numpy/core/src/multiarray/compiled_base.c)
double np_interp(double x, const double *xp, const double *fp, int n) {
  if (x <= xp[0]) return fp[0];
  if (x >= xp[n - 1]) return fp[n - 1];
  int j = 0;
  while (j + 1 < n && xp[j + 1] <= x) ++j;
  if (x == xp[j]) return fp[j];
  const double slope = (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j]);
  return slope * (x - xp[j]) + fp[j];
}

void build_lut(const char *name, uint8_t *lut) {
  const ColorStops *cm = &kColormaps[0];  // any other name -> 'Default' (S:1613-1614)
  for (const ColorStops &c : kColormaps)
    if (name && std::strcmp(name, c.name) == 0) cm = &c;
  const double step = 1.0 / 255.0;  // np.linspace(0, 1, 256): arange * step, last = stop
  for (int i = 0; i < 256; ++i) {
    const double x = i == 255 ? 1.0 : (double)i * step;
    for (int ch = 0; ch < 3; ++ch) {
      double fp[6];
      for (int k = 0; k < cm->n; ++k) fp[k] = (double)cm->rgba[k][ch];
      lut[4 * i + ch] = (uint8_t)np_interp(x, cm->pos, fp, cm->n);  // astype(ubyte): truncation
    }
    lut[4 * i + 3] = 255;
  }
}

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 1);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T *as() const { return static_cast<T *>(p); }
};

bool is_pow2(int64_t v) { return v > 0 && (v & (v - 1)) == 0; }
int ilog2(int64_t v) {
  int r = 0;
  while ((int64_t(1) << r) < v) ++r;
  return r;
}

int fail(int code, const std::string &msg) {
  set_error(msg);
  return code;
}

int hip_fail(hipError_t e, const char *where) {
  return fail(ZFFT_EHIP, std::string(where) + ": " + hipGetErrorString(e));
}

}  // namespace
}  // namespace zfft

using namespace zfft;

struct zfft_plan {
  zfft_config cfg{};
  int K = 0;  // log2(zoom) decimation stages
  hipStream_t stream = nullptr;
  std::vector<float> user_window;
  DevBuf lo, win, tw, in, in2, yf, ping, pong, rows, ring, img, one_row, dec;
  hipStream_t copy_st = nullptr;            // H2D of the next batch in zfft_process
  hipEvent_t h2d_ev[2] = {}, comp_ev[2] = {};
  int64_t lo_len = 0;                       // entries per LO row (0: not built)
  std::vector<double> lo_freqs;             // set_lo_frames: one LO row per entry (config 4)
  int lo_per = 1;                           // frames per LO row
  int lo_first = 0;                         // first frame of the current batch (zfft_process)
  int win_len = -1;
  double win_ss = 0.0;
  int block_override = 0, warm_override = 0;
  int H = 0, W = 0;
  int64_t off = 0;
  bool wf_ready = false;
  const float *last_row = nullptr;  // device row of the last processed frame
  bool timing = false;
  std::vector<hipEvent_t> events;    // one per mark when timing is on
  std::vector<std::string> mark_names;
  std::string names_buf;
  int n_marks = 0;
  int path = 0;  // 0 auto, 1 exact blocked pipeline, 2 fused interior + edge windows,
                // 3 XA tiles (all-pole + FIR + half-rate all-pole), 4 PC (polyphase cascade,
                // zoom 8)
  int welch = 0;  // 0 auto, 1 one workgroup per frame, 2 four-step
  DevBuf edge, xk, xa_tab, tws, means, z4, winf;
  DevBuf pc_tab, pc_edge;  // PC decimator: PcTab; edge maps U0 V0 U1 V1 (floats)
  DevBuf pc_tab4;  // PC zoom 4: PcTab4
  DevBuf pc_tab2;  // PC zoom 2: PcTab2
  DevBuf wparts;   // split DIF Welch: partial PSDs (frames x split x n_win floats)
  DevBuf lo1;      // unit LO table (the blocked passes after the PC head mix with it)
  int64_t lo1_n = 0;  // entries of lo1 filled (a failed fill leaves it short: refilled next call)
                           // (pc_edge: all nine maps of pc_edge_maps.h, uploaded once)
  int64_t n_quiesce = 0;   // host waits on enqueued work (test hook zfft__plan_quiesce_count)
  // waterfall rendering: colormap LUT (host copy + device), levels
  uint8_t lut[256 * 4] = {};
  bool lut_ready = false;         // lut holds the chosen map (built on first use)
  bool lut_uploaded = false;      // lut_d holds lut
  std::string cmap = "Default";
  double lev_lo = -220.0, lev_hi = -120.0;  // Waterfall.__init__ (S:1593-1598)
  DevBuf lut_d, rgba, al_hist, al_bins;
  DevBuf img64;                    // float64 image of the display entries
  float *row_pin = nullptr;        // page-locked staging of host rows the display kernels read
  size_t row_pin_cap = 0;          //   in place (no H2D copy command); bytes
  // Ordering across streams: every call that enqueues work first makes its stream wait for
  // the plan's previous work (done_ev, recorded on done_st), then records done_ev after its
  // own; the workspaces, tables and the ring are thus used in call order whatever streams the
  // caller picks, and a synchronous table upload waits for done_ev first.
  hipEvent_t done_ev = nullptr;
  hipStream_t done_st = nullptr;
  bool has_work = false;
  // the walk's frame-end sums V^T x run on side_st beside it (fork_ev / join_ev), into edge_v
  hipStream_t side_st = nullptr;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
  DevBuf edge_v;
  // FC decimator (path 6): W_1024 twiddles, then one C row per LO frequency; fc_built holds the
  // f_lo / fs ratios the rows were built for (rebuilt when they change)
  DevBuf fc_tab;
  std::vector<double> fc_built;
};

namespace {

// Timing marks: an event before the first launch and after each launch (or launch group)
// of a call, with the name of what ran since the previous mark.
void mark(zfft_plan *p, hipStream_t st, const char *what = "") {
  if (!p->timing) return;
  if ((int)p->events.size() <= p->n_marks) {
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return;
    p->events.push_back(ev);
  }
  if ((int)p->mark_names.size() <= p->n_marks) p->mark_names.resize(p->n_marks + 1);
  p->mark_names[p->n_marks] = what;
  (void)hipEventRecord(p->events[p->n_marks++], st);
}

// Stage lengths: n_0 = L, n_{k+1} = ceil(n_k / 2)  (decimate(...)[::2]).
std::vector<int64_t> stage_lengths(int64_t L, int K) {
  std::vector<int64_t> n{L};
  for (int k = 0; k < K; ++k) n.push_back((n.back() + 1) / 2);
  return n;
}

int choose_block(const zfft_plan *p, int64_t n, int ngroups) {
  if (p->block_override > 0) return (p->block_override + 15) & ~15;
  // Enough waves (one per block of a 64-frame group) to fill 256 CUs many times over;
  // larger blocks amortise the warm-up.  A few frames of <= 2^19 samples (one per call:
  // the reference's use) go down to 256-sample blocks, whose shorter serial runs took one
  // cfg2 frame from 0.48 to 0.38 ms of kernels (cfg5's 2^20-sample frames: no gain).
  const int s_min = n <= ((int64_t)1 << 19) ? 256 : 512;
  int S = 4096;
  while (S > s_min && (int64_t)ngroups * ((n + kPad + S - 1) / S) < 8192) S >>= 1;
  return S;
}

int warmup(const zfft_plan *p) { return p->warm_override > 0 ? (p->warm_override + 15) & ~15 : 192; }

int quiesce(zfft_plan *p);
int use_stream(zfft_plan *p, hipStream_t st);
int done_on(zfft_plan *p, hipStream_t st);

#ifndef ZFFT_WELCH_ONEWG_MAX
#define ZFFT_WELCH_ONEWG_MAX 16384
#endif
constexpr int kWelchOneWgMax = ZFFT_WELCH_ONEWG_MAX;  // auto Welch: one workgroup per frame up to here

// LO table: one row of lo_len entries per LO frequency (the plan's f_lo, or the
// zfft_plan_set_lo_frames list), rows lo_len apart.
constexpr size_t kMaxLoBytes = (size_t)4 << 30;  // the LO table, all rows
int ensure_lo(zfft_plan *p, int64_t L) {
  if (p->lo_len >= L) return ZFFT_OK;
  int rc = quiesce(p);
  if (rc) return rc;
  // the XA kernels read lo[lane] for every lane; rows 64-entry aligned
  const int64_t cap = (std::max<int64_t>(L, 64) + 63) & ~(int64_t)63;
  const std::vector<double> freqs = p->lo_freqs.empty() ? std::vector<double>{p->cfg.f_lo} : p->lo_freqs;
  if ((double)cap * (double)freqs.size() * sizeof(float2) > (double)kMaxLoBytes)
    return fail(ZFFT_ENOMEM, "LO table (set_lo_frames rows x frame length x 8 B) over 4 GiB");
  std::vector<float2> h;
  try {
    h.resize(cap * freqs.size());
  } catch (const std::bad_alloc &) {
    return fail(ZFFT_ENOMEM, "LO table host staging allocation failed");
  }
  const double sq2 = std::sqrt(2.0);
  for (size_t k = 0; k < freqs.size(); ++k) {
    const double r = freqs[k] / p->cfg.fs;
    for (int64_t n = 0; n < cap; ++n) {
      // lo[n] = sqrt(2) exp(-2 pi i f_lo n / fs) on integer n (S:2091-2093)
      const double turns = std::fmod((double)n * r, 1.0);
      const double ph = -2.0 * M_PI * turns;
      h[k * cap + n] = make_float2((float)(sq2 * std::cos(ph)), (float)(sq2 * std::sin(ph)));
    }
  }
  hipError_t e = p->lo.ensure(h.size() * sizeof(float2));
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "LO table allocation failed");
  e = hipMemcpy(p->lo.p, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "LO table upload");
  p->lo_len = cap;
  return ZFFT_OK;
}

// In-place radix-2 DFT (forward, exp(-2 pi i k n / N)), N a power of two, float64.
void fft64(std::vector<double> &re, std::vector<double> &im) {
  const size_t n = re.size();
  for (size_t i = 1, j = 0; i < n; ++i) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j |= bit;
    if (i < j) std::swap(re[i], re[j]), std::swap(im[i], im[j]);
  }
  for (size_t len = 2; len <= n; len <<= 1) {
    const double a = -2.0 * M_PI / (double)len;
    for (size_t i = 0; i < n; i += len)
      for (size_t k = 0; k < len / 2; ++k) {
        const double c = std::cos(a * (double)k), sn = std::sin(a * (double)k);
        const size_t u = i + k, v = u + len / 2;
        const double tr = re[v] * c - im[v] * sn, ti = re[v] * sn + im[v] * c;
        re[v] = re[u] - tr, im[v] = im[u] - ti;
        re[u] += tr, im[u] += ti;
      }
  }
}

// welch builds get_window(window, nperseg); nperseg = min(N, L_d) (short-input branch).
int ensure_window(zfft_plan *p, int nperseg) {
  if (p->win_len == nperseg) return ZFFT_OK;
  int rc = quiesce(p);
  if (rc) return rc;
  std::vector<double> w;
  if (p->cfg.window_kind == ZFFT_WIN_ARRAY) {
    if (nperseg != p->cfg.n_fft)
      return fail(ZFFT_EINVAL, "window is longer than input signal (array window of length "
                               "n_fft, decimated frame shorter than n_fft)");
    w.assign(p->user_window.begin(), p->user_window.end());
  } else if (!make_window(p->cfg.window_kind, p->cfg.window_param, nperseg, w)) {
    return fail(ZFFT_EINVAL, "window generation failed");
  }
  std::vector<float> wf(nperseg);
  double ss = 0.0;
  for (int i = 0; i < nperseg; ++i) {
    wf[i] = (float)w[i];
    ss += w[i] * w[i];
  }
  hipError_t e = p->win.ensure(p->cfg.n_fft * sizeof(float));
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "window allocation failed");
  e = hipMemcpy(p->win.p, wf.data(), nperseg * sizeof(float), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "window upload");
  if (nperseg == p->cfg.n_fft && p->cfg.n_fft >= 4096) {  // (four-step capable sizes)
    // the four-step Welch subtracts the segment mean after its transform: X = FFT(x w) -
    // mean FFT(w) (scipy's detrend='constant' is linear); FFT(w) of the float32 window, fp64
    std::vector<double> re(wf.begin(), wf.end()), im(nperseg, 0.0);
    fft64(re, im);
    std::vector<float2> wft(nperseg);
    for (int k = 0; k < nperseg; ++k) wft[k] = make_float2((float)re[k], (float)im[k]);
    e = p->winf.ensure(nperseg * sizeof(float2));
    if (e == hipSuccess) e = hipMemcpy(p->winf.p, wft.data(), nperseg * sizeof(float2), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(e, "window transform upload");
  }
  p->win_len = nperseg;
  p->win_ss = ss;
  return ZFFT_OK;
}

int check_lengths(const zfft_plan *p, int64_t L, int32_t frames, std::vector<int64_t> &n) {
  if (L < 1 || frames < 1) return fail(ZFFT_EINVAL, "n_samples and n_frames must be >= 1");
  if (L > (int64_t)1 << 30) return fail(ZFFT_EINVAL, "n_samples too large (max 2^30)");
  n = stage_lengths(L, p->K);
  for (int k = 0; k < p->K; ++k)
    if (n[k] <= kPad)
      return fail(ZFFT_ESHORT, "The length of the input vector x must be greater than padlen, "
                               "which is 27 (decimation stage " + std::to_string(k) + " has " +
                               std::to_string(n[k]) + " samples)");
  return ZFFT_OK;
}

// Exact decimation cascade (reference pass order, odd padding, zi initial conditions) on
// `frames` frames of n[0] samples each at frame stride `stride` (natural layout in; lo points
// at the LO value of the first sample).  Intermediates in FGI layout, the result (last
// stage) in natural layout in *out.
// With split > 0 (a multiple of 64) the frames [split, split + frames) are a second window
// set starting alt_off samples into the same frames; the output then has split + frames rows.
// k0 > 0: stages k0 .. K-1 only, `in` holding stage k0's input (already mixed: lo a unit
// table), e.g. after the PC head.
int run_exact(zfft_plan *p, const InDesc &in, const float2 *lo, int frames,
              const std::vector<int64_t> &n, const float2 **out, hipStream_t st, int split = 0,
              int64_t alt_off = 0, int k0 = 0) {
  const int rows = split > 0 ? split + frames : frames;
  const int ngroups = (rows + 63) / 64;
  const size_t G = (size_t)ngroups * 64;
  hipError_t e = p->yf.ensure(G * (n[k0] + 2 * kPad) * sizeof(float2));
  if (e == hipSuccess) e = p->ping.ensure(G * n[k0 + 1] * sizeof(float2));
  if (e == hipSuccess && p->K > k0 + 1) e = p->pong.ensure(G * n[k0 + 2] * sizeof(float2));
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "decimator workspace allocation failed");
  const float2 *cur = nullptr;
  for (int k = k0; k < p->K; ++k) {
    StageGeom g;
    g.n = (int)n[k];
    g.block = choose_block(p, n[k], ngroups);
    g.nblk = (int)((n[k] + kPad + g.block - 1) / g.block);
    g.warmup = warmup(p);
    g.ngroups = ngroups;
    g.split = split;
    g.alt_off = alt_off;
    if (k == k0)
      e = launch_iir_forward_mix(in, frames, lo, p->yf.as<float2>(), g, st);
    else
      e = launch_iir_forward_fgi(cur, p->yf.as<float2>(), g, st);
    if (e != hipSuccess) return hip_fail(e, "iir_forward launch");
    mark(p, st, k == 0 ? "exact_forward_mix" : "exact_forward");
    float2 *dst = ((k - k0) & 1) ? p->pong.as<float2>() : p->ping.as<float2>();
    e = launch_iir_backward(p->yf.as<float2>(), dst, k == p->K - 1, rows, g, st);
    if (e != hipSuccess) return hip_fail(e, "iir_backward launch");
    mark(p, st, "exact_backward");
    cur = dst;
  }
  *out = cur;
  return ZFFT_OK;
}

#ifndef ZFFT_WELCH4_CHUNK_MB
#define ZFFT_WELCH4_CHUNK_MB 0  // chunks of 48/96/192 MB measured 3.1x/1.8x/1.4x slower (cfg5)
#endif
constexpr size_t kWelch4ChunkBytes = (size_t)ZFFT_WELCH4_CHUNK_MB << 20;  // 0: one launch set
constexpr int kMaxLoRows = 256;  // LO rows of set_lo_frames (each n_samples x 8 B)

// Edge width (final-stage samples) recomputed exactly, and the exact window length.
constexpr int kEdge = 384;
int64_t edge_window(int K) { return ((int64_t)1 << K) * (kEdge + 640); }

// Auto choice between XA (one wave per frame) and the blocked schedules, from the sweep
// tools/sweep_schedule.py (profiles/r03i/sweep_schedule.json: ms per call, N = 4096, zoom 8):
// XA needs enough frames to fill 2 waves x 1024 SIMDs; for ~300k-sample frames it is the
// fastest from 384 frames (1.66 ms against 1.80 fused / 1.83 exact; 256 frames: 1.62 against
// 1.25 exact), for 2^20-sample frames from 768 (5.67 against 7.69 fused; 512: 5.56 against 5.28).
constexpr int kXaMinFrames = 768;
constexpr int kXaMinFramesShort = 384;
constexpr int64_t kXaShortFrame = (int64_t)1 << 19;
// zfft_process pipelining: inputs of >= 64 MB go in batches of about 1 GB (at least two).
constexpr size_t kPipeMinBytes = (size_t)64 << 20;
constexpr size_t kPipeBatchBytes = (size_t)1 << 30;
bool auto_xa(int frames, int64_t L) {
  return frames >= kXaMinFrames || (frames >= kXaMinFramesShort && L <= kXaShortFrame);
}

// XA addresses a frame's stage input and output through 32-bit buffer resources.
bool xa_fits(const zfft_plan *p, int64_t L) {
  return L * (int64_t)in_elem_bytes(p->cfg.in_dtype) < ((int64_t)1 << 31) &&
         L * (int64_t)sizeof(float2) < ((int64_t)1 << 31);
}

// The fused blocked schedule (path 2) saves passes over the frame interior but adds the
// exact edge-window runs, whose launches cost about as much as a whole pass over a few
// frames: it wins only for large batches.  Same sweep (frames x samples, ms, path 1 / path 2):
// 2^20-sample frames 64: 1.15 / 1.33, 128: 2.20 / 2.04, 256: 4.04 / 3.30; ~300k-sample frames
// 256: 1.25 / 1.43 (and from 384 frames XA beats both).
constexpr int64_t kFusedMinSamples = (int64_t)1 << 27;  // per call
bool use_fused(const zfft_plan *p, int64_t L, int frames) {
  if (p->path == 1 || p->K < 2) return false;
  if (8 * edge_window(p->K) > L) return false;  // windows cost <= 1/4 of a frame
  return p->path == 2 || (int64_t)frames * L >= kFusedMinSamples;
}

int fused_block(int64_t n_mid, int ngroups) {
  int S = 2048;
  while (S > 256 && (int64_t)ngroups * ((n_mid + S - 1) / S) < 4096) S >>= 1;
  return S;
}

// Interior in commuted pass order with fused same-direction pass pairs, edges exact:
//   [C0] [A0 A1] [C1 C2] [A2 A3] ... [last pass of stage K-1, decimated, natural layout]
// then the first/last kEdge outputs are replaced by the exact pipeline on prefix/suffix
// windows of the frames (run first, their edge outputs parked in p->edge).
int run_fused(zfft_plan *p, const InDesc &in, int64_t L, int frames,
              const std::vector<int64_t> &n, const float2 **out, hipStream_t st) {
  const int K = p->K;
  const int64_t nK = n[K];
  const int ngroups = (frames + 63) / 64;
  const size_t G = (size_t)ngroups * 64;
  const int64_t P = edge_window(K);
  const int64_t L0 = ((L - P) >> K) << K;  // suffix window start, multiple of 2^K
  // both window sets have length Pw = L - L0 in [P, P + 2^K): the suffix ends at the frame end
  const std::vector<int64_t> npre = stage_lengths(L - L0, K), nsuf = npre;
  // all workspace first (the window runs reuse the interior chain's buffers)
  hipError_t e = p->edge.ensure((size_t)frames * 2 * kEdge * sizeof(float2));
  if (e == hipSuccess) e = p->xk.ensure((size_t)frames * nK * sizeof(float2));
  if (e == hipSuccess) e = p->yf.ensure(G * (L + 2 * kPad) * sizeof(float2));
  if (e == hipSuccess) e = p->ping.ensure(G * n[1] * sizeof(float2));
  if (e == hipSuccess) e = p->pong.ensure(G * n[2] * sizeof(float2));
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "decimator workspace allocation failed");
  float2 *edge = p->edge.as<float2>();
  // exact edges: one run over prefix windows (rows [0, F)) and suffix windows (rows
  // [Fp, Fp + F), Fp = F rounded up to 64); then prefix cols [0, E) and suffix cols
  // [nsuf_K - E, nsuf_K) -> p->edge [F][2E]
  const int Fp = ngroups * 64;
  const float2 *w;
  int rc = run_exact(p, in, p->lo.as<float2>(), frames, npre, &w, st, Fp, L0);
  if (rc) return rc;
  e = hipMemcpy2DAsync(edge, 2 * kEdge * sizeof(float2), w, npre[K] * sizeof(float2),
                       kEdge * sizeof(float2), frames, hipMemcpyDeviceToDevice, st);
  if (e != hipSuccess) return hip_fail(e, "edge copy");
  e = hipMemcpy2DAsync(edge + kEdge, 2 * kEdge * sizeof(float2),
                       w + (int64_t)Fp * npre[K] + (nsuf[K] - kEdge), npre[K] * sizeof(float2),
                       kEdge * sizeof(float2), frames, hipMemcpyDeviceToDevice, st);
  if (e != hipSuccess) return hip_fail(e, "edge copy");
  mark(p, st, "edge_windows");

  // interior chain
  StageGeom g0;
  g0.n = (int)L;
  g0.block = choose_block(p, L, ngroups);
  g0.nblk = (int)((L + kPad + g0.block - 1) / g0.block);
  g0.warmup = warmup(p);
  g0.ngroups = ngroups;
  e = launch_iir_forward_mix(in, frames, p->lo.as<float2>(), p->yf.as<float2>(), g0, st);
  if (e != hipSuccess) return hip_fail(e, "iir_forward launch");
  mark(p, st, "C0_forward_mix");
  const float2 *cur = p->yf.as<float2>();
  int64_t cur_len = L + 2 * kPad;
  int cur_off = kPad;
  for (int i = 0; i <= K - 1; ++i) {  // kernel i: 2nd pass of stage i (+ 1st of stage i+1)
    const bool two = i < K - 1;
    FusedGeom fg;
    fg.in_len = (int)cur_len;
    fg.in_off = cur_off;
    fg.n_mid = (int)n[i + 1];
    fg.block = fused_block(fg.n_mid, ngroups);
    fg.nblk = (fg.n_mid + fg.block - 1) / fg.block;
    fg.w1 = fg.w2 = warmup(p);
    fg.ngroups = ngroups;
    float2 *dst = !two ? p->xk.as<float2>() : ((i & 1) ? p->pong.as<float2>() : p->ping.as<float2>());
    e = launch_fused_pass(cur, dst, (i & 1) == 0, two, !two, fg, frames, st);
    if (e != hipSuccess) return hip_fail(e, "fused pass launch");
    mark(p, st, two ? ((i & 1) ? "fused_asc_pair" : "fused_desc_pair")
                    : ((i & 1) ? "fused_asc_last" : "fused_desc_last"));
    cur = dst;
    cur_len = n[i + 1];
    cur_off = 0;
  }
  // patch the exact edges into the interior result
  float2 *xk = p->xk.as<float2>();
  e = hipMemcpy2DAsync(xk, nK * sizeof(float2), edge, 2 * kEdge * sizeof(float2),
                       kEdge * sizeof(float2), frames, hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess)
    e = hipMemcpy2DAsync(xk + (nK - kEdge), nK * sizeof(float2), edge + kEdge,
                         2 * kEdge * sizeof(float2), kEdge * sizeof(float2), frames,
                         hipMemcpyDeviceToDevice, st);
  if (e != hipSuccess) return hip_fail(e, "edge patch");
  mark(p, st, "edge_patch");
  *out = xk;
  return ZFFT_OK;
}

// XA path: one wave per frame and stage launch, stage outputs in natural layout (ping /
// pong).  Two or three stages per launch through per-frame rings measured slower.
int run_xa(zfft_plan *p, const InDesc &in, int frames, const std::vector<int64_t> &n,
           const float2 **out, hipStream_t st) {
  hipError_t e = p->ping.ensure((size_t)frames * n[1] * sizeof(float2));
  if (e == hipSuccess && p->K > 1) e = p->pong.ensure((size_t)frames * n[2] * sizeof(float2));
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "decimator workspace allocation failed");
  const float2 *cur = nullptr;
  for (int k = 0; k < p->K; ++k) {
    float2 *dst = (k & 1) ? p->pong.as<float2>() : p->ping.as<float2>();
    const InDesc src = k == 0 ? in : InDesc{cur, n[k], n[k], kInC64, 0};
    e = launch_xa_stage(src, (int)n[k], p->lo.as<float2>(), k == 0, dst, frames,
                        p->xa_tab.as<XaTab>(), st);
    if (e != hipSuccess) return hip_fail(e, "xa_stage launch");
    mark(p, st, k == 0 ? "xa_stage_mix" : "xa_stage");
    cur = dst;
  }
  *out = cur;
  return ZFFT_OK;
}

// PC decimator (pc_kernels.hip): zoom 8, frames long enough that the two frame ends'
// maps do not meet (kPcMinL), grid y = frames.
constexpr int64_t kPcMinL = 16384;
// KW (one workgroup per frame) from this many frames per call; below, K1 + K2's tiles.
// tools/sweep_walk.py (profiles/r06k/sweep_walk.json, round 6's walk; ms per call, tiles / walk):
// 299,008-sample frames 512: 0.78 / 0.78, 768: 1.08 / 1.12, 1024: 1.44 / 1.43, 2048: 2.64 /
// 2.53, 4096: 5.21 / 4.87; 2^20-sample frames 768: 3.34 / 3.44, 1024: 4.40 / 4.36, 2048: 8.54 /
// 8.27 (cfg5), 4096: 16.8 / 16.0.  One workgroup per frame needs about two rounds of the chip's
// 512 resident workgroups to fill it; KW also keeps y2 (2 B per input sample) off HBM.  (Round
// 4 measured the walk level with the tiles up to 4096 frames: the threshold was 4096.)
constexpr int kPcWalkMinFrames = 1024;
// Zoom 4: the two-stage walk from this many frames per call, the tiles below; XA no longer
// wins anywhere PC fits (cfg1's 262,144-sample frames, ms per call, XA / tiles / walk: 256:
// 1.24 / 0.47 / 0.50, 512: 1.32 / 0.90 / 0.78, 1024: 1.69 / 1.69 / 1.44, 4096 (cfg1): 5.17 /
// 6.27 / 4.89; profiles/r06k/sweep_walk.json).
constexpr int kPc4WalkMinFrames = 512;
// Zoom 8 (and the zoom >= 16 head): FC (path 6, fc_kernels.hip) from this many frames per call,
// PC's tiles below.  ms per call, tiles / walk / FC (tools/fc_ab.py, profiles/r06fc3/fc_ab.json):
// 299,008-sample frames 1: 0.053 / 0.39 / 0.064, 16: 0.078 / 0.41 / 0.078, 64: 0.124 / 0.41 /
// 0.107, 512: 0.75 / 0.74 / 0.52, 4096: - / 4.69 / 3.44; 2^20-sample frames 1: 0.057 / 1.23 /
// 0.066, 64: 0.37 / 1.30 / 0.26, 2048: - / 9.05 / 6.61.
constexpr int kFcMinFrames = 16;
// Zoom 4 (cfg1's 262,144-sample frames, ms per call, tiles / walk / FC, profiles/r06fc/r06fc8):
// 1: 0.055 / 0.39 / 0.062, 16: 0.080 / 0.41 / 0.083, 64: 0.146 / 0.43 / 0.129, 512: 0.93 / 0.80 /
// 0.61, 4096: - / 5.06 / 3.77.
constexpr int kFc4MinFrames = 32;
// FC takes frames of >= kFcN samples below 2^31 bytes (its buffer loads' 32-bit offsets).
bool fc_fits(const zfft_plan *p, int64_t L) {
  return L >= kFcN && L * (int64_t)in_elem_bytes(p->cfg.in_dtype) < ((int64_t)1 << 31);
}
bool pc_fits(const zfft_plan *p, int64_t L, int frames) {
  return p->K == kPcStages && L >= kPcMinL && frames <= 65535;
}
// Zoom 4 (two stages): the walk (pc_walk_kernel<4>, path 5, automatic from kPc4WalkMinFrames:
// round 5's form lost to XA at cfg1, 4.49 against 4.34 ms, profiles/r05h; round 6's walk wins)
// and the tiles (K1 = FIR alpha into y1, K2 = the zoom-8 tail kernel on zoom 4's tables: path 4,
// automatic below the walk's batch).
bool pc4_fits(const zfft_plan *p, int64_t L, int frames) {
  return p->K == 2 && L >= kPcMinL && frames <= 65535;
}
// Zoom-4 tiles against XA (cfg1's 262,144-sample frames, profiles/r05u, ms per call): 1 frame
// 0.061 / 1.14 (blocked passes 0.22), 64: 0.14 / 1.21 (0.28), 256: 0.46 / 1.24, 384: 0.65 /
// 1.26 -- XA, one wave per frame, needs about a thousand frames to fill the chip; from 512
// frames the zoom-4 walk beats both (kPc4WalkMinFrames).
// Zoom 2 (one stage): the tail kernel on the mixed input in XA's factorisation (D forward at
// the input rate, the 25-tap FIR M, D2 backward at half rate), automatic below
// 512 frames per call: cfg2's 299,008-sample frames, ms per call, tiles / XA (profiles/r05y):
// 1 frame 0.048 / 0.89 (blocked passes 0.16), 64: 0.16 / 0.95 (0.28), 384: 0.85 / 1.18,
// 1024: 2.05 / 1.53 -- equal near 640.
constexpr int kPc2TilesMaxFrames = 512;
bool pc2_fits(const zfft_plan *p, int64_t L, int frames) {
  return p->K == 1 && L >= kPcMinL && frames <= 65535;
}
// Zoom >= 16: PC takes the first three stages (decimate x 3 exactly, frame-end maps included)
// and XA the remaining K - 3 on its 1/8-rate output -- the reference's stages are applied one
// after another (S:2096-2098), so the composition is the same cascade.
bool pc_head_fits(const zfft_plan *p, int64_t L, int frames) {
  return p->K > kPcStages && L >= kPcMinL && frames <= 65535;
}

// Host copy of the PC tables: built once per process (fp64, microseconds); the frame-end maps
// are the constants of pc_edge_maps.h (tools/gen_pc_edge.py).
const PcTab *pc_host_tab() {
  static const std::unique_ptr<PcTab> t = [] {
    std::unique_ptr<PcTab> x(new PcTab());
    if (!pc_build_tables(*x)) x.reset();
    return x;
  }();
  return t.get();
}
const PcTab2 *pc_host_tab2() {
  static const std::unique_ptr<PcTab2> t = [] {
    std::unique_ptr<PcTab2> x(new PcTab2());
    if (!pc_build_tables2(*x)) x.reset();
    return x;
  }();
  return t.get();
}
const PcTab4 *pc_host_tab4() {
  static const std::unique_ptr<PcTab4> t = [] {
    std::unique_ptr<PcTab4> x(new PcTab4());
    if (!pc_build_tables4(*x)) x.reset();
    return x;
  }();
  return t.get();
}
// The PC tables and all nine frame-end maps, uploaded on the plan's first PC call; nothing is
// uploaded afterwards, so a change of L mod 8 between calls never waits on enqueued work.
int ensure_pc(zfft_plan *p) {
  if (p->pc_tab.p && p->pc_tab4.p && p->pc_tab2.p && p->pc_edge.p) return ZFFT_OK;
  const PcTab *t = pc_host_tab();
  const PcTab4 *t4 = pc_host_tab4();
  const PcTab2 *t2 = pc_host_tab2();
  if (!t || !t4 || !t2) return fail(ZFFT_EINTERNAL, "PC tables: scan depth or correction length too short");
  for (const PcEdgeConst &m : kPcEdge2Idx)
    if (m.r > kPcEdgeRank || m.R > kPcEdgeR || m.R > 256)
      return fail(ZFFT_EINTERNAL, "PC frame-end maps exceed the kernel's capacities");
  for (const PcEdgeConst &m : kPcEdgeIdx)
    if (m.r > kPcEdgeRank || m.R > kPcEdgeR || m.R > 256)
      return fail(ZFFT_EINTERNAL, "PC frame-end maps exceed the kernel's capacities");
  for (const PcEdgeConst &m : kPcEdge4Idx)
    if (m.r > kPcEdgeRank || m.R > kPcEdgeR || m.R > 256)
      return fail(ZFFT_EINTERNAL, "PC frame-end maps exceed the kernel's capacities");
  hipError_t e = p->pc_tab.ensure(sizeof(PcTab));
  if (e == hipSuccess) e = hipMemcpy(p->pc_tab.p, t, sizeof(PcTab), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = p->pc_tab4.ensure(sizeof(PcTab4));
  if (e == hipSuccess) e = hipMemcpy(p->pc_tab4.p, t4, sizeof(PcTab4), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = p->pc_tab2.ensure(sizeof(PcTab2));
  if (e == hipSuccess) e = hipMemcpy(p->pc_tab2.p, t2, sizeof(PcTab2), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = p->pc_edge.ensure(sizeof(kPcEdgeData));
  if (e == hipSuccess) e = hipMemcpy(p->pc_edge.p, kPcEdgeData, sizeof(kPcEdgeData), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "PC table upload");
  return ZFFT_OK;
}

// FC's zoom on this plan: 4 at zoom 4, else 8 (zoom 8 and the head of zoom >= 16)
int fc_zoom(const zfft_plan *p) { return p->K == 2 ? 4 : 8; }
// FC tables for the plan's LO rows (host fp64 build, fc_build_row; one synchronous upload when
// the LO frequencies change, after the plan's enqueued work)
int ensure_fc(zfft_plan *p) {
  const std::vector<double> freqs = p->lo_freqs.empty() ? std::vector<double>{p->cfg.f_lo} : p->lo_freqs;
  std::vector<double> ratios;
  for (double fr : freqs) ratios.push_back(fr / p->cfg.fs);
  if (p->fc_tab.p && p->fc_built == ratios) return ZFFT_OK;
  int rc = quiesce(p);
  if (rc) return rc;
  const int zoom = fc_zoom(p), M = kFcN / zoom;
  std::vector<float2> h;
  try {
    h.resize(M + ratios.size() * (size_t)kFcRow);
  } catch (const std::bad_alloc &) {
    return fail(ZFFT_ENOMEM, "FC table host staging allocation failed");
  }
  fc_build_twiddles(M, h.data());
  for (size_t k = 0; k < ratios.size(); ++k)
    if (!fc_build_row(zoom, ratios[k], h.data() + M + k * kFcRow))
      return fail(ZFFT_EINTERNAL, "FC table: model response unavailable");
  hipError_t e = p->fc_tab.ensure(h.size() * sizeof(float2));
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "FC table allocation failed");
  e = hipMemcpy(p->fc_tab.p, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "FC table upload");
  p->fc_built = ratios;
  return ZFFT_OK;
}

// PC path: K1 (FIRs) -> y2 (ping) -> K2 (own-rate sections, FIR, output-rate sections) ->
// out (pong) -> K3 (frame-end maps, in place).
// K = the stages PC runs: p->K (zoom 4 or 8), or 3 as the head of a longer cascade.
// fc (zoom 8, K = 3, with walk): the FC kernel in the walk's place (fc_kernels.hip, path 6).
int run_pc(zfft_plan *p, const InDesc &in, int64_t L, int frames, const std::vector<int64_t> &n,
           bool walk, const float2 **out, hipStream_t st, int K, bool fc = false) {
  int rc = ensure_pc(p);
  if (rc) return rc;
  fc = fc && walk && (K == kPcStages || K == 2);
  if (fc && (rc = ensure_fc(p))) return rc;
  const int64_t n3 = n[K];
  const PcTab *tab = p->pc_tab.as<PcTab>();
  hipError_t e;
  if (K == 1) {  // zoom 2: the tail kernel straight on the mixed input
    e = p->pong.ensure((size_t)frames * n3 * sizeof(float2));
    if (e != hipSuccess) return fail(ZFFT_ENOMEM, "decimator workspace allocation failed");
    e = launch_pc2_tail(in, p->lo.as<float2>(), p->pong.as<float2>(), n3, frames, p->pc_tab2.as<PcTab2>(), st);
    if (e != hipSuccess) return hip_fail(e, "pc_tail launch");
    mark(p, st, "pc_tail");
  } else if (K == 2 && !walk) {  // zoom 4 as tiles: K1 (FIR alpha) -> y1 (ping) -> K2 -> out (pong)
    const int64_t y1s = (pc4_y1_len(L) + kPc4K1M - 1) / kPc4K1M * kPc4K1M;
    e = p->ping.ensure((size_t)frames * y1s * sizeof(float2));
    if (e == hipSuccess) e = p->pong.ensure((size_t)frames * n3 * sizeof(float2));
    if (e != hipSuccess) return fail(ZFFT_ENOMEM, "decimator workspace allocation failed");
    e = launch_pc4_fir(in, p->lo.as<float2>(), p->ping.as<float2>(), y1s, frames, p->pc_tab4.as<PcTab4>(), st);
    if (e != hipSuccess) return hip_fail(e, "pc_fir launch");
    mark(p, st, "pc_fir");
    e = launch_pc4_tail(p->ping.as<float2>(), y1s, y1s, p->pong.as<float2>(), n3, frames,
                        p->pc_tab4.as<PcTab4>(), st);
    if (e != hipSuccess) return hip_fail(e, "pc_tail launch");
    mark(p, st, "pc_tail");
  } else if (walk) {  // one launch, y2 (zoom 4: y1) in LDS; the frame-end sums beside it
    e = p->pong.ensure((size_t)frames * n3 * sizeof(float2));
    if (e == hipSuccess) e = p->edge_v.ensure((size_t)frames * 2 * kPcEdgeRank * sizeof(float2));
    if (e != hipSuccess) return fail(ZFFT_ENOMEM, "decimator workspace allocation failed");
    e = hipEventRecord(p->fork_ev, st);
    if (e == hipSuccess) e = hipStreamWaitEvent(p->side_st, p->fork_ev, 0);
    if (e != hipSuccess) return hip_fail(e, "side stream fork");
    if (fc) e = launch_fc_decim(in, p->lo.as<float2>(), p->fc_tab.as<float2>(), kFcRow, p->pong.as<float2>(), n3, frames,
                                K == 2 ? 4 : 8, st);
    else if (K == 2) e = launch_pc_walk4(in, p->lo.as<float2>(), p->pong.as<float2>(), n3, frames, p->pc_tab4.as<PcTab4>(), st);
    else e = launch_pc_walk(in, p->lo.as<float2>(), p->pong.as<float2>(), n3, frames, tab, st);
    if (e != hipSuccess) return hip_fail(e, fc ? "fc_decim launch" : "pc_walk launch");
    mark(p, st, fc ? "fc_decim" : K == 2 ? "pc_walk4" : "pc_walk");
    const float *eb = p->pc_edge.as<float>();
    const PcEdgeConst &m0 = K == 2 ? kPcEdge4Idx[0] : kPcEdgeIdx[0];
    const PcEdgeConst &m1 = K == 2 ? kPcEdge4Idx[1 + (L & 3)] : kPcEdgeIdx[1 + (L & 7)];
    const float *const V[2] = {eb + m0.v, eb + m1.v};
    const int J[2] = {m0.J, m1.J}, r[2] = {m0.r, m1.r};
    // submitted after the walk's launch (before it: the same step time, profiles/r06r)
    e = launch_pc_edge_v(in, p->lo.as<float2>(), p->edge_v.as<float2>(), frames, V, J, r, p->side_st);
    if (e != hipSuccess) return hip_fail(e, "pc_edge_v launch");
  } else {
    const int64_t y2s = (pc_y2_len(L) + kPcK1Q - 1) / kPcK1Q * kPcK1Q;
    e = p->ping.ensure((size_t)frames * y2s * sizeof(float2));
    if (e == hipSuccess) e = p->pong.ensure((size_t)frames * n3 * sizeof(float2));
    if (e != hipSuccess) return fail(ZFFT_ENOMEM, "decimator workspace allocation failed");
    e = launch_pc_fir(in, p->lo.as<float2>(), p->ping.as<float2>(), y2s, frames, tab, st);
    if (e != hipSuccess) return hip_fail(e, "pc_fir launch");
    mark(p, st, "pc_fir");
    e = launch_pc_tail(p->ping.as<float2>(), y2s, p->pong.as<float2>(), n3, frames, tab, st);
    if (e != hipSuccess) return hip_fail(e, "pc_tail launch");
    mark(p, st, "pc_tail");
  }
  // map 0 = frame start, 1 + (L mod 2^K) = frame end (pc_edge_maps.h)
  const float *eb = p->pc_edge.as<float>();
  const PcEdgeConst &m0 = K == 1 ? kPcEdge2Idx[0] : K == 2 ? kPcEdge4Idx[0] : kPcEdgeIdx[0];
  const PcEdgeConst &m1 = K == 1   ? kPcEdge2Idx[1 + (L & 1)]
                          : K == 2 ? kPcEdge4Idx[1 + (L & 3)]
                                   : kPcEdgeIdx[1 + (L & 7)];
  const float *const U[2] = {eb + m0.u, eb + m1.u};
  const float *const V[2] = {eb + m0.v, eb + m1.v};
  const int R[2] = {m0.R, m1.R}, J[2] = {m0.J, m1.J}, r[2] = {m0.r, m1.r};
  if (walk && K >= 2) {  // V^T x ran on the side stream beside the walk: join, then out += U v
    e = hipEventRecord(p->join_ev, p->side_st);
    if (e == hipSuccess) e = hipStreamWaitEvent(st, p->join_ev, 0);
    if (e == hipSuccess) e = launch_pc_edge_u(p->edge_v.as<float2>(), p->pong.as<float2>(), n3, frames, U, R, r, st);
  } else {
    e = launch_pc_edge(in, p->lo.as<float2>(), p->pong.as<float2>(), n3, frames, U, V, R, J, r, st);
  }
  if (e != hipSuccess) return hip_fail(e, "pc_edge launch");
  mark(p, st, "pc_edge");
  *out = p->pong.as<float2>();
  return ZFFT_OK;
}

// PC head (3 stages into pong), then stages 3 .. K-1 on its output (no LO mix): XA where XA
// takes the batch (ping, pong, ... in turn), else the exact blocked passes (few frames per
// call, the reference's one: a unit LO table stands for the mix their first pass applies).
int run_pc_head(zfft_plan *p, const InDesc &in, int64_t L, int frames, const std::vector<int64_t> &n,
                bool walk, const float2 **out, hipStream_t st, bool fc = false) {
  const float2 *cur = nullptr;
  const int64_t n3 = n[kPcStages];
  // XA where it takes the batch, except where zoom 2's tiles still beat it (< 512 frames)
  const bool xa_tail = auto_xa(frames, n3) && !(frames < kPc2TilesMaxFrames && n3 >= kPcMinL);
  hipError_t e = hipSuccess;
  if (!xa_tail) {  // ping / pong must not move under a stage's input once the tail sizes them
    const size_t G = (size_t)(frames + 63) / 64 * 64;
    e = p->pong.ensure(std::max((size_t)frames * n3, p->K > kPcStages + 1 ? G * n[kPcStages + 2] : 0) *
                       sizeof(float2));
    if (e == hipSuccess) e = p->ping.ensure(G * n[kPcStages + 1] * sizeof(float2));
    if (e == hipSuccess && p->lo1_n < n3) {  // filled length, set only once the fill is enqueued
      e = p->lo1.ensure((size_t)n3 * sizeof(float2));
      if (e == hipSuccess) e = launch_fill_c64(p->lo1.as<float2>(), n3, 1.f, 0.f, st);
      if (e == hipSuccess) p->lo1_n = n3;
    }
    if (e != hipSuccess) return fail(ZFFT_ENOMEM, "decimator workspace allocation failed");
  }
  int rc = run_pc(p, in, L, frames, n, walk, &cur, st, kPcStages, fc);
  if (rc) return rc;
  if (!xa_tail) {
    // zoom 2's tiles (XA's factorisation, the unit LO table) while a stage's input has >= 16384
    // samples, ping, pong, ... in turn; the blocked passes for the stages after that
    int k = kPcStages;
    for (; k < p->K && n[k] >= kPcMinL; ++k) {
      float2 *dst = ((k - kPcStages) & 1) ? p->pong.as<float2>() : p->ping.as<float2>();
      const InDesc src{cur, n[k], n[k], kInC64, 0};
      e = launch_pc2_tail(src, p->lo1.as<float2>(), dst, n[k + 1], frames, p->pc_tab2.as<PcTab2>(), st);
      if (e != hipSuccess) return hip_fail(e, "pc_tail launch");
      mark(p, st, "pc_tail");
      const float *eb = p->pc_edge.as<float>();
      const PcEdgeConst &m0 = kPcEdge2Idx[0], &m1 = kPcEdge2Idx[1 + (n[k] & 1)];
      const float *const U[2] = {eb + m0.u, eb + m1.u};
      const float *const V[2] = {eb + m0.v, eb + m1.v};
      const int R[2] = {m0.R, m1.R}, J[2] = {m0.J, m1.J}, r[2] = {m0.r, m1.r};
      e = launch_pc_edge(src, p->lo1.as<float2>(), dst, n[k + 1], frames, U, V, R, J, r, st);
      if (e != hipSuccess) return hip_fail(e, "pc_edge launch");
      mark(p, st, "pc_edge");
      cur = dst;
    }
    if (k == p->K) {
      *out = cur;
      return ZFFT_OK;
    }
    const InDesc src{cur, n[k], n[k], kInC64, 0};
    return run_exact(p, src, p->lo1.as<float2>(), frames, n, out, st, 0, 0, k);
  }
  e = p->ping.ensure((size_t)frames * n[kPcStages + 1] * sizeof(float2));
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "decimator workspace allocation failed");
  for (int k = kPcStages; k < p->K; ++k) {
    float2 *dst = ((k - kPcStages) & 1) ? p->pong.as<float2>() : p->ping.as<float2>();
    const InDesc src{cur, n[k], n[k], kInC64, 0};
    e = launch_xa_stage(src, (int)n[k], p->lo.as<float2>(), false, dst, frames, p->xa_tab.as<XaTab>(), st);
    if (e != hipSuccess) return hip_fail(e, "xa_stage launch");
    mark(p, st, "xa_stage");
    cur = dst;
  }
  *out = cur;
  return ZFFT_OK;
}

int run_decimator(zfft_plan *p, const InDesc &in, int64_t L, int frames,
                  const std::vector<int64_t> &n, const float2 **out, hipStream_t st) {
  if (p->path == 3 && !xa_fits(p, L))
    return fail(ZFFT_EUNSUPPORTED, "XA tiles (path 3) address a frame's stage arrays with 32-bit "
                                   "offsets: frames of >= 2^31 bytes need path 0, 1 or 2");
  int rc = ensure_lo(p, L);
  if (rc) return rc;
  // exact tiles run one wave per frame: the schedule for batches that fill the GPU; the
  // blocked schedules split each frame over many waves and win for a few frames per call
  const bool pc8 = pc_fits(p, L, frames), head = pc_head_fits(p, L, frames), pc4 = pc4_fits(p, L, frames),
             pc2 = pc2_fits(p, L, frames);
  if (p->path >= 4 && !pc8 && !head && !pc4 && !pc2)
    return fail(ZFFT_EUNSUPPORTED, "PC decimator needs frames of >= 16384 samples and <= 65535 "
                                   "frames per call");
  // the tiles hand a batch over to XA only where XA takes it (auto_xa: from 768 frames of
  // > 2^19 samples), never to the blocked passes, which lose to the tiles at every batch
  const bool xa_auto = auto_xa(frames, L) && xa_fits(p, L);
  // zoom 2: the tiles on request (paths 4, 5) and automatic below 512 frames per call
  if (pc2 && (p->path >= 4 || (p->path == 0 && (frames < kPc2TilesMaxFrames || !xa_auto))))
    return run_pc(p, in, L, frames, n, false, out, st, 1);
  // zoom 4: the tiles below 512 frames per call, the walk from there (both on request too)
  if (pc4 && (p->path >= 4 || p->path == 0)) {
    const bool fc4 = fc_fits(p, L) && (p->path == 6 || (p->path == 0 && frames >= kFc4MinFrames));
    return run_pc(p, in, L, frames, n, fc4 || p->path >= 5 || (p->path == 0 && frames >= kPc4WalkMinFrames),
                  out, st, p->K, fc4);
  }
  const bool walk = p->path >= 5 || (p->path == 0 && frames >= kPcWalkMinFrames);
  // FC in the walk's place: on request (6) and automatic from kFcMinFrames frames per call
  const bool fc = fc_fits(p, L) && (p->path == 6 || (p->path == 0 && frames >= kFcMinFrames));
  // PC (tiles below kFcMinFrames frames per call, FC from there) is the fastest schedule
  // wherever it applies, from one frame per call (the reference's use: 0.053 against 0.37 ms
  // for path 1) to full batches (4096 frames: FC 3.44 against the walk's 4.69 ms) --
  // tools/sweep_schedule.py, profiles/r04l; tools/fc_ab.py, profiles/r06fc3
  if (pc8 && (p->path == 0 || p->path >= 4))
    return run_pc(p, in, L, frames, n, walk || fc, out, st, p->K, fc);
  // zoom >= 16: the head, then XA or the blocked passes for the rest (by the tail's batch)
  if (p->path >= 4 || (p->path == 0 && head && xa_fits(p, L)))
    return run_pc_head(p, in, L, frames, n, walk || fc, out, st, fc);
  if (p->path == 3 || (p->path == 0 && auto_xa(frames, L) && xa_fits(p, L)))
    return run_xa(p, in, frames, n, out, st);
  if (use_fused(p, L, frames)) return run_fused(p, in, L, frames, n, out, st);
  return run_exact(p, in, p->lo.as<float2>(), frames, n, out, st);
}

// Real input at zoom 1 takes scipy.signal.welch's one-sided branch.
bool onesided(const zfft_plan *p) { return p->cfg.in_dtype == kInF32R && p->K == 0; }

// Valid entries per row: the length of the reference's slice fftshift(P)[N//2 - W//2 :
// N//2 + W//2] (S:2114): 2 (W//2), or in the one-sided case that slice of the N/2+1 bins.
int row_length(const zfft_plan *p) {
  const int N = p->cfg.n_fft, W = p->cfg.n_win;
  if (!onesided(p)) return W & ~1;  // [N/2 - W//2, N/2 + W//2): W - 1 entries for odd W
  const int a = N / 2 - W / 2, b = std::min(N / 2 + W / 2, N / 2 + 1);
  return std::max(0, b - a);
}

InDesc input_of(const zfft_plan *p, const void *d_iq, int64_t L) {
  InDesc d{d_iq, L, L, p->cfg.in_dtype, p->cfg.flip_input};
  if (p->lo_freqs.size() > 1) {
    d.lo_stride = p->lo_len;  // (ensure_lo runs before any kernel reads the rows)
    d.lo_n = (int)p->lo_freqs.size();
    d.lo_per = p->lo_per;
    d.lo_first = p->lo_first;
  }
  return d;
}

int process_device(zfft_plan *p, const void *d_iq, int64_t L, int32_t frames, float *d_rows,
                   hipStream_t st) {
  std::vector<int64_t> n;
  int rc = check_lengths(p, L, frames, n);
  if (rc) return rc;
  const int64_t Ld = n[p->K];
  const int N = p->cfg.n_fft;
  const int nperseg = (int)(Ld < N ? Ld : N);
  rc = ensure_window(p, nperseg);
  if (rc) return rc;
  if (p->K > 0) {  // the LO rows exist (and have their stride) before input_of reads it
    rc = ensure_lo(p, L);
    if (rc) return rc;
  }
  const InDesc in = input_of(p, d_iq, L);
  const float2 *x = (const float2 *)d_iq;
  if (p->n_marks == 0) mark(p, st, "start");  // (the entry points reset the marks per call)
  if (p->K > 0) {
    rc = run_decimator(p, in, L, frames, n, &x, st);
    if (rc) return rc;
  } else if (in.dtype != kInC64 || in.flip) {  // zoom 1: Welch reads complex64 frames
    hipError_t e = p->dec.ensure((size_t)frames * L * sizeof(float2));
    if (e != hipSuccess) return fail(ZFFT_ENOMEM, "ingest workspace allocation failed");
    e = launch_ingest(in, nullptr, p->dec.as<float2>(), frames, st);
    if (e != hipSuccess) return hip_fail(e, "ingest launch");
    mark(p, st, "ingest");
    x = p->dec.as<float2>();
  }
  WelchGeom w;
  w.n_fft = N;
  w.log2n = ilog2(N);
  w.n_win = p->cfg.n_win;
  w.nperseg = nperseg;
  w.step = nperseg - nperseg / 2;
  w.nseg = (int)((Ld - nperseg) / w.step + 1);
  // density scaling 1/(fs*sum(w^2)) and the segment mean (csd average='mean')
  w.scale = (float)(1.0 / (p->cfg.fs * p->win_ss * (double)w.nseg));
  if (onesided(p)) {
    w.onesided = 1;
    w.row_a = N / 2 - p->cfg.n_win / 2;
    w.row_len = row_length(p);
  }
  // auto: four-step above 16384 (the only form there); N <= 16384 runs one workgroup per
  // frame (the in-place DIF kernel from N = 1024)
  const bool four = p->welch == 2 || (p->welch == 0 && N > kWelchOneWgMax);
  hipError_t e;
  if (four) {
    // frames in chunks whose intermediate Z (nseg x N complex64 per frame) stays in the
    // 256 MB Infinity Cache between the column and the row pass instead of round-tripping
    // through HBM
    const size_t zf = (size_t)w.nseg * N * sizeof(float2);
    const int chunk = kWelch4ChunkBytes > 0
                          ? (int)std::max<size_t>(1, std::min<size_t>(frames, kWelch4ChunkBytes / zf))
                          : frames;
    w.fused_mean = nperseg == N ? 1 : 0;  // partial sums from the column pass (kN2-column groups)
    e = p->means.ensure((size_t)chunk * w.nseg * std::max(1, N / 256 / 16) * sizeof(float2));
    if (e == hipSuccess) e = p->z4.ensure((size_t)chunk * zf);
    if (e != hipSuccess) return fail(ZFFT_ENOMEM, "four-step Welch workspace allocation failed");
    for (int f0 = 0; f0 < frames; f0 += chunk) {
      const int nf = std::min(chunk, frames - f0);
      e = launch_welch4(x + (int64_t)f0 * Ld, Ld, p->win.as<float>(), p->tw.as<float2>(),
                        p->tws.as<float2>(), w.fused_mean ? p->winf.as<float2>() : nullptr, w,
                        p->means.as<float2>(), p->z4.as<float2>(),
                        d_rows + (int64_t)f0 * p->cfg.n_win, nf, st);
      if (e != hipSuccess) return hip_fail(e, "welch4 launch");
    }
    mark(p, st, "welch4");
  } else {
    // few frames per call (the reference's one): each frame's segments over several
    // workgroups (welch_dif_split), partial PSDs summed by a second launch
    if (nperseg == N) w.split = welch_dif_split(N, w.nseg, frames);
    if (w.split > 1) {
      e = p->wparts.ensure((size_t)frames * w.split * p->cfg.n_win * sizeof(float));
      if (e != hipSuccess) return fail(ZFFT_ENOMEM, "Welch workspace allocation failed");
      w.parts = p->wparts.as<float>();
    }
    e = launch_welch_rows(x, Ld, p->win.as<float>(), p->tw.as<float2>(), w, d_rows, frames, st);
    if (e != hipSuccess) return hip_fail(e, "welch_rows launch");
    mark(p, st, "welch_rows");
  }
  p->last_row = d_rows + (int64_t)(frames - 1) * p->cfg.n_win;
  return ZFFT_OK;
}

int ensure_waterfall(zfft_plan *p) {
  const int W = p->cfg.n_win;
  if (p->wf_ready && p->W == W) return ZFFT_OK;
  if (W < 10 || (p->cfg.scroll > 0 && W / 4 < 15) || (p->cfg.scroll < 0 && W / 4 < 10))
    return fail(ZFFT_EINVAL, "waterfall needs n_win >= 60 (scroll=+1) or >= 40 (scroll=-1): "
                             "Waterfall.image_update indexes rows 5..14 / -10..-3 (S:1655-1662)");
  const int H = W / 4;
  hipError_t e = p->ring.ensure((size_t)H * W * sizeof(float));
  if (e == hipSuccess) e = p->img.ensure((size_t)H * W * sizeof(float));
  if (e == hipSuccess) e = p->one_row.ensure((size_t)W * sizeof(float));
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "waterfall allocation failed");
  int rc = use_stream(p, p->stream);
  if (rc) return rc;
  e = launch_waterfall_init(p->ring.as<float>(), H, W, p->stream);
  if (e != hipSuccess) return hip_fail(e, "waterfall init");
  rc = done_on(p, p->stream);
  if (rc) return rc;
  p->H = H;
  p->W = W;
  p->off = 0;
  p->wf_ready = true;
  return ZFFT_OK;
}

// A NULL stream handle means HIP's default (null) stream, as everywhere in HIP.
hipStream_t pick_stream(zfft_plan *, void *s) { return (hipStream_t)s; }

// Order `st` after everything the plan enqueued before (on any stream).
int use_stream(zfft_plan *p, hipStream_t st) {
  if (p->has_work && p->done_st != st) {
    hipError_t e = hipStreamWaitEvent(st, p->done_ev, 0);
    if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent");
  }
  return ZFFT_OK;
}
// Mark the end of the plan's work enqueued so far on `st`.
int done_on(zfft_plan *p, hipStream_t st) {
  hipError_t e = hipEventRecord(p->done_ev, st);
  if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
  p->done_st = st;
  p->has_work = true;
  return ZFFT_OK;
}
// Wait on the host until the plan's enqueued work is done (before a synchronous upload
// overwrites a table that work may still read).
int quiesce(zfft_plan *p) {
  if (!p->has_work) return ZFFT_OK;
  ++p->n_quiesce;
  hipError_t e = hipEventSynchronize(p->done_ev);
  return e == hipSuccess ? ZFFT_OK : hip_fail(e, "hipEventSynchronize");
}

int enter(zfft_plan *p) {
  if (!p) return fail(ZFFT_EINVAL, "null plan");
  hipError_t e = hipSetDevice(p->cfg.device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  return ZFFT_OK;
}

}  // namespace

// Test hook (not part of include/zfft.h): how often the plan has waited on the host for its
// enqueued work (a table upload that must not overwrite data in use, a synchronous call).
extern "C" int64_t zfft__plan_quiesce_count(const zfft_plan *p) { return p ? p->n_quiesce : -1; }

extern "C" {

const char *zfft_last_error(void) { return g_err.c_str(); }
int zfft_version(void) { return ZFFT_VERSION; }

int zfft_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int64_t zfft_decimated_length(int64_t n_samples, int32_t zoom) {
  if (n_samples < 0 || !is_pow2(zoom)) return -1;
  for (int z = zoom; z > 1; z >>= 1) n_samples = (n_samples + 1) / 2;
  return n_samples;
}

int zfft_plan_create(const zfft_config *cfg, const float *window_or_null, zfft_plan **out) {
  if (!cfg || !out) return fail(ZFFT_EINVAL, "null config or output pointer");
  *out = nullptr;
  const zfft_config &c = *cfg;
  if (!is_pow2(c.n_fft) || c.n_fft < 32 || c.n_fft > 65536)
    return fail(ZFFT_EINVAL, "n_fft must be a power of two in [32, 65536]");
  if (!is_pow2(c.zoom) || c.zoom > 512) return fail(ZFFT_EINVAL, "zoom must be 1, 2, 4, ..., 512");
  if (c.n_win < 2 || c.n_win > c.n_fft)
    return fail(ZFFT_EINVAL, "n_win must be in [2, n_fft]");
  if (!(c.fs > 0) || !std::isfinite(c.fs) || !std::isfinite(c.f_lo))
    return fail(ZFFT_EINVAL, "fs must be positive and finite, f_lo finite");
  if (c.scroll != 1 && c.scroll != -1) return fail(ZFFT_EINVAL, "scroll must be +1 or -1");
  if (c.in_dtype < kInC64 || c.in_dtype > kInF32R)
    return fail(ZFFT_EINVAL, "in_dtype must be 0 (complex64), 1 (complex32 f16), 2 (RTL-SDR u8) or 3 (real f32)");
  if (c.flip_input != 0 && c.flip_input != 1) return fail(ZFFT_EINVAL, "flip_input must be 0 or 1");
  if (c.window_kind == ZFFT_WIN_ARRAY) {
    if (!window_or_null) return fail(ZFFT_EINVAL, "ZFFT_WIN_ARRAY needs a window array");
  } else if (!window_kind_native(c.window_kind)) {
    return fail(ZFFT_EINVAL, "unknown window kind");
  }
  int ndev = zfft_device_count();
  if (ndev < 1) return fail(ZFFT_ENODEV, "no HIP device");
  if (c.device < 0 || c.device >= ndev) return fail(ZFFT_ENODEV, "device ordinal out of range");
  hipError_t e = hipSetDevice(c.device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");

  zfft_plan *p = new zfft_plan();
  p->cfg = c;
  p->K = ilog2(c.zoom);
  if (c.window_kind == ZFFT_WIN_ARRAY)
    p->user_window.assign(window_or_null, window_or_null + c.n_fft);
  e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->copy_st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->side_st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&p->done_ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&p->fork_ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&p->join_ev, hipEventDisableTiming);
  for (int i = 0; i < 2 && e == hipSuccess; ++i) {
    e = hipEventCreateWithFlags(&p->h2d_ev[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->comp_ev[i], hipEventDisableTiming);
  }
  if (e != hipSuccess) {
    zfft_plan_destroy(p);
    return hip_fail(e, "hipStreamCreate / hipEventCreate");
  }
  // FFT twiddles tw[m] = exp(-2 pi i m / N), computed in fp64
  std::vector<float2> tw(c.n_fft);
  for (int m = 0; m < c.n_fft; ++m) {
    const double a = -2.0 * M_PI * (double)m / (double)c.n_fft;
    tw[m] = make_float2((float)std::cos(a), (float)std::sin(a));
  }
  e = p->tw.ensure(c.n_fft * sizeof(float2));
  if (e == hipSuccess)
    e = hipMemcpy(p->tw.p, tw.data(), c.n_fft * sizeof(float2), hipMemcpyHostToDevice);
  if (e == hipSuccess && c.n_fft >= 4096) {  // four-step sub-FFT twiddles: W_256 ++ W_N1
    const int n1 = c.n_fft / 256;
    std::vector<float2> ts(256 + n1);
    for (int m = 0; m < 256; ++m) ts[m] = tw[(size_t)m * n1];
    for (int m = 0; m < n1; ++m) ts[256 + m] = tw[(size_t)m * 256];
    e = p->tws.ensure(ts.size() * sizeof(float2));
    if (e == hipSuccess)
      e = hipMemcpy(p->tws.p, ts.data(), ts.size() * sizeof(float2), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    static XaTab xa[1]{};
    static const bool xa_ok = xa_build_tables(xa[0], kXaB);
    if (!xa_ok) {
      zfft_plan_destroy(p);
      return fail(ZFFT_EHIP, "XA tables: scan levels too shallow for the filter poles");
    }
    e = p->xa_tab.ensure(sizeof(xa));
    if (e == hipSuccess) e = hipMemcpy(p->xa_tab.p, xa, sizeof(xa), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    zfft_plan_destroy(p);
    return hip_fail(e, "twiddle upload");
  }
  *out = p;
  return ZFFT_OK;
}

int zfft_plan_destroy(zfft_plan *p) {
  if (!p) return ZFFT_OK;
  (void)hipSetDevice(p->cfg.device);
  if (p->has_work) (void)hipEventSynchronize(p->done_ev);
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  for (DevBuf *b : {&p->lo, &p->win, &p->tw, &p->in, &p->in2, &p->yf, &p->ping, &p->pong, &p->rows,
                    &p->ring, &p->img, &p->one_row, &p->dec, &p->edge, &p->xk, &p->xa_tab,
                    &p->tws, &p->means, &p->z4, &p->winf, &p->pc_tab, &p->pc_edge, &p->pc_tab4,
                    &p->wparts, &p->lo1, &p->pc_tab2, &p->lut_d, &p->rgba, &p->al_hist, &p->al_bins,
                    &p->edge_v, &p->img64, &p->fc_tab})
    b->release();
  if (p->row_pin) (void)hipHostFree(p->row_pin);
  for (hipEvent_t ev : p->events) (void)hipEventDestroy(ev);
  if (p->done_ev) (void)hipEventDestroy(p->done_ev);
  if (p->fork_ev) (void)hipEventDestroy(p->fork_ev);
  if (p->join_ev) (void)hipEventDestroy(p->join_ev);
  if (p->side_st) (void)hipStreamSynchronize(p->side_st), (void)hipStreamDestroy(p->side_st);
  for (int i = 0; i < 2; ++i) {
    if (p->h2d_ev[i]) (void)hipEventDestroy(p->h2d_ev[i]);
    if (p->comp_ev[i]) (void)hipEventDestroy(p->comp_ev[i]);
  }
  if (p->copy_st) (void)hipStreamSynchronize(p->copy_st), (void)hipStreamDestroy(p->copy_st);
  if (p->stream) (void)hipStreamDestroy(p->stream);
  delete p;
  return ZFFT_OK;
}

int zfft_plan_row_length(const zfft_plan *p) {
  if (!p) return fail(ZFFT_EINVAL, "null plan");
  return row_length(p);
}

int zfft_plan_config(const zfft_plan *p, zfft_config *out) {
  if (!p || !out) return fail(ZFFT_EINVAL, "null argument");
  *out = p->cfg;
  return ZFFT_OK;
}

int zfft_plan_tune(zfft_plan *p, int32_t block, int32_t warm) {
  if (!p || block < 0 || warm < 0) return fail(ZFFT_EINVAL, "bad tune arguments");
  if (block && (block < 64 || block > (1 << 20)))
    return fail(ZFFT_EINVAL, "block must be in [64, 2^20]");
  p->block_override = block;
  p->warm_override = warm;
  return ZFFT_OK;
}

int zfft_plan_timing(zfft_plan *p, int32_t enable) {
  if (!p) return fail(ZFFT_EINVAL, "null plan");
  p->timing = enable != 0;  // marks of the last timed call stay readable
  return ZFFT_OK;
}

int zfft_plan_path(zfft_plan *p, int32_t path) {
  if (!p || path < 0 || path > 6)
    return fail(ZFFT_EINVAL, "path must be 0 (auto), 1 (exact), 2 (fused), 3 (XA tiles), 4 (PC "
                             "tiles), 5 (PC walk) or 6 (FC at zoom 8, else as 5)");
  p->path = path;
  return ZFFT_OK;
}

int zfft_plan_set_lo_frames(zfft_plan *p, const double *f_lo, int32_t n, int32_t frames_per_lo) {
  int rc = enter(p);
  if (rc) return rc;
  if (n < 0 || n > kMaxLoRows || (n > 0 && (!f_lo || frames_per_lo < 1)))
    return fail(ZFFT_EINVAL, "set_lo_frames: 0 <= n <= 256 frequencies, frames_per_lo >= 1");
  if (n > 1 && p->K == 0)  // rows never mix at zoom 1: the reference skips zoomfft (S:2108)
    return fail(ZFFT_EINVAL, "set_lo_frames: several LO rows need zoom > 1 (zoom 1 does not mix)");
  for (int i = 0; i < n; ++i)
    if (!std::isfinite(f_lo[i])) return fail(ZFFT_EINVAL, "set_lo_frames: f_lo must be finite");
  rc = quiesce(p);  // the old table may still be read by enqueued work
  if (rc) return rc;
  p->lo_freqs.assign(f_lo, f_lo + n);
  if (n == 1) p->cfg.f_lo = f_lo[0];
  if (n <= 1) p->lo_freqs.clear();
  p->lo_per = n > 0 ? frames_per_lo : 1;
  p->lo_len = 0;  // rebuilt by the next call
  return ZFFT_OK;
}

int zfft_plan_welch(zfft_plan *p, int32_t mode) {
  if (!p || mode < 0 || mode > 2)
    return fail(ZFFT_EINVAL, "welch mode must be 0 (auto), 1 (one workgroup) or 2 (four-step)");
  if (mode == 1 && p->cfg.n_fft > kMaxLdsFft)
    return fail(ZFFT_EUNSUPPORTED, "one-workgroup Welch holds at most 16384 points in LDS");
  if (mode == 2 && p->cfg.n_fft < 4096)
    return fail(ZFFT_EINVAL, "four-step Welch needs n_fft >= 4096 (N1 = n_fft/256 >= 16)");
  p->welch = mode;
  return ZFFT_OK;
}

const char *zfft_plan_timing_names(zfft_plan *p) {
  if (!p) return "";
  p->names_buf.clear();
  for (int k = 1; k < p->n_marks; ++k) {
    if (k > 1) p->names_buf += ",";
    p->names_buf += p->mark_names[k];
  }
  return p->names_buf.c_str();
}

int zfft_plan_timings(zfft_plan *p, float *ms_out, int32_t max, int32_t *count) {
  int rc = enter(p);
  if (rc) return rc;
  if (!ms_out || !count) return fail(ZFFT_EINVAL, "null output");
  const int n = p->n_marks > 0 ? p->n_marks - 1 : 0;
  if (n > 0) {
    hipError_t e = hipEventSynchronize(p->events[n]);
    if (e != hipSuccess) return hip_fail(e, "event sync");
  }
  int k = 0;
  for (; k < n && k < max; ++k) {
    float ms = 0.f;
    hipError_t e = hipEventElapsedTime(&ms, p->events[k], p->events[k + 1]);
    if (e != hipSuccess) return hip_fail(e, "event elapsed");
    ms_out[k] = ms;
  }
  *count = k;
  return ZFFT_OK;
}

int zfft_process_device(zfft_plan *p, const void *d_iq, int64_t L, int32_t frames, float *d_rows,
                        void *hip_stream) {
  int rc = enter(p);
  if (rc) return rc;
  if (!d_iq || !d_rows) return fail(ZFFT_EINVAL, "null device pointer");
  hipStream_t st = pick_stream(p, hip_stream);
  rc = use_stream(p, st);
  if (rc) return rc;
  p->n_marks = 0;
  rc = process_device(p, d_iq, L, frames, d_rows, st);
  if (rc) return rc;
  return done_on(p, st);
}

int zfft_process(zfft_plan *p, const void *iq, int64_t L, int32_t frames, float *rows_out) {
  int rc = enter(p);
  if (rc) return rc;
  if (!iq || !rows_out) return fail(ZFFT_EINVAL, "null host pointer");
  if (L < 1 || frames < 1) return fail(ZFFT_EINVAL, "n_samples and n_frames must be >= 1");
  const size_t frame_bytes = (size_t)L * in_elem_bytes(p->cfg.in_dtype);
  const size_t row_bytes = (size_t)frames * p->cfg.n_win * sizeof(float);
  // Batches: one for a small call; otherwise >= 2 so that the H2D copy of batch k+1 (copy
  // stream) runs while batch k is computed (plan stream).  From pinned memory both are
  // asynchronous; from pageable memory HIP stages the copy on this thread, which then copies
  // batch k+1 while the GPU computes batch k.  Every batch takes the schedule its own frame
  // count earns; a call the XA tiles would take keeps them in every batch: its batches hold at
  // least the XA threshold for this frame length (or the call is one batch), so splitting
  // never drops a large call onto a schedule that loses at its batch size.  At zoom 8 and 4
  // (PC at every batch) and zoom 2 below 512 frames a batch takes what its own frame count
  // earns: the tiles below the walk's batch (e.g. 418-frame cfg2 batches run zoom 8's tiles).
  int B = frames;
  const size_t total = (size_t)frames * frame_bytes;
  if (total >= kPipeMinBytes && frames >= 2) {
    int nb = std::max<int64_t>(2, (int64_t)((total + kPipeBatchBytes - 1) / kPipeBatchBytes));
    B = (frames + nb - 1) / nb;
    const int need = L <= kXaShortFrame ? kXaMinFramesShort : kXaMinFrames;
    if (p->path == 0 && p->K > 0 && !pc_fits(p, L, frames) && !pc4_fits(p, L, frames) &&
        !(pc2_fits(p, L, frames) && frames < kPc2TilesMaxFrames) && auto_xa(frames, L) && B < need) {
      nb = std::max(1, frames / need);
      B = (frames + nb - 1) / nb;
    }
  }
  const int nb = (frames + B - 1) / B;
  hipError_t e = p->in.ensure((size_t)B * frame_bytes);
  if (e == hipSuccess && nb > 1) e = p->in2.ensure((size_t)B * frame_bytes);
  if (e == hipSuccess) e = p->rows.ensure(row_bytes);
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "staging allocation failed");
  rc = use_stream(p, p->stream);
  if (rc == ZFFT_OK && nb > 1) rc = use_stream(p, p->copy_st);
  if (rc) return rc;
  const char *src = (const char *)iq;
  p->n_marks = 0;  // timings cover every batch of this call
  mark(p, p->stream, "start");
  for (int k = 0; k < nb; ++k) {
    const int f0 = k * B, nk = std::min(B, frames - f0), buf = k & 1;
    void *dst = buf ? p->in2.p : p->in.p;
    hipStream_t cs = nb > 1 ? p->copy_st : p->stream;
    if (k >= 2) e = hipStreamWaitEvent(cs, p->comp_ev[buf], 0);  // batch k-2 done with dst
    if (e == hipSuccess) e = hipMemcpyAsync(dst, src + (size_t)f0 * frame_bytes, (size_t)nk * frame_bytes,
                                            hipMemcpyHostToDevice, cs);
    if (e == hipSuccess && nb > 1) e = hipEventRecord(p->h2d_ev[buf], cs);
    if (e == hipSuccess && nb > 1) e = hipStreamWaitEvent(p->stream, p->h2d_ev[buf], 0);
    if (e != hipSuccess) return hip_fail(e, "H2D copy");
    if (k > 0) mark(p, p->stream, "batch_wait");
    p->lo_first = f0;  // batch frame 0 is call frame f0 (its LO row, config 4)
    rc = process_device(p, dst, L, nk, p->rows.as<float>() + (int64_t)f0 * p->cfg.n_win, p->stream);
    p->lo_first = 0;
    if (rc) return rc;
    if (nb > 1 && (e = hipEventRecord(p->comp_ev[buf], p->stream)) != hipSuccess)
      return hip_fail(e, "event record");
  }
  e = hipMemcpyAsync(rows_out, p->rows.p, row_bytes, hipMemcpyDeviceToHost, p->stream);
  if (e != hipSuccess) return hip_fail(e, "D2H copy");
  rc = done_on(p, p->stream);
  if (rc) return rc;
  e = hipStreamSynchronize(p->stream);
  return e == hipSuccess ? ZFFT_OK : hip_fail(e, "sync");
}

int zfft_decimate(zfft_plan *p, const void *iq, int64_t L, void *out_iq, int64_t *out_len) {
  int rc = enter(p);
  if (rc) return rc;
  if (!iq || !out_iq) return fail(ZFFT_EINVAL, "null host pointer");
  std::vector<int64_t> n;
  rc = check_lengths(p, L, 1, n);
  if (rc) return rc;
  const size_t in_bytes = (size_t)L * in_elem_bytes(p->cfg.in_dtype);
  rc = ensure_lo(p, L);  // (a table upload waits for the plan's earlier work)
  if (rc) return rc;
  hipError_t e = p->in.ensure(in_bytes);
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "staging allocation failed");
  rc = use_stream(p, p->stream);
  if (rc) return rc;
  e = hipMemcpyAsync(p->in.p, iq, in_bytes, hipMemcpyHostToDevice, p->stream);
  if (e != hipSuccess) return hip_fail(e, "H2D copy");
  p->n_marks = 0;  // timings of this call's launches (the first one was unnamed before)
  mark(p, p->stream, "start");
  const float2 *x;
  if (p->K == 0) {  // zoomfft(x, 1) still mixes (S:2093-2094)
    e = p->dec.ensure((size_t)L * sizeof(float2));
    if (e != hipSuccess) return fail(ZFFT_ENOMEM, "allocation failed");
    e = launch_ingest(input_of(p, p->in.p, L), p->lo.as<float2>(), p->dec.as<float2>(), 1,
                      p->stream);
    if (e != hipSuccess) return hip_fail(e, "mix launch");
    x = p->dec.as<float2>();
  } else {
    rc = run_decimator(p, input_of(p, p->in.p, L), L, 1, n, &x, p->stream);
    if (rc) return rc;
  }
  const int64_t m = n[p->K];
  e = hipMemcpyAsync(out_iq, x, (size_t)m * sizeof(float2), hipMemcpyDeviceToHost, p->stream);
  if (e != hipSuccess) return hip_fail(e, "D2H copy");
  rc = done_on(p, p->stream);
  if (rc) return rc;
  e = hipStreamSynchronize(p->stream);
  if (e != hipSuccess) return hip_fail(e, "sync");
  if (out_len) *out_len = m;
  return ZFFT_OK;
}

int zfft_waterfall_shape(const zfft_plan *p, int32_t *rows, int32_t *cols) {
  if (!p || !rows || !cols) return fail(ZFFT_EINVAL, "null argument");
  *rows = p->cfg.n_win / 4;
  *cols = p->cfg.n_win;
  return ZFFT_OK;
}

int zfft_waterfall_reset(zfft_plan *p, int32_t scroll) {
  int rc = enter(p);
  if (rc) return rc;
  if (scroll != 1 && scroll != -1) return fail(ZFFT_EINVAL, "scroll must be +1 or -1");
  p->cfg.scroll = scroll;
  p->wf_ready = false;  // init_image on the next push / read (S:2074-2077)
  return ensure_waterfall(p);
}

int zfft_waterfall_push_device(zfft_plan *p, const float *d_rows, int32_t count,
                               void *hip_stream) {
  int rc = enter(p);
  if (rc) return rc;
  if (!d_rows || count < 1) return fail(ZFFT_EINVAL, "bad rows / count");
  rc = ensure_waterfall(p);
  if (rc) return rc;
  hipStream_t st = pick_stream(p, hip_stream);
  rc = use_stream(p, st);  // after the ring init and the rows' producer, on any stream
  if (rc) return rc;
  hipError_t e = launch_waterfall_push(p->ring.as<float>(), p->H, p->W, d_rows, p->W, count,
                                       p->off, p->cfg.scroll, st);
  if (e != hipSuccess) return hip_fail(e, "waterfall push");
  p->off = ((p->off + (int64_t)count * p->cfg.scroll) % p->H + p->H) % p->H;
  return done_on(p, st);
}

int zfft_waterfall_push(zfft_plan *p, const float *row) {
  int rc = enter(p);
  if (rc) return rc;
  rc = ensure_waterfall(p);
  if (rc) return rc;
  const float *src = p->last_row;
  if (row) {
    rc = use_stream(p, p->stream);  // one_row may still be read by the previous push
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(p->one_row.p, row, (size_t)p->W * sizeof(float),
                                  hipMemcpyHostToDevice, p->stream);
    if (e != hipSuccess) return hip_fail(e, "H2D row");
    src = p->one_row.as<float>();
  }
  if (!src) return fail(ZFFT_EINVAL, "no row given and no frame processed yet");
  if (!row && row_length(p) < p->W)  // columns >= row_length were never written
    return fail(ZFFT_EINVAL, "the plan's rows are shorter than n_win (odd n_win, or the one-sided "
                             "real-input crop): img_array[-1:] = psd raises in the reference "
                             "(S:1640); push a full-width row instead");
  rc = zfft_waterfall_push_device(p, src, 1, p->stream);
  if (rc) return rc;
  hipError_t e = hipStreamSynchronize(p->stream);
  return e == hipSuccess ? ZFFT_OK : hip_fail(e, "sync");
}

int zfft_waterfall_read(zfft_plan *p, float *img_out) {
  int rc = enter(p);
  if (rc) return rc;
  if (!img_out) return fail(ZFFT_EINVAL, "null output");
  rc = ensure_waterfall(p);
  if (rc) return rc;
  rc = use_stream(p, p->stream);
  if (rc) return rc;
  hipError_t e = launch_waterfall_read(p->ring.as<float>(), p->H, p->W, p->off, p->img.as<float>(),
                                       p->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(img_out, p->img.p, (size_t)p->H * p->W * sizeof(float),
                       hipMemcpyDeviceToHost, p->stream);
  if (e == hipSuccess) e = done_on(p, p->stream) == ZFFT_OK ? hipSuccess : hipErrorUnknown;
  if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
  return e == hipSuccess ? ZFFT_OK : hip_fail(e, "waterfall read");
}

int zfft_colormap_lut(const char *name, uint8_t *lut_rgba) {
  if (!lut_rgba) return fail(ZFFT_EINVAL, "null output");
  build_lut(name, lut_rgba);
  return ZFFT_OK;
}

int zfft_waterfall_colormap(zfft_plan *p, const char *name) {
  int rc = enter(p);
  if (rc) return rc;
  p->cmap = name ? name : "Default";
  p->lut_ready = p->lut_uploaded = false;
  return ZFFT_OK;
}

int zfft_waterfall_levels(zfft_plan *p, double minlev, double maxlev) {
  int rc = enter(p);
  if (rc) return rc;
  if (!std::isfinite(minlev) || !std::isfinite(maxlev)) return fail(ZFFT_EINVAL, "levels must be finite");
  p->lev_lo = minlev;
  p->lev_hi = maxlev;
  return ZFFT_OK;
}

int zfft_waterfall_get_levels(const zfft_plan *p, double *minlev, double *maxlev) {
  if (!p || !minlev || !maxlev) return fail(ZFFT_EINVAL, "null argument");
  *minlev = p->lev_lo;
  *maxlev = p->lev_hi;
  return ZFFT_OK;
}

namespace {
// The colormap LUT on the device (built and uploaded on first use, on st) and makeARGB's
// levels (pyqtgraph functions.py): equal levels -> max = nextafter(max, 2 max); scale = lut
// size / (max - min) (1 when the range is 0)
int render_setup(zfft_plan *p, hipStream_t st, double *lo, double *scale) {
  if (!p->lut_ready) {
    build_lut(p->cmap.c_str(), p->lut);
    p->lut_ready = true;
  }
  if (!p->lut_uploaded) {
    hipError_t e = p->lut_d.ensure(sizeof(p->lut));
    if (e == hipSuccess) e = hipMemcpyAsync(p->lut_d.p, p->lut, sizeof(p->lut), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return hip_fail(e, "LUT upload");
    p->lut_uploaded = true;
  }
  double l = p->lev_lo, h = p->lev_hi;
  if (l == h) h = std::nextafter(h, 2.0 * h);
  double rng = h - l;
  if (rng == 0.0) rng = 1.0;
  *lo = l;
  *scale = 256.0 / rng;
  return ZFFT_OK;
}

// zfft_waterfall_push_render / _push_read64: count host rows pushed, then the image emitted
// (RGBA8 or float64) and copied to the host -- one kernel for the per-line case, one copy, one
// wait.  The rows are staged in page-locked memory the kernels read in place.
constexpr size_t kDisplayZeroCopyMax = (size_t)4 << 20;
int push_emit(zfft_plan *p, const float *rows, int32_t count, bool f64, void *host_out) {
  int rc = enter(p);
  if (rc) return rc;
  if (!host_out) return fail(ZFFT_EINVAL, "null output");
  if (count < 0 || (count > 0 && !rows)) return fail(ZFFT_EINVAL, "bad rows / count");
  rc = ensure_waterfall(p);
  if (rc) return rc;
  const int H = p->H, W = p->W;
  const size_t npx = (size_t)H * W, bytes = npx * (f64 ? sizeof(double) : 4);
  hipError_t e = f64 ? p->img64.ensure(bytes) : p->rgba.ensure(bytes);
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "image buffer allocation failed");
  const float *drows = nullptr;
  if (count > 0) {
    const size_t rb = (size_t)count * W * sizeof(float);
    if (rb > p->row_pin_cap) {
      if (p->row_pin) (void)hipHostFree(p->row_pin);
      p->row_pin = nullptr;
      p->row_pin_cap = 0;
      e = hipHostMalloc((void **)&p->row_pin, rb, hipHostMallocDefault);
      if (e != hipSuccess) return fail(ZFFT_ENOMEM, "page-locked row staging allocation failed");
      p->row_pin_cap = rb;
    }
    // every display call waits for its kernels before returning: no kernel still reads row_pin
    std::memcpy(p->row_pin, rows, rb);
    void *d = nullptr;
    e = hipHostGetDevicePointer(&d, p->row_pin, 0);
    if (e != hipSuccess) return hip_fail(e, "hipHostGetDevicePointer");
    drows = (const float *)d;
  }
  rc = use_stream(p, p->stream);
  if (rc) return rc;
  double lo = 0.0, scale = 1.0;
  if (!f64) {
    rc = render_setup(p, p->stream, &lo, &scale);
    if (rc) return rc;
  }
  // a small image into page-locked host memory is written by the kernel in place (no copy
  // command: the UI's widths, W <= 1024, are 64 KB .. 1 MB per image); a large one goes through
  // the device buffer and one DMA copy (at W = 8192 the 67 MB RGBA image copies faster so)
  void *dout = f64 ? p->img64.p : p->rgba.p;
  void *hout = nullptr;
  if (bytes <= kDisplayZeroCopyMax && hipHostGetDevicePointer(&hout, host_out, 0) == hipSuccess && hout)
    dout = hout;
  else
    (void)hipGetLastError(), hout = nullptr;
  if (count > 1) {  // the batch through the push kernels, then the image
    e = launch_waterfall_push(p->ring.as<float>(), H, W, drows, W, count, p->off, p->cfg.scroll, p->stream);
    if (e != hipSuccess) return hip_fail(e, "waterfall push");
    p->off = ((p->off + (int64_t)count * p->cfg.scroll) % H + H) % H;
    drows = nullptr;
  }
  e = launch_waterfall_push_emit(p->ring.as<float>(), H, W, p->off, p->cfg.scroll, drows, p->lut_d.p, lo,
                                 scale, dout, f64, p->stream);
  if (e != hipSuccess) return hip_fail(e, "waterfall push + emit");
  if (drows) p->off = ((p->off + p->cfg.scroll) % H + H) % H;
  if (!hout) e = hipMemcpyAsync(host_out, dout, bytes, hipMemcpyDeviceToHost, p->stream);
  if (e == hipSuccess) e = done_on(p, p->stream) == ZFFT_OK ? hipSuccess : hipErrorUnknown;
  if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
  return e == hipSuccess ? ZFFT_OK : hip_fail(e, "waterfall image copy");
}
}  // namespace

int zfft_waterfall_push_render(zfft_plan *p, const float *rows, int32_t count, uint8_t *rgba_out) {
  return push_emit(p, rows, count, false, rgba_out);
}

int zfft_waterfall_push_read64(zfft_plan *p, const float *rows, int32_t count, double *img_out) {
  return push_emit(p, rows, count, true, img_out);
}

int zfft_waterfall_render_device(zfft_plan *p, uint8_t *d_rgba, void *hip_stream) {
  int rc = enter(p);
  if (rc) return rc;
  if (!d_rgba) return fail(ZFFT_EINVAL, "null output");
  rc = ensure_waterfall(p);
  if (rc) return rc;
  hipStream_t st = pick_stream(p, hip_stream);
  rc = use_stream(p, st);
  if (rc) return rc;
  double lo, scale;
  rc = render_setup(p, st, &lo, &scale);
  if (rc) return rc;
  hipError_t e = launch_waterfall_render(p->ring.as<float>(), p->H, p->W, p->off, p->lut_d.p, lo, scale,
                                         d_rgba, st);
  if (e != hipSuccess) return hip_fail(e, "waterfall render");
  return done_on(p, st);
}

int zfft_waterfall_render(zfft_plan *p, uint8_t *rgba_out) {
  int rc = enter(p);
  if (rc) return rc;
  if (!rgba_out) return fail(ZFFT_EINVAL, "null output");
  rc = ensure_waterfall(p);
  if (rc) return rc;
  const size_t bytes = (size_t)p->H * p->W * 4;
  hipError_t e = p->rgba.ensure(bytes);
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "render buffer allocation failed");
  rc = zfft_waterfall_render_device(p, p->rgba.as<uint8_t>(), p->stream);
  if (rc) return rc;
  e = hipMemcpyAsync(rgba_out, p->rgba.p, bytes, hipMemcpyDeviceToHost, p->stream);
  if (e == hipSuccess) e = done_on(p, p->stream) == ZFFT_OK ? hipSuccess : hipErrorUnknown;
  if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
  return e == hipSuccess ? ZFFT_OK : hip_fail(e, "render copy");
}

int zfft_host_alloc(size_t bytes, void **out) {
  if (!out || bytes == 0) return fail(ZFFT_EINVAL, "zfft_host_alloc: null output or zero size");
  *out = nullptr;
  hipError_t e = hipHostMalloc(out, bytes, hipHostMallocDefault);
  if (e != hipSuccess) {
    *out = nullptr;
    return fail(ZFFT_ENOMEM, "page-locked host allocation failed");
  }
  return ZFFT_OK;
}

int zfft_host_free(void *ptr) {
  if (!ptr) return ZFFT_OK;
  hipError_t e = hipHostFree(ptr);
  return e == hipSuccess ? ZFFT_OK : hip_fail(e, "hipHostFree");
}

int zfft_waterfall_autolevel(zfft_plan *p, double *minlev, double *maxlev) {
  int rc = enter(p);
  if (rc) return rc;
  rc = ensure_waterfall(p);
  if (rc) return rc;
  const int64_t n = (int64_t)p->H * p->W;
  hipError_t e = p->al_hist.ensure(4 * 65536 * sizeof(unsigned));
  if (e == hipSuccess) e = p->al_bins.ensure(4 * sizeof(unsigned));
  if (e != hipSuccess) return fail(ZFFT_ENOMEM, "autolevel workspace allocation failed");
  // pass 1: counts per top-16-bit key of the pixels < 0
  std::vector<unsigned> h1(65536);
  rc = use_stream(p, p->stream);
  if (rc) return rc;
  e = hipMemsetAsync(p->al_hist.p, 0, 65536 * sizeof(unsigned), p->stream);
  if (e == hipSuccess) e = launch_autolevel_hist_hi(p->ring.as<float>(), n, p->al_hist.as<unsigned>(), p->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(h1.data(), p->al_hist.p, 65536 * sizeof(unsigned), hipMemcpyDeviceToHost, p->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
  if (e != hipSuccess) return hip_fail(e, "autolevel pass 1");
  int64_t cnt = 0;
  for (unsigned c : h1) cnt += c;
  if (cnt == 0) return fail(ZFFT_EINVAL, "autolevel: no pixel below 0");  // np.percentile of an empty array raises
  // numpy percentile, method 'linear': virtual index (n-1) q, q = p/100; the order
  // statistics at floor and floor+1 (clipped to n-1)
  const double qs[2] = {2.0 / 100.0, 98.0 / 100.0};
  double vi[2];
  int64_t ranks[4];
  for (int k = 0; k < 2; ++k) {
    vi[k] = (double)(cnt - 1) * qs[k];
    const int64_t prev = (int64_t)std::floor(vi[k]);
    ranks[2 * k] = std::min<int64_t>(std::max<int64_t>(prev, 0), cnt - 1);
    ranks[2 * k + 1] = std::min<int64_t>(std::max<int64_t>(prev + 1, 0), cnt - 1);
  }
  // the top bin and the rank inside it of each wanted rank
  unsigned bin_of[4];
  int64_t within[4];
  for (int r = 0; r < 4; ++r) {
    int64_t acc = 0;
    unsigned b = 0;
    while (acc + h1[b] <= ranks[r]) acc += h1[b++];
    bin_of[r] = b;
    within[r] = ranks[r] - acc;
  }
  unsigned bins[4];
  int nb = 0, slot[4];
  for (int r = 0; r < 4; ++r) {
    int j = 0;
    while (j < nb && bins[j] != bin_of[r]) ++j;
    if (j == nb) bins[nb++] = bin_of[r];
    slot[r] = j;
  }
  std::vector<unsigned> h2((size_t)nb * 65536);
  e = hipMemcpyAsync(p->al_bins.p, bins, nb * sizeof(unsigned), hipMemcpyHostToDevice, p->stream);
  if (e == hipSuccess) e = hipMemsetAsync(p->al_hist.p, 0, (size_t)nb * 65536 * sizeof(unsigned), p->stream);
  if (e == hipSuccess)
    e = launch_autolevel_hist_lo(p->ring.as<float>(), n, p->al_bins.as<unsigned>(), nb, p->al_hist.as<unsigned>(), p->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(h2.data(), p->al_hist.p, (size_t)nb * 65536 * sizeof(unsigned), hipMemcpyDeviceToHost, p->stream);
  if (e == hipSuccess) e = done_on(p, p->stream) == ZFFT_OK ? hipSuccess : hipErrorUnknown;
  if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
  if (e != hipSuccess) return hip_fail(e, "autolevel pass 2");
  double val[4];
  for (int r = 0; r < 4; ++r) {
    const unsigned *hb = h2.data() + (size_t)slot[r] * 65536;
    int64_t acc = 0;
    unsigned lo16 = 0;
    while (acc + hb[lo16] <= within[r]) acc += hb[lo16++];
    const uint32_t key = (bin_of[r] << 16) | lo16;
    uint32_t bits = ~key;  // neg_key inverse
    float f;
    std::memcpy(&f, &bits, 4);
    val[r] = (double)f;
  }
  // numpy _lerp(a, b, t): a + (b - a) t, or b - (b - a)(1 - t) when t >= 0.5
  double lev[2];
  for (int k = 0; k < 2; ++k) {
    const double a = val[2 * k], b = val[2 * k + 1];
    const double t = vi[k] - std::floor(vi[k]);
    const double d = b - a;
    lev[k] = t >= 0.5 ? b - d * (1.0 - t) : a + d * t;
  }
  p->lev_lo = lev[0];
  p->lev_hi = lev[1];
  if (minlev) *minlev = lev[0];
  if (maxlev) *maxlev = lev[1];
  return ZFFT_OK;
}

}  // extern "C"
