// pc_tables.cpp -- host-side tables of the "PC" decimator (pc_kernels.hip): the polyphase
// FIR taps, the all-pole sections left at their own rate and at the output rate with their
// lane-scan tables, and the frame-end maps.  Design model and derivation: tools/pc_model.py,
// tools/pc_proto.py; DESIGN.md §3.5.
//
// The reference decimates with log2(zoom) x scipy.signal.decimate(x, 2)
// (pypanadapter_spectrum.py:2096-2098): cheby1(8, 0.05, 0.4) as 4 SOS, sosfiltfilt (odd
// extension 27, sosfilt_zi states), [::2].  With H = N(z) / D(z), the interior of three
// stages is the LTI filter G(z) = prod_k |H(z^(2^k))|^2 followed by [::8].  Every all-pole
// factor 1 / D_s(z^(2^k)) can be moved to a lower rate with
//   1 / D(z) = D(-z) D2(-z^2) D4(-z^4) ... / D_(2^j)(z^(2^j)),  D_2(z^2) = D(z) D(-z),
// whose numerator factors in z, z^2, z^4 join the FIR of the stage at that rate.  Stages 0
// and 1 move all their poles to the output rate (radius <= .765 there); stage 2 keeps its
// two slowest sections at its own rate (moving them amplified fp32 rounding 5-500x) and
// moves the other two by one rate.  The frame ends differ from this LTI model only by a
// linear map of the first / last input samples onto the first / last ~150 outputs, computed
// here (exact cascade minus model, on impulses) and stored as a rank <= 16 factorisation.
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstring>
#include <system_error>
#include <thread>
#include <vector>

#include "cheby1_q2.h"
#include "pc_edge_maps.h"
#include "zfft_internal.h"

namespace zfft {
namespace {

typedef std::vector<double> Poly;  // coefficients of z^0, z^-1, ...

Poly conv(const Poly &a, const Poly &b) {
  Poly r(a.size() + b.size() - 1, 0.0);
  for (size_t i = 0; i < a.size(); ++i)
    for (size_t j = 0; j < b.size(); ++j) r[i + j] += a[i] * b[j];
  return r;
}
Poly neg(Poly p) {  // p(z) -> p(-z)
  for (size_t i = 1; i < p.size(); i += 2) p[i] = -p[i];
  return p;
}

struct Secs {
  double a1[4], a2[4];
};
// the sections of D_(2^(j+1)) from those of D_(2^j): poles squared
Secs square(const Secs &s) {
  Secs r;
  for (int k = 0; k < 4; ++k) {
    r.a1[k] = 2.0 * s.a2[k] - s.a1[k] * s.a1[k];
    r.a2[k] = s.a2[k] * s.a2[k];
  }
  return r;
}
Poly sec_poly(const Secs &s, std::initializer_list<int> idx) {
  Poly p{1.0};
  for (int k : idx) p = conv(p, Poly{1.0, s.a1[k], s.a2[k]});
  return p;
}

struct Lev {
  Secs d[4];  // D, D2, D4, D8
  Poly n9;
};
const Lev &levels() {
  static const Lev L = [] {
    Lev l;
    for (int k = 0; k < 4; ++k) {
      l.d[0].a1[k] = kDecimSos[k][4];
      l.d[0].a2[k] = kDecimSos[k][5];
    }
    for (int j = 1; j < 4; ++j) l.d[j] = square(l.d[j - 1]);
    l.n9.resize(9);
    for (int i = 0; i < 9; ++i) {
      double bin = 1.0;
      for (int r = 0; r < i; ++r) bin = bin * (8 - r) / (r + 1);
      l.n9[i] = kDecimSos[0][0] * bin;  // N = b0 (1 + z^-1)^8 (sections 1..3 are [1, 2, 1])
    }
    return l;
  }();
  return L;
}

Poly zero_phase(const Poly &f) {
  Poly r(f.rbegin(), f.rend());
  return conv(f, r);
}

typedef double M2[2][2];
void mul2(const M2 a, const M2 b, M2 out) {
  M2 t;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) t[i][j] = a[i][0] * b[0][j] + a[i][1] * b[1][j];
  std::memcpy(out, t, sizeof(t));
}
void pow2(const M2 a, int p, M2 out) {
  M2 r = {{1, 0}, {0, 1}}, b;
  std::memcpy(b, a, sizeof(b));
  for (; p > 0; p >>= 1) {
    if (p & 1) mul2(r, b, r);
    mul2(b, b, b);
  }
  std::memcpy(out, r, sizeof(r));
}

// Tables of one section for lane blocks of B; false when the kernel's compiled scan depth or
// correction length would not reach 1e-9 / 1e-10.
bool sec_tables(double a1, double a2, int B, int levels, int dcut, PcSec &s) {
  s.a1 = (float)a1;
  s.a2 = (float)a2;
  s.pad_[0] = s.pad_[1] = 0.f;
  const M2 A = {{-a1, -a2}, {1.0, 0.0}};
  for (int d = 0; d < 5; ++d) {
    M2 P;
    pow2(A, B << d, P);
    for (int i = 0; i < 4; ++i) s.pw[d][i] = (float)P[i / 2][i % 2];
  }
  // reach: lanes whose exit state still matters, |lambda|^(B reach) < 1e-9
  const double r = std::sqrt(std::max(a2, 0.0));
  int reach = 1;
  while (std::pow(r, (double)B * reach) > 1e-9) ++reach;
  const int need_levels = reach > 1 ? (int)std::ceil(std::log2((double)reach)) : 0;
  if (need_levels > levels) return false;
  double mx = 0, row[kPcCt][2];
  M2 P = {{-a1, -a2}, {1.0, 0.0}};
  for (int t = 0; t < kPcCt; ++t) {
    row[t][0] = P[0][0];
    row[t][1] = P[0][1];
    mx = std::max(mx, std::max(std::fabs(P[0][0]), std::fabs(P[0][1])));
    mul2(A, P, P);
  }
  int last = 0;
  for (int t = 0; t < kPcCt; ++t) {
    if (t < B && std::max(std::fabs(row[t][0]), std::fabs(row[t][1])) > 1e-10 * mx) last = t + 1;
    s.ct[t][0] = (float)row[t][0];
    s.ct[t][1] = (float)row[t][1];
  }
  return last <= dcut;
}

// ---- frame-end maps ----

// scipy.signal.sosfiltfilt(sos, x)[::2] for cheby1(8, .05, .4) (padlen 27, sosfilt_zi
// states; _signaltools.py:4718-4828), fp64, real input.
void exact_stage(const std::vector<double> &x, std::vector<double> &out) {
  const int n = (int)x.size(), P = kPad, e = n + 2 * P;
  std::vector<double> ext(e), f(e);
  for (int i = 0; i < P; ++i) ext[i] = 2 * x[0] - x[P - i];
  for (int i = 0; i < n; ++i) ext[P + i] = x[i];
  for (int k = 0; k < P; ++k) ext[P + n + k] = 2 * x[n - 1] - x[n - 2 - k];
  auto pass = [](const double *in, double *o, int len, int dir) {
    // sosfilt with zi * in[first] (transposed direct form II), in order dir
    double z[4][2];
    const double u0 = in[dir > 0 ? 0 : len - 1];
    for (int k = 0; k < 4; ++k) z[k][0] = kDecimZi[k][0] * u0, z[k][1] = kDecimZi[k][1] * u0;
    for (int c = 0; c < len; ++c) {
      const int i = dir > 0 ? c : len - 1 - c;
      double u = in[i];
      for (int k = 0; k < 4; ++k) {
        const double *b = kDecimSos[k];
        const double y = b[0] * u + z[k][0];
        z[k][0] = b[1] * u - b[4] * y + z[k][1];
        z[k][1] = b[2] * u - b[5] * y;
        u = y;
      }
      o[i] = u;
    }
  };
  pass(ext.data(), f.data(), e, +1);
  pass(f.data(), ext.data(), e, -1);
  out.resize((n + 1) / 2);
  for (int j = 0; j < (int)out.size(); ++j) out[j] = ext[P + 2 * j];
}

void exact_k(std::vector<double> x, int K, std::vector<double> &out) {  // decimate(., 2)^K
  for (int k = 0; k < K; ++k) {
    exact_stage(x, out);
    x.swap(out);
  }
  out.swap(x);
}

void fft_inplace(std::vector<std::complex<double>> &a, bool inverse) {
  const size_t n = a.size();
  for (size_t i = 1, j = 0; i < n; ++i) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j |= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
  for (size_t len = 2; len <= n; len <<= 1) {
    const double ang = (inverse ? 2.0 : -2.0) * M_PI / (double)len;
    for (size_t i = 0; i < n; i += len)
      for (size_t k = 0; k < len / 2; ++k) {
        const std::complex<double> w(std::cos(ang * (double)k), std::sin(ang * (double)k));
        const std::complex<double> u = a[i + k], v = a[i + k + len / 2] * w;
        a[i + k] = u + v;
        a[i + k + len / 2] = u - v;
      }
  }
}

// Impulse response of the LTI model G(z) = prod_(k < K) |H(z^(2^k))|^2 at the input rate,
// h[n] for |n| < kHz (the model output m is sum_n h[2^K m - n] x[n]).
constexpr int kHzFft = 1 << 16, kHz = 1 << 15;
std::vector<double> model_hz_build(int K) {
  {
    std::vector<std::complex<double>> g(kHzFft);
    for (int k = 0; k < kHzFft; ++k) {
      const double w = 2.0 * M_PI * k / kHzFft;
      double G = 1.0;
      for (int s = 0; s < K; ++s) {
        const double ws = w * (double)(1 << s);
        std::complex<double> h(1.0, 0.0);
        const std::complex<double> e1 = std::polar(1.0, -ws), e2 = std::polar(1.0, -2 * ws);
        for (int q = 0; q < 4; ++q) {
          const double *b = kDecimSos[q];
          h *= (b[0] + b[1] * e1 + b[2] * e2) / (1.0 + b[4] * e1 + b[5] * e2);
        }
        G *= std::norm(h);
      }
      g[k] = G;
    }
    fft_inplace(g, true);
    std::vector<double> h(2 * kHz + 1);
    for (int n = -kHz; n <= kHz; ++n) h[n + kHz] = g[(n + kHzFft) % kHzFft].real() / kHzFft;
    return h;
  }
}
const std::vector<double> &model_hz(int K) {
  static const std::vector<double> H1 = model_hz_build(1), H2 = model_hz_build(2), H3 = model_hz_build(3);
  return K == 1 ? H1 : K == 2 ? H2 : H3;
}

// C[m][j] = (exact - model)(e_j) at output m of K stages; side 0 from the frame start, side 1
// from the frame end (frame length = lmod mod 2^K).
void edge_matrix(int K, int side, int lmod, int R, int J, std::vector<double> &C) {
  const int Lc = 4096 + lmod;
  int n3 = Lc;
  for (int k = 0; k < K; ++k) n3 = (n3 + 1) / 2;
  const std::vector<double> &hz = model_hz(K);
  C.assign((size_t)R * J, 0.0);
  const int nt = std::max(1, std::min<int>(8, (int)std::thread::hardware_concurrency()));
  auto work = [&](int w) {
    std::vector<double> x(Lc), out;
    for (int j = w; j < J; j += nt) {
      const int pos = side == 0 ? j : Lc - 1 - j;
      std::fill(x.begin(), x.end(), 0.0);
      x[pos] = 1.0;
      exact_k(x, K, out);
      for (int m = 0; m < R; ++m) {
        const int mo = side == 0 ? m : n3 - 1 - m;
        const long n = (1L << K) * mo - pos;
        const double model = (n >= -kHz && n <= kHz) ? hz[n + kHz] : 0.0;
        C[(size_t)m * J + j] = out[mo] - model;
      }
    }
  };
  std::vector<std::thread> pool;
  for (int w = 0; w < nt; ++w) {
    try {
      pool.emplace_back(work, w);
    } catch (const std::system_error &) {  // no thread: this share on the calling thread
      work(w);
    }
  }
  for (auto &t : pool) t.join();
}

}  // namespace

int64_t pc_y2_len(int64_t L) {
  const int64_t m_hi = (L + 15) / 2;
  return (m_hi + 24) / 2 + 1 - kPcQ0;
}

int64_t pc4_y1_len(int64_t L) { return (L + 15) / 2 + 1 - kPc4Q0; }

bool pc_build_tables(PcTab &tab) {
  std::memset(&tab, 0, sizeof(tab));
  const Lev &l = levels();
  const Poly f0 = conv(l.n9, neg(sec_poly(l.d[0], {0, 1, 2, 3})));
  const Poly f1 = conv(conv(l.n9, neg(sec_poly(l.d[1], {0, 1, 2, 3}))), neg(sec_poly(l.d[0], {0, 1, 2, 3})));
  const Poly f2 = conv(conv(conv(l.n9, neg(sec_poly(l.d[2], {0, 1, 2, 3}))),
                            neg(sec_poly(l.d[1], {0, 1, 2, 3}))),
                       neg(sec_poly(l.d[0], {0, 1})));
  const Poly g0 = zero_phase(f0), g1 = zero_phase(f1), g2 = zero_phase(f2);
  if ((int)g0.size() != kPcG0 || (int)g1.size() != kPcG1 || (int)g2.size() != kPcG2) return false;
  for (int i = 0; i < kPcG0; ++i) tab.g0[i] = (float)g0[i];
  for (int i = 0; i < kPcG1; ++i) tab.g1[i] = (float)g1[i];
  for (int i = 0; i < kPcG2; ++i) tab.g2[i] = (float)g2[i];
  // own-rate sections: stage 2's sections 2 and 3 (radius .808, .935), in that order
  const int own_idx[kPcOwn] = {2, 3};
  for (int s = 0; s < kPcOwn; ++s) {
    const double a1 = l.d[0].a1[own_idx[s]], a2 = l.d[0].a2[own_idx[s]];
    if (!sec_tables(a1, a2, kPcOwnBlk, pc_own_levels(s), kPcOwnBlk, tab.own[s]) ||
        !sec_tables(a1, a2, kPcWf, pc_wf_levels(s), kPcWf, tab.wf[s]) ||
        !sec_tables(a1, a2, kPcWb, pc_wb_levels(s), kPcWb, tab.wb[s]))
      return false;
    const M2 A = {{-a1, -a2}, {1.0, 0.0}};
    auto cross = [&](int B, float (*x)[4]) {
      for (int i = 0; i < 64; ++i) {
        M2 P;
        pow2(A, B * (i + 1), P);
        for (int q = 0; q < 4; ++q) x[i][q] = (float)P[q / 2][q % 2];
      }
    };
    cross(kPcOwnBlk, tab.own_x[s]);
    cross(kPcWf, tab.wf_x[s]);
    cross(kPcWb, tab.wb_x[s]);
  }
  // output-rate sections: D8 (stage 0), D4 (stage 1), D2 sections 0, 1 (stage 2), slowest
  // first
  std::vector<std::pair<double, double>> ap;
  for (int k = 0; k < 4; ++k) ap.emplace_back(l.d[3].a1[k], l.d[3].a2[k]);
  for (int k = 0; k < 4; ++k) ap.emplace_back(l.d[2].a1[k], l.d[2].a2[k]);
  for (int k = 0; k < 2; ++k) ap.emplace_back(l.d[1].a1[k], l.d[1].a2[k]);
  std::stable_sort(ap.begin(), ap.end(), [](auto &a, auto &b) { return a.second > b.second; });
  for (int s = 0; s < kPcAp; ++s)
    if (!sec_tables(ap[s].first, ap[s].second, kPcApBlk, pc_ap_levels(s), pc_ap_dcut(s), tab.ap[s]))
      return false;
  return true;
}

bool pc_build_tables4(PcTab4 &tab) {
  std::memset(&tab, 0, sizeof(tab));
  const Lev &l = levels();
  const Poly f0 = conv(l.n9, neg(sec_poly(l.d[0], {0, 1, 2, 3})));
  const Poly f1 = conv(conv(l.n9, neg(sec_poly(l.d[1], {0, 1, 2, 3}))), neg(sec_poly(l.d[0], {0, 1})));
  const Poly g0 = zero_phase(f0), g1 = zero_phase(f1);
  if ((int)g0.size() != kPcG0 || (int)g1.size() != kPc4G1) return false;
  for (int i = 0; i < kPcG0; ++i) tab.g0[i] = (float)g0[i];
  for (int i = 0; i < kPc4G1; ++i) tab.g1[i] = (float)g1[i];
  PcTab t8;  // the own-rate sections are zoom 8's (the base filter's sections 2, 3)
  if (!pc_build_tables(t8)) return false;
  std::memcpy(tab.wf, t8.wf, sizeof(tab.wf));
  std::memcpy(tab.wb, t8.wb, sizeof(tab.wb));
  std::memcpy(tab.wf_x, t8.wf_x, sizeof(tab.wf_x));
  std::memcpy(tab.wb_x, t8.wb_x, sizeof(tab.wb_x));
  std::memcpy(tab.own, t8.own, sizeof(tab.own));
  std::memcpy(tab.own_x, t8.own_x, sizeof(tab.own_x));
  // output-rate sections: D4 (stage 0 moved twice), D2 sections 0, 1 (stage 1), slowest first
  std::vector<std::pair<double, double>> ap;
  for (int k = 0; k < 4; ++k) ap.emplace_back(l.d[2].a1[k], l.d[2].a2[k]);
  for (int k = 0; k < 2; ++k) ap.emplace_back(l.d[1].a1[k], l.d[1].a2[k]);
  std::stable_sort(ap.begin(), ap.end(), [](auto &a, auto &b) { return a.second > b.second; });
  for (int s = 0; s < kPc4Ap; ++s)
    if (!sec_tables(ap[s].first, ap[s].second, kPcApBlk, pc4_ap_levels(s), pc4_ap_dcut(s), tab.ap[s]))
      return false;
  return true;
}

bool pc_build_tables2(PcTab2 &tab) {
  std::memset(&tab, 0, sizeof(tab));
  const Lev &l = levels();
  // M(z) = N(z) N(1/z) D(-1/z): with N(1/z) and D(-1/z) written as the reversed lists of N and
  // D(-z) (entry j <-> z^(8 - j)), entry i of the product list is the power z^(16 - i)
  const Poly dneg = neg(sec_poly(l.d[0], {0, 1, 2, 3}));  // D(-z): entry k <-> z^-k
  const Poly nrev(l.n9.rbegin(), l.n9.rend());
  const Poly drev(dneg.rbegin(), dneg.rend());
  const Poly m = conv(l.n9, conv(nrev, drev));
  if ((int)m.size() != kPc2G) return false;
  for (int i = 0; i < kPc2G; ++i) tab.g[i] = (float)m[16 - (i + kPc2M0)];  // z^(i - 8)
  std::vector<std::pair<double, double>> own, ap;
  for (int k = 0; k < 4; ++k) own.emplace_back(l.d[0].a1[k], l.d[0].a2[k]), ap.emplace_back(l.d[1].a1[k], l.d[1].a2[k]);
  auto slow_first = [](auto &a, auto &b) { return a.second > b.second; };
  std::stable_sort(own.begin(), own.end(), slow_first);
  std::stable_sort(ap.begin(), ap.end(), slow_first);
  for (int s = 0; s < kPc2Own; ++s) {
    const double a1 = own[s].first, a2 = own[s].second;
    if (!sec_tables(a1, a2, kPcOwnBlk, pc2_own_levels(s), kPcOwnBlk, tab.own[s])) return false;
    const M2 A = {{-a1, -a2}, {1.0, 0.0}};
    for (int i = 0; i < 64; ++i) {
      M2 P;
      pow2(A, kPcOwnBlk * (i + 1), P);
      for (int q = 0; q < 4; ++q) tab.own_x[s][i][q] = (float)P[q / 2][q % 2];
    }
  }
  for (int s = 0; s < kPc2Ap; ++s)
    if (!sec_tables(ap[s].first, ap[s].second, kPcApBlk, pc2_ap_levels(s), pc2_ap_dcut(s), tab.ap[s]))
      return false;
  return true;
}

bool pc_edge_map(int side, int lmod8, PcEdge &out) { return pc_edge_map_k(3, side, lmod8, out); }

// ---- FC tables (fc_kernels.hip; tools/fc_model.py c_table) ----

void fc_build_twiddles(int M, float2 *tw) {
  for (int k = 0; k < M; ++k) {
    const double a = -2.0 * M_PI * k / M;
    tw[k] = make_float2((float)std::cos(a), (float)std::sin(a));
  }
}

// Zoom Z (8 or 4): g'[k] = g[k] e^(2 pi i lo_ratio k), |k| <= K (g = the zoom-Z model's input-rate
// response, model_hz(log2 Z); K = kFcK or kFc4K), placed circularly in N = kFcN; G = its DFT;
// C[k][r] = W_N^(rk) sum_(q < Z) G[k + M q] W_Z^(rq) / (N sqrt 2) for k < M = N / Z (the 1 / sqrt 2:
// the outputs take lo[Z m] as the composite lo[a] lo[b] = sqrt 2 lo[a + b]).  Stored for pass C's
// thread t (k' = (t >> 4) + 16 (t & 15), k = k' + 256 k3) as v4f pairs: float2 index
// (((Z / 2) k3 + r / 2) 256 + t) 2 + r % 2 holds C[k][r].
bool fc_build_row(int zoom, double lo_ratio, float2 *row) {
  if (zoom != 8 && zoom != 4) return false;
  const int N = kFcN, M = kFcN / zoom, K = zoom == 8 ? kFcK : kFc4K, R1 = M / 256;
  const std::vector<double> &h = model_hz(zoom == 8 ? 3 : 2);
  if ((int)h.size() < 2 * K + 1) return false;
  const int hc = ((int)h.size() - 1) / 2;
  std::vector<std::complex<double>> g(N, 0.0);
  for (int k = -K; k <= K; ++k) {
    const double turns = std::fmod(lo_ratio * (double)k, 1.0);
    g[(k + N) % N] = h[hc + k] * std::polar(1.0, 2.0 * M_PI * turns);
  }
  fft_inplace(g, false);
  const double s = 1.0 / ((double)N * std::sqrt(2.0));
  for (int t = 0; t < 256; ++t) {
    const int kp = (t >> 4) + 16 * (t & 15);
    for (int k3 = 0; k3 < R1; ++k3) {
      const int k = kp + 256 * k3;
      for (int r = 0; r < zoom; ++r) {
        std::complex<double> c = 0.0;
        for (int q = 0; q < zoom; ++q) c += g[k + M * q] * std::polar(1.0, -2.0 * M_PI * ((r * q) % zoom) / zoom);
        c *= std::polar(s, -2.0 * M_PI * (double)((int64_t)r * k % N) / N);
        row[(((zoom / 2) * k3 + r / 2) * 256 + t) * 2 + (r & 1)] = make_float2((float)c.real(), (float)c.imag());
      }
    }
  }
  return true;
}

bool pc_edge_map_k(int K, int side, int lmod, PcEdge &out) {
  const int R = kPcEdgeR, J = side == 0 ? 768 : kPcEdgeJ;
  std::vector<double> C;
  edge_matrix(K, side, lmod & ((1 << K) - 1), R, J, C);
  // entries are responses to unit input samples: below kTol they cannot move an output by
  // more than ~1e-9 of the input's peak even summed over a whole edge
  constexpr double kTol = 1e-11;
  // the support must end well inside the computed block
  for (int m = 0; m < R; ++m)
    for (int j = J - 64; j < J; ++j)
      if (std::fabs(C[(size_t)m * J + j]) > kTol) return false;
  for (int m = R - 16; m < R; ++m)
    for (int j = 0; j < J; ++j)
      if (std::fabs(C[(size_t)m * J + j]) > kTol) return false;
  // rank-revealing modified Gram-Schmidt on the rows: C ~= A Q^T, Q (J x r) orthonormal
  std::vector<double> Wk(C), Q;
  std::vector<double> nrm(R);
  for (int m = 0; m < R; ++m) {
    double s = 0;
    for (int j = 0; j < J; ++j) s += Wk[(size_t)m * J + j] * Wk[(size_t)m * J + j];
    nrm[m] = std::sqrt(s);
  }
  int r = 0;
  while (true) {
    int piv = 0;
    for (int m = 1; m < R; ++m)
      if (nrm[m] > nrm[piv]) piv = m;
    if (nrm[piv] <= 10 * kTol) break;
    if (r == kPcEdgeRank) return false;
    std::vector<double> q(Wk.begin() + (size_t)piv * J, Wk.begin() + (size_t)(piv + 1) * J);
    for (int pass = 0; pass < 2; ++pass) {  // re-orthogonalise against the earlier q
      for (int k = 0; k < r; ++k) {
        double d = 0;
        for (int j = 0; j < J; ++j) d += q[j] * Q[(size_t)k * J + j];
        for (int j = 0; j < J; ++j) q[j] -= d * Q[(size_t)k * J + j];
      }
    }
    double s = 0;
    for (double v : q) s += v * v;
    s = std::sqrt(s);
    for (double &v : q) v /= s;
    Q.insert(Q.end(), q.begin(), q.end());
    ++r;
    for (int m = 0; m < R; ++m) {
      double *row = &Wk[(size_t)m * J];
      double d = 0;
      for (int j = 0; j < J; ++j) d += row[j] * q[j];
      double ss = 0;
      for (int j = 0; j < J; ++j) {
        row[j] -= d * q[j];
        ss += row[j] * row[j];
      }
      nrm[m] = std::sqrt(ss);
    }
  }
  // trim rows and columns that carry nothing
  int Rt = 0, Jt = 0;
  for (int m = 0; m < R; ++m)
    for (int j = 0; j < J; ++j)
      if (std::fabs(C[(size_t)m * J + j]) > kTol) Rt = std::max(Rt, m + 1), Jt = std::max(Jt, j + 1);
  out.R = Rt;
  out.J = Jt;
  out.r = r;
  out.U.assign((size_t)Rt * r, 0.f);
  out.V.assign((size_t)Jt * r, 0.f);
  for (int m = 0; m < Rt; ++m)
    for (int k = 0; k < r; ++k) {
      double d = 0;
      for (int j = 0; j < J; ++j) d += C[(size_t)m * J + j] * Q[(size_t)k * J + j];
      out.U[(size_t)m * r + k] = (float)d;
    }
  for (int j = 0; j < Jt; ++j)
    for (int k = 0; k < r; ++k) out.V[(size_t)j * r + k] = (float)Q[(size_t)k * J + j];
  return true;
}

}  // namespace zfft

// Test hook (not part of include/zfft.h): the PC tables, for the CPU suite.
//   what 0: FIR taps g0 | g1 | g2 (139 floats); 1: PcTab as raw floats;
//   2 / 3: left / right edge map for L mod 8 = arg built now (fp64): R, J, r then U (R x r), V (J x r);
//   4: the shipped constant map arg of pc_edge_maps.h: R, J, r then U (R x r), V^T (r x J);
//   5: zoom 4 FIR taps g0 | g1 (74 floats); 12 / 13: zoom-4 left / right map for L mod 4 = arg
//   built now; 14: the shipped zoom-4 map arg; 6: zoom 2 FIR taps M + its input-rate and
//   output-rate sections' a1, a2 (41 floats); 15 / 16: zoom-2 left / right map for L mod 2 = arg
//   built now; 17: the shipped zoom-2 map arg; 18 / 20: the FC twiddles W_M^k of zoom 8 / 4
//   (M = 1024 / 2048, as floats); 19 / 21: the FC filter row of zoom 8 / 4 for f_lo / fs =
//   arg / 2^20 (kFcRow complex as floats, kernel order).
extern "C" int zfft__pc_tables(int what, int arg, float *out, int cap) {
  using namespace zfft;
  if (what >= 18 && what <= 21) {
    const int zoom = what <= 19 ? 8 : 4;
    const bool tw = what == 18 || what == 20;
    const int n = tw ? 2 * (kFcN / zoom) : 2 * kFcRow;
    if (cap < n) return -2;
    if (tw) fc_build_twiddles(kFcN / zoom, (float2 *)out);
    else if (!fc_build_row(zoom, (double)arg / (double)(1 << 20), (float2 *)out)) return -1;
    return n;
  }
  if (what == 0 || what == 1) {
    PcTab t;
    if (!pc_build_tables(t)) return -1;
    if (what == 0) {
      const int n = kPcG0 + kPcG1 + kPcG2;
      if (cap < n) return -2;
      std::memcpy(out, t.g0, kPcG0 * 4);
      std::memcpy(out + kPcG0, t.g1, kPcG1 * 4);
      std::memcpy(out + kPcG0 + kPcG1, t.g2, kPcG2 * 4);
      return n;
    }
    const int n = (int)(sizeof(PcTab) / 4);
    if (cap < n) return -2;
    std::memcpy(out, &t, sizeof(t));
    return n;
  }
  if (what == 5) {  // zoom 4: FIR taps g0 | g1 (33 + 41 floats)
    PcTab4 t;
    if (!pc_build_tables4(t)) return -1;
    if (cap < kPcG0 + kPc4G1) return -2;
    std::memcpy(out, t.g0, kPcG0 * 4);
    std::memcpy(out + kPcG0, t.g1, kPc4G1 * 4);
    return kPcG0 + kPc4G1;
  }
  if (what == 6) {  // zoom 2: FIR taps M (25 floats, z^-8 first), then the input-rate and the
                    // output-rate sections' a1, a2 (4 + 4 pairs)
    PcTab2 t;
    if (!pc_build_tables2(t)) return -1;
    const int n = kPc2G + 2 * (kPc2Own + kPc2Ap);
    if (cap < n) return -2;
    std::memcpy(out, t.g, kPc2G * 4);
    float *o = out + kPc2G;
    for (int s = 0; s < kPc2Own; ++s) *o++ = t.own[s].a1, *o++ = t.own[s].a2;
    for (int s = 0; s < kPc2Ap; ++s) *o++ = t.ap[s].a1, *o++ = t.ap[s].a2;
    return n;
  }
  if (what == 12 || what == 13 || what == 15 || what == 16) {  // zoom 4 (12, 13) / zoom 2 (15, 16):
    PcEdge e;                                                  // left / right map, built now
    const int K = what < 15 ? 2 : 1;
    try {
      if (!pc_edge_map_k(K, (what - 12) % 3, arg & ((1 << K) - 1), e)) return -1;
    } catch (...) {
      return -4;
    }
    const int n = 3 + e.R * e.r + e.J * e.r;
    if (cap < n) return -2;
    out[0] = (float)e.R;
    out[1] = (float)e.J;
    out[2] = (float)e.r;
    std::copy(e.U.begin(), e.U.end(), out + 3);
    std::copy(e.V.begin(), e.V.end(), out + 3 + e.R * e.r);
    return n;
  }
  if (what == 4 || what == 14 || what == 17) {  // the shipped constant map arg (0 start, 1 + k
                                                // end for L mod 2^K = k): zoom 8, 4, 2
    const int nmaps = what == 4 ? kPcEdgeMaps : what == 14 ? kPcEdge4Maps : kPcEdge2Maps;
    if (arg < 0 || arg >= nmaps) return -3;
    const PcEdgeConst &m = what == 4 ? kPcEdgeIdx[arg] : what == 14 ? kPcEdge4Idx[arg] : kPcEdge2Idx[arg];
    const int n = 3 + m.R * m.r + m.J * m.r;
    if (cap < n) return -2;
    out[0] = (float)m.R;
    out[1] = (float)m.J;
    out[2] = (float)m.r;
    std::memcpy(out + 3, kPcEdgeData + m.u, sizeof(float) * (size_t)(m.R * m.r + m.J * m.r));
    return n;  // U (R x r) then V^T (r x J), as stored
  }
  PcEdge e;
  try {  // fp64 builder (threads, large vectors): nothing may cross the C ABI
    if (!pc_edge_map(what - 2, arg & 7, e)) return -1;
  } catch (...) {
    return -4;
  }
  const int n = 3 + e.R * e.r + e.J * e.r;
  if (cap < n) return -2;
  out[0] = (float)e.R;
  out[1] = (float)e.J;
  out[2] = (float)e.r;
  std::copy(e.U.begin(), e.U.end(), out + 3);
  std::copy(e.V.begin(), e.V.end(), out + 3 + e.R * e.r);
  return n;
}
