// Native (fp64) window generation: scipy.signal.get_window(kind, M, fftbins=True).
//
// The reference hands `AppState.fft_tapering` (a name or (name, params) tuple chosen in
// FFTTaperingControl, pypanadapter_spectrum.py:1222-1243, 1358-1363) to welch, which calls
// get_window(window, nperseg) -> a PERIODIC window: the symmetric window of length M+1
// with the last sample dropped (scipy/signal/windows/_windows.py `_extend`/`_truncate`).
// The formulas below restate scipy.signal.windows (scipy 1.15.3) for every kind in the
// taper list; 'slepian' is not a window in that scipy either (get_window raises).
// Absent parameters arrive as NaN and take scipy's defaults; the kinds scipy refuses to
// build without parameters (kaiser, gaussian, general_gaussian, chebwin, dpss) fail.
#include <cmath>
#include <complex>
#include <vector>

#include "zfft.h"
#include "zfft_internal.h"

namespace zfft {
namespace {

std::vector<double> linspace(double a, double b, int M) {
  std::vector<double> v(M);
  if (M == 1) { v[0] = a; return v; }
  const double step = (b - a) / (M - 1);
  for (int i = 0; i < M; ++i) v[i] = a + i * step;
  if (M > 1) v[M - 1] = b;  // numpy.linspace endpoint is exact
  return v;
}

// general_cosine(M, a, sym=True)
std::vector<double> general_cosine(int M, const std::vector<double> &a) {
  std::vector<double> fac = linspace(-M_PI, M_PI, M), w(M, 0.0);
  for (size_t k = 0; k < a.size(); ++k)
    for (int i = 0; i < M; ++i) w[i] += a[k] * std::cos(k * fac[i]);
  return w;
}

// modified Bessel I0 by its power series (beta <= ~700): sum ((x/2)^k / k!)^2
double bessel_i0(double x) {
  double s = 1.0, t = 1.0, q = 0.25 * x * x;
  for (int k = 1; k < 1000; ++k) {
    t *= q / (double(k) * double(k));
    s += t;
    if (t < s * 1e-17) break;
  }
  return s;
}

using cd = std::complex<double>;

// in-place radix-2 FFT (forward, exp(-i...)), n a power of two
void fft_pow2(std::vector<cd> &a) {
  const size_t n = a.size();
  for (size_t i = 1, j = 0; i < n; ++i) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
  for (size_t len = 2; len <= n; len <<= 1) {
    const double ang = -2 * M_PI / (double)len;
    for (size_t i = 0; i < n; i += len)
      for (size_t k = 0; k < len / 2; ++k) {
        const cd w = std::polar(1.0, ang * (double)k);
        const cd u = a[i + k], v = a[i + k + len / 2] * w;
        a[i + k] = u + v;
        a[i + k + len / 2] = u - v;
      }
  }
}

// DFT of any length n (Bluestein: chirp z-transform on a power-of-two FFT), fp64
std::vector<cd> dft_any(const std::vector<cd> &x) {
  const size_t n = x.size();
  size_t m = 1;
  while (m < 2 * n - 1) m <<= 1;
  std::vector<cd> chirp(n), a(m, 0.0), b(m, 0.0);
  for (size_t k = 0; k < n; ++k) {  // exp(-i pi k^2 / n) with k^2 reduced mod 2n exactly
    const unsigned long long k2 = (unsigned long long)k * k % (2ULL * n);
    chirp[k] = std::polar(1.0, -M_PI * (double)k2 / (double)n);
  }
  for (size_t k = 0; k < n; ++k) a[k] = x[k] * chirp[k];
  b[0] = std::conj(chirp[0]);
  for (size_t k = 1; k < n; ++k) b[k] = b[m - k] = std::conj(chirp[k]);
  fft_pow2(a);
  fft_pow2(b);
  for (size_t i = 0; i < m; ++i) a[i] *= b[i];
  for (auto &v : a) v = std::conj(v);  // inverse FFT via conjugation
  fft_pow2(a);
  std::vector<cd> out(n);
  for (size_t k = 0; k < n; ++k) out[k] = std::conj(a[k]) / (double)m * chirp[k];
  return out;
}

// chebwin(M, at, sym=True): Dolph-Chebyshev window from its DFT coefficients
std::vector<double> chebwin_sym(int M, double at) {
  const double order = M - 1.0;
  const double beta = std::cosh(1.0 / order * std::acosh(std::pow(10.0, std::fabs(at) / 20.0)));
  std::vector<cd> p(M);
  for (int k = 0; k < M; ++k) {
    const double x = beta * std::cos(M_PI * k / M);
    double v;
    if (x > 1) v = std::cosh(order * std::acosh(x));
    else if (x < -1) v = (2 * (M % 2) - 1) * std::cosh(order * std::acosh(-x));
    else v = std::cos(order * std::acos(x));
    p[k] = M % 2 ? cd(v, 0.0) : v * std::polar(1.0, M_PI / M * k);
  }
  const std::vector<cd> P = dft_any(p);
  std::vector<double> w;
  if (M % 2) {
    const int n = (M + 1) / 2;
    for (int i = n - 1; i >= 1; --i) w.push_back(P[i].real());
    for (int i = 0; i < n; ++i) w.push_back(P[i].real());
  } else {
    const int n = M / 2 + 1;
    for (int i = n - 1; i >= 1; --i) w.push_back(P[i].real());
    for (int i = 1; i < n; ++i) w.push_back(P[i].real());
  }
  double mx = w[0];
  for (double v : w) mx = std::max(mx, v);
  for (double &v : w) v /= mx;
  return w;
}

// dpss(M, NW) single window, sym=True: eigenvector of the largest eigenvalue of the
// Percival-Walden tridiagonal (d_t = ((M-1-2t)/2)^2 cos(2 pi W), e_t = t (M-t) / 2,
// W = NW/M), by Sturm-count bisection for the eigenvalue and inverse iteration for the
// vector; positive mean, max-normalised, even-M "approximate" correction M^2/(M^2+NW).
std::vector<double> dpss_sym(int M, double NW) {
  const double W = NW / M;
  std::vector<double> d(M), e(M, 0.0);
  for (int t = 0; t < M; ++t) {
    const double c = (M - 1 - 2.0 * t) / 2.0;
    d[t] = c * c * std::cos(2 * M_PI * W);
    if (t > 0) e[t] = t * (M - (double)t) / 2.0;  // e[t] couples t-1 and t
  }
  auto count_below = [&](double x) {  // eigenvalues < x (Sturm sequence)
    int cnt = 0;
    double q = d[0] - x;
    if (q < 0) ++cnt;
    for (int t = 1; t < M; ++t) {
      if (q == 0) q = 1e-300;
      q = d[t] - x - e[t] * e[t] / q;
      if (q < 0) ++cnt;
    }
    return cnt;
  };
  double lo = 0, hi = 0;  // Gershgorin bounds
  for (int t = 0; t < M; ++t) {
    const double r = std::fabs(e[t]) + (t + 1 < M ? std::fabs(e[t + 1]) : 0.0);
    lo = std::min(lo, d[t] - r);
    hi = std::max(hi, d[t] + r);
  }
  for (int it = 0; it < 200 && hi - lo > 1e-15 * std::max(std::fabs(lo), std::fabs(hi)); ++it) {
    const double mid = 0.5 * (lo + hi);
    if (count_below(mid) >= M) hi = mid;  // all eigenvalues below mid
    else lo = mid;
  }
  const double lam = hi;
  // inverse iteration on -(T - lam I), positive semidefinite: LU without pivoting
  std::vector<double> v(M, 1.0), diag(M), x(M);
  for (int iter = 0; iter < 3; ++iter) {
    for (int t = 0; t < M; ++t) diag[t] = lam - d[t];  // -(T - lam I) diagonal
    x = v;
    for (int t = 1; t < M; ++t) {  // forward elimination (off-diagonals are -e)
      if (diag[t - 1] == 0) diag[t - 1] = 1e-300;
      const double f = -e[t] / diag[t - 1];
      diag[t] -= f * -e[t];
      x[t] -= f * x[t - 1];
    }
    if (diag[M - 1] == 0) diag[M - 1] = 1e-300 * (std::fabs(lam) + 1);
    x[M - 1] /= diag[M - 1];
    for (int t = M - 2; t >= 0; --t) x[t] = (x[t] + e[t + 1] * x[t + 1]) / diag[t];
    double nrm = 0;
    for (double u : x) nrm += u * u;
    nrm = std::sqrt(nrm);
    for (int t = 0; t < M; ++t) v[t] = x[t] / nrm;
  }
  double sum = 0, mx = 0;
  for (double u : v) sum += u;
  if (sum < 0)
    for (double &u : v) u = -u;
  for (double u : v) mx = std::max(mx, u);
  for (double &u : v) u /= mx;
  if (M % 2 == 0) {
    const double corr = (double)M * M / ((double)M * M + NW);
    for (double &u : v) u *= corr;
  }
  return v;
}

std::vector<double> symmetric(int kind, const double *p, int M) {
  std::vector<double> w(M);
  switch (kind) {
    case ZFFT_WIN_HAMMING: return general_cosine(M, {0.54, 1.0 - 0.54});
    case ZFFT_WIN_HANN: return general_cosine(M, {0.5, 0.5});
    case ZFFT_WIN_BLACKMAN: return general_cosine(M, {0.42, 0.50, 0.08});
    case ZFFT_WIN_BLACKMANHARRIS: return general_cosine(M, {0.35875, 0.48829, 0.14128, 0.01168});
    case ZFFT_WIN_NUTTALL: return general_cosine(M, {0.3635819, 0.4891775, 0.1365995, 0.0106411});
    case ZFFT_WIN_FLATTOP:
      return general_cosine(M, {0.21557895, 0.41663158, 0.277263158, 0.083578947, 0.006947368});
    case ZFFT_WIN_BARTHANN:
      for (int n = 0; n < M; ++n) {
        double fac = std::fabs(n / double(M - 1) - 0.5);
        w[n] = 0.62 - 0.48 * fac + 0.38 * std::cos(2 * M_PI * fac);
      }
      return w;
    case ZFFT_WIN_BARTLETT:
      for (int n = 0; n < M; ++n)
        w[n] = (n <= (M - 1) / 2.0) ? 2.0 * n / (M - 1) : 2.0 - 2.0 * n / (M - 1);
      return w;
    case ZFFT_WIN_TRIANG: {
      int h = (M + 1) / 2;
      std::vector<double> v(h);
      for (int i = 0; i < h; ++i) {
        int n = i + 1;
        v[i] = (M % 2 == 0) ? (2.0 * n - 1.0) / M : 2.0 * n / (M + 1.0);
      }
      for (int i = 0; i < h; ++i) w[i] = v[i];
      if (M % 2 == 0)
        for (int i = 0; i < h; ++i) w[h + i] = v[h - 1 - i];
      else
        for (int i = 0; i < h - 1; ++i) w[h + i] = v[h - 2 - i];
      return w;
    }
    case ZFFT_WIN_BOHMAN: {
      std::vector<double> f = linspace(-1.0, 1.0, M);
      w[0] = 0.0;
      w[M - 1] = 0.0;
      for (int i = 1; i < M - 1; ++i) {
        double fac = std::fabs(f[i]);
        w[i] = (1 - fac) * std::cos(M_PI * fac) + 1.0 / M_PI * std::sin(M_PI * fac);
      }
      return w;
    }
    case ZFFT_WIN_PARZEN: {
      // n = arange(-(M-1)/2, (M-1)/2 + 0.5, 1.0)
      for (int i = 0; i < M; ++i) {
        double n = -(M - 1) / 2.0 + i, an = std::fabs(n);
        if (an <= (M - 1) / 4.0) {
          double r = an / (M / 2.0);
          w[i] = 1 - 6 * r * r + 6 * r * r * r;
        } else {
          double r = 1 - an / (M / 2.0);
          w[i] = 2 * r * r * r;
        }
      }
      return w;
    }
    case ZFFT_WIN_BOXCAR:
      for (int n = 0; n < M; ++n) w[n] = 1.0;
      return w;
    case ZFFT_WIN_KAISER: {
      double beta = p ? p[0] : 14.0, alpha = (M - 1) / 2.0, den = bessel_i0(beta);
      for (int n = 0; n < M; ++n) {
        double r = (n - alpha) / alpha;
        double a = 1.0 - r * r;
        w[n] = bessel_i0(beta * std::sqrt(a < 0 ? 0 : a)) / den;
      }
      return w;
    }
    case ZFFT_WIN_GAUSSIAN: {
      double sd = p ? p[0] : 7.0;
      for (int i = 0; i < M; ++i) {
        double n = i - (M - 1.0) / 2.0;
        w[i] = std::exp(-n * n / (2 * sd * sd));
      }
      return w;
    }
    case ZFFT_WIN_GENERAL_GAUSSIAN: {
      double pw = p ? p[0] : 1.5, sig = p ? p[1] : 7.0;
      for (int i = 0; i < M; ++i) {
        double n = i - (M - 1.0) / 2.0;
        w[i] = std::exp(-0.5 * std::pow(std::fabs(n / sig), 2 * pw));
      }
      return w;
    }
    case ZFFT_WIN_TUKEY: {
      double alpha = p ? p[0] : 0.5;
      if (alpha <= 0) {
        for (int n = 0; n < M; ++n) w[n] = 1.0;
        return w;
      }
      if (alpha >= 1.0) return general_cosine(M, {0.5, 0.5});
      int width = int(std::floor(alpha * (M - 1) / 2.0));
      for (int n = 0; n < M; ++n) {
        if (n <= width)
          w[n] = 0.5 * (1 + std::cos(M_PI * (-1 + 2.0 * n / alpha / (M - 1))));
        else if (n < M - width - 1)
          w[n] = 1.0;
        else
          w[n] = 0.5 * (1 + std::cos(M_PI * (-2.0 / alpha + 1 + 2.0 * n / alpha / (M - 1))));
      }
      return w;
    }
    case ZFFT_WIN_EXPONENTIAL: {  // exponential(M, center=None, tau=1.0)
      const double center = std::isnan(p[0]) ? (M - 1) / 2.0 : p[0];
      const double tau = std::isnan(p[1]) ? 1.0 : p[1];
      for (int n = 0; n < M; ++n) w[n] = std::exp(-std::fabs(n - center) / tau);
      return w;
    }
    case ZFFT_WIN_CHEBWIN: return chebwin_sym(M, p[0]);
    case ZFFT_WIN_DPSS: return dpss_sym(M, p[0]);
    default: return {};
  }
}

// scipy.signal.get_window refuses these without parameters ("needs one or more parameters")
bool params_ok(int kind, const double *p) {
  switch (kind) {
    case ZFFT_WIN_KAISER:
    case ZFFT_WIN_GAUSSIAN:
    case ZFFT_WIN_CHEBWIN:
    case ZFFT_WIN_DPSS: return !std::isnan(p[0]);
    case ZFFT_WIN_GENERAL_GAUSSIAN: return !std::isnan(p[0]) && !std::isnan(p[1]);
    default: return true;
  }
}

}  // namespace

bool window_kind_native(int kind) { return kind >= ZFFT_WIN_HAMMING && kind <= ZFFT_WIN_DPSS; }

// get_window(kind, M) with fftbins=True: symmetric length M+1, drop the last sample.
bool make_window(int kind, const double *param, int M, std::vector<double> &out) {
  const double nan = std::nan("");
  const double none[2] = {nan, nan};
  if (!param) param = none;
  if (!window_kind_native(kind) || M < 1 || !params_ok(kind, param)) return false;
  if (kind == ZFFT_WIN_DPSS && !(param[0] > 0 && param[0] < M / 2.0)) return false;  // scipy checks
  double pd[2] = {param[0], param[1]};
  if (kind == ZFFT_WIN_TUKEY && std::isnan(pd[0])) pd[0] = 0.5;  // tukey(M, alpha=0.5)
  param = pd;
  if (M == 1) {  // _len_guards: M <= 1 -> ones(M)
    out.assign(1, 1.0);
    return true;
  }
  std::vector<double> w = symmetric(kind, param, M + 1);
  if ((int)w.size() != M + 1) return false;
  w.pop_back();
  out.swap(w);
  return true;
}

}  // namespace zfft

extern "C" int zfft_window_values(int32_t kind, const double *param, int32_t length, double *out) {
  std::vector<double> w;
  if (!out || length < 1 || !zfft::make_window(kind, param, length, w)) {
    zfft::set_error("zfft_window_values: unsupported window kind or bad length");
    return ZFFT_EINVAL;
  }
  for (int i = 0; i < length; ++i) out[i] = w[i];
  return ZFFT_OK;
}
