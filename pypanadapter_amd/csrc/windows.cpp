// Native (fp64) window generation: scipy.signal.get_window(kind, M, fftbins=True).
//
// The reference hands `AppState.fft_tapering` (a name or (name, params) tuple chosen in
// FFTTaperingControl, pypanadapter_spectrum.py:1222-1243, 1358-1363) to welch, which calls
// get_window(window, nperseg) -> a PERIODIC window: the symmetric window of length M+1
// with the last sample dropped (scipy/signal/windows/_windows.py `_extend`/`_truncate`).
// The formulas below restate scipy.signal.windows for the kinds in the taper list that
// have closed forms; chebwin / dpss / slepian come in as caller arrays (ZFFT_WIN_ARRAY).
#include <cmath>
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
    default: return {};
  }
}

}  // namespace

bool window_kind_native(int kind) { return kind >= ZFFT_WIN_HAMMING && kind <= ZFFT_WIN_TUKEY; }

// get_window(kind, M) with fftbins=True: symmetric length M+1, drop the last sample.
bool make_window(int kind, const double *param, int M, std::vector<double> &out) {
  if (!window_kind_native(kind) || M < 1) return false;
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
