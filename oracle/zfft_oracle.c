/*
 * zfft_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped or measured
 * as the product).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it.
 *
 * A plain-C float64 restatement of the reference's IQ -> log-PSD row path:
 *
 *   pypanadapter_spectrum.py:2088-2100  ApplicationDisplay.zoomfft  (LO mix, decimate loop)
 *   pypanadapter_spectrum.py:2102-2119  ApplicationDisplay.update   (welch, fftshift/crop, dB)
 *   pypanadapter_thread.py:1513-1548    PSD.update                  (same path, threaded)
 *
 * The arithmetic lives in a third-party dependency that is NOT vendored in the reference:
 * SciPy (container: 1.15.3, unpinned by the reference -- README.md:3-9).  Its published
 * algorithms are restated here:
 *   scipy/signal/_signaltools.py:4831 decimate(x, 2): sos = cheby1(8, 0.05, 0.8/2, 'sos')
 *                                     -> sosfiltfilt (:4718), padtype 'odd', padlen 27
 *   scipy/signal/_arraytools.py       odd_ext
 *   scipy/signal/_filter_design.py    sosfilt_zi (steady-state step response per section)
 *   scipy/signal/_sosfilt.pyx         sosfilt: transposed direct form II per section
 *   scipy/signal/_spectral_py.py:490  welch -> csd -> _spectral_helper(:1863) -> _fft_helper
 *                                     (constant detrend, window, nfft FFT, |X|^2, mean,
 *                                      1/(fs*sum(w^2)) density scaling, two-sided)
 * The SOS coefficients and sosfilt_zi table are passed in by the caller (generated from
 * scipy and pinned in pypanadapter_amd/csrc/cheby1_q2.h; tests check both against scipy).
 *
 * Deliberate, documented deviation: the LO is defined on integer n,
 * lo[n] = sqrt(2) * exp(-2*pi*i*f_lo*n/fs), instead of the reference's float arange, which
 * sometimes yields L+1 points and then raises.  Where the reference works the two agree
 * to ~1e-13 relative.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NSEC 4
#define PADLEN 27 /* 3 * ntaps, ntaps = 2*4+1 (sosfiltfilt, _signaltools.py:4811-4814) */

typedef struct { double re, im; } cplx;

/* sosfilt (one complex signal, real coefficients), DF2T, state z[s][0..1] per channel */
static void sosfilt_c(const double *sos, const cplx *x, cplx *y, int64_t n, cplx z[NSEC][2]) {
  for (int64_t i = 0; i < n; ++i) {
    cplx xn = x[i];
    for (int s = 0; s < NSEC; ++s) {
      const double *c = sos + 6 * s; /* b0 b1 b2 a0 a1 a2, a0 == 1 */
      cplx yc;
      yc.re = c[0] * xn.re + z[s][0].re;
      yc.im = c[0] * xn.im + z[s][0].im;
      z[s][0].re = c[1] * xn.re - c[4] * yc.re + z[s][1].re;
      z[s][0].im = c[1] * xn.im - c[4] * yc.im + z[s][1].im;
      z[s][1].re = c[2] * xn.re - c[5] * yc.re;
      z[s][1].im = c[2] * xn.im - c[5] * yc.im;
      xn = yc;
    }
    y[i] = xn;
  }
}

/* sosfiltfilt(sos, x) with padtype='odd', padlen=27; _signaltools.py:4807-4828 */
static int sosfiltfilt_c(const double *sos, const double *zi, const cplx *x, int64_t n, cplx *out) {
  if (n <= PADLEN) return -1; /* "The length of the input vector x must be greater than padlen" */
  int64_t e = n + 2 * PADLEN;
  cplx *ext = (cplx *)malloc(sizeof(cplx) * e);
  cplx *y = (cplx *)malloc(sizeof(cplx) * e);
  if (!ext || !y) { free(ext); free(y); return -2; }
  /* odd_ext: left 2*x[0]-x[27..1], right 2*x[-1]-x[-2..-28] */
  for (int i = 0; i < PADLEN; ++i) {
    ext[i].re = 2 * x[0].re - x[PADLEN - i].re;
    ext[i].im = 2 * x[0].im - x[PADLEN - i].im;
    ext[n + PADLEN + i].re = 2 * x[n - 1].re - x[n - 2 - i].re;
    ext[n + PADLEN + i].im = 2 * x[n - 1].im - x[n - 2 - i].im;
  }
  memcpy(ext + PADLEN, x, sizeof(cplx) * n);
  cplx z[NSEC][2];
  /* forward pass, zi * ext[0] */
  for (int s = 0; s < NSEC; ++s)
    for (int k = 0; k < 2; ++k) {
      z[s][k].re = zi[2 * s + k] * ext[0].re;
      z[s][k].im = zi[2 * s + k] * ext[0].im;
    }
  sosfilt_c(sos, ext, y, e, z);
  /* backward pass on the reversed output, zi * y[-1] */
  for (int64_t i = 0; i < e / 2; ++i) { cplx t = y[i]; y[i] = y[e - 1 - i]; y[e - 1 - i] = t; }
  for (int s = 0; s < NSEC; ++s)
    for (int k = 0; k < 2; ++k) {
      z[s][k].re = zi[2 * s + k] * y[0].re;
      z[s][k].im = zi[2 * s + k] * y[0].im;
    }
  sosfilt_c(sos, y, ext, e, z);
  for (int64_t i = 0; i < n; ++i) out[i] = ext[e - 1 - PADLEN - i];
  free(ext);
  free(y);
  return 0;
}

/* zoomfft: S:2088-2100.  x (complex64 interleaved) -> out (complex128), returns length or <0.
 * `mix`: the reference's zoomfft always mixes (S:2093-2094) but update() only calls it
 * when fft_ratio > 1 (S:2108-2109), so the row path passes mix = (zoom > 1). */
int64_t oracle_zoomfft(const float *iq, int64_t L, double fs, double f_lo, int zoom, int mix,
                       const double *sos, const double *zi, double *out) {
  if (zoom < 1 || (zoom & (zoom - 1))) return -3;
  cplx *a = (cplx *)malloc(sizeof(cplx) * (L > 0 ? L : 1));
  cplx *b = (cplx *)malloc(sizeof(cplx) * (L > 0 ? L : 1));
  if (!a || !b) { free(a); free(b); return -2; }
  const double sq2 = sqrt(2.0), r = f_lo / fs;
  for (int64_t n = 0; n < L; ++n) {
    double xr = iq[2 * n], xi = iq[2 * n + 1];
    if (mix) {
      double turns = fmod((double)n * r, 1.0); /* exact phase reduction for large n */
      double ph = -2.0 * M_PI * turns, c = sq2 * cos(ph), s = sq2 * sin(ph);
      a[n].re = xr * c - xi * s;
      a[n].im = xr * s + xi * c;
    } else {
      a[n].re = xr;
      a[n].im = xi;
    }
  }
  int64_t n = L;
  for (int z = zoom; z > 1; z >>= 1) {
    int rc = sosfiltfilt_c(sos, zi, a, n, b);
    if (rc) { free(a); free(b); return rc == -1 ? -4 : -2; }
    int64_t m = (n + 1) / 2; /* y[::2] */
    for (int64_t i = 0; i < m; ++i) a[i] = b[2 * i];
    n = m;
  }
  memcpy(out, a, sizeof(cplx) * n);
  free(a);
  free(b);
  return n;
}

/* in-place iterative radix-2 DIT FFT, forward (exp(-2 pi i k n / N)) */
static void fft_c(cplx *v, int N) {
  for (int i = 1, j = 0; i < N; ++i) {
    int bit = N >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) { cplx t = v[i]; v[i] = v[j]; v[j] = t; }
  }
  for (int len = 2; len <= N; len <<= 1) {
    int half = len >> 1, step = N / len;
    for (int i = 0; i < N; i += len)
      for (int k = 0; k < half; ++k) {
        double ang = -2.0 * M_PI * (double)(k * step) / (double)N;
        double c = cos(ang), s = sin(ang);
        cplx u = v[i + k], w = v[i + k + half];
        cplx t = {w.re * c - w.im * s, w.re * s + w.im * c};
        v[i + k].re = u.re + t.re;
        v[i + k].im = u.im + t.im;
        v[i + k + half].re = u.re - t.re;
        v[i + k + half].im = u.im - t.im;
      }
  }
}

/*
 * Welch + fftshift/crop + 20*log10: S:2111-2119.  x complex128 interleaved, length Ld.
 * win has length nperseg = min(n_fft, Ld) (_triage_segments: short input -> nperseg = Ld).
 * row[j] = 20*log10(P[(j - W//2) mod N]), j in [0, 2 (W//2)): the slice
 * fftshift(P)[N//2 - W//2 : N//2 + W//2] (W - 1 entries for odd W).
 */
int oracle_welch_row(const double *x, int64_t Ld, double fs, int n_fft, int n_win,
                     const double *win, int nperseg, double *row) {
  if (n_fft < 1 || (n_fft & (n_fft - 1)) || nperseg < 1 || nperseg > n_fft || Ld < nperseg)
    return -3;
  const cplx *xc = (const cplx *)x;
  int noverlap = nperseg / 2, step = nperseg - noverlap;
  int64_t nseg = (Ld - nperseg) / step + 1;
  double *acc = (double *)calloc(n_fft, sizeof(double));
  cplx *buf = (cplx *)malloc(sizeof(cplx) * n_fft);
  if (!acc || !buf) { free(acc); free(buf); return -2; }
  double wss = 0;
  for (int i = 0; i < nperseg; ++i) wss += win[i] * win[i];
  for (int64_t sidx = 0; sidx < nseg; ++sidx) {
    const cplx *seg = xc + sidx * step;
    double mr = 0, mi = 0;
    for (int i = 0; i < nperseg; ++i) { mr += seg[i].re; mi += seg[i].im; }
    mr /= nperseg;
    mi /= nperseg;
    for (int i = 0; i < n_fft; ++i) {
      if (i < nperseg) {
        buf[i].re = (seg[i].re - mr) * win[i];
        buf[i].im = (seg[i].im - mi) * win[i];
      } else {
        buf[i].re = buf[i].im = 0;
      }
    }
    fft_c(buf, n_fft);
    for (int k = 0; k < n_fft; ++k) acc[k] += buf[k].re * buf[k].re + buf[k].im * buf[k].im;
  }
  double scale = 1.0 / (fs * wss);
  for (int j = 0; j < (n_win & ~1); ++j) {
    int k = ((j - n_win / 2) % n_fft + n_fft) % n_fft;
    double p = acc[k] * scale / (double)nseg;
    row[j] = 20.0 * log10(fabs(p));
  }
  free(acc);
  free(buf);
  return 0;
}

/*
 * Waterfall ring, restating Waterfall.init_image / image_update (S:1625-1664) with the
 * roll expressed as an offset: img[i] == ring[(i + off) mod H].  The product keeps the
 * same ring on the device; this is the checker.
 *   state: ring (H*W doubles), off (int64)
 */
void oracle_waterfall_init(double *ring, int W, int64_t *off) {
  int H = W / 4;
  for (int i = 0; i < H; ++i)
    for (int x = 0; x < W; ++x) ring[(int64_t)i * W + x] = (x == 0 || x == W - 1) ? 0.0 : -500.0;
  *off = 0;
}

void oracle_waterfall_push(double *ring, int W, int64_t *off, int scroll, double *psd) {
  int H = W / 4;
  psd[0] = 0;
  psd[W / 2] = 0;
  psd[W - 1] = 0;
  int64_t o = *off;
  int64_t last = ((H - 1 + o) % H + H) % H;
  memcpy(ring + last * W, psd, sizeof(double) * W);
  o = ((o + scroll) % H + H) % H; /* np.roll(img, -scroll, 0) */
  *off = o;
  int tick = W / 10;
  for (int i = 0, x = 0; x < W - 1; ++i, x += tick) {
    if (i == 5 || i == 10) continue;
    if (scroll > 0) {
      for (int y = 5; y < 15; ++y) ring[((y + o) % H) * (int64_t)W + x] = 0;
    } else {
      for (int y = -10; y < -2; ++y) ring[((((y + H) % H) + o) % H) * (int64_t)W + x] = 0;
    }
  }
}

void oracle_waterfall_read(const double *ring, int W, int64_t off, double *img) {
  int H = W / 4;
  for (int i = 0; i < H; ++i)
    memcpy(img + (int64_t)i * W, ring + ((i + off) % H) * (int64_t)W, sizeof(double) * W);
}
