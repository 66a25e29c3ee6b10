/*
 * zfft.h -- C-ABI of the MI355X Zoom-FFT spectrum/waterfall engine (libzfft.so).
 *
 * Drop-in boundary for pypanadapter's IQ -> waterfall-line hot path.  The reference has
 * no FFI: the path is inline numpy/scipy.  Each entry point below replaces a reference
 * call site (file:line under alfille/pypanadapter):
 *
 *   zfft_process        ApplicationDisplay.update (pypanadapter_spectrum.py:2102-2119):
 *                       zoomfft -> welch -> fftshift/crop -> 20*log10, one row per frame;
 *                       PSD.update (pypanadapter_thread.py:1513-1548), threaded caller.
 *   zfft_decimate       ApplicationDisplay.zoomfft (pypanadapter_spectrum.py:2088-2100).
 *   zfft_waterfall_*    Waterfall.init_image / image_update (pypanadapter_spectrum.py:
 *                       1625-1664), kept as a device ring + offset instead of np.roll.
 *   zfft_waterfall_reset ApplicationDisplay.on_invertscroll_clicked (S:2074-2077).
 *
 * Conventions: IQ is interleaved float32 (complex64, numpy's layout).  Rows are float32,
 * length n_win, dB = 20*log10(PSD) exactly as the reference computes it.  Every function
 * returns 0 on success or a negative ZFFT_E* code; zfft_last_error() (thread-local)
 * holds the message.  A plan is not re-entrant: one plan per calling thread; plans on
 * different devices run concurrently.  The caller owns all host buffers; the plan owns
 * its device buffers, HIP stream and tables.
 */
#ifndef ZFFT_H
#define ZFFT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZFFT_VERSION 1

/* error codes */
#define ZFFT_OK 0
#define ZFFT_EINVAL (-1)       /* bad argument / config (ValueError in the Python shim) */
#define ZFFT_ESHORT (-2)       /* frame too short: a decimation stage has <= 27 samples  */
#define ZFFT_EHIP (-3)         /* HIP runtime failure                                    */
#define ZFFT_ENOMEM (-4)       /* device or host allocation failed                       */
#define ZFFT_ENODEV (-5)       /* no HIP device                                          */
#define ZFFT_EUNSUPPORTED (-6) /* valid in the reference but not built in this version   */
#define ZFFT_EINTERNAL (-7)    /* the library's own filter tables failed a consistency check */

/* window kinds: scipy.signal.get_window(kind, M) with fftbins=True (periodic), the taper
 * list of FFTTaperingControl (pypanadapter_spectrum.py:1222-1243) */
enum zfft_window_kind {
  ZFFT_WIN_HAMMING = 0, /* AppState.fft_tapering default, S:1492 */
  ZFFT_WIN_HANN = 1,
  ZFFT_WIN_BLACKMAN = 2,
  ZFFT_WIN_BLACKMANHARRIS = 3,
  ZFFT_WIN_NUTTALL = 4,
  ZFFT_WIN_FLATTOP = 5,
  ZFFT_WIN_BARTHANN = 6,
  ZFFT_WIN_BARTLETT = 7,
  ZFFT_WIN_TRIANG = 8,
  ZFFT_WIN_BOHMAN = 9,
  ZFFT_WIN_PARZEN = 10,
  ZFFT_WIN_BOXCAR = 11,
  ZFFT_WIN_KAISER = 12,           /* window_param[0] = beta              */
  ZFFT_WIN_GAUSSIAN = 13,         /* window_param[0] = std               */
  ZFFT_WIN_GENERAL_GAUSSIAN = 14, /* window_param = {p, sig}              */
  ZFFT_WIN_TUKEY = 15,            /* window_param[0] = alpha (NaN: 0.5)  */
  ZFFT_WIN_EXPONENTIAL = 16,      /* window_param = {center, tau}; NaN = scipy default
                                     (get_window(('exponential', 3), N) binds 3 to center) */
  ZFFT_WIN_CHEBWIN = 17,          /* window_param[0] = attenuation, dB   */
  ZFFT_WIN_DPSS = 18,             /* window_param[0] = NW (single taper)  */
  ZFFT_WIN_ARRAY = 100            /* caller-supplied float window (any scipy window) */
};

typedef struct zfft_config {
  int32_t n_fft;           /* N: power of two, 32..65536 (AppState.fft_size, S:1397; cfg5)  */
  int32_t zoom;            /* power of two, 1..512 (AppState.fft_ratio, S:2079-2086)        */
  int32_t n_win;           /* W: row stride, 2..N (N_WIN S:1757; T:1542); odd W gives the
                              reference's W - 1 entries (zfft_plan_row_length)            */
  int32_t window_kind;     /* enum zfft_window_kind                                         */
  double fs;               /* sample rate, Hz (panadapter.SampleRate)                       */
  double f_lo;             /* LO frequency, Hz; the reference hard-codes 1.0 (S:2090)       */
  double window_param[2];  /* see window kinds; NaN = parameter absent (scipy's default)      */
  int32_t scroll;          /* waterfall direction, +1 or -1 (AppState.scroll, S:1496)       */
  int32_t in_dtype;        /* 0 = complex64 (interleaved f32, 8 B/sample); 1 = complex32
                              (interleaved f16, 4 B/sample, BASELINE cfg5); 2 = RTL-SDR
                              interleaved uint8 I,Q (2 B/sample), value b/127.5 - 1 as
                              pyrtlsdr's packed_bytes_to_iq; 3 = real f32
                              (4 B/sample: AudioPan's paFloat32 stream, S:712-713, §8f-4)  */
  int32_t device;          /* HIP device ordinal                                            */
  int32_t flip_input;      /* 1 = reverse each frame on load: the np.flip the RTL-SDR
                              sources apply (S:541-543, 459-460), fused into stage 0       */
} zfft_config;

typedef struct zfft_plan zfft_plan;

/* Create a plan.  window_or_null: with ZFFT_WIN_ARRAY, a float window of length n_fft (the
 * array welch receives; frames whose decimated length is < n_fft are then rejected, as
 * scipy rejects a window longer than the input). */
int zfft_plan_create(const zfft_config *cfg, const float *window_or_null, zfft_plan **out);
int zfft_plan_destroy(zfft_plan *plan);
int zfft_plan_config(const zfft_plan *plan, zfft_config *out);  /* the configuration in use */
/* Valid floats per row (rows keep the stride n_win): the length of the reference's slice
 * fftshift(P)[N//2 - W//2 : N//2 + W//2] (S:2114), i.e. n_win rounded down to even, except
 * for real input (in_dtype 3) at zoom 1, where the reference's welch is one-sided and that
 * slice of the N/2+1 bins is shorter.  A waterfall of any width >= 40/60
 * (the one-sided rows are odd) is a plan with n_win = that width. */
int zfft_plan_row_length(const zfft_plan *plan);

/* Host-buffer path: n_frames frames of n_samples IQ each (frame-major), rows_out holds
 * n_frames*n_win floats.  Synchronous.  PCIe-inclusive. */
int zfft_process(zfft_plan *plan, const void *iq, int64_t n_samples, int32_t n_frames,
                 float *rows_out);

/* Device-buffer path: d_iq and d_rows are device pointers on the plan's device.  Enqueued
 * on `hip_stream` (a hipStream_t; NULL = HIP's default stream); returns without syncing. */
int zfft_process_device(zfft_plan *plan, const void *d_iq, int64_t n_samples, int32_t n_frames,
                        float *d_rows, void *hip_stream);

/* zoomfft (S:2088-2100): LO mix then log2(zoom) x decimate(x, 2).  out_iq receives
 * zfft_decimated_length(n_samples, zoom) complex64 samples.  Synchronous, host buffers. */
int zfft_decimate(zfft_plan *plan, const void *iq, int64_t n_samples, void *out_iq,
                  int64_t *out_len);
int64_t zfft_decimated_length(int64_t n_samples, int32_t zoom);

/* Waterfall ring: H = n_win/4 rows of n_win floats, reference row order on read. */
int zfft_waterfall_push(zfft_plan *plan, const float *row /* host, n_win; NULL = last row of
                                                             the last zfft_process* frame:
                                                             ZFFT_EINVAL when the plan's rows
                                                             are shorter than n_win */);
/* d_rows: count rows of n_win floats, every column defined (a row shorter than n_win --
 * zfft_plan_row_length < n_win -- leaves its tail columns unwritten: pad them first). */
int zfft_waterfall_push_device(zfft_plan *plan, const float *d_rows, int32_t count,
                               void *hip_stream);
int zfft_waterfall_read(zfft_plan *plan, float *img_out /* host, H*n_win */);
int zfft_waterfall_reset(zfft_plan *plan, int32_t scroll);
int zfft_waterfall_shape(const zfft_plan *plan, int32_t *rows, int32_t *cols);

/* Host IQ accumulation ring: pypanadapter_thread.py's `Data` (T:1400-1483)
 * between the reader thread and the PSD worker, in pinned host memory.  capacity =
 * 16 * chunk_size (T:1409); zfft_ring_add = Data.add without the pacing sleep: a chunk that
 * would run past the end is written at 0 instead (T:1437-1442), real_size is the high-water
 * mark and total_size the samples added since the last drain; zfft_ring_take =
 * get_data_start / data[:real_size] / get_data_end (T:1516-1520): it returns that frame
 * (after a fold-back: newest chunks first, as the reference reads it) and resets the
 * counts.  Two buffers alternate, so the returned frame stays intact until the next take
 * while add() continues (the reference's consumer keeps a view the reader may overwrite).
 * zfft_ring_process = PSD.update (T:1513-1548): take, skip frames shorter than n_fft
 * (*produced = 0), else one row through zfft_process from the pinned frame.  Thread-safe:
 * one producer and one consumer. */
typedef struct zfft_ring zfft_ring;
int zfft_ring_create(int64_t chunk_size, int32_t in_dtype, zfft_ring **out);
int zfft_ring_destroy(zfft_ring *ring);
int zfft_ring_add(zfft_ring *ring, const void *chunk, int64_t n_samples);
int zfft_ring_state(zfft_ring *ring, int64_t *size, int64_t *real_size, int64_t *total_size);
int zfft_ring_take(zfft_ring *ring, const void **frame, int64_t *n_samples, int64_t *total_size);
int zfft_ring_process(zfft_ring *ring, zfft_plan *plan, float *row_out /* host, n_win */,
                      int32_t *produced);

/* On-device waterfall rendering.  The reference hands img_array.T to a
 * pyqtgraph ImageItem with a 256-entry colormap LUT and fixed levels (Waterfall.__init__ /
 * lookuptable / newlevel / autolevel, pypanadapter_spectrum.py:1579-1623, 1667-1685); these
 * produce the RGBA pixels that ImageItem draws for the ring image, on the device:
 *   pixel = LUT[clip(trunc((v - min) * 256 / (max - min)), 0, 255)], alpha 255
 * (pyqtgraph makeARGB / rescaleData / applyLookupTable), rows in zfft_waterfall_read order.
 * Colormaps 'Default', 'Matrix', 'Red Green', 'Tropical' (S:1580-1585; any other name ->
 * 'Default', S:1613-1616); the LUT is linspace(0, 1, 256) through the stops, channels
 * truncated to uint8 (ColorMap.getLookupTable(0, 1, 256)).  'Default' carries the
 * reference's out-of-range stop value 2020 as numpy < 2 stored it in a uint8 (2020 mod 256
 * = 228; numpy 2 raises OverflowError there).  Initial levels -220 .. -120 (S:1593-1598).
 * autolevel sets the levels to the 2nd and 98th percentiles (numpy 'linear') of the pixels
 * below 0 -- what S:1676 computes; the reference then assigns them to unused attributes,
 * so its autolevel never changes the levels (a bug, SURVEY §8 a-6 note). */
int zfft_colormap_lut(const char *name, uint8_t *lut_rgba /* 256*4; no plan, no GPU */);
int zfft_waterfall_colormap(zfft_plan *plan, const char *name);
int zfft_waterfall_levels(zfft_plan *plan, double minlev, double maxlev);
int zfft_waterfall_get_levels(const zfft_plan *plan, double *minlev, double *maxlev);
int zfft_waterfall_autolevel(zfft_plan *plan, double *minlev, double *maxlev);
int zfft_waterfall_render(zfft_plan *plan, uint8_t *rgba_out /* host, H*n_win*4 */);
int zfft_waterfall_render_device(zfft_plan *plan, uint8_t *d_rgba /* H*n_win*4 */,
                                 void *hip_stream);
/* The per-line display in one round trip (Waterfall.image_update then the image the Qt side
 * draws, S:1638-1664): `count` host rows of n_win floats pushed as zfft_waterfall_push would
 * (0 = none), then the image emitted -- RGBA8 as zfft_waterfall_render, or float64 as the
 * reference's img_array (zfft_waterfall_read's floats widened) -- and copied to the host, with
 * one kernel for a single row, one copy and one wait (the rows are staged in page-locked
 * memory the kernel reads in place).  Same ring and image as the separate calls. */
int zfft_waterfall_push_render(zfft_plan *plan, const float *rows, int32_t count,
                               uint8_t *rgba_out /* host, H*n_win*4 */);
int zfft_waterfall_push_read64(zfft_plan *plan, const float *rows, int32_t count,
                               double *img_out /* host, H*n_win */);

/* Page-locked host memory (hipHostMalloc on the current device), e.g. for rgba_out: a render
 * (or a zfft_process row block) copied into it moves at PCIe DMA rate; into pageable memory
 * the runtime stages the copy through its own bounce buffer at a fraction of that (W = 8192:
 * 67 MB per image).  Free with zfft_host_free. */
int zfft_host_alloc(size_t bytes, void **out);
int zfft_host_free(void *ptr);

/* Native window generation (fp64), for tests and for callers without scipy. */
int zfft_window_values(int32_t kind, const double *param, int32_t length, double *out);

/* Block size / warm-up of the device decimator (0 = automatic).  Diagnostics. */
int zfft_plan_tune(zfft_plan *plan, int32_t block, int32_t warmup);

/* Per-launch HIP-event timing of zfft_process*: when enabled, the plan brackets every
 * kernel it launches with events on the launch stream; zfft_plan_timings then returns the
 * durations (ms) of the last call, in launch order, named by zfft_plan_timing_names: per
 * decimation stage one "xa_stage_mix"/"xa_stage" interval (XA schedule) or a forward and a
 * backward pass (blocked schedules), then the Welch kernel ("welch_rows" / "welch4").  A
 * batched zfft_process call reports every batch ("batch_wait" = the gap before batch k >= 1,
 * mostly its H2D copy).  Diagnostics; adds event records. */
int zfft_plan_timing(zfft_plan *plan, int32_t enable);
int zfft_plan_timings(zfft_plan *plan, float *ms_out, int32_t max, int32_t *count);
/* Comma-separated names of the intervals zfft_plan_timings returns (owned by the plan). */
const char *zfft_plan_timing_names(zfft_plan *plan);

/* Decimator schedule: 0 = automatic -- for zoom 8 and frames of >= 16384 samples 4 below
 * 16 frames per call and 6 from there (zoom >= 16: the same for the first three stages;
 * zoom 4: 4 below 32 frames per call and 6 from there; zoom 2: 4 below 512); otherwise 3 for
 * batches of >= 768 frames, or >= 384 frames of <= 2^19
 * samples, else 2 for batches of >= 2^27 samples whose frames are long enough for the edge
 * windows, else 1 -- e.g. one frame per call, the reference's use.  Each batch of a
 * zfft_process call is judged by its own frame count (host calls are split into batches of
 * about 1 GiB of input -- 418 cfg2 frames); crossovers measured by tools/sweep_schedule.py,
 * tools/sweep_walk.py and tools/fc_ab.py (profiles/r04v, r06k, r06fc).  Default tolerance:
 * path 6 gives the float64 reference's decimated IQ within 6.5e-7 of its peak (measured
 * worst 6.0e-7, tests/test_gpu_fc.py FC_TOL); the PC choices (zoom 8 below 16 frames per call,
 * zoom 4 below 32, zoom 2 below 512) within 6.5e-6, the head of zoom >= 16 (x8 + zoom 2's tiles or the
 * blocked passes) within 7.5e-6 -- the measured worst of the GPU tests + ~20 % (5.35e-6 and
 * 6.02e-6; the walk on the zf_n512_z8 fixture 6.07e-6; tests/test_gpu_pc.py PC_TOL / HEAD_TOL);
 * path 1: 2e-6.
 * 1 = blocked warm-up passes in the reference order (frames split over many waves),
 * 2 = blocked, fused commuted-order interior + exact edge windows, 3 = XA tiles (one wave per
 * frame and stage: all-pole cascade + 25-tap FIR + half-rate all-pole, lane states scanned;
 * each stage is one launch whose decimated output -- n_k/2 complex64 per frame -- is the next
 * stage's input in device memory), 4 = PC polyphase cascade (zoom 8: FIRs at falling
 * rates + the slow poles as zero-phase sections at rates 1/4 and 1/8, two launches, plus
 * rank-~10 frame-end maps; frames >= 16384 samples, <= 65535 frames per launch; zoom 4, 2
 * and the head of zoom >= 16 as below), 5 = the
 * same arithmetic as one launch with one workgroup per frame (the rate-1/4 intermediate
 * stays on chip); at zoom 4, path 5 is the two-stage
 * form of the walk (FIR, own-rate sections at rate 1/2, 41-tap FIR, 6 output-rate sections)
 * and path 4 its tiles (automatic below 32 frames per call); at zoom 2,
 * paths 4 / 5 run one-stage tiles in XA's factorisation (the
 * 4 sections forward at the input rate, a 25-tap FIR, their squares backward at half rate;
 * automatic below 512 frames per call); at zoom >= 16, paths 4 / 5 / 6 run PC / FC for the
 * first three stages and XA for the rest on its 1/8-rate output -- the automatic choice
 * wherever XA would take the batch (zoom 16 on cfg2's frames: 3.64 ms per 4096 frames with FC,
 * 5.01 with the walk, 6.35 with XA alone); 6 = FC, fast convolution (zoom 8, zoom 4 and the head
 * of zoom >= 16; elsewhere as 5): the model's impulse response truncated at |k| <= 768 (zoom 8)
 * / 512 (zoom 4) input samples (tail <= 1e-6 of its absolute sum) applied by overlap-save in
 * 8192-sample windows -- the residues' DFTs, the decimation folded into the spectrum with the
 * filter and the LO's modulation, one inverse DFT per window, one launch with one workgroup
 * per frame (or per run of windows below 1024 frames per call), the frame-end maps as for 5;
 * frames of >= 8192 samples below 2^31 bytes (cfg2's 4096 frames: 2.66 ms against the walk's
 * 4.18; cfg1's: 2.82 against the zoom-4 walk's 4.22).  Path 3
 * needs every stage array below 2^31 bytes per frame; a forced path outside its domain
 * returns ZFFT_EUNSUPPORTED.  All produce the reference's rows within the fp32 parity gate
 * (zfft_plan.cpp auto_xa, use_fused, pc_fits, fc_fits). */
int zfft_plan_path(zfft_plan *plan, int32_t path);

/* Batched multi-IF (BASELINE config 4): one LO frequency per group of frames in a single
 * plan and launch chain.  Frame f of every zfft_process* / zfft_decimate call (f counted from
 * the call's first frame) is mixed with f_lo[(f / frames_per_lo) % n] instead of cfg.f_lo --
 * the reference's mixer (S:2090-2094) with f_demod per IF.  frames_per_lo = 1 interleaves
 * the IFs frame by frame; n = 0 restores cfg.f_lo; n = 1 replaces cfg.f_lo.  The LO table
 * holds n rows of n_samples complex64 (n <= 256, at most 4 GiB: ZFFT_ENOMEM beyond).  Zoom 1
 * never mixes (the reference skips zoomfft at ratio 1, S:2108): n > 1 is ZFFT_EINVAL there.
 * Waits for the plan's enqueued work. */
int zfft_plan_set_lo_frames(zfft_plan *plan, const double *f_lo, int32_t n, int32_t frames_per_lo);

/* Welch FFT schedule: 0 = automatic (one workgroup per frame for n_fft <= 16384, four-step
 * beyond), 1 = one workgroup per frame (n_fft <= 16384), 2 = four-step N1 x 256 (n_fft in
 * [4096, 65536]; its row pass forms only the bins the crop keeps when n_win <= n_fft / 8).
 * Same rows within the parity gate; diagnostics / A-B only. */
int zfft_plan_welch(zfft_plan *plan, int32_t mode);

const char *zfft_last_error(void);
int zfft_device_count(void);
int zfft_version(void);

#ifdef __cplusplus
}
#endif

#endif /* ZFFT_H */
