// zfft_ring.cpp -- host IQ accumulation ring: the pinned-memory analogue of
// pypanadapter_thread.py's `Data` (T:1400-1483), the buffer between the SDR reader thread
// (`add`, T:2191) and the PSD worker (`get_data_start` / `data[:real_size]` /
// `get_data_end`, T:1516-1520).
//
// Semantics kept from Data: capacity max_size = 16 * chunk_size (T:1409); `add` writes at
// `size` and, when the chunk would run past max_size, folds back and writes it at 0 (T:1437-
// 1442); real_size = the high-water mark since the last drain, total_size = samples added
// since then (T:1448-1451); a drain hands over data[:real_size] -- after a fold-back that is
// the newest chunks first and the older ones behind them, exactly as the reference reads it
// -- and resets size, real_size and total_size (T:1462-1466).
//
// What changes: the reference's consumer keeps a *view* of the buffer after unlocking, so
// the reader thread can overwrite the frame while the DSP runs on it (the T
// race).  Here two buffers alternate: a drain swaps them under the lock, the producer fills
// the other one, and the drained frame stays intact until the next drain.  The buffers are
// pinned host memory (hipHostMalloc) so the frame's H2D copy in zfft_ring_process is a
// direct DMA; without a device (CPU-only hosts, tests) they are ordinary memory.  The
// NewtRap pacing (`delay_time`, T:1411-1412, 1455-1458) is out of scope.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "zfft.h"
#include "zfft_internal.h"

struct zfft_ring {
  std::mutex mu;
  int64_t chunk_size = 0, max_size = 0;
  int dtype = 0;
  size_t esz = 8;
  void *buf[2] = {nullptr, nullptr};
  bool pinned[2] = {false, false};
  int fill = 0;                                       // buffer `add` writes
  int64_t size = 0, real_size = 0, total_size = 0;    // Data.size / real_size / total_size
};

namespace {

void *ring_alloc(size_t bytes, bool *pinned) {
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess && p) {
    *pinned = true;
    return p;
  }
  (void)hipGetLastError();  // no device: ordinary memory (the copy is then staged by HIP)
  *pinned = false;
  return std::malloc(bytes);
}

void ring_free(void *p, bool pinned) {
  if (!p) return;
  if (pinned) (void)hipHostFree(p);
  else std::free(p);
}

}  // namespace

extern "C" {

int zfft_ring_create(int64_t chunk_size, int32_t in_dtype, zfft_ring **out) {
  if (!out) return zfft::set_error("null output"), ZFFT_EINVAL;
  *out = nullptr;
  if (chunk_size < 1 || chunk_size > ((int64_t)1 << 26))
    return zfft::set_error("chunk_size must be in [1, 2^26]"), ZFFT_EINVAL;
  if (in_dtype < 0 || in_dtype > 3)  // 3: real float32 (Data.new_real, T:1413-1417)
    return zfft::set_error("in_dtype must be 0, 1, 2 or 3"), ZFFT_EINVAL;
  zfft_ring *r = new zfft_ring;
  r->chunk_size = chunk_size;
  r->max_size = 16 * chunk_size;
  r->dtype = in_dtype;
  r->esz = zfft::in_elem_bytes(in_dtype);
  for (int i = 0; i < 2; ++i) {
    r->buf[i] = ring_alloc((size_t)r->max_size * r->esz, &r->pinned[i]);
    if (!r->buf[i]) {
      zfft_ring_destroy(r);
      return zfft::set_error("ring allocation failed"), ZFFT_ENOMEM;
    }
    std::memset(r->buf[i], 0, (size_t)r->max_size * r->esz);  // np.zeros(max_size) (T:1416, 1422)
  }
  *out = r;
  return ZFFT_OK;
}

int zfft_ring_destroy(zfft_ring *r) {
  if (!r) return ZFFT_OK;
  for (int i = 0; i < 2; ++i) ring_free(r->buf[i], r->pinned[i]);
  delete r;
  return ZFFT_OK;
}

int zfft_ring_add(zfft_ring *r, const void *chunk, int64_t n) {
  if (!r || (!chunk && n > 0)) return zfft::set_error("null argument"), ZFFT_EINVAL;
  if (n < 0) return zfft::set_error("negative chunk length"), ZFFT_EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  if (n > r->max_size) {
    // the reference folds back (size = 0, T:1439-1442) and then fails the slice assignment
    // data[0:n] = chunk (T:1447) with a ValueError: nothing is written or counted
    r->size = 0;
    return zfft::set_error("chunk longer than the ring (max_size = 16 * chunk_size)"), ZFFT_EINVAL;
  }
  int64_t new_size = r->size + n;
  if (new_size > r->max_size) {  // fold back: overwrite from the start (T:1437-1442)
    r->size = 0;
    new_size = n;
  }
  std::memcpy((char *)r->buf[r->fill] + (size_t)r->size * r->esz, chunk, (size_t)n * r->esz);
  r->size = new_size;
  r->real_size = std::max(r->real_size, r->size);
  r->total_size += n;
  return ZFFT_OK;
}

int zfft_ring_state(zfft_ring *r, int64_t *size, int64_t *real_size, int64_t *total_size) {
  if (!r) return zfft::set_error("null ring"), ZFFT_EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  if (size) *size = r->size;
  if (real_size) *real_size = r->real_size;
  if (total_size) *total_size = r->total_size;
  return ZFFT_OK;
}

int zfft_ring_take(zfft_ring *r, const void **frame, int64_t *n, int64_t *total) {
  if (!r || !frame || !n) return zfft::set_error("null argument"), ZFFT_EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  *frame = r->buf[r->fill];
  *n = r->real_size;
  if (total) *total = r->total_size;
  r->fill ^= 1;  // the producer continues in the other buffer; this frame stays intact
  r->size = r->real_size = r->total_size = 0;
  return ZFFT_OK;
}

int zfft_ring_process(zfft_ring *r, zfft_plan *plan, float *row_out, int32_t *produced) {
  if (!r || !plan || !row_out || !produced) return zfft::set_error("null argument"), ZFFT_EINVAL;
  *produced = 0;
  const void *frame = nullptr;
  int64_t n = 0;
  int rc = zfft_ring_take(r, &frame, &n, nullptr);
  if (rc) return rc;
  zfft_config c;
  rc = zfft_plan_config(plan, &c);
  if (rc) return rc;
  if (c.in_dtype != r->dtype) return zfft::set_error("ring and plan in_dtype differ"), ZFFT_EINVAL;
  if (n < c.n_fft) return ZFFT_OK;  // PSD.update skips frames shorter than fft_size (T:1522-1523)
  rc = zfft_process(plan, frame, n, 1, row_out);
  if (rc == ZFFT_OK) *produced = 1;
  return rc;
}

}  // extern "C"
