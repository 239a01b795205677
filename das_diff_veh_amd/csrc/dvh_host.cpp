// Host staging copies for the drop-in classes' NumPy windows (device.py:stage_windows).  The reference's
// classes take a list of host windows (VirtualShotGathersFromWindows, apis/imaging_classes.py:91-126); the
// product packs them into a pinned buffer, chunk by chunk, while the previous chunk crosses PCIe.  This is that
// packing copy: n blocks of nbytes, src[i] -> dst + i * nbytes.  Several Python threads call it at once, each
// on its own run of windows (ctypes releases the interpreter lock for the call), so the copy runs in parallel
// without per-window interpreter work.  Stores are non-temporal: the pinned buffer is read next by the GPU's
// DMA engine, not by this core, and streaming stores skip the read-for-ownership of every destination line.
#include <emmintrin.h>
#include <algorithm>
#include <stdint.h>
#include <string.h>

#include "dvh_common.h"
#include "dvh.h"

namespace {

void stream_copy(char* d, const char* s, int64_t nbytes) {
  // head: up to the destination's 16-byte alignment
  const int64_t head = std::min<int64_t>(nbytes, (16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15);
  memcpy(d, s, (size_t)head);
  d += head;
  s += head;
  nbytes -= head;
  int64_t i = 0;
  for (; i + 64 <= nbytes; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 32));
    const __m128i e = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 48), e);
  }
  memcpy(d + i, s + i, (size_t)(nbytes - i));
}

}  // namespace

DVH_API int dvh_host_gather(void* dst, const void* const* src, int64_t nbytes, int32_t n) {
  if ((!dst || !src) && n > 0) return dvh::set_error(-2, "null pointer argument");
  if (nbytes < 0 || n < 0) return dvh::set_error(-2, "negative size or count");
  for (int32_t i = 0; i < n; ++i)
    if (!src[i]) return dvh::set_error(-2, "null source window");
  char* d = static_cast<char*>(dst);
  for (int32_t i = 0; i < n; ++i) {
    stream_copy(d + (int64_t)i * nbytes, static_cast<const char*>(src[i]), nbytes);
  }
  _mm_sfence();  // the streaming stores are globally visible before the caller issues the H2D copy
  return 0;
}
