// RIFF/WAVE header parsing for sedx_wav_parse (include/sedx.h): the first
// step of librosa.core.load -> soundfile (pytorch/predict.py:295,
// pytorch/main_strong.py:787).  Host-only C++ with no HIP dependency, so the
// parser of untrusted file bytes also builds under AddressSanitizer /
// UBSan (Makefile target `asan`, tests/native/asan_driver.cpp).
#include <cstdint>
#include <cstring>

#include "../../include/sedx.h"

extern "C" {

sedx_status sedx_wav_parse(const void* bytes, size_t n_bytes, sedx_wav_info* info) {
  if (!bytes || !info || n_bytes < 12) return SEDX_EINVAL;
  const unsigned char* b = static_cast<const unsigned char*>(bytes);
  auto u16 = [&](size_t o) { return (uint32_t)b[o] | ((uint32_t)b[o + 1] << 8); };
  auto u32 = [&](size_t o) { return u16(o) | (u16(o + 2) << 16); };
  if (std::memcmp(b, "RIFF", 4) != 0 || std::memcmp(b + 8, "WAVE", 4) != 0) return SEDX_EINVAL;
  std::memset(info, 0, sizeof(*info));
  bool have_fmt = false, have_data = false;
  uint32_t fmt_tag = 0, block_align = 0;
  size_t o = 12;
  while (o + 8 <= n_bytes) {
    const uint32_t sz = u32(o + 4);
    const size_t body = o + 8;
    if (std::memcmp(b + o, "fmt ", 4) == 0) {
      if (sz < 16 || body + 16 > n_bytes) return SEDX_EINVAL;
      fmt_tag = u16(body);
      info->channels = (int32_t)u16(body + 2);
      info->sample_rate = (int32_t)u32(body + 4);
      block_align = u16(body + 12);
      info->bits_per_sample = (int32_t)u16(body + 14);
      if (fmt_tag == 0xFFFE) {              // WAVE_FORMAT_EXTENSIBLE: sub-format GUID
        if (sz < 40 || body + 40 > n_bytes) return SEDX_EINVAL;
        fmt_tag = u16(body + 24);
      }
      have_fmt = true;
    } else if (std::memcmp(b + o, "data", 4) == 0) {
      info->data_offset = (int64_t)body;
      // streamed writers leave 0 / 0xFFFFFFFF: take the rest of the buffer
      const size_t avail = n_bytes - body;
      info->data_bytes = (int64_t)((sz == 0 || sz == 0xFFFFFFFFu || sz > avail) ? avail : sz);
      have_data = true;
      break;
    }
    o = body + sz + (sz & 1);               // chunks are word aligned
  }
  if (!have_fmt || !have_data || info->channels <= 0 || info->sample_rate <= 0) return SEDX_EINVAL;
  const int bps = info->bits_per_sample;
  if (fmt_tag == 1 && (bps == 8 || bps == 16 || bps == 24 || bps == 32))
    info->format = SEDX_WAV_PCM;
  else if (fmt_tag == 3 && (bps == 32 || bps == 64))
    info->format = SEDX_WAV_FLOAT;
  else
    return SEDX_EINVAL;
  const int64_t frame_bytes = (int64_t)info->channels * (bps / 8);
  if (block_align && (int64_t)block_align != frame_bytes) return SEDX_EINVAL;
  info->frames = info->data_bytes / frame_bytes;
  return SEDX_OK;
}

}  // extern "C"
