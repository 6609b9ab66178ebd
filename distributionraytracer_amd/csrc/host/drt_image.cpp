// drt_image.cpp — the output image of a frame: the reference's img_Data fill
// (main.cpp:705-719, u8fromfloat maths.h:126-130) and saveImgFile (main.cpp:251-266, DevIL PNG).
#include <stdint.h>
#include <stdio.h>
#include <zlib.h>

#include <vector>

#include "../../../include/drt.h"
#include "../../../include/drt_host.h"

namespace {

inline uint8_t u8fromfloat(float x) {  // maths.h:126-130; the float->uint8 cast of a negative is
  const float v = x * 255.99f;         // undefined in C++, 0 here (colours are clamped anyway)
  if (v >= 255.0f) return 255;
  if (!(v > 0.0f)) return 0;
  return (uint8_t)v;
}

void put_u32(std::vector<uint8_t>& b, uint32_t v) {
  b.push_back((uint8_t)(v >> 24)); b.push_back((uint8_t)(v >> 16)); b.push_back((uint8_t)(v >> 8)); b.push_back((uint8_t)v);
}

void chunk(std::vector<uint8_t>& png, const char type[4], const uint8_t* data, size_t n) {
  put_u32(png, (uint32_t)n);
  const size_t start = png.size();
  png.insert(png.end(), type, type + 4);
  if (n) png.insert(png.end(), data, data + n);
  const uint32_t crc = (uint32_t)crc32(0L, png.data() + start, (uInt)(n + 4));
  put_u32(png, crc);
}

}  // namespace

extern "C" int drt_image_rgb8(const float* rgb, int32_t res_x, int32_t res_y, uint8_t* out) {
  if (!rgb || !out || res_x <= 0 || res_y <= 0) return DRT_E_INVALID;
  const size_t n = (size_t)res_x * res_y * 3;
  for (size_t i = 0; i < n; i++) out[i] = u8fromfloat(rgb[i]);
  return DRT_OK;
}

extern "C" int drt_image_write_png(const char* path, const float* rgb, int32_t res_x, int32_t res_y) {
  if (!path || !rgb || res_x <= 0 || res_y <= 0) return DRT_E_INVALID;
  const size_t row = (size_t)res_x * 3;
  std::vector<uint8_t> raw;
  try {
    raw.resize((row + 1) * (size_t)res_y);
  } catch (...) {
    return DRT_E_OOM;
  }
  for (int32_t r = 0; r < res_y; r++) {  // PNG row r = frame row res_y-1-r (lower-left origin)
    uint8_t* dst = raw.data() + (row + 1) * (size_t)r;
    dst[0] = 0;  // filter: none
    const float* src = rgb + row * (size_t)(res_y - 1 - r);
    for (size_t i = 0; i < row; i++) dst[1 + i] = u8fromfloat(src[i]);
  }
  uLongf zn = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zn);
  if (compress2(z.data(), &zn, raw.data(), (uLong)raw.size(), 6) != Z_OK) return DRT_E_OOM;
  std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<uint8_t> ihdr;
  put_u32(ihdr, (uint32_t)res_x);
  put_u32(ihdr, (uint32_t)res_y);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit, RGB, deflate, adaptive filter, no interlace
  chunk(png, "IHDR", ihdr.data(), ihdr.size());
  chunk(png, "IDAT", z.data(), zn);
  chunk(png, "IEND", nullptr, 0);
  FILE* f = fopen(path, "wb");
  if (!f) return -7;
  const bool ok = fwrite(png.data(), 1, png.size(), f) == png.size();
  return (fclose(f) == 0 && ok) ? DRT_OK : -7;
}
