// image_io.cpp — the reference's output surface.
//
// SaveImage (internal/renderer/renderer.go:438-451) writes PNG through
// image/png, which encodes an opaque *image.RGBA as 8-bit truecolour RGB
// (colour type 2).  The pixel bytes here are identical; the compressed
// stream differs (zlib vs Go's compress/flate).  A P3 PPM writer in the
// format of internal/output/ppm.go:34-59 is provided for ".ppm" outputs
// (the Go CLI writes PNG bytes whatever the extension — a documented
// deviation).
#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <zlib.h>

#include <string>
#include <vector>

#include "rt_internal.h"

namespace rtgo {

static double go_max(double x, double y) {
  if ((isinf(x) && x > 0) || (isinf(y) && y > 0)) return INFINITY;
  if (isnan(x) || isnan(y)) return NAN;
  if (x == 0 && x == y) return signbit(x) ? y : x;
  return x > y ? x : y;
}
static double go_min(double x, double y) {
  if ((isinf(x) && x < 0) || (isinf(y) && y < 0)) return -INFINITY;
  if (isnan(x) || isnan(y)) return NAN;
  if (x == 0 && x == y) return signbit(x) ? x : y;
  return x < y ? x : y;
}

double go_pow_tonemap(double x) {
  const double y = 1.0 / 2.2;
  if (x == 1) return 1;
  if (isnan(x)) return x;
  if (x == 0) return 0;
  if (isinf(x)) return x > 0 ? x : INFINITY;
  if (x < 0) return NAN;
  return exp(y * log(x));  // Pow's fractional part: Exp(yf*Log(x)), pow.go
}

static uint8_t go_u8(double f) {
  if (isnan(f) || f >= 9.2233720368547758e18 || f < -9.2233720368547758e18) return 0;
  return (uint8_t)(int64_t)f;
}

void tonemap_to_rgba(const double c[3], uint8_t out[4]) {
  for (int k = 0; k < 3; ++k) {
    double v = c[k] * 1.0;
    v = 1.0 - exp(-v);
    v = go_pow_tonemap(v);
    v = go_max(0.0, go_min(1.0, v));
    v = go_max(0.0, go_min(1.0, v));  // ToRGB's Clamp(0, 1)
    out[k] = go_u8(v * 255);
  }
  out[3] = 255;
}

static void put_be32(std::vector<uint8_t>& b, uint32_t v) {
  b.push_back((uint8_t)(v >> 24));
  b.push_back((uint8_t)(v >> 16));
  b.push_back((uint8_t)(v >> 8));
  b.push_back((uint8_t)v);
}

static void chunk(std::vector<uint8_t>& out, const char* type, const uint8_t* data, size_t n) {
  put_be32(out, (uint32_t)n);
  size_t start = out.size();
  out.insert(out.end(), type, type + 4);
  out.insert(out.end(), data, data + n);
  uint32_t crc = (uint32_t)crc32(0L, out.data() + start, (uInt)(n + 4));
  put_be32(out, crc);
}

// os.MkdirAll(filepath.Dir(filename), 0755), renderer.go:439-442
static bool mkdir_parents(const std::string& path) {
  size_t slash = path.find_last_of('/');
  if (slash == std::string::npos || slash == 0) return true;
  std::string dir = path.substr(0, slash);
  std::string cur;
  for (size_t i = 0; i <= dir.size(); ++i) {
    if (i == dir.size() || dir[i] == '/') {
      if (!cur.empty()) {
        if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
      }
    }
    if (i < dir.size()) cur += dir[i];
  }
  return true;
}

}  // namespace rtgo

using namespace rtgo;

extern "C" {

void rt_tonemap_rgba(const float* lin, int32_t npix, uint8_t* out) {
  if (!lin || !out) return;
  for (int32_t i = 0; i < npix; ++i) {
    double c[3] = {lin[i * 3 + 0], lin[i * 3 + 1], lin[i * 3 + 2]};
    tonemap_to_rgba(c, out + (size_t)i * 4);
  }
}

int rt_write_png(const char* path, const uint8_t* rgba, int32_t w, int32_t h) {
  if (!path || !rgba || w <= 0 || h <= 0) {
    set_error("invalid PNG arguments");
    return RT_E_INVALID;
  }
  if (!mkdir_parents(path)) {
    set_error(std::string("mkdir for ") + path + ": " + strerror(errno));
    return RT_E_IO;
  }
  // image/png encodes an opaque *image.RGBA as RGB8 (every render: alpha 255,
  // renderer.go:96) and any other as RGBA8 with the colour un-premultiplied
  // ((c * 0xffff / a) >> 8 on 16-bit values; the CLI's empty frame of a
  // negative size is all zero)
  bool opaque = true;
  for (size_t i = 0; i < (size_t)w * h && opaque; ++i) opaque = rgba[i * 4 + 3] == 255;
  const int ch = opaque ? 3 : 4;
  // raw scanlines, filter type 0
  std::vector<uint8_t> raw;
  raw.reserve((size_t)h * (1 + (size_t)w * ch));
  for (int32_t y = 0; y < h; ++y) {
    raw.push_back(0);
    const uint8_t* row = rgba + (size_t)y * w * 4;
    for (int32_t x = 0; x < w; ++x) {
      const uint8_t* q = row + x * 4;
      if (opaque) {
        raw.push_back(q[0]);
        raw.push_back(q[1]);
        raw.push_back(q[2]);
        continue;
      }
      const uint32_t a = q[3] * 0x101u;
      for (int c = 0; c < 3; ++c) raw.push_back(a == 0 ? 0 : (uint8_t)(((q[c] * 0x101u) * 0xffffu / a) >> 8));
      raw.push_back(q[3]);
    }
  }
  uLongf zcap = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zcap);
  if (compress2(z.data(), &zcap, raw.data(), (uLong)raw.size(), Z_DEFAULT_COMPRESSION) != Z_OK) {
    set_error("zlib compression failed");
    return RT_E_IO;
  }
  z.resize(zcap);
  std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
  uint8_t ihdr[13];
  ihdr[0] = (uint8_t)(w >> 24);
  ihdr[1] = (uint8_t)(w >> 16);
  ihdr[2] = (uint8_t)(w >> 8);
  ihdr[3] = (uint8_t)w;
  ihdr[4] = (uint8_t)(h >> 24);
  ihdr[5] = (uint8_t)(h >> 16);
  ihdr[6] = (uint8_t)(h >> 8);
  ihdr[7] = (uint8_t)h;
  ihdr[8] = 8;   // bit depth
  ihdr[9] = opaque ? 2 : 6;  // truecolour, or truecolour with alpha
  ihdr[10] = 0;  // deflate
  ihdr[11] = 0;  // adaptive filtering
  ihdr[12] = 0;  // no interlace
  chunk(png, "IHDR", ihdr, 13);
  chunk(png, "IDAT", z.data(), z.size());
  chunk(png, "IEND", nullptr, 0);
  FILE* f = fopen(path, "wb");
  if (!f) {
    set_error(std::string("open ") + path + ": " + strerror(errno));
    return RT_E_IO;
  }
  size_t n = fwrite(png.data(), 1, png.size(), f);
  int cerr = fclose(f);
  if (n != png.size() || cerr != 0) {
    set_error(std::string("write ") + path + " failed");
    return RT_E_IO;
  }
  return RT_OK;
}

int rt_write_ppm(const char* path, const uint8_t* rgba, int32_t w, int32_t h) {
  if (!path || !rgba || w <= 0 || h <= 0) {
    set_error("invalid PPM arguments");
    return RT_E_INVALID;
  }
  if (!mkdir_parents(path)) {
    set_error(std::string("mkdir for ") + path + ": " + strerror(errno));
    return RT_E_IO;
  }
  FILE* f = fopen(path, "wb");
  if (!f) {
    set_error(std::string("open ") + path + ": " + strerror(errno));
    return RT_E_IO;
  }
  // SavePPMFromVec3 format: header, then per row "r g b " triples and '\n'
  fprintf(f, "P3\n%d %d\n255\n", w, h);
  for (int32_t y = 0; y < h; ++y) {
    for (int32_t x = 0; x < w; ++x) {
      const uint8_t* p = rgba + ((size_t)y * w + x) * 4;
      fprintf(f, "%d %d %d ", p[0], p[1], p[2]);
    }
    fputc('\n', f);
  }
  if (fclose(f) != 0) {
    set_error(std::string("write ") + path + " failed");
    return RT_E_IO;
  }
  return RT_OK;
}

}  // extern "C"
