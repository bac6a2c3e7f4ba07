// sfrt_png.cpp -- PNG -> RGBA8 decoder (the asset pipeline).
//
// The reference loads every texture with sf::Image::loadFromFile (SFML 2.4.2,
// which decodes through stb_image and asks for 4 channels), e.g. Floor.png at
// /root/reference/Raytracing/SphereWorld.cpp:52-53 and the World textures at
// World.cpp:40-45.  This decoder produces the bytes stb_image's 4-channel path
// produces:
//  * colour types 0 (grey), 2 (RGB), 3 (palette), 4 (grey+alpha), 6 (RGBA);
//    bit depths 1, 2, 4, 8, 16; Adam7 interlacing;
//  * grey below 8 bits is scaled by 0xff / (2^depth - 1) (stb's depth scale
//    table); palette indices are not scaled; 16-bit samples keep the high byte;
//  * tRNS: palette alpha per entry; for grey / RGB a pixel equal to the key
//    (compared at the image's bit depth, after the same scaling) gets alpha 0,
//    every other pixel 255; no tRNS -> alpha 255;
//  * gAMA / sRGB / iCCP are ignored and chunk CRCs are not checked (stb does
//    neither); unknown ancillary chunks are skipped.
// Errors (truncation, bad header, failed inflate, missing PLTE) return
// SFRT_E_INVALID; nothing is written then.
#include <zlib.h>

#include <cstdint>
#include <cstring>
#include <vector>

#include "sfrt.h"

namespace {

uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

struct Header {
  uint32_t w = 0, h = 0;
  int depth = 0, color = 0, interlace = 0;
  int channels = 0;
};

struct Png {
  Header hd;
  uint8_t pal[256][4];
  int pal_n = 0;
  bool has_trns = false;
  uint16_t key[3] = {0, 0, 0};
  std::vector<uint8_t> idat;
};

int channels_of(int color) {
  switch (color) {
    case 0: return 1;
    case 2: return 3;
    case 3: return 1;
    case 4: return 2;
    case 6: return 4;
    default: return 0;
  }
}

bool depth_ok(int color, int depth) {
  switch (color) {
    case 0: return depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16;
    case 3: return depth == 1 || depth == 2 || depth == 4 || depth == 8;
    case 2: case 4: case 6: return depth == 8 || depth == 16;
    default: return false;
  }
}

int parse(const uint8_t* d, int64_t n, Png& png, bool header_only) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  if (!d || n < 8 + 25 || std::memcmp(d, sig, 8) != 0) return SFRT_E_INVALID;
  int64_t pos = 8;
  bool first = true, seen_idat = false;
  for (;;) {
    if (pos + 12 > n) return SFRT_E_INVALID;
    const uint32_t len = be32(d + pos);
    const uint8_t* type = d + pos + 4;
    const uint8_t* body = d + pos + 8;
    if (len > (uint32_t)0x7fffffff || pos + 12 + (int64_t)len > n) return SFRT_E_INVALID;
    if (first) {
      if (std::memcmp(type, "IHDR", 4) != 0 || len != 13) return SFRT_E_INVALID;
      Header& h = png.hd;
      h.w = be32(body);
      h.h = be32(body + 4);
      h.depth = body[8];
      h.color = body[9];
      h.interlace = body[12];
      if (h.w == 0 || h.h == 0 || h.w > (1u << 24) || h.h > (1u << 24)) return SFRT_E_INVALID;
      if (body[10] != 0 || body[11] != 0 || h.interlace > 1) return SFRT_E_INVALID;
      if (!depth_ok(h.color, h.depth)) return SFRT_E_INVALID;
      h.channels = channels_of(h.color);
      first = false;
      if (header_only) return SFRT_OK;
    } else if (!std::memcmp(type, "PLTE", 4)) {
      if (len % 3 != 0 || len / 3 > 256 || len == 0) return SFRT_E_INVALID;
      png.pal_n = (int)(len / 3);
      for (int k = 0; k < png.pal_n; k++) {
        png.pal[k][0] = body[3 * k];
        png.pal[k][1] = body[3 * k + 1];
        png.pal[k][2] = body[3 * k + 2];
        png.pal[k][3] = 255;
      }
    } else if (!std::memcmp(type, "tRNS", 4)) {
      if (seen_idat) return SFRT_E_INVALID;
      const Header& h = png.hd;
      if (h.color == 3) {
        if (png.pal_n == 0 || (int)len > png.pal_n) return SFRT_E_INVALID;
        for (uint32_t k = 0; k < len; k++) png.pal[k][3] = body[k];
      } else if (h.color == 0) {
        if (len != 2) return SFRT_E_INVALID;
        png.key[0] = (uint16_t)((body[0] << 8) | body[1]);
      } else if (h.color == 2) {
        if (len != 6) return SFRT_E_INVALID;
        for (int c = 0; c < 3; c++) png.key[c] = (uint16_t)((body[2 * c] << 8) | body[2 * c + 1]);
      } else {
        return SFRT_E_INVALID;  // stb: tRNS with an alpha channel is an error
      }
      png.has_trns = h.color != 3;
    } else if (!std::memcmp(type, "IDAT", 4)) {
      seen_idat = true;
      png.idat.insert(png.idat.end(), body, body + len);
    } else if (!std::memcmp(type, "IEND", 4)) {
      break;
    } else if (!(type[0] & 0x20)) {
      return SFRT_E_INVALID;  // unknown critical chunk
    }
    pos += 12 + (int64_t)len;
  }
  if (!seen_idat || (png.hd.color == 3 && png.pal_n == 0)) return SFRT_E_INVALID;
  return SFRT_OK;
}

int paeth(int a, int b, int c) {
  const int p = a + b - c;
  const int pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

// Reverses the scanline filters of one (sub)image in place; raw has 1 + stride bytes per row.
bool unfilter(uint8_t* raw, uint32_t rows, size_t stride, int bpp, std::vector<uint8_t>& out) {
  out.assign((size_t)rows * stride, 0);
  for (uint32_t y = 0; y < rows; y++) {
    const uint8_t f = raw[(size_t)y * (stride + 1)];
    const uint8_t* in = raw + (size_t)y * (stride + 1) + 1;
    uint8_t* cur = out.data() + (size_t)y * stride;
    const uint8_t* prev = y ? cur - stride : nullptr;
    for (size_t x = 0; x < stride; x++) {
      const int a = x >= (size_t)bpp ? cur[x - bpp] : 0;
      const int b = prev ? prev[x] : 0;
      const int c = (prev && x >= (size_t)bpp) ? prev[x - bpp] : 0;
      int v;
      switch (f) {
        case 0: v = in[x]; break;
        case 1: v = in[x] + a; break;
        case 2: v = in[x] + b; break;
        case 3: v = in[x] + ((a + b) >> 1); break;
        case 4: v = in[x] + paeth(a, b, c); break;
        default: return false;
      }
      cur[x] = (uint8_t)v;
    }
  }
  return true;
}

// Sample k (0-based within the row) of a row at the image's bit depth.
uint16_t sample(const uint8_t* row, size_t k, int depth) {
  if (depth == 8) return row[k];
  if (depth == 16) return (uint16_t)((row[2 * k] << 8) | row[2 * k + 1]);
  const size_t bit = k * depth;
  const int shift = 8 - depth - (int)(bit & 7);
  return (uint16_t)((row[bit >> 3] >> shift) & ((1 << depth) - 1));
}

// Expands one unfiltered (sub)image row to RGBA8 at out (stride 4 per pixel, step apart).
void expand_row(const Png& png, const uint8_t* row, uint32_t width, uint8_t* out, size_t step) {
  const Header& h = png.hd;
  static const uint8_t scale[9] = {0, 0xff, 0x55, 0, 0x11, 0, 0, 0, 0x01};
  for (uint32_t x = 0; x < width; x++, out += step) {
    if (h.color == 3) {
      const uint16_t idx = sample(row, x, h.depth);
      if (idx < png.pal_n) {
        std::memcpy(out, png.pal[idx], 4);
      } else {
        out[0] = out[1] = out[2] = 0;  // stb reads an unset palette slot here (undefined); fixed to opaque black
        out[3] = 255;
      }
      continue;
    }
    const int ch = h.channels;
    uint16_t s[4];
    for (int c = 0; c < ch; c++) s[c] = sample(row, (size_t)x * ch + c, h.depth);
    auto to8 = [&](uint16_t v) -> uint8_t {
      if (h.depth == 16) return (uint8_t)(v >> 8);
      return (uint8_t)(v * scale[h.depth]);
    };
    if (ch <= 2) {
      const uint8_t g = to8(s[0]);
      out[0] = out[1] = out[2] = g;
      if (ch == 2) out[3] = to8(s[1]);
      else if (!png.has_trns) out[3] = 255;
      else if (h.depth == 16) out[3] = s[0] == png.key[0] ? 0 : 255;
      else out[3] = g == (uint8_t)((png.key[0] & 255) * scale[h.depth]) ? 0 : 255;  // stb's scaled key
    } else {
      out[0] = to8(s[0]);
      out[1] = to8(s[1]);
      out[2] = to8(s[2]);
      if (ch == 4) {
        out[3] = to8(s[3]);
      } else if (png.has_trns) {
        const bool m = h.depth == 16 ? (s[0] == png.key[0] && s[1] == png.key[1] && s[2] == png.key[2])
                                     : (s[0] == (png.key[0] & 255) && s[1] == (png.key[1] & 255) &&
                                        s[2] == (png.key[2] & 255));
        out[3] = m ? 0 : 255;
      } else {
        out[3] = 255;
      }
    }
  }
}

size_t row_bytes(uint32_t width, const Header& h) {
  return ((size_t)width * h.channels * h.depth + 7) / 8;
}

}  // namespace

extern "C" {

int sfrt_png_info(const uint8_t* data, int64_t len, int* width, int* height) {
  if (!width || !height) return SFRT_E_INVALID;
  Png png;
  const int rc = parse(data, len, png, true);
  if (rc) return rc;
  *width = (int)png.hd.w;
  *height = (int)png.hd.h;
  return SFRT_OK;
}

int sfrt_png_decode(const uint8_t* data, int64_t len, uint8_t* rgba, int64_t capacity,
                    int* width, int* height) {
  if (!rgba || !width || !height) return SFRT_E_INVALID;
  Png png;
  int rc = parse(data, len, png, false);
  if (rc) return rc;
  const Header& h = png.hd;
  if ((int64_t)h.w * h.h * 4 > capacity) return SFRT_E_INVALID;
  const int bpp = (h.channels * h.depth + 7) / 8;
  // Adam7 passes: (x0, y0, dx, dy); one pass covering everything when not interlaced.
  static const int adam7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                  {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
  const int npass = h.interlace ? 7 : 1;
  size_t total = 0;
  uint32_t pw[7], ph[7];
  for (int p = 0; p < npass; p++) {
    const int x0 = h.interlace ? adam7[p][0] : 0, y0 = h.interlace ? adam7[p][1] : 0;
    const int dx = h.interlace ? adam7[p][2] : 1, dy = h.interlace ? adam7[p][3] : 1;
    pw[p] = h.w > (uint32_t)x0 ? (h.w - x0 + dx - 1) / dx : 0;
    ph[p] = h.h > (uint32_t)y0 ? (h.h - y0 + dy - 1) / dy : 0;
    if (pw[p] && ph[p]) total += (size_t)ph[p] * (row_bytes(pw[p], h) + 1);
  }
  std::vector<uint8_t> raw(total);
  uLongf got = (uLongf)total;
  if (uncompress(raw.data(), &got, png.idat.data(), (uLong)png.idat.size()) != Z_OK ||
      got != total)
    return SFRT_E_INVALID;
  std::vector<uint8_t> img((size_t)h.w * h.h * 4);
  std::vector<uint8_t> rows;
  size_t off = 0;
  for (int p = 0; p < npass; p++) {
    if (!pw[p] || !ph[p]) continue;
    const size_t stride = row_bytes(pw[p], h);
    if (!unfilter(raw.data() + off, ph[p], stride, bpp, rows)) return SFRT_E_INVALID;
    off += (size_t)ph[p] * (stride + 1);
    const int x0 = h.interlace ? adam7[p][0] : 0, y0 = h.interlace ? adam7[p][1] : 0;
    const int dx = h.interlace ? adam7[p][2] : 1, dy = h.interlace ? adam7[p][3] : 1;
    for (uint32_t y = 0; y < ph[p]; y++)
      expand_row(png, rows.data() + (size_t)y * stride, pw[p],
                 img.data() + (((size_t)(y0 + y * dy)) * h.w + x0) * 4, (size_t)dx * 4);
  }
  std::memcpy(rgba, img.data(), img.size());
  *width = (int)h.w;
  *height = (int)h.h;
  return SFRT_OK;
}

}  // extern "C"
