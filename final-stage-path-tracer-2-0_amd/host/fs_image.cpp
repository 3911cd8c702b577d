// fs_image.cpp — BMP and OpenEXR texture loaders (see fs_image.h).
#include "fs_image.h"

#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>

namespace base {

// ============================================================================
// BMP — bitmap.cpp:40-104
// ============================================================================
namespace {
#pragma pack(push, 2)
struct BmpFileHeader {  // PTCX_BITMAP_FILE_HEADER (bitmap.cpp:13-20)
  uint16_t type;
  uint32_t size;
  uint16_t reserved[2];
  uint32_t off_bits;
};
struct BmpInfoHeader {  // PTCX_BITMAP_INFO_HEADER (bitmap.cpp:22-35)
  uint32_t size;
  int32_t width;
  int32_t height;
  uint16_t planes;
  uint16_t bit_count;
  uint32_t compression;
  uint32_t size_image;
  int32_t x_pels_per_meter;
  int32_t y_pels_per_meter;
  uint32_t clr_used;
  uint32_t clr_important;
};
#pragma pack(pop)
static_assert(sizeof(BmpFileHeader) == 14 && sizeof(BmpInfoHeader) == 40, "BMP header layout");

uint32_t greater_multiple(uint32_t value, uint32_t multiple) {  // scalar.h:196-204
  uint32_t mod = value % multiple;
  if (mod) value += multiple - mod;
  return value;
}
}  // namespace

bool LoadBitmap(const std::string& filename, std::vector<float>* output, uint32_t* width, uint32_t* height) {
  if (filename.empty() || !output) return false;
  std::printf("Loading bitmap file: %s.\n", filename.c_str());
  BmpFileHeader fh;
  BmpInfoHeader ih;
  std::ifstream in(filename, std::ios::in | std::ios::binary);
  if (!in.read(reinterpret_cast<char*>(&fh), sizeof(fh))) {
    std::printf("Failed to read bitmap file header for file %s.\n", filename.c_str());
    return false;
  }
  if (!in.read(reinterpret_cast<char*>(&ih), sizeof(ih))) {
    std::printf("Failed to read bitmap info header for file %s.\n", filename.c_str());
    return false;
  }
  if (ih.bit_count != 24) {
    std::printf("Unsupported bitmap file type for file %s.\n", filename.c_str());
    return false;
  }
  // The reference sizes the buffer from int32 dimensions; a negative or zero
  // product is rejected here instead of being handed to vector::resize.
  int64_t n = (int64_t)ih.width * ih.height * 3;
  if (ih.width <= 0 || ih.height <= 0 || n > (int64_t)0x7FFFFFFF) return false;
  output->assign((size_t)n, 0.0f);
  *width = (uint32_t)ih.width;
  *height = (uint32_t)ih.height;
  // Pixel rows follow the 54 header bytes directly: off_bits is not used.
  uint32_t row_stride = (uint32_t)ih.width * 3;
  uint32_t pad = greater_multiple(row_stride, 4) - row_stride;
  std::vector<uint8_t> row(row_stride);
  for (uint32_t i = 0; i < (uint32_t)ih.height; i++) {
    if (!in.read(reinterpret_cast<char*>(row.data()), row_stride)) return false;
    uint32_t dummy = 0;
    if (!in.read(reinterpret_cast<char*>(&dummy), pad)) return false;
    for (uint32_t j = 0; j < (uint32_t)ih.width; j++) {  // BGR -> RGB
      (*output)[i * row_stride + j * 3 + 0] = row[j * 3 + 2] / 255.0f;
      (*output)[i * row_stride + j * 3 + 1] = row[j * 3 + 1] / 255.0f;
      (*output)[i * row_stride + j * 3 + 2] = row[j * 3 + 0] / 255.0f;
    }
  }
  return true;
}

// ============================================================================
// OpenEXR — the LoadEXR path of tiny_exr_loader.h
// ============================================================================
namespace {
constexpr int kSuccess = 0, kInvalidMagic = -1, kInvalidVersion = -2, kInvalidArgument = -3, kInvalidData = -4,
              kCantOpen = -6, kUnsupportedFormat = -7, kInvalidHeader = -8, kUnsupportedFeature = -9;
constexpr int kUint = 0, kHalf = 1, kFloat = 2;                 // TINYEXR_PIXELTYPE_*
constexpr int kNone = 0, kRle = 1, kZips = 2, kZip = 3, kPiz = 4;  // TINYEXR_COMPRESSIONTYPE_*

struct Channel {
  std::string name;
  int pixel_type = 0;
};
struct Header {
  std::vector<Channel> channels;
  int compression = -1;
  int data_window[4] = {0, 0, 0, 0};
  int line_order = 0;
  bool tiled = false;
  int tile_x = 0, tile_y = 0, tile_level_mode = 0;
};

thread_local std::string g_exr_err;
int exr_fail(const char** err, int code, const std::string& msg) {
  g_exr_err = msg;
  if (err) *err = g_exr_err.c_str();
  return code;
}

template <class T>
T rd(const uint8_t* p) {  // little-endian file, little-endian host
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

// FP16 -> FP32 (tinyexr half_to_float, IEEE binary16 semantics).
float half_to_float(uint16_t h) {
  uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1F, m = h & 0x3FF, bits;
  if (e == 0) {
    if (m == 0) {
      bits = s;
    } else {  // subnormal: normalise
      int shift = 0;
      while (!(m & 0x400)) {
        m <<= 1;
        shift++;
      }
      m &= 0x3FF;
      bits = s | ((uint32_t)(127 - 15 - shift + 1) << 23) | (m << 13);
    }
  } else if (e == 31) {
    bits = s | 0x7F800000u | (m << 13);
  } else {
    bits = s | ((e - 15 + 127) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

// Predictor + byte reorder shared by ZIP and RLE (DecompressZip/Rle).
void undo_predictor_reorder(std::vector<uint8_t>& tmp, uint8_t* dst) {
  size_t n = tmp.size();
  for (size_t i = 1; i < n; i++) tmp[i] = (uint8_t)((int)tmp[i - 1] + (int)tmp[i] - 128);
  const uint8_t* t1 = tmp.data();
  const uint8_t* t2 = tmp.data() + (n + 1) / 2;
  size_t k = 0;
  for (;;) {
    if (k < n) dst[k++] = *t1++;
    else break;
    if (k < n) dst[k++] = *t2++;
    else break;
  }
}
bool decompress_zip(uint8_t* dst, size_t dst_len, const uint8_t* src, size_t src_len) {
  if (dst_len == src_len) {  // stored uncompressed (tinyexr issue 40)
    std::memcpy(dst, src, src_len);
    return true;
  }
  std::vector<uint8_t> tmp(dst_len);
  uLongf out = (uLongf)dst_len;
  if (uncompress(tmp.data(), &out, src, (uLong)src_len) != Z_OK) return false;
  tmp.resize(out);
  if (out != dst_len) tmp.resize(dst_len, 0);
  undo_predictor_reorder(tmp, dst);
  return true;
}
bool decompress_rle(uint8_t* dst, size_t dst_len, const uint8_t* src, size_t src_len) {
  if (dst_len == src_len) {
    std::memcpy(dst, src, src_len);
    return true;
  }
  std::vector<uint8_t> tmp(dst_len);
  // rleUncompress (OpenEXR ImfRle): negative count = literal run, else count+1 repeats
  const int8_t* in = reinterpret_cast<const int8_t*>(src);
  long in_len = (long)src_len, max_len = (long)dst_len;
  uint8_t* out = tmp.data();
  while (in_len > 0) {
    if (*in < 0) {
      int count = -(int)(*in++);
      in_len -= count + 1;
      if (0 > (max_len -= count)) return false;
      std::memcpy(out, in, (size_t)count);
      out += count;
      in += count;
    } else {
      int count = *in++;
      in_len -= 2;
      if (0 > (max_len -= count + 1)) return false;
      std::memset(out, *reinterpret_cast<const uint8_t*>(in), (size_t)count + 1);
      out += count + 1;
      in++;
    }
  }
  if ((size_t)(out - tmp.data()) != dst_len) return false;
  undo_predictor_reorder(tmp, dst);
  return true;
}

int type_size(int t) { return t == kHalf ? 2 : 4; }

// ---- PIZ: tinyexr's DecompressPiz (tiny_exr_loader.h:9303-9415), the
// OpenEXR PIZ scheme: a bitmap of the 16-bit values that occur and its
// reverse lookup table (:9155-9173), a canonical Huffman code with run
// lengths (:8201-9110), and a 2D Haar wavelet per channel layer
// (:7909-8187). Restated from those routines; the Huffman decoder keeps
// their table layout (14-bit primary table, long codes listed per entry)
// and their error points, and, as tinyexr does, the decoder's failures
// are not fatal: the buffer keeps what was decoded (DecompressPiz only
// fails on a bad bitmap range).
//
// The decoder below (wav2_decode in particular) is derived from tinyexr,
// which carries OpenEXR's PIZ code; both notices apply:
//
//   Copyright (c) 2014 - 2018, Syoyo Fujita and many contributors.
//   Copyright (c) 2002, Industrial Light & Magic, a division of Lucas
//   Digital Ltd. LLC. All rights reserved.
//   Redistribution and use in source and binary forms, with or without
//   modification, are permitted provided that the following conditions are
//   met:
//   * Redistributions of source code must retain the above copyright
//     notice, this list of conditions and the following disclaimer.
//   * Redistributions in binary form must reproduce the above copyright
//     notice, this list of conditions and the following disclaimer in the
//     documentation and/or other materials provided with the distribution.
//   * Neither the name of Syoyo Fujita / Industrial Light & Magic nor the
//     names of its contributors may be used to endorse or promote products
//     derived from this software without specific prior written permission.
//   THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS
//   IS" AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO,
//   THE IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A PARTICULAR
//   PURPOSE ARE DISCLAIMED. IN NO EVENT SHALL THE COPYRIGHT OWNER OR
//   CONTRIBUTORS BE LIABLE FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL,
//   EXEMPLARY, OR CONSEQUENTIAL DAMAGES (INCLUDING, BUT NOT LIMITED TO,
//   PROCUREMENT OF SUBSTITUTE GOODS OR SERVICES; LOSS OF USE, DATA, OR
//   PROFITS; OR BUSINESS INTERRUPTION) HOWEVER CAUSED AND ON ANY THEORY OF
//   LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY, OR TORT (INCLUDING
//   NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE OF THIS
//   SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
namespace piz {
constexpr int kEncSize = (1 << 16) + 1;  // HUF_ENCSIZE
constexpr int kDecBits = 14, kDecSize = 1 << kDecBits, kDecMask = kDecSize - 1;
constexpr int kShortZeroRun = 59, kLongZeroRun = 63;
constexpr int kShortestLongRun = 2 + kLongZeroRun - kShortZeroRun;
constexpr int kBitmapSize = (1 << 16) >> 3;

struct Bits {  // MSB-first bit reader over [p, end); reads past the end give zero bytes
  const uint8_t* p;
  const uint8_t* end;
  uint64_t c = 0;
  int lc = 0;
  void byte() {
    c = (c << 8) | (p < end ? *p : 0u);
    p++;
    lc += 8;
  }
  uint64_t take(int n) {  // getBits
    while (lc < n) byte();
    lc -= n;
    return (c >> lc) & ((1ull << n) - 1);
  }
};

// hufUnpackEncTable + hufCanonicalCodeTable: code lengths for [im, iM] with
// zero runs, then canonical codes (hcode = length | code << 6).
bool unpack_table(Bits& b, const uint8_t* start, long ni, int im, int iM, std::vector<uint64_t>& hcode) {
  std::fill(hcode.begin(), hcode.end(), 0);
  for (; im <= iM; im++) {
    if (b.p - start > ni) return false;
    uint64_t l = hcode[im] = b.take(6);
    if (l == (uint64_t)kLongZeroRun) {
      if (b.p - start > ni) return false;
      int zerun = (int)b.take(8) + kShortestLongRun;
      if (im + zerun > iM + 1) return false;
      while (zerun--) hcode[im++] = 0;
      im--;
    } else if (l >= (uint64_t)kShortZeroRun) {
      int zerun = (int)l - kShortZeroRun + 2;
      if (im + zerun > iM + 1) return false;
      while (zerun--) hcode[im++] = 0;
      im--;
    }
  }
  uint64_t n[59] = {0};
  for (int i = 0; i < kEncSize; i++) n[hcode[i]]++;  // lengths are < 59 here
  uint64_t c = 0;
  for (int l = 58; l > 0; l--) {  // lowest code of each length, longest first
    uint64_t nc = (c + n[l]) >> 1;
    n[l] = c;
    c = nc;
  }
  for (int i = 0; i < kEncSize; i++) {
    uint64_t l = hcode[i];
    if (l > 0) hcode[i] = l | (n[l]++ << 6);
  }
  return true;
}

struct DecEntry {
  int len = 0;            // short code: its length
  int lit = 0;            // short code: the symbol
  std::vector<int> longs; // symbols of the long codes whose top 14 bits index this entry
};

// hufBuildDecTable
bool build_dec(const std::vector<uint64_t>& hcode, int im, int iM, std::vector<DecEntry>& dec) {
  for (; im <= iM; im++) {
    const uint64_t c = hcode[im] >> 6;
    const int l = (int)(hcode[im] & 63);
    if (c >> l) return false;
    if (l > kDecBits) {
      DecEntry& e = dec[c >> (l - kDecBits)];
      if (e.len) return false;
      e.longs.push_back(im);
    } else if (l) {
      const uint64_t first = c << (kDecBits - l);
      for (uint64_t i = 0; i < (1ull << (kDecBits - l)); i++) {
        DecEntry& e = dec[first + i];
        if (e.len || !e.longs.empty()) return false;
        e.len = l;
        e.lit = im;
      }
    }
  }
  return true;
}

// getCode: a symbol, or (the run-length pseudo-symbol rlc) an 8-bit count of
// repeats of the previous output value.
bool emit(int sym, int rlc, Bits& b, const uint8_t* in_end, uint16_t*& out, const uint16_t* ob, const uint16_t* oe) {
  if (sym == rlc) {
    if (b.lc < 8) {
      if (b.p + 1 >= in_end) return false;
      b.byte();
    }
    b.lc -= 8;
    uint8_t cs = (uint8_t)(b.c >> b.lc);
    if (out + cs > oe) return false;
    if (out - 1 <= ob) return false;  // (tinyexr: a run needs two earlier values)
    const uint16_t v = out[-1];
    while (cs-- > 0) *out++ = v;
  } else if (out < oe) {
    *out++ = (uint16_t)sym;
  } else {
    return false;
  }
  return true;
}

// hufDecode over ni bits
bool decode(const std::vector<uint64_t>& hcode, const std::vector<DecEntry>& dec, const uint8_t* in, long ni, int rlc,
            uint16_t* out, size_t no) {
  Bits b{in, in + (ni + 7) / 8};
  const uint8_t* ie = b.end;
  uint16_t* const ob = out;
  const uint16_t* oe = out + no;
  while (b.p < ie) {
    b.byte();
    while (b.lc >= kDecBits) {
      const DecEntry& e = dec[(b.c >> (b.lc - kDecBits)) & kDecMask];
      if (e.len) {
        b.lc -= e.len;
        if (!emit(e.lit, rlc, b, ie, out, ob, oe)) return false;
      } else {
        if (e.longs.empty()) return false;
        size_t j = 0;
        for (; j < e.longs.size(); j++) {
          const int l = (int)(hcode[e.longs[j]] & 63);
          while (b.lc < l && b.p < ie) b.byte();
          if (b.lc >= l && (hcode[e.longs[j]] >> 6) == ((b.c >> (b.lc - l)) & ((1ull << l) - 1))) {
            b.lc -= l;
            if (!emit(e.longs[j], rlc, b, ie, out, ob, oe)) return false;
            break;
          }
        }
        if (j == e.longs.size()) return false;
      }
    }
  }
  const int i = (int)((8 - ni) & 7);  // the padding bits of the last byte
  b.c >>= i;
  b.lc -= i;
  while (b.lc > 0) {
    const DecEntry& e = dec[(b.c << (kDecBits - b.lc)) & kDecMask];
    if (!e.len) return false;
    b.lc -= e.len;
    if (!emit(e.lit, rlc, b, ie, out, ob, oe)) return false;
  }
  return (size_t)(out - ob) == no;
}

// hufUncompress; its callers ignore the result, and so do we.
void huf_uncompress(const uint8_t* comp, long n_comp, std::vector<uint16_t>& raw) {
  if (n_comp < 20) return;
  const int im = (int)rd<uint32_t>(comp), iM = (int)rd<uint32_t>(comp + 4);
  const int n_bits = (int)rd<uint32_t>(comp + 12);
  if (im < 0 || im >= kEncSize || iM < 0 || iM >= kEncSize) return;
  std::vector<uint64_t> hcode(kEncSize);
  Bits b{comp + 20, comp + n_comp};
  // (a table that fails to unpack leaves the data pointer at the table)
  const uint8_t* data = unpack_table(b, comp + 20, n_comp - 20, im, iM, hcode) ? b.p : comp + 20;
  if (n_bits < 0 || (long)n_bits > 8 * (n_comp - (long)(data - comp))) return;
  std::vector<DecEntry> dec(kDecSize);
  build_dec(hcode, im, iM, dec);
  decode(hcode, dec, data, n_bits, iM, raw.data(), raw.size());
}

// wdec14 / wdec16: one inverse Haar step (14-bit without, 16-bit with modulo
// arithmetic)
inline void wdec14(uint16_t l, uint16_t h, uint16_t& a, uint16_t& b) {
  const int hi = (int16_t)h;
  const int ai = (int16_t)l + (hi & 1) + (hi >> 1);
  a = (uint16_t)(int16_t)ai;
  b = (uint16_t)(int16_t)(ai - hi);
}
inline void wdec16(uint16_t l, uint16_t h, uint16_t& a, uint16_t& b) {
  const int m = l, d = h;
  const int bb = (m - (d >> 1)) & 0xFFFF;
  const int aa = (d + bb - (1 << 15)) & 0xFFFF;
  b = (uint16_t)bb;
  a = (uint16_t)aa;
}

// wav2Decode: the 2D inverse transform of one layer (nx x ny values at
// strides ox, oy), coarsest level first.
void wav2_decode(uint16_t* in, int nx, int ox, int ny, int oy, uint16_t mx) {
  const bool w14 = mx < (1 << 14);
  auto dec = [w14](uint16_t l, uint16_t h, uint16_t& a, uint16_t& b) {
    if (w14)
      wdec14(l, h, a, b);
    else
      wdec16(l, h, a, b);
  };
  const int n = nx > ny ? ny : nx;
  int p = 1;
  while (p <= n) p <<= 1;
  p >>= 1;
  int p2 = p;
  p >>= 1;
  while (p >= 1) {
    uint16_t* py = in;
    uint16_t* const ey = in + (ptrdiff_t)oy * (ny - p2);
    const int oy1 = oy * p, oy2 = oy * p2, ox1 = ox * p, ox2 = ox * p2;
    uint16_t i00, i01, i10, i11;
    for (; py <= ey; py += oy2) {
      uint16_t* px = py;
      uint16_t* const ex = py + (ptrdiff_t)ox * (nx - p2);
      for (; px <= ex; px += ox2) {
        uint16_t* p01 = px + ox1;
        uint16_t* p10 = px + oy1;
        uint16_t* p11 = p10 + ox1;
        dec(*px, *p10, i00, i10);
        dec(*p01, *p11, i01, i11);
        dec(i00, i01, *px, *p01);
        dec(i10, i11, *p10, *p11);
      }
      if (nx & p) {  // odd column
        uint16_t* p10 = px + oy1;
        dec(*px, *p10, i00, *p10);
        *px = i00;
      }
    }
    if (ny & p) {  // odd line
      uint16_t* px = py;
      uint16_t* const ex = py + (ptrdiff_t)ox * (nx - p2);
      for (; px <= ex; px += ox2) {
        uint16_t* p01 = px + ox1;
        dec(*px, *p01, i00, *p01);
        *px = i00;
      }
    }
    p2 = p;
    p >>= 1;
  }
}
}  // namespace piz

// DecompressPiz: dst_len bytes of `num_lines` lines of `width` pixels, the
// channels planar per line as the other codecs produce them.
bool decompress_piz(uint8_t* dst, size_t dst_len, const uint8_t* src, size_t src_len, const std::vector<Channel>& chans,
                    int width, int num_lines) {
  if (src_len == dst_len) {  // stored uncompressed (tinyexr issue 40)
    std::memcpy(dst, src, src_len);
    return true;
  }
  if (src_len < 4) return false;
  const uint16_t min_nz = rd<uint16_t>(src), max_nz = rd<uint16_t>(src + 2);
  const uint8_t* ptr = src + 4;
  if (max_nz >= piz::kBitmapSize) return false;
  std::vector<uint8_t> bitmap(piz::kBitmapSize, 0);
  if (min_nz <= max_nz) {
    const size_t n = (size_t)(max_nz - min_nz + 1);
    if ((size_t)(ptr - src) + n > src_len) return false;
    std::memcpy(bitmap.data() + min_nz, ptr, n);
    ptr += n;
  }
  // reverseLutFromBitmap: lut[k] = the k-th value present (0 always is)
  std::vector<uint16_t> lut(1 << 16, 0);
  int k = 0;
  for (int i = 0; i < (1 << 16); i++)
    if (i == 0 || (bitmap[i >> 3] & (1 << (i & 7)))) lut[k++] = (uint16_t)i;
  const uint16_t max_value = (uint16_t)(k - 1);
  if ((size_t)(ptr - src) + 4 > src_len) return false;
  const int32_t length = rd<int32_t>(ptr);
  ptr += 4;
  // tinyexr sizes the 16-bit buffer in bytes (twice the values it holds);
  // the Huffman stream fills the first half.
  std::vector<uint16_t> tmp(dst_len, 0);
  const long avail = (long)(src_len - (size_t)(ptr - src));
  piz::huf_uncompress(ptr, std::min<long>(length, avail), tmp);
  // per channel: size/2 interleaved 16-bit layers of nx x ny values
  uint16_t* at = tmp.data();
  std::vector<uint16_t*> starts(chans.size());
  std::vector<int> layers(chans.size());
  for (size_t c = 0; c < chans.size(); c++) {
    layers[c] = type_size(chans[c].pixel_type) / 2;
    starts[c] = at;
    at += (size_t)width * num_lines * layers[c];
  }
  for (size_t c = 0; c < chans.size(); c++)
    for (int j = 0; j < layers[c]; j++)
      piz::wav2_decode(starts[c] + j, width, layers[c], num_lines, width * layers[c], max_value);
  for (uint16_t& v : tmp) v = lut[v];  // applyLut over the whole buffer
  uint8_t* out = dst;
  std::vector<uint16_t*> cur(starts);
  for (int y = 0; y < num_lines; y++)
    for (size_t c = 0; c < chans.size(); c++) {
      const size_t n = (size_t)width * layers[c];
      std::memcpy(out, cur[c], n * 2);
      out += n * 2;
      cur[c] += n;
    }
  return true;
}

// DecodePixelData: one block of `num_lines` lines, `width` pixels, into the
// per-channel float planes (HALF converted; UINT bits kept, as LoadEXR later
// reads every plane as float). Rows follow tinyexr's line_order handling.
bool decode_block(const Header& h, std::vector<std::vector<float>>& planes, const uint8_t* data, size_t data_len,
                  int width, int height, int x_stride, int line_no, int num_lines) {
  size_t pixel_size = 0;
  std::vector<size_t> off(h.channels.size());
  for (size_t c = 0; c < h.channels.size(); c++) {
    off[c] = pixel_size;
    pixel_size += (size_t)type_size(h.channels[c].pixel_type);
  }
  size_t raw_len = (size_t)width * num_lines * pixel_size;
  std::vector<uint8_t> raw(raw_len);
  if (h.compression == kNone) {
    if (data_len < raw_len) return false;
    std::memcpy(raw.data(), data, raw_len);
  } else if (h.compression == kZip || h.compression == kZips) {
    if (!decompress_zip(raw.data(), raw_len, data, data_len)) return false;
  } else if (h.compression == kRle) {
    if (!decompress_rle(raw.data(), raw_len, data, data_len)) return false;
  } else if (h.compression == kPiz) {
    if (!decompress_piz(raw.data(), raw_len, data, data_len, h.channels, width, num_lines)) return false;
  } else {
    return false;
  }
  for (size_t c = 0; c < h.channels.size(); c++) {
    int t = h.channels[c].pixel_type;
    for (int v = 0; v < num_lines; v++) {
      const uint8_t* line = raw.data() + (size_t)v * pixel_size * width + off[c] * width;
      size_t row = h.line_order == 0 ? (size_t)(line_no + v) : (size_t)(height - 1 - (line_no + v));
      float* dst = planes[c].data() + row * (size_t)x_stride;
      for (int u = 0; u < width; u++) {
        if (t == kHalf) {
          dst[u] = half_to_float(rd<uint16_t>(line + 2 * u));
        } else {
          uint32_t bits = rd<uint32_t>(line + 4 * u);
          std::memcpy(&dst[u], &bits, 4);
        }
      }
    }
  }
  return true;
}

int parse_header(const uint8_t* p, size_t size, size_t* pos, Header* h, const char** err) {
  bool has_channels = false, has_compression = false, has_dw = false;
  size_t i = *pos;
  for (;;) {
    if (i >= size) return exr_fail(err, kInvalidHeader, "Insufficient data size for attributes.");
    if (p[i] == 0) {  // end of header
      i++;
      break;
    }
    std::string name, type;
    while (i < size && p[i]) name.push_back((char)p[i++]);
    i++;
    while (i < size && p[i]) type.push_back((char)p[i++]);
    i++;
    if (i + 4 > size) return exr_fail(err, kInvalidHeader, "Insufficient data size for attributes.");
    uint32_t len = rd<uint32_t>(p + i);
    i += 4;
    if (i + len > size) return exr_fail(err, kInvalidHeader, "Insufficient data size for attributes.");
    const uint8_t* v = p + i;
    if (name == "channels") {
      size_t k = 0;
      while (k < len && v[k]) {
        Channel ch;
        while (k < len && v[k]) ch.name.push_back((char)v[k++]);
        k++;
        if (k + 16 > len) return exr_fail(err, kInvalidHeader, "Invalid channels format.");
        ch.pixel_type = rd<int32_t>(v + k);
        k += 16;  // pixel_type, pLinear + 3 reserved, xSampling, ySampling
        h->channels.push_back(ch);
      }
      has_channels = true;
    } else if (name == "compression" && len >= 1) {
      h->compression = v[0];
      has_compression = true;
    } else if (name == "dataWindow" && len >= 16) {
      for (int k = 0; k < 4; k++) h->data_window[k] = rd<int32_t>(v + 4 * k);
      has_dw = true;
    } else if (name == "lineOrder" && len >= 1) {
      h->line_order = v[0];
    } else if (name == "tiles" && len >= 9) {
      h->tile_x = (int)rd<uint32_t>(v);
      h->tile_y = (int)rd<uint32_t>(v + 4);
      h->tile_level_mode = v[8] & 0x3;
    }
    i += len;
  }
  if (!has_channels || !has_compression || !has_dw)
    return exr_fail(err, kInvalidHeader, "Required attribute (channels/compression/dataWindow) missing.");
  if (h->compression > kPiz) return exr_fail(err, kUnsupportedFormat, "Unsupported compression type.");
  for (const Channel& c : h->channels)
    if (c.pixel_type != kUint && c.pixel_type != kHalf && c.pixel_type != kFloat)
      return exr_fail(err, kInvalidHeader, "Invalid pixel type.");
  *pos = i;
  return kSuccess;
}
}  // namespace

int LoadEXR(float** out_rgba, int* width, int* height, const char* filename, const char** err) {
  if (!out_rgba) return exr_fail(err, kInvalidArgument, "Invalid argument for LoadEXR()");
  FILE* fp = std::fopen(filename, "rb");
  if (!fp) return exr_fail(err, kCantOpen, "Cannot read file " + std::string(filename));
  std::vector<uint8_t> buf;
  {
    uint8_t tmp[65536];
    size_t n;
    while ((n = std::fread(tmp, 1, sizeof(tmp), fp)) > 0) buf.insert(buf.end(), tmp, tmp + n);
    std::fclose(fp);
  }
  const uint8_t* p = buf.data();
  size_t size = buf.size();
  if (size < 8) return exr_fail(err, kInvalidHeader, "Invalid EXR header.");
  static const uint8_t magic[4] = {0x76, 0x2f, 0x31, 0x01};
  if (std::memcmp(p, magic, 4)) return exr_fail(err, kInvalidMagic, "Invalid EXR header.");
  if (p[4] != 2) return exr_fail(err, kInvalidVersion, "Invalid EXR header.");
  Header h;
  h.tiled = (p[5] & 0x2) != 0;
  bool non_image = (p[5] & 0x8) != 0, multipart = (p[5] & 0x10) != 0;
  if (multipart || non_image)
    return exr_fail(err, kInvalidData, "Loading multipart or DeepImage is not supported  in LoadEXR() API");
  size_t pos = 8;
  int rc = parse_header(p, size, &pos, &h, err);
  if (rc) return rc;
  int dw = h.data_window[2] - h.data_window[0] + 1, dh = h.data_window[3] - h.data_window[1] + 1;
  if (dw <= 0 || dh <= 0) return exr_fail(err, kInvalidData, "Invalid data window.");
  size_t nch = h.channels.size();
  // channel indices (LoadEXR, tiny_exr_loader.h:11230-11245)
  int iR = -1, iG = -1, iB = -1, iA = -1;
  for (size_t c = 0; c < nch; c++) {
    const std::string& n = h.channels[c].name;
    if (n == "R") iR = (int)c;
    else if (n == "G") iG = (int)c;
    else if (n == "B") iB = (int)c;
    else if (n == "A") iA = (int)c;
  }
  bool alpha_only = iA == 0 && iR < 0 && iG < 0 && iB < 0;
  std::vector<float> rgba((size_t)4 * dw * dh);
  if (!h.tiled) {
    int lines = h.compression == kZip ? 16 : h.compression == kPiz ? 32 : 1;  // num_scanline_blocks
    int nblocks = dh / lines + (dh % lines ? 1 : 0);
    if (pos + 8ull * nblocks > size) return exr_fail(err, kInvalidData, "Insufficient data size in offset table.");
    std::vector<std::vector<float>> planes(nch, std::vector<float>((size_t)dw * dh, 0.0f));
    for (int b = 0; b < nblocks; b++) {
      uint64_t off = rd<uint64_t>(p + pos + 8ull * b);
      if (off + 8 > size) return exr_fail(err, kInvalidData, "Invalid offset table.");
      int line_no = rd<int32_t>(p + off), len = rd<int32_t>(p + off + 4);
      if (len < 0 || (size_t)len > size - (off + 8)) return exr_fail(err, kInvalidData, "Invalid chunk size.");
      int end = std::min(line_no + lines, h.data_window[3] + 1);
      int num = end - line_no;
      line_no -= h.data_window[1];
      if (num <= 0 || line_no < 0 || line_no + num > dh)
        return exr_fail(err, kInvalidData, "Invalid line number in chunk.");
      if (!decode_block(h, planes, p + off + 8, (size_t)len, dw, dh, dw, line_no, num))
        return exr_fail(err, kInvalidData, "Failed to decode a scanline block.");
    }
    if (alpha_only) {
      for (size_t i = 0; i < (size_t)dw * dh; i++)
        rgba[4 * i] = rgba[4 * i + 1] = rgba[4 * i + 2] = rgba[4 * i + 3] = planes[0][i];
    } else {
      if (iR < 0) return exr_fail(err, kInvalidData, "R channel not found");
      if (iG < 0) return exr_fail(err, kInvalidData, "G channel not found");
      if (iB < 0) return exr_fail(err, kInvalidData, "B channel not found");
      for (size_t i = 0; i < (size_t)dw * dh; i++) {
        rgba[4 * i + 0] = planes[iR][i];
        rgba[4 * i + 1] = planes[iG][i];
        rgba[4 * i + 2] = planes[iB][i];
        rgba[4 * i + 3] = iA >= 0 ? planes[iA][i] : 1.0f;
      }
    }
  } else {
    if (h.tile_x <= 0 || h.tile_y <= 0) return exr_fail(err, kInvalidHeader, "Invalid tile description.");
    if (h.tile_level_mode != 0) return exr_fail(err, kUnsupportedFeature, "Only ONE_LEVEL tiles are supported.");
    int ntx = (dw + h.tile_x - 1) / h.tile_x, nty = (dh + h.tile_y - 1) / h.tile_y;
    int ntiles = ntx * nty;
    if (pos + 8ull * ntiles > size) return exr_fail(err, kInvalidData, "Insufficient data size in offset table.");
    if (alpha_only) return exr_fail(err, kUnsupportedFeature, "Alpha-only tiled images are not supported.");
    if (iR < 0) return exr_fail(err, kInvalidData, "R channel not found");
    if (iG < 0) return exr_fail(err, kInvalidData, "G channel not found");
    if (iB < 0) return exr_fail(err, kInvalidData, "B channel not found");
    std::vector<std::vector<float>> tile(nch, std::vector<float>((size_t)h.tile_x * h.tile_y, 0.0f));
    for (int t = 0; t < ntiles; t++) {
      uint64_t off = rd<uint64_t>(p + pos + 8ull * t);
      if (off + 20 > size) return exr_fail(err, kInvalidData, "Insufficient data size.");
      int tx = rd<int32_t>(p + off), ty = rd<int32_t>(p + off + 4);
      int lx = rd<int32_t>(p + off + 8), ly = rd<int32_t>(p + off + 12);
      int len = rd<int32_t>(p + off + 16);
      if (lx != 0 || ly != 0) return exr_fail(err, kUnsupportedFeature, "Tile levels are not supported.");
      if (len < 4 || (size_t)len > size - (off + 20)) return exr_fail(err, kInvalidData, "Insufficient data length.");
      if (tx < 0 || ty < 0 || tx * h.tile_x >= dw || ty * h.tile_y >= dh)
        return exr_fail(err, kInvalidData, "Invalid tile coordinates.");
      // DecodeTiledPixelData: actual tile extent; rows within the tile follow line_order
      int w = (tx + 1) * h.tile_x >= dw ? dw - tx * h.tile_x : h.tile_x;
      int hh = (ty + 1) * h.tile_y >= dh ? dh - ty * h.tile_y : h.tile_y;
      for (auto& pl : tile) std::fill(pl.begin(), pl.end(), 0.0f);
      if (!decode_block(h, tile, p + off + 20, (size_t)len, w, h.tile_y, h.tile_x, 0, hh))
        return exr_fail(err, kInvalidData, "Failed to decode a tile.");
      for (int j = 0; j < h.tile_y; j++)
        for (int i = 0; i < h.tile_x; i++) {
          int ii = tx * h.tile_x + i, jj = ty * h.tile_y + j;
          if (ii >= dw || jj >= dh) continue;
          size_t idx = (size_t)ii + (size_t)jj * dw, src = (size_t)i + (size_t)j * h.tile_x;
          rgba[4 * idx + 0] = tile[iR][src];
          rgba[4 * idx + 1] = tile[iG][src];
          rgba[4 * idx + 2] = tile[iB][src];
          rgba[4 * idx + 3] = iA >= 0 ? tile[iA][src] : 1.0f;
        }
    }
  }
  *out_rgba = static_cast<float*>(std::malloc(sizeof(float) * rgba.size()));
  std::memcpy(*out_rgba, rgba.data(), sizeof(float) * rgba.size());
  *width = dw;
  *height = dh;
  return kSuccess;
}

}  // namespace base
