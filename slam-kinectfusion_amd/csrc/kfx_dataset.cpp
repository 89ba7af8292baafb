// kfx_dataset.cpp — the reference's DATASET front-end without OpenCV.
//
// depth_sensor::open / getFrame (kfusion/src/depth_sensor.cpp:11-46, 186-196)
// read a directory `<dir>/color/*.png`, `<dir>/depth/*.png` (cv::glob: sorted
// names) and `<dir>/intr.txt`, and hand each frame to kinectfusion::pipeline
// as `imread(color, IMREAD_COLOR)` (8-bit BGR) and
// `imread(depth, IMREAD_UNCHANGED).convertTo(CV_32F)` (millimetres).  This
// file restates those calls: a PNG decoder on zlib (all PNG colour types and
// bit depths, Adam7, CRC-checked) with OpenCV's conversions (16 → 8 bit by the
// high byte, alpha stripped, grey replicated to BGR, palette expanded), and
// the intr.txt parse of depth_sensor.cpp:22-44.  Host code only.
#include <dirent.h>
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "../../include/kfx.h"

namespace kfx {
void set_error_text(const std::string &msg);  // kfx_api.hip: the text kfx_last_error returns
}

namespace {

int fail(int code, const std::string &msg) {
  kfx::set_error_text(msg);
  return code;
}

uint32_t be32(const uint8_t *p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

// A decoded PNG: samples as stored (8 or 16 bit, big-endian order resolved),
// `chan` per pixel in PNG order (grey, grey+alpha, RGB, RGBA; palette expanded
// to RGB(A)).
struct Image {
  int w = 0, h = 0, chan = 0, depth = 0;  // depth: 8 or 16 after expansion
  std::vector<uint16_t> px;               // w*h*chan samples
};

struct PngHeader {
  uint32_t w = 0, h = 0;
  int bit = 0, ctype = 0, interlace = 0;
};

int channels_of(int ctype) {
  switch (ctype) {
    case 0: return 1;
    case 2: return 3;
    case 3: return 1;
    case 4: return 2;
    case 6: return 4;
  }
  return 0;
}

bool valid_depth(int ctype, int bit) {
  switch (ctype) {
    case 0: return bit == 1 || bit == 2 || bit == 4 || bit == 8 || bit == 16;
    case 3: return bit == 1 || bit == 2 || bit == 4 || bit == 8;
    case 2: case 4: case 6: return bit == 8 || bit == 16;
  }
  return false;
}

int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

// Undo the per-scanline filters of one (sub)image in place; `bpp` = bytes per
// complete pixel (>= 1), `stride` = bytes per scanline without the filter byte.
int unfilter(uint8_t *data, size_t rows, size_t stride, size_t bpp, uint8_t *out) {
  std::vector<uint8_t> prev(stride, 0);
  for (size_t y = 0; y < rows; ++y) {
    const uint8_t ft = data[y * (stride + 1)];
    const uint8_t *in = data + y * (stride + 1) + 1;
    uint8_t *cur = out + y * stride;
    for (size_t i = 0; i < stride; ++i) {
      const int a = i >= bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
      int v = in[i];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: v += paeth(a, b, c); break;
        default: return fail(KFX_ERR_ARG, "PNG: bad filter type");
      }
      cur[i] = (uint8_t)v;
    }
    std::memcpy(prev.data(), cur, stride);
  }
  return KFX_OK;
}

// Sample k of a packed scanline at `bit` bits per sample.
int sample_at(const uint8_t *row, size_t k, int bit) {
  if (bit == 8) return row[k];
  if (bit == 16) return (row[2 * k] << 8) | row[2 * k + 1];
  const size_t b = k * bit;
  return (row[b >> 3] >> (8 - bit - (b & 7))) & ((1 << bit) - 1);
}

int decode_png(const std::string &path, Image &img, bool header_only, PngHeader *hdr_out = nullptr) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(KFX_ERR_ARG, "cannot open " + path);
  std::vector<uint8_t> file((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (file.size() < 8 || std::memcmp(file.data(), sig, 8) != 0) return fail(KFX_ERR_ARG, path + ": not a PNG");
  PngHeader h;
  std::vector<uint8_t> idat, plte;
  bool have_hdr = false, done = false;
  size_t pos = 8;
  while (!done) {
    if (pos + 12 > file.size()) return fail(KFX_ERR_ARG, path + ": truncated PNG");
    const uint32_t len = be32(&file[pos]);
    if (len > file.size() - pos - 12) return fail(KFX_ERR_ARG, path + ": truncated PNG chunk");
    const uint8_t *type = &file[pos + 4], *data = &file[pos + 8];
    const uint32_t crc = be32(&file[pos + 8 + len]);
    if ((uint32_t)crc32(crc32(0L, Z_NULL, 0), type, len + 4) != crc)
      return fail(KFX_ERR_ARG, path + ": PNG CRC mismatch");
    const std::string t((const char *)type, 4);
    if (t == "IHDR") {
      if (len != 13) return fail(KFX_ERR_ARG, path + ": bad IHDR");
      h.w = be32(data);
      h.h = be32(data + 4);
      h.bit = data[8];
      h.ctype = data[9];
      h.interlace = data[12];
      if (data[10] != 0 || data[11] != 0 || h.interlace > 1 || !valid_depth(h.ctype, h.bit) ||
          h.w == 0 || h.h == 0 || h.w > (1u << 16) || h.h > (1u << 16))
        return fail(KFX_ERR_ARG, path + ": unsupported PNG header");
      have_hdr = true;
      if (header_only) break;
    } else if (t == "PLTE") {
      plte.assign(data, data + len);
    } else if (t == "IDAT") {
      idat.insert(idat.end(), data, data + len);
    } else if (t == "IEND") {
      done = true;
    } else if (!(type[0] & 0x20)) {
      return fail(KFX_ERR_ARG, path + ": unknown critical PNG chunk " + t);
    }
    pos += 12 + len;
  }
  if (!have_hdr) return fail(KFX_ERR_ARG, path + ": no IHDR");
  if (hdr_out) *hdr_out = h;
  const int spp = channels_of(h.ctype);  // samples per pixel as stored
  img.w = (int)h.w;
  img.h = (int)h.h;
  if (h.ctype == 3) {
    img.chan = 3;
    img.depth = 8;
  } else {
    img.chan = spp;
    img.depth = h.bit == 16 ? 16 : 8;
  }
  if (header_only) return KFX_OK;
  if (h.ctype == 3 && (plte.empty() || plte.size() % 3)) return fail(KFX_ERR_ARG, path + ": bad palette");

  // Adam7 passes (or the whole image once)
  struct Pass { int x0, y0, dx, dy; };
  static const Pass adam7[7] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
  const Pass whole = {0, 0, 1, 1};
  const int npass = h.interlace ? 7 : 1;
  const size_t bits_pp = (size_t)spp * h.bit, bpp = std::max<size_t>(1, bits_pp / 8);
  size_t raw_size = 0;
  for (int p = 0; p < npass; ++p) {
    const Pass &ps = h.interlace ? adam7[p] : whole;
    const size_t pw = (h.w > (uint32_t)ps.x0) ? (h.w - ps.x0 + ps.dx - 1) / ps.dx : 0;
    const size_t ph = (h.h > (uint32_t)ps.y0) ? (h.h - ps.y0 + ps.dy - 1) / ps.dy : 0;
    if (pw && ph) raw_size += ph * (1 + (pw * bits_pp + 7) / 8);
  }
  std::vector<uint8_t> raw(raw_size);
  uLongf out_len = (uLongf)raw_size;
  if (uncompress(raw.data(), &out_len, idat.data(), (uLong)idat.size()) != Z_OK || out_len != raw_size)
    return fail(KFX_ERR_ARG, path + ": bad PNG image data");

  img.px.assign((size_t)img.w * img.h * img.chan, 0);
  size_t off = 0;
  for (int p = 0; p < npass; ++p) {
    const Pass &ps = h.interlace ? adam7[p] : whole;
    const size_t pw = (h.w > (uint32_t)ps.x0) ? (h.w - ps.x0 + ps.dx - 1) / ps.dx : 0;
    const size_t ph = (h.h > (uint32_t)ps.y0) ? (h.h - ps.y0 + ps.dy - 1) / ps.dy : 0;
    if (!pw || !ph) continue;
    const size_t stride = (pw * bits_pp + 7) / 8;
    std::vector<uint8_t> rows(ph * stride);
    int r = unfilter(raw.data() + off, ph, stride, bpp, rows.data());
    if (r) return fail(r, path + ": bad PNG filter type");
    off += ph * (stride + 1);
    for (size_t yy = 0; yy < ph; ++yy) {
      const uint8_t *row = rows.data() + yy * stride;
      const size_t y = ps.y0 + yy * ps.dy;
      for (size_t xx = 0; xx < pw; ++xx) {
        const size_t x = ps.x0 + xx * ps.dx;
        uint16_t *dst = &img.px[(y * img.w + x) * img.chan];
        if (h.ctype == 3) {
          const size_t idx = (size_t)sample_at(row, xx, h.bit);
          if (3 * idx + 2 >= plte.size()) return fail(KFX_ERR_ARG, path + ": palette index out of range");
          for (int c = 0; c < 3; ++c) dst[c] = plte[3 * idx + c];
        } else {
          for (int c = 0; c < spp; ++c) {
            int v = sample_at(row, xx * spp + c, h.bit);
            if (h.bit < 8) v = v * 255 / ((1 << h.bit) - 1);  // libpng expands grey to 8 bit
            dst[c] = (uint16_t)v;
          }
        }
      }
    }
  }
  return KFX_OK;
}

// imread(path, IMREAD_COLOR): 8-bit BGR (16-bit samples keep the high byte,
// alpha stripped, grey replicated).
int to_bgr8(const Image &img, uint8_t *bgr) {
  const size_t n = (size_t)img.w * img.h;
  const int sh = img.depth == 16 ? 8 : 0;
  for (size_t i = 0; i < n; ++i) {
    const uint16_t *s = &img.px[i * img.chan];
    uint8_t r, g, b;
    if (img.chan <= 2) {
      r = g = b = (uint8_t)(s[0] >> sh);
    } else {
      r = (uint8_t)(s[0] >> sh);
      g = (uint8_t)(s[1] >> sh);
      b = (uint8_t)(s[2] >> sh);
    }
    bgr[3 * i] = b;
    bgr[3 * i + 1] = g;
    bgr[3 * i + 2] = r;
  }
  return KFX_OK;
}

// imread(path, IMREAD_UNCHANGED).convertTo(CV_32F) of a one-channel depth map.
int to_depth(const Image &img, float *out, const std::string &path) {
  if (img.chan != 1) return fail(KFX_ERR_ARG, path + ": depth PNG must have one channel");
  const size_t n = (size_t)img.w * img.h;
  for (size_t i = 0; i < n; ++i) out[i] = (float)img.px[i];
  return KFX_OK;
}

std::vector<std::string> glob_png(const std::string &dir) {
  std::vector<std::string> out;
  DIR *d = opendir(dir.c_str());
  if (!d) return out;
  while (dirent *e = readdir(d)) {
    const std::string n = e->d_name;
    if (n.size() > 4 && n.compare(n.size() - 4, 4, ".png") == 0) out.push_back(dir + "/" + n);
  }
  closedir(d);
  std::sort(out.begin(), out.end());  // cv::glob sorts its result
  return out;
}

}  // namespace

struct kfx_dataset {
  std::string dir;
  std::vector<std::string> color, depth;
  kfx_intrinsics intr{};
  int has_intr = 0;
};

extern "C" {

int kfx_png_info(const char *path, int *width, int *height, int *channels, int *bit_depth) {
  if (!path) return fail(KFX_ERR_ARG, "null path");
  Image img;
  PngHeader h;
  int r = decode_png(path, img, true, &h);
  if (r) return r;
  if (width) *width = img.w;
  if (height) *height = img.h;
  if (channels) *channels = channels_of(h.ctype);
  if (bit_depth) *bit_depth = h.bit;
  return KFX_OK;
}

int kfx_png_read_bgr8(const char *path, uint8_t *bgr, int width, int height) {
  if (!path || !bgr) return fail(KFX_ERR_ARG, "null argument");
  Image img;
  int r = decode_png(path, img, false);
  if (r) return r;
  if (img.w != width || img.h != height) return fail(KFX_ERR_ARG, std::string(path) + ": size mismatch");
  return to_bgr8(img, bgr);
}

int kfx_png_read_depth(const char *path, float *depth, int width, int height) {
  if (!path || !depth) return fail(KFX_ERR_ARG, "null argument");
  Image img;
  int r = decode_png(path, img, false);
  if (r) return r;
  if (img.w != width || img.h != height) return fail(KFX_ERR_ARG, std::string(path) + ": size mismatch");
  return to_depth(img, depth, path);
}

int kfx_parse_intr(const char *path, float out5[5]) {
  if (!path || !out5) return fail(KFX_ERR_ARG, "null argument");
  // depth_sensor.cpp:22-35: nine `>>` reads (a failed read stores 0 and
  // leaves the stream failed), keeping the values > 0.1
  std::ifstream f(path);
  if (!f.is_open()) return fail(KFX_ERR_ARG, std::string("cannot open ") + path);
  std::vector<float> v;
  for (int i = 0; i < 9; ++i) {
    float t = 0;
    if (!(f >> t)) t = 0;
    if (t > 0.1f) v.push_back(t);
  }
  if (v.size() != 5) return fail(KFX_ERR_ARG, std::string(path) + ": expected 5 values > 0.1 in the 3x3 matrix");
  std::copy(v.begin(), v.end(), out5);
  return KFX_OK;
}

int kfx_dataset_open(const char *dir, kfx_dataset **out) {
  if (!dir || !out) return fail(KFX_ERR_ARG, "null argument");
  *out = nullptr;
  auto *ds = new kfx_dataset();
  ds->dir = dir;
  ds->color = glob_png(ds->dir + "/color");
  ds->depth = glob_png(ds->dir + "/depth");
  if (ds->color.empty() || ds->depth.empty()) {  // depth_sensor.cpp:17-21 ("no camera")
    delete ds;
    return fail(KFX_ERR_ARG, std::string(dir) + ": no color/*.png or depth/*.png");
  }
  float p[5];
  // 640x480 unless intr.txt gives the camera (depth_sensor.h:37-40, .cpp:36-44)
  ds->intr.width = 640;
  ds->intr.height = 480;
  if (kfx_parse_intr((ds->dir + "/intr.txt").c_str(), p) == KFX_OK) {
    int w = 0, h = 0;
    int r = kfx_png_info(ds->color[0].c_str(), &w, &h, nullptr, nullptr);
    if (r) {
      delete ds;
      return r;
    }
    ds->intr = {w, h, p[0], p[2], p[1], p[3]};  // fx, cx, fy, cy order in the file
    ds->has_intr = 1;
  }
  *out = ds;
  return KFX_OK;
}

int kfx_dataset_info(const kfx_dataset *ds, kfx_intrinsics *intr, int *n_frames, int *has_intr) {
  if (!ds) return fail(KFX_ERR_ARG, "null dataset");
  if (intr) *intr = ds->intr;
  if (n_frames) *n_frames = (int)std::min(ds->color.size(), ds->depth.size());
  if (has_intr) *has_intr = ds->has_intr;
  return KFX_OK;
}

int kfx_dataset_read(const kfx_dataset *ds, int index, uint8_t *bgr, float *depth_mm) {
  if (!ds) return fail(KFX_ERR_ARG, "null dataset");
  const int n = (int)std::min(ds->color.size(), ds->depth.size());
  if (index < 0 || index >= n) return fail(KFX_ERR_ARG, "frame index out of range");
  int r = KFX_OK;
  if (bgr) r = kfx_png_read_bgr8(ds->color[index].c_str(), bgr, ds->intr.width, ds->intr.height);
  if (!r && depth_mm) r = kfx_png_read_depth(ds->depth[index].c_str(), depth_mm, ds->intr.width, ds->intr.height);
  return r;
}

int kfx_dataset_close(kfx_dataset *ds) {
  delete ds;
  return KFX_OK;
}

}  // extern "C"
