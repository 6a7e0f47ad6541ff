// Host-side (CPU) data-pipeline ops for raft_stir_amd, registered as
// torch.ops.raft_stir_host.*  and built into raft_stir_amd/_host.so with g++
// (no GPU dependency, so DataLoader worker processes can use it freely).
//
// The reference's data path (core/utils/frame_utils.py, core/utils/augmentor.py)
// leans on OpenCV + torchvision C++ internals for exactly these primitives;
// neither library exists in this image, so the engine carries its own:
//
//   png_decode(bytes)               8/16-bit gray/GA/RGB/RGBA PNG -> (H,W,C) uint8|int32(16b)
//   png_encode16(img uint16 HxWxC)  -> bytes   (KITTI 16-bit flow PNGs, writeFlowKITTI)
//   resize_bilinear(img, oh, ow)    cv2.INTER_LINEAR semantics (half-pixel centres,
//                                   edge clamp), uint8 (rounded) or float32, HxWxC
//   color_jitter(img u8 HxWx3, b, c, s, h, order[4])
//                                   torchvision ColorJitter-on-PIL semantics with
//                                   the random factors drawn by the caller
//   resize_crop(img, oh, ow, fy, fx, y0, x0, ch, cw, hflip, vflip, mul)
//                                   crop(flip(resize(img))) * mul[c] without the full resize
//   sparse_flow_resize(flow, valid, fx, fy)  scatter-resize of sparse KITTI flow
//                                   (reference core/utils/augmentor.py:161-193)
//
// 16-bit images come back as int32 tensors (torch has no uint16 arithmetic in
// every build); callers cast.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <xmmintrin.h>
#include <vector>

namespace {

// ------------------------------------------------------------------ PNG
uint32_t be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}
void put_be32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back(uint8_t(x >> 24)); v.push_back(uint8_t(x >> 16));
  v.push_back(uint8_t(x >> 8)); v.push_back(uint8_t(x));
}

int paeth(int a, int b, int c) {
  int p = a + b - c;
  int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  if (pb <= pc) return b;
  return c;
}

at::Tensor png_decode(const at::Tensor& data) {
  TORCH_CHECK(data.scalar_type() == at::kByte && data.dim() == 1, "png_decode: 1-D uint8 bytes");
  auto buf = data.contiguous();
  const uint8_t* p = buf.data_ptr<uint8_t>();
  const int64_t n = buf.numel();
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  TORCH_CHECK(n >= 8 && std::memcmp(p, sig, 8) == 0, "png_decode: not a PNG");
  int64_t off = 8;
  uint32_t W = 0, H = 0;
  int depth = 0, ctype = 0, interlace = 0;
  std::vector<uint8_t> idat;
  while (off + 8 <= n) {
    uint32_t len = be32(p + off);
    const uint8_t* type = p + off + 4;
    const uint8_t* body = p + off + 8;
    TORCH_CHECK(off + 12 + int64_t(len) <= n, "png_decode: truncated chunk");
    if (!std::memcmp(type, "IHDR", 4)) {
      TORCH_CHECK(len >= 13, "png_decode: short IHDR");
      W = be32(body); H = be32(body + 4);
      depth = body[8]; ctype = body[9]; interlace = body[12];
    } else if (!std::memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), body, body + len);
    } else if (!std::memcmp(type, "IEND", 4)) {
      break;
    }
    off += 12 + len;
  }
  TORCH_CHECK(W > 0 && H > 0, "png_decode: missing IHDR");
  TORCH_CHECK(interlace == 0, "png_decode: interlaced PNG unsupported");
  TORCH_CHECK(depth == 8 || depth == 16, "png_decode: bit depth ", depth, " unsupported");
  int C;
  switch (ctype) {
    case 0: C = 1; break;
    case 2: C = 3; break;
    case 4: C = 2; break;
    case 6: C = 4; break;
    default: TORCH_CHECK(false, "png_decode: colour type ", ctype, " unsupported (palette?)");
  }
  const int bps = depth / 8;               // bytes per sample
  const int bpp = C * bps;                 // bytes per pixel (filter unit)
  // untrusted header: bound the allocation (and keep every size in 32 bits for zlib)
  TORCH_CHECK(W <= (1u << 16) && H <= (1u << 16) && uint64_t(W) * H * bpp + H <= (uint64_t(1) << 31),
              "png_decode: image ", W, "x", H, " too large");
  const size_t stride = size_t(W) * bpp;
  std::vector<uint8_t> raw((stride + 1) * H);
  z_stream zs{};
  TORCH_CHECK(inflateInit(&zs) == Z_OK, "png_decode: inflateInit");
  zs.next_in = idat.data();
  zs.avail_in = uInt(idat.size());
  zs.next_out = raw.data();
  zs.avail_out = uInt(raw.size());
  int zr = inflate(&zs, Z_FINISH);
  inflateEnd(&zs);
  TORCH_CHECK((zr == Z_STREAM_END || zr == Z_OK || zr == Z_BUF_ERROR) && zs.avail_out == 0,
              "png_decode: corrupt or truncated image data");
  std::vector<uint8_t> img(stride * H);
  for (uint32_t y = 0; y < H; ++y) {
    const uint8_t* src = raw.data() + y * (stride + 1);
    uint8_t* dst = img.data() + y * stride;
    const uint8_t* up = y ? img.data() + (y - 1) * stride : nullptr;
    const int f = src[0];
    ++src;
    for (size_t i = 0; i < stride; ++i) {
      int a = i >= size_t(bpp) ? dst[i - bpp] : 0;
      int b = up ? up[i] : 0;
      int c = (up && i >= size_t(bpp)) ? up[i - bpp] : 0;
      int v = src[i];
      switch (f) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: v += paeth(a, b, c); break;
        default: TORCH_CHECK(false, "png_decode: bad filter ", f);
      }
      dst[i] = uint8_t(v);
    }
  }
  if (depth == 8) {
    auto out = at::empty({int64_t(H), int64_t(W), C}, at::kByte);
    std::memcpy(out.data_ptr<uint8_t>(), img.data(), img.size());
    return out;
  }
  auto out = at::empty({int64_t(H), int64_t(W), C}, at::kInt);
  int32_t* o = out.data_ptr<int32_t>();
  const size_t cnt = size_t(W) * H * C;
  for (size_t i = 0; i < cnt; ++i) o[i] = (int32_t(img[2 * i]) << 8) | img[2 * i + 1];
  return out;
}

void png_chunk(std::vector<uint8_t>& out, const char* type, const uint8_t* body, size_t len) {
  put_be32(out, uint32_t(len));
  size_t start = out.size();
  out.insert(out.end(), type, type + 4);
  out.insert(out.end(), body, body + len);
  uLong crc = crc32(0L, out.data() + start, uInt(len + 4));
  put_be32(out, uint32_t(crc));
}

at::Tensor png_encode16(const at::Tensor& img_in) {
  TORCH_CHECK(img_in.dim() == 3, "png_encode16: HxWxC");
  auto img = img_in.to(at::kInt).contiguous();
  const int64_t H = img.size(0), W = img.size(1), C = img.size(2);
  int ctype = C == 1 ? 0 : C == 2 ? 4 : C == 3 ? 2 : C == 4 ? 6 : -1;
  TORCH_CHECK(ctype >= 0, "png_encode16: C in 1..4");
  const size_t stride = size_t(W) * C * 2;
  std::vector<uint8_t> raw((stride + 1) * H);
  const int32_t* s = img.data_ptr<int32_t>();
  for (int64_t y = 0; y < H; ++y) {
    uint8_t* d = raw.data() + y * (stride + 1);
    d[0] = 0;  // filter: none
    for (int64_t i = 0; i < W * C; ++i) {
      int32_t v = std::min<int32_t>(65535, std::max<int32_t>(0, s[y * W * C + i]));
      d[1 + 2 * i] = uint8_t(v >> 8);
      d[2 + 2 * i] = uint8_t(v & 255);
    }
  }
  uLongf zcap = compressBound(uLong(raw.size()));
  std::vector<uint8_t> z(zcap);
  TORCH_CHECK(compress2(z.data(), &zcap, raw.data(), uLong(raw.size()), 6) == Z_OK,
              "png_encode16: deflate failed");
  std::vector<uint8_t> out = {137, 80, 78, 71, 13, 10, 26, 10};
  uint8_t ihdr[13];
  ihdr[0] = uint8_t(W >> 24); ihdr[1] = uint8_t(W >> 16); ihdr[2] = uint8_t(W >> 8); ihdr[3] = uint8_t(W);
  ihdr[4] = uint8_t(H >> 24); ihdr[5] = uint8_t(H >> 16); ihdr[6] = uint8_t(H >> 8); ihdr[7] = uint8_t(H);
  ihdr[8] = 16; ihdr[9] = uint8_t(ctype); ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
  png_chunk(out, "IHDR", ihdr, 13);
  png_chunk(out, "IDAT", z.data(), zcap);
  png_chunk(out, "IEND", nullptr, 0);
  auto t = at::empty({int64_t(out.size())}, at::kByte);
  std::memcpy(t.data_ptr<uint8_t>(), out.data(), out.size());
  return t;
}

// ------------------------------------------------------- bilinear resize
// cv2.resize(INTER_LINEAR) with explicit output size: sx = in/out,
// src = (dst + 0.5) * sx - 0.5, clamped to [0, in-1].
struct Tap { int i0, i1; float w1; };

std::vector<Tap> taps(int in, int out, double scale_inv) {
  std::vector<Tap> t(out);
  for (int d = 0; d < out; ++d) {
    double s = (d + 0.5) * scale_inv - 0.5;
    int i0 = int(std::floor(s));
    float w1 = float(s - i0);
    if (i0 < 0) { i0 = 0; w1 = 0.f; }
    if (i0 >= in - 1) { i0 = in - 1; w1 = 0.f; }
    t[d] = {i0, std::min(i0 + 1, in - 1), w1};
  }
  return t;
}

template <typename T>
void resize_impl(const T* src, T* dst, int H, int W, int C, int OH, int OW, double sy, double sx) {
  auto ty = taps(H, OH, sy), tx = taps(W, OW, sx);
  std::vector<float> row0(size_t(OW) * C), row1(size_t(OW) * C);
  for (int y = 0; y < OH; ++y) {
    const T* r0 = src + size_t(ty[y].i0) * W * C;
    const T* r1 = src + size_t(ty[y].i1) * W * C;
    for (int x = 0; x < OW; ++x) {
      const Tap& t = tx[x];
      for (int c = 0; c < C; ++c) {
        float a0 = float(r0[t.i0 * C + c]), a1 = float(r0[t.i1 * C + c]);
        float b0 = float(r1[t.i0 * C + c]), b1 = float(r1[t.i1 * C + c]);
        row0[x * C + c] = a0 + t.w1 * (a1 - a0);
        row1[x * C + c] = b0 + t.w1 * (b1 - b0);
      }
    }
    const float wy = ty[y].w1;
    T* d = dst + size_t(y) * OW * C;
    for (int i = 0; i < OW * C; ++i) {
      float v = row0[i] + wy * (row1[i] - row0[i]);
      if constexpr (std::is_same<T, uint8_t>::value)
        d[i] = uint8_t(std::min(255.f, std::max(0.f, std::nearbyint(v))));
      else
        d[i] = T(v);
    }
  }
}

at::Tensor resize_bilinear(const at::Tensor& img_in, int64_t OH, int64_t OW, double fy, double fx) {
  TORCH_CHECK(img_in.dim() == 3 || img_in.dim() == 2, "resize_bilinear: HxW[xC]");
  auto img = img_in.dim() == 2 ? img_in.unsqueeze(-1) : img_in;
  img = img.contiguous();
  const int H = int(img.size(0)), W = int(img.size(1)), C = int(img.size(2));
  TORCH_CHECK(OH > 0 && OW > 0, "resize_bilinear: empty output");
  // cv2 uses 1/fx (when given scale factors) or in/out (explicit size) as the map scale.
  const double sy = fy > 0 ? 1.0 / fy : double(H) / OH;
  const double sx = fx > 0 ? 1.0 / fx : double(W) / OW;
  at::Tensor out;
  if (img.scalar_type() == at::kByte) {
    out = at::empty({OH, OW, C}, at::kByte);
    resize_impl<uint8_t>(img.data_ptr<uint8_t>(), out.data_ptr<uint8_t>(), H, W, C, int(OH), int(OW), sy, sx);
  } else {
    img = img.to(at::kFloat);
    out = at::empty({OH, OW, C}, at::kFloat);
    resize_impl<float>(img.data_ptr<float>(), out.data_ptr<float>(), H, W, C, int(OH), int(OW), sy, sx);
  }
  return img_in.dim() == 2 ? out.squeeze(-1) : out;
}

// ------------------------------------------- fused resize + flip + crop
// crop(flip(resize(img, OH x OW))) [* mul[c]] without materialising the
// resized image: FlowAugmentor.spatial_transform draws the crop offset from the
// resized size, then only the ch x cw window is interpolated (the resize was
// up to 4x the crop's pixels).  Same taps and the same float operations as
// resize_impl, so the window is bitwise equal to slicing the full resize.
// Output row i reads resized row (vflip ? OH-1-(y0+i) : y0+i); likewise columns.
template <typename T>
void resize_crop_impl(const T* src, T* dst, int H, int W, int C, int OH, int OW, double sy, double sx, int y0,
                      int x0, int ch, int cw, bool hflip, bool vflip, const float* mul) {
  auto ty = taps(H, OH, sy), tx = taps(W, OW, sx);
  std::vector<Tap> cx(cw);
  for (int j = 0; j < cw; ++j) cx[j] = tx[hflip ? OW - 1 - (x0 + j) : x0 + j];
  for (int i = 0; i < ch; ++i) {
    const Tap& t = ty[vflip ? OH - 1 - (y0 + i) : y0 + i];
    const T* r0 = src + size_t(t.i0) * W * C;
    const T* r1 = src + size_t(t.i1) * W * C;
    const float wy = t.w1;
    T* d = dst + size_t(i) * cw * C;
    for (int j = 0; j < cw; ++j) {
      const Tap& u = cx[j];
      for (int c = 0; c < C; ++c) {
        const float a0 = float(r0[u.i0 * C + c]), a1 = float(r0[u.i1 * C + c]);
        const float b0 = float(r1[u.i0 * C + c]), b1 = float(r1[u.i1 * C + c]);
        const float h0 = a0 + u.w1 * (a1 - a0);
        const float h1 = b0 + u.w1 * (b1 - b0);
        const float v = h0 + wy * (h1 - h0);
        if constexpr (std::is_same<T, uint8_t>::value)
          d[j * C + c] = uint8_t(std::min(255.f, std::max(0.f, std::nearbyint(v))));
        else
          d[j * C + c] = T(mul ? v * mul[c] : v);
      }
    }
  }
}

at::Tensor resize_crop(const at::Tensor& img_in, int64_t OH, int64_t OW, double fy, double fx, int64_t y0,
                       int64_t x0, int64_t ch, int64_t cw, bool hflip, bool vflip, at::ArrayRef<double> mul) {
  TORCH_CHECK(img_in.dim() == 3, "resize_crop: HxWxC");
  auto img = img_in.contiguous();
  const int H = int(img.size(0)), W = int(img.size(1)), C = int(img.size(2));
  TORCH_CHECK(OH > 0 && OW > 0 && ch > 0 && cw > 0, "resize_crop: empty");
  TORCH_CHECK(y0 >= 0 && x0 >= 0 && y0 + ch <= OH && x0 + cw <= OW, "resize_crop: window outside the resized image");
  TORCH_CHECK(mul.empty() || int64_t(mul.size()) == C, "resize_crop: one multiplier per channel");
  const double sy = fy > 0 ? 1.0 / fy : double(H) / OH;
  const double sx = fx > 0 ? 1.0 / fx : double(W) / OW;
  at::Tensor out;
  if (img.scalar_type() == at::kByte) {
    TORCH_CHECK(mul.empty(), "resize_crop: no multipliers on uint8 images");
    out = at::empty({ch, cw, C}, at::kByte);
    resize_crop_impl<uint8_t>(img.data_ptr<uint8_t>(), out.data_ptr<uint8_t>(), H, W, C, int(OH), int(OW), sy, sx,
                              int(y0), int(x0), int(ch), int(cw), hflip, vflip, nullptr);
  } else {
    img = img.to(at::kFloat);
    std::vector<float> m(mul.begin(), mul.end());
    out = at::empty({ch, cw, C}, at::kFloat);
    resize_crop_impl<float>(img.data_ptr<float>(), out.data_ptr<float>(), H, W, C, int(OH), int(OW), sy, sx,
                            int(y0), int(x0), int(ch), int(cw), hflip, vflip, m.empty() ? nullptr : m.data());
  }
  return out;
}

// ---------------------------------------------------------- colour jitter
// torchvision ColorJitter applied to a PIL RGB image: the four adjustments in
// the order given (0 brightness, 1 contrast, 2 saturation, 3 hue), each a PIL
// operation with uint8 rounding between steps.
inline int rne(float x) { return _mm_cvtss_si32(_mm_set_ss(x)); }  // nearest, ties to even
inline float ffloor(float x) {
  const float t = float(int(x));
  return t > x ? t - 1.f : t;
}
inline uint8_t clip8(float v) { return uint8_t(std::min(255.f, std::max(0.f, v))); }
inline int luma(int r, int g, int b) { return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16; }

void rgb2hsv(int r, int g, int b, int& h, int& s, int& v) {
  // PIL ImagingConvert RGB->HSV (uint8 channels)
  int maxc = std::max(r, std::max(g, b)), minc = std::min(r, std::min(g, b));
  v = maxc;
  if (maxc == minc) { h = 0; s = 0; return; }
  float cr = float(maxc - minc);
  s = int(cr / maxc * 255.f);
  float rc = (maxc - r) / cr, gc = (maxc - g) / cr, bc = (maxc - b) / cr;
  float hf;
  if (r == maxc) hf = bc - gc;
  else if (g == maxc) hf = 2.f + rc - bc;
  else hf = 4.f + gc - rc;
  hf = hf / 6.f;
  hf = hf - std::floor(hf);
  h = int(hf * 255.f);
}

void hsv2rgb(int h, int s, int v, int& r, int& g, int& b) {
  if (s == 0) { r = g = b = v; return; }
  float hf = h / 255.f, sf = s / 255.f;
  int i = int(std::floor(hf * 6.f));
  float f = hf * 6.f - i;
  int p = int(std::nearbyint(v * (1.f - sf)));
  int q = int(std::nearbyint(v * (1.f - sf * f)));
  int t = int(std::nearbyint(v * (1.f - sf * (1.f - f))));
  switch (((i % 6) + 6) % 6) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
}

at::Tensor color_jitter(const at::Tensor& img_in, double bright, double contrast, double sat,
                        double hue, at::IntArrayRef order) {
  TORCH_CHECK(img_in.scalar_type() == at::kByte && img_in.dim() == 3 && img_in.size(2) == 3,
              "color_jitter: HxWx3 uint8");
  auto out = img_in.contiguous().clone();
  uint8_t* p = out.data_ptr<uint8_t>();
  const int64_t n = out.size(0) * out.size(1);
  uint8_t lut[256];
  for (int64_t op : order) {
    if (op == 0) {  // per-value map: a 256-entry table
      const float f = float(bright);
      for (int v = 0; v < 256; ++v) lut[v] = clip8(v * f);
      for (int64_t i = 0; i < 3 * n; ++i) p[i] = lut[p[i]];
    } else if (op == 1) {
      // PIL ImageEnhance.Contrast: blend with the (rounded) mean grey level.
      int64_t acc = 0;
      for (int64_t i = 0; i < n; ++i) acc += luma(p[3 * i], p[3 * i + 1], p[3 * i + 2]);
      const float mean = float(int(double(acc) / n + 0.5));
      const float f = float(contrast);
      for (int v = 0; v < 256; ++v) lut[v] = clip8(mean + f * (v - mean));
      for (int64_t i = 0; i < 3 * n; ++i) p[i] = lut[p[i]];
    } else if (op == 2) {
      const float f = float(sat);
      for (int64_t i = 0; i < n; ++i) {
        uint8_t* q = p + 3 * i;
        const float g = float(luma(q[0], q[1], q[2]));
        q[0] = clip8(g + f * (q[0] - g));
        q[1] = clip8(g + f * (q[1] - g));
        q[2] = clip8(g + f * (q[2] - g));
      }
    } else if (op == 3) {
      if (hue == 0.0) continue;
      const int shift = int(hue * 255.0);
      // rgb2hsv -> shift -> hsv2rgb with the divisions of the reference
      // formulas kept (a one-step hue quantisation change moves a channel by
      // up to ~6 levels), floor / round-to-nearest-even as inline SSE
      // conversions instead of libm calls (baseline x86-64 has no roundss)
      for (int64_t i = 0; i < n; ++i) {
        uint8_t* q = p + 3 * i;
        const int r = q[0], g = q[1], b = q[2];
        const int maxc = std::max(r, std::max(g, b)), minc = std::min(r, std::min(g, b));
        if (maxc == minc) continue;  // grey: s = 0, the hue shift leaves it unchanged
        const float cr = float(maxc - minc);
        const int s_ = int(cr / maxc * 255.f);
        const float rc = (maxc - r) / cr, gc = (maxc - g) / cr, bc = (maxc - b) / cr;
        float hf;
        if (r == maxc) hf = bc - gc;
        else if (g == maxc) hf = 2.f + rc - bc;
        else hf = 4.f + gc - rc;
        hf = hf / 6.f;
        hf = hf - ffloor(hf);
        const int h = (int(hf * 255.f) + shift) & 255;  // uint8 wrap, as torchvision does on the H plane
        // hsv2rgb (s > 0 here unless the quantised s is 0)
        if (s_ == 0) { q[0] = q[1] = q[2] = uint8_t(maxc); continue; }
        const float hh = h / 255.f, sf = s_ / 255.f;
        const int k = int(hh * 6.f);  // hh >= 0: truncation is floor
        const float f = hh * 6.f - k;
        const int v = maxc;
        const int pp = rne(v * (1.f - sf)), qq = rne(v * (1.f - sf * f)), tt = rne(v * (1.f - sf * (1.f - f)));
        int ro, go, bo;
        switch (k % 6) {
          case 0: ro = v; go = tt; bo = pp; break;
          case 1: ro = qq; go = v; bo = pp; break;
          case 2: ro = pp; go = v; bo = tt; break;
          case 3: ro = pp; go = qq; bo = v; break;
          case 4: ro = tt; go = pp; bo = v; break;
          default: ro = v; go = pp; bo = qq; break;
        }
        q[0] = uint8_t(ro); q[1] = uint8_t(go); q[2] = uint8_t(bo);
      }
    }
  }
  return out;
}

// -------------------------------------------------- sparse flow resize
std::vector<at::Tensor> sparse_flow_resize(const at::Tensor& flow_in, const at::Tensor& valid_in,
                                           double fx, double fy) {
  auto flow = flow_in.to(at::kFloat).contiguous();
  auto valid = valid_in.to(at::kFloat).contiguous();
  const int64_t H = flow.size(0), W = flow.size(1);
  const int64_t H1 = int64_t(std::nearbyint(H * fy)), W1 = int64_t(std::nearbyint(W * fx));
  auto fo = at::zeros({H1, W1, 2}, at::kFloat);
  auto vo = at::zeros({H1, W1}, at::kInt);
  const float* f = flow.data_ptr<float>();
  const float* v = valid.data_ptr<float>();
  float* F = fo.data_ptr<float>();
  int32_t* V = vo.data_ptr<int32_t>();
  for (int64_t y = 0; y < H; ++y)
    for (int64_t x = 0; x < W; ++x) {
      const int64_t i = y * W + x;
      if (v[i] < 1.f) continue;
      const int64_t xx = int64_t(std::nearbyint(float(x) * float(fx)));
      const int64_t yy = int64_t(std::nearbyint(float(y) * float(fy)));
      if (xx > 0 && xx < W1 && yy > 0 && yy < H1) {
        F[(yy * W1 + xx) * 2] = f[2 * i] * float(fx);
        F[(yy * W1 + xx) * 2 + 1] = f[2 * i + 1] * float(fy);
        V[yy * W1 + xx] = 1;
      }
    }
  return {fo, vo};
}

}  // namespace

TORCH_LIBRARY(raft_stir_host, m) {
  m.def("png_decode(Tensor data) -> Tensor", &png_decode);
  m.def("png_encode16(Tensor img) -> Tensor", &png_encode16);
  m.def("resize_bilinear(Tensor img, int oh, int ow, float fy=0., float fx=0.) -> Tensor", &resize_bilinear);
  m.def("color_jitter(Tensor img, float brightness, float contrast, float saturation, float hue, int[] order) -> Tensor",
        &color_jitter);
  m.def("resize_crop(Tensor img, int oh, int ow, float fy, float fx, int y0, int x0, int ch, int cw, bool hflip, "
        "bool vflip, float[] mul) -> Tensor", &resize_crop);
  m.def("sparse_flow_resize(Tensor flow, Tensor valid, float fx, float fy) -> Tensor[]", &sparse_flow_resize);
}
