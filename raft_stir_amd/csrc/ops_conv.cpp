// torch.ops.raft_stir.conv_fused / flow_encode: the fused update-block
// convolution (csrc/conv.hip).  All shape, alignment and bounds checks happen
// here on the host; the kernel assumes them.
#include <ATen/ATen.h>
#include "host_common.h"
#include "enc_epi.h"
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <algorithm>

namespace rs {
struct ConvLaunch {
  const void* seg_ptr[3];
  int seg_C[3], seg_stride[3];
  int nseg;
  const void* w;
  const float* bias;
  int B, H, W, KH, KW, PH, PW, Cout, Cout_pad, Ktot;
  int epi;
  float scale;
  int hd;
  void* out; int ostr, ooff;
  void* out2; int o2str, o2off;
  void* out3; int o3str, o3off;
  const void* aux1; int a1str, a1off;
  const void* aux2; int a2str, a2off;
  int tile;
  unsigned seg_bytes[3];  // bytes from seg_ptr to the end of its tensor (buffer range checks)
  unsigned w_bytes;
  int geo;  // 1: strided / remapped geometry below (conv_lds tiles 2-4, 6-8)
  int Hi, Wi, SY, SX, oH, oW, OSY, OSX, OOY, OOX;
  // EPI_NORM per-channel scale (conv_common.h Args)
  const float* chs;
  int f32;  // fp32 activations / outputs (split-bf16 tiles 6-8, conv_lds_kernel<..., F32>)
};
bool conv_launch(const ConvLaunch& L, hipStream_t stream);
struct SconvLaunch {
  const void* x;
  int xstr, Cin, B, Hi, Wi;
  const float* w;
  const float* bias;
  void* y;
  int ystr, yoff, Cout, Ho, Wo, KH, KW, S, P, relu;
  const void* res;
  int rstr;
  bool f32;
};
int sconv_max_weights();
struct SconvWgradLaunch {
  const void* x;
  const void* dy;
  int xstr, ystr, Cin, Cout, B, Hi, Wi, Ho, Wo, KH, KW, S, P;
  bool f32;
  float* dw;
  float* part;
};
int sconv_wgrad_blocks(int B, int Ho, int OUT, int* rows_per_block);
void sconv_wgrad_launch(const SconvWgradLaunch& L, int nblk, int rows_per_block, hipStream_t stream);
void sconv_launch(const SconvLaunch& L, hipStream_t stream);
struct EncWgradLaunch {
  const void* x;
  const void* dy;
  int xstr, ystr;
  long x_bytes, dy_bytes;
  int B, H, W, Cin, Cout;
  float* part;
  float* dw;
  int nsplit, tpb;
};
int enc_wgrad_splits(int B, int H, int W, int Cin, int Cout, int* tpb);
void enc_wgrad_launch(const EncWgradLaunch& L, hipStream_t stream);
void flow_enc_launch(const float* coords, int B, int H, int W, const float* w, const float* bias,
                     int Cout, void* out, int ostr, int ooff, void* fout, int fstr, int foff, bool f32,
                     hipStream_t stream);
void flowhead_fwd_launch(const void* x, int xstr, int xoff, int cin, const float* w, const float* bias, int B,
                         int H, int W, float* crd, const float* src, bool x_f32, hipStream_t s);
void flowhead_dgrad_launch(const float* dflow, const float* w, int cin, int B, int H, int W, const void* act,
                           int astr, int aoff, void* out, int ostr, int ooff, bool f32, hipStream_t s);
void gru_gate_bwd_launch(float* dh, int dhstr, const void* z, int zstr, const void* q, int qstr, const void* h,
                         int hstr, int hoff, void* dq, int dqstr, void* dzr, int dzrstr, long P, int hd, bool f32,
                         hipStream_t stream);
void relu_take_launch(float* G, int gstr, int goff, int n, int nz, const void* act, int astr, int aoff, void* out,
                      int ostr, long P, bool f32, hipStream_t stream);
struct WgradLaunch {
  const void* dy;
  int ystr, yoff, Cout;
  const void* seg_ptr[3];
  int seg_C[3], seg_stride[3], seg_period[3];
  int nseg;
  int Bp, H, W, KH, KW, Ktot;
  float* dw;
  float* db;
  int bn128;  unsigned dy_bytes, seg_bytes[3];  // buffer range checks
  int dma;  // 1: buffer-DMA kernel
  float* part;  // deterministic mode: split partials (see wgrad_splits), else null
  int Hi, Wi, SY, SX;  // strided conv (DMA kernel): X grid and stride; 0 = dY's grid, stride 1
};
void wgrad_launch(const WgradLaunch& L, hipStream_t stream);
int wgrad_splits(const WgradLaunch& L);
int colsum_blocks(int P);
void colsum_launch(const void* dy, int ystr, int yoff, int C, int P, float* db, float* part, hipStream_t stream);
int flow_wgrad_blocks(int Bp, int H);
void flow_wgrad_launch(const float* coords, int Bp, int H, int W, const void* df, int fstr, int Cout, float* dw,
                       float* db, float* part, bool f32, hipStream_t stream);
bool deterministic();
bool enc_halo_launch(const uint16_t* x, int xstr, const uint16_t* w, int Ktot, uint16_t* y, int ystr, int B, int H,
                     int W, int cin, int cout, int num_cus, const EncEpi& e, hipStream_t stream);
bool enc_halo_supported(int cin, int cout);
struct StemLaunch {  // must match stem.hip
  const void* x;
  int x_bf16, B, Hi, Wi, Ho, Wo;
  const void* w;
  const float* bias;
  int Cout, epi, relu;
  void* out;
  int ostr, ooff;
  const void* res;
  int rstr;
  const float* chs;
  int f32;
};
void stem_launch(const StemLaunch& L, hipStream_t stream);
int stem_wgrad_blocks(int B, int Ho, int Wo, int* chunks_per_block);
void stem_wgrad_launch(const void* x, bool x_bf16, int B, int Hi, int Wi, int Ho, int Wo, const uint16_t* dy, int ystr,
                       int Cout, float* part, int nblk, int px_per_block, float* dw, hipStream_t stream);
}  // namespace rs

namespace {
using at::Tensor;

constexpr int EPI_GRU_ZR = 3, EPI_GRU_Q = 4, EPI_FLOW = 5, EPI_RELU_BWD = 6, EPI_ACC_F32 = 7, EPI_GRU_QBWD = 8,
              EPI_NORM = 9;

hipStream_t stream() { return rs::current_stream(); }

void check_nhwc(const Tensor& t, int B, int H, int W, const char* n, at::ScalarType dt = at::kBFloat16) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.dim() == 4, n, ": contiguous NHWC GPU tensor required");
  TORCH_CHECK(t.size(0) == B && t.size(1) == H && t.size(2) == W, n, ": spatial shape mismatch");
  TORCH_CHECK(t.scalar_type() == dt, n, ": ", dt, " required");
}

// Encoder-normalisation extra shared by conv_fused / conv_geo / conv3x3_halo / stem_conv:
//   nscale (fp32, >= round_up(Cout, 4), 16-B aligned; epi EPI_NORM only) with
//     the bias as the shift: out = [relu](acc * nscale + bias) [then relu(. + aux1)].
struct NormX {
  const float* chs = nullptr;
};
void check_vec4(const c10::optional<Tensor>& t, int Cout, const char* op, const char* n) {
  TORCH_CHECK(t && t->is_cuda() && t->is_contiguous() && t->scalar_type() == at::kFloat &&
                  t->numel() >= (Cout + 3) / 4 * 4 && (uintptr_t)t->data_ptr() % 16 == 0,
              op, ": ", n, " must be 16-B aligned fp32 with round_up(Cout, 4) values");
}
NormX norm_extras(const c10::optional<Tensor>& nscale, const c10::optional<Tensor>& bias, int epi, int Cout,
                  const char* op) {
  NormX x;
  TORCH_CHECK(bool(nscale) == (epi == EPI_NORM), op, ": nscale is the EPI_NORM scale (and only that)");
  if (nscale) {
    check_vec4(nscale, Cout, op, "nscale");
    check_vec4(bias, Cout, op, "bias (the EPI_NORM shift)");
    x.chs = nscale->data_ptr<float>();
  }
  return x;
}

void conv_impl(const std::vector<Tensor>& segs, at::IntArrayRef seg_off, at::IntArrayRef seg_C,
               const Tensor& w, const c10::optional<Tensor>& bias, int64_t KH, int64_t KW, int64_t Cout,
               int64_t epi, double scale, int64_t hd, const Tensor& out, int64_t ooff,
               const c10::optional<Tensor>& out2, int64_t o2off, const c10::optional<Tensor>& out3,
               int64_t o3off, const c10::optional<Tensor>& aux1, int64_t a1off,
               const c10::optional<Tensor>& aux2, int64_t a2off, int64_t tile,
               const NormX& nx = NormX()) {
  TORCH_CHECK(!segs.empty() && segs.size() <= 3, "conv_fused: 1..3 input segments");
  TORCH_CHECK(seg_off.size() == segs.size() && seg_C.size() == segs.size(), "conv_fused: segment spec");
  const int B = segs[0].size(0), H = segs[0].size(1), W = segs[0].size(2);
  const c10::DeviceGuard guard(segs[0].device());
  rs::ConvLaunch L{};
  // fp32 activations: the split-bf16 register-staged tiles (conv.hip conv_lds_kernel<..., F32>)
  const bool f32 = segs[0].scalar_type() == at::kFloat;
  const at::ScalarType adt = f32 ? at::kFloat : at::kBFloat16;
  // tiles 81-84 (conv_v3f.hip): fp32 weight streaming, split fragment-major weights
  const bool v3f = f32 && tile >= 81 && tile <= 85;
  if (f32) {
    TORCH_CHECK(tile == 6 || tile == 7 || tile == 8 || (tile >= 38 && tile <= 40) || v3f,
                "conv_fused: fp32 activations run on tiles 6, 7, 8, 38-40, 81-85 only");
    TORCH_CHECK(epi != EPI_FLOW, "conv_fused: fp32 activations: no flow epilogue (csrc/flowhead.hip serves it)");
  }
  L.f32 = f32 ? 1 : 0;
  int Ktot = 0;
  for (size_t s = 0; s < 3; ++s) {
    if (s < segs.size()) {
      check_nhwc(segs[s], B, H, W, "segment", adt);
      const int C = seg_C[s], off = seg_off[s], Cb = segs[s].size(3);
      TORCH_CHECK(C > 0 && C % 32 == 0, "conv_fused: segment channels must be a positive multiple of 32");
      TORCH_CHECK(off >= 0 && off % 8 == 0 && Cb % 8 == 0 && off + C <= Cb,
                  "conv_fused: segment window out of bounds or misaligned");
      L.seg_ptr[s] = static_cast<const char*>(segs[s].data_ptr()) + (size_t)off * segs[s].element_size();
      L.seg_C[s] = C;
      L.seg_stride[s] = Cb;
      TORCH_CHECK(segs[s].numel() * segs[s].element_size() < (int64_t(1) << 31),
                  "conv_fused: segment tensor must be < 2 GiB");
      L.seg_bytes[s] = (unsigned)((segs[s].numel() - off) * segs[s].element_size());
      Ktot += C;
    } else {
      L.seg_ptr[s] = L.seg_ptr[0];
      L.seg_C[s] = 32;
      L.seg_stride[s] = L.seg_stride[0];
      L.seg_bytes[s] = L.seg_bytes[0];
    }
  }
  L.nseg = segs.size();
  TORCH_CHECK(KH >= 1 && KW >= 1 && KH % 2 == 1 && KW % 2 == 1, "conv_fused: odd kernel sizes only");
  TORCH_CHECK((tile >= 0 && tile <= 54) || tile == 56 || tile == 57 || tile == 61 || tile == 65 || tile == 66 ||
                  tile == 68 || tile == 70 || v3f,
              "conv_fused: tile must be in [0,54], 56, 57, 61, 65, 66, 68 or 70");
  if (tile == 70) {  // conv_gemm1.hip: 1x1 GEMM over 64-channel K chunks
    TORCH_CHECK(KH == 1 && KW == 1 && !f32, "conv_fused: tile 70 is the bf16 1x1 GEMM");
    for (size_t s = 0; s < segs.size(); ++s)
      TORCH_CHECK(seg_C[s] % 64 == 0, "conv_fused: tile 70 needs segment channels % 64 == 0");
  }
  const bool v3 = tile >= 56 && tile <= 68;  // conv_v3.hip: fragment-major weights (ops/conv.py frag_weight)
  if (v3f) {
    for (size_t s = 0; s < segs.size(); ++s)
      TORCH_CHECK(seg_C[s] % 64 == 0, "conv_fused: tiles 81-85 need segment channels % 64 == 0");
    TORCH_CHECK(tile != 85 || Ktot == 64, "conv_fused: tile 85 (one halo buffer) needs exactly one 64-channel K chunk");
  }
  if ((tile >= 42 && tile <= 54) || v3 || v3f)
    TORCH_CHECK((KH == 3 && KW == 3) || (KH == 1 && KW == 5) || (KH == 5 && KW == 1),
                "conv_fused: tiles 42-68 are instantiated for 3x3, 1x5 and 5x1 kernels only");
  TORCH_CHECK(tile < 16 || KH * KW <= 32, "conv_fused: buffer-DMA tiles (16-37) support at most 32 taps");
  TORCH_CHECK(!(tile >= 38 && tile <= 40) || f32, "conv_fused: tiles 38-40 are the fp32 split-K tiles");
  TORCH_CHECK(tile != 5 || Cout <= 16, "conv_fused: tile 5 (small-N) needs Cout <= 16");
  if (tile >= 24 && tile <= 26) {  // halo tiles: the (TH+KH-1) x (16+KW-1) halo must fit the LDS buffer
    const int TH = tile == 26 ? 4 : 8, HCAP = tile == 26 ? 128 : 192;
    TORCH_CHECK((TH + KH - 1) * (16 + KW - 1) <= HCAP, "conv_fused: kernel too large for halo tile ", tile);
  }
  const bool bm128 = tile == 4 || tile == 7 || tile == 8 || (tile >= 10 && tile <= 13) || tile == 16 ||
                     tile == 18 || tile == 20 || tile == 22 || tile == 24 || tile == 26 || tile == 36 ||
                     tile == 39;
  const bool bm128w = tile == 28 || tile == 31 || tile == 33;
  const int tileM = (tile == 48 || tile == 49 || tile == 53 || tile == 70) ? 128
                    : (tile == 50 || tile == 51 || tile == 52) ? 256
                    : tile == 54 ? 192
                    : (tile == 42 || tile >= 45) ? 64 : tile == 43 ? 32 : tile == 44 ? 128
                    : tile == 0 ? 32
                    : (tile == 27 || tile == 30 || tile == 32) ? 256
                    : tile == 29 ? 192
                    : (bm128 || bm128w) ? 128 : (tile == 5 ? 16 : 64);
  if (tile >= 6 && tile != 12 && tile != 13 && tile != 14 && tile != 41 && !f32)  // 64-deep K steps
    for (size_t s = 0; s < segs.size(); ++s)
      TORCH_CHECK(seg_C[s] % 64 == 0, "conv_fused: 64-deep-K tiles need segment channels % 64 == 0");
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == at::kBFloat16 && w.dim() == 3,
              "conv_fused: packed weight must be contiguous bf16 (Cout_pad, taps, Ktot)");
  TORCH_CHECK(w.size(1) == KH * KW && w.size(2) == (f32 && !v3f ? 2 : 1) * Ktot,
              "conv_fused: packed weight K mismatch", f32 && !v3f ? " (fp32: split [wh | wl] weights, 2 x Ktot)" : "");
  if (v3f) {  // [frag(wh) ; frag(wl)]: two halves of round_up(Cout, 32)+ rows each
    TORCH_CHECK(w.size(0) % 64 == 0 && w.size(0) / 2 >= (Cout + 31) / 32 * 32 && w.numel() * 2 < (int64_t(1) << 31),
                "conv_fused: tiles 81-85 need split fragment-major weights [frag(wh); frag(wl)] (ops/conv.py "
                "frag_weight_split)");
  } else if (v3) {  // fragment-major rows in 32-row blocks; blocks past the weight read as zeros
    TORCH_CHECK(w.size(0) % 32 == 0 && w.size(0) >= (Cout + 31) / 32 * 32 && w.numel() * 2 < (int64_t(1) << 31),
                "conv_fused: tiles 56-68 need fragment-major weights with round_up(Cout, 32) rows (< 2 GiB)");
  } else {
    TORCH_CHECK(w.size(0) >= (Cout + tileM - 1) / tileM * tileM,
                "conv_fused: packed weight needs >= round_up(Cout, ", tileM, ") rows");
  }
  if (bias) {
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kFloat && bias->numel() >= Cout &&
                    bias->is_contiguous(),
                "conv_fused: bias must be fp32 (Cout,)");
  }
  L.w = w.data_ptr();
  L.w_bytes = (unsigned)(w.numel() * 2);
  L.bias = bias ? bias->data_ptr<float>() : nullptr;
  L.B = B; L.H = H; L.W = W; L.KH = KH; L.KW = KW; L.PH = KH / 2; L.PW = KW / 2;
  L.Cout = Cout; L.Cout_pad = w.size(0); L.Ktot = w.size(2);  // weight row length
  L.epi = epi; L.scale = scale; L.hd = hd; L.tile = tile;
  if (epi == EPI_FLOW) {
    TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.scalar_type() == at::kFloat && out.dim() == 4 &&
                    out.size(0) == B && out.size(1) == 2 && out.size(2) == H && out.size(3) == W,
                "conv_fused(flow): out must be fp32 coords (B,2,H,W)");
    TORCH_CHECK(Cout == 2, "conv_fused(flow): Cout must be 2");
    L.out = out.data_ptr(); L.ostr = 0; L.ooff = 0;
    if (out2) {  // out-of-place: out = out2 + delta
      TORCH_CHECK(out2->is_cuda() && out2->is_contiguous() && out2->scalar_type() == at::kFloat &&
                      out2->sizes() == out.sizes(),
                  "conv_fused(flow): out2 (source coords) must match out");
      L.out2 = out2->data_ptr();
    }
  } else {
    const bool f32out = f32 || epi == EPI_ACC_F32 || epi == EPI_GRU_QBWD;
    check_nhwc(out, B, H, W, "out", f32out ? at::kFloat : at::kBFloat16);
    const int cw = epi == EPI_GRU_ZR ? hd : Cout;
    TORCH_CHECK(ooff >= 0 && ooff + cw <= out.size(3), "conv_fused: output window out of bounds");
    L.out = out.data_ptr(); L.ostr = out.size(3); L.ooff = ooff;
  }
  auto opt_nhwc = [&](const c10::optional<Tensor>& t, int64_t off, int width, const char* n, void** p,
                      int* str, int* o) {
    if (!t) { *p = nullptr; *str = 0; *o = 0; return; }
    check_nhwc(*t, B, H, W, n, adt);
    TORCH_CHECK(off >= 0 && off + width <= t->size(3), "conv_fused: ", n, " window out of bounds");
    *p = t->data_ptr(); *str = t->size(3); *o = off;
  };
  void* p;
  if (epi == EPI_GRU_ZR) {
    TORCH_CHECK(Cout == 2 * hd && hd % 4 == 0 && out2 && aux1, "conv_fused(gru_zr): needs Cout=2*hd, out2 (r*h), aux1 (h)");
    opt_nhwc(out2, o2off, hd, "out2", &L.out2, &L.o2str, &L.o2off);
    opt_nhwc(out3, o3off, hd, "out3", &L.out3, &L.o3str, &L.o3off);
    opt_nhwc(aux1, a1off, hd, "aux1", &p, &L.a1str, &L.a1off); L.aux1 = p;
  } else if (epi == EPI_GRU_Q) {
    TORCH_CHECK(Cout % 4 == 0 && aux1 && aux2, "conv_fused(gru_q): needs aux1 (h) and aux2 (z)");
    opt_nhwc(out2, o2off, Cout, "out2", &L.out2, &L.o2str, &L.o2off);
    opt_nhwc(aux1, a1off, Cout, "aux1", &p, &L.a1str, &L.a1off); L.aux1 = p;
    opt_nhwc(aux2, a2off, Cout, "aux2", &p, &L.a2str, &L.a2off); L.aux2 = p;
  } else if (epi == EPI_RELU_BWD) {
    TORCH_CHECK(aux1, "conv_fused(relu_bwd): needs aux1 (the ReLU output)");
    opt_nhwc(aux1, a1off, Cout, "aux1", &p, &L.a1str, &L.a1off); L.aux1 = p;
  } else if (epi == EPI_NORM) {
    if (aux1) { opt_nhwc(aux1, a1off, Cout, "aux1", &p, &L.a1str, &L.a1off); L.aux1 = p; }
  } else if (epi == EPI_GRU_QBWD) {
    TORCH_CHECK(hd % 4 == 0 && hd <= Cout && out2 && aux1 && aux2,
                "conv_fused(gru_qbwd): needs out2 (dr_pre), aux1 (h), aux2 (r)");
    opt_nhwc(out2, o2off, hd, "out2", &L.out2, &L.o2str, &L.o2off);
    opt_nhwc(aux1, a1off, hd, "aux1", &p, &L.a1str, &L.a1off); L.aux1 = p;
    opt_nhwc(aux2, a2off, hd, "aux2", &p, &L.a2str, &L.a2off); L.aux2 = p;
  }
  TORCH_CHECK(epi >= 0 && epi <= EPI_NORM, "conv_fused: unknown epilogue kind");
  if (nx.chs)
    TORCH_CHECK(!(tile >= 42 && tile <= 54) && !v3 && tile != 70 && (!(tile >= 81 && tile <= 85) || f32),
                "conv_fused: EPI_NORM needs a tile with the shared epilogue (not 42-70)");
  L.chs = nx.chs;
  TORCH_CHECK(rs::conv_launch(L, stream()), "conv_fused: tile ", L.tile, " is not instantiated for a ", KH, "x", KW,
              " kernel");
  RS_CHECK_LAUNCH();
}

void conv_fused(const std::vector<Tensor>& segs, at::IntArrayRef seg_off, at::IntArrayRef seg_C,
                const Tensor& w, const c10::optional<Tensor>& bias, int64_t KH, int64_t KW, int64_t Cout,
                int64_t epi, double scale, int64_t hd, const Tensor& out, int64_t ooff,
                const c10::optional<Tensor>& out2, int64_t o2off, const c10::optional<Tensor>& out3,
                int64_t o3off, const c10::optional<Tensor>& aux1, int64_t a1off,
                const c10::optional<Tensor>& aux2, int64_t a2off, int64_t tile, const c10::optional<Tensor>& nscale) {
  const NormX nx = norm_extras(nscale, bias, epi, Cout, "conv_fused");
  conv_impl(segs, seg_off, seg_C, w, bias, KH, KW, Cout, epi, scale, hd, out, ooff, out2, o2off, out3, o3off,
            aux1, a1off, aux2, a2off, tile, nx);
}

// convf1 of the motion encoder from coords1 (flow = coords1 - grid), ReLU, bf16
// NHWC into out[..., ooff:ooff+Cout]; the flow itself (bf16) into fout[..., foff:foff+2].
// Strided / remapped implicit-GEMM convolution: the encoder's stride-2 3x3 and
// 1x1 convolutions and the phase-split input gradients of them
// (ops/enc_conv.py; csrc/conv.hip conv_lds_kernel<..., GEO>).
//   segs : NHWC bf16 [B, Hi, Wi, Cb], one grid;  GEMM pixel grid B x Ho x Wo
//   GEMM pixel (b, y, x) reads input (b, y*SY + ky - PH, x*SX + kx - PW) (zero outside)
//   and writes out[b, y*OSY + OOY, x*OSX + OOX, ooff : ooff + Cout]  (out: NHWC bf16)
void conv_geo(const std::vector<Tensor>& segs, at::IntArrayRef seg_off, at::IntArrayRef seg_C, const Tensor& w,
              const c10::optional<Tensor>& bias, int64_t KH, int64_t KW, int64_t PH, int64_t PW, int64_t SY,
              int64_t SX, int64_t Ho, int64_t Wo, int64_t Cout, const Tensor& out, int64_t ooff, int64_t OSY,
              int64_t OSX, int64_t OOY, int64_t OOX, int64_t tile, const c10::optional<Tensor>& nscale, bool relu) {
  TORCH_CHECK(!segs.empty() && segs.size() <= 3 && seg_off.size() == segs.size() && seg_C.size() == segs.size(),
              "conv_geo: 1..3 input segments");
  TORCH_CHECK(tile == 2 || tile == 3 || tile == 4 || tile == 6 || tile == 7 || tile == 8,
              "conv_geo: tile must be one of the register-staged variants 2, 3, 4, 6, 7, 8");
  const bool f32 = segs[0].scalar_type() == at::kFloat;  // split-bf16 F32 tiles (32 input channels per step)
  const at::ScalarType adt = f32 ? at::kFloat : at::kBFloat16;
  const int bk = (tile >= 6 && !f32) ? 64 : 32;
  const int tileM = (tile == 2 || tile == 3 || tile == 6) ? 64 : 128;
  const int B = segs[0].size(0), Hi = segs[0].size(1), Wi = segs[0].size(2);
  const c10::DeviceGuard guard(segs[0].device());
  rs::ConvLaunch L{};
  int Ktot = 0;
  for (size_t s = 0; s < 3; ++s) {
    if (s < segs.size()) {
      check_nhwc(segs[s], B, Hi, Wi, "conv_geo segment", adt);
      const int C = seg_C[s], off = seg_off[s], Cb = segs[s].size(3);
      TORCH_CHECK(C > 0 && C % bk == 0, "conv_geo: segment channels must be a multiple of ", bk, " for tile ", tile);
      TORCH_CHECK(off >= 0 && off % 8 == 0 && Cb % 8 == 0 && off + C <= Cb, "conv_geo: segment window");
      L.seg_ptr[s] = static_cast<const char*>(segs[s].data_ptr()) + (size_t)off * segs[s].element_size();
      L.seg_C[s] = C;
      L.seg_stride[s] = Cb;
      Ktot += C;
    } else {
      L.seg_ptr[s] = L.seg_ptr[0];
      L.seg_C[s] = bk;
      L.seg_stride[s] = L.seg_stride[0];
    }
  }
  L.nseg = segs.size();
  TORCH_CHECK(KH >= 1 && KW >= 1 && SY >= 1 && SX >= 1 && Ho >= 1 && Wo >= 1 && Cout >= 1, "conv_geo: geometry");
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == at::kBFloat16 && w.dim() == 3 &&
                  w.size(1) == KH * KW && w.size(2) == (f32 ? 2 : 1) * Ktot &&
                  w.size(0) >= (Cout + tileM - 1) / tileM * tileM,
              "conv_geo: packed weight must be bf16 [>= round_up(Cout, ", tileM, ")][KH*KW][Ktot]");
  if (bias)
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kFloat && bias->is_contiguous() &&
                    bias->numel() >= Cout,
                "conv_geo: bias fp32 (Cout,)");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.dim() == 4 && out.scalar_type() == adt &&
                  out.size(0) == B && ooff >= 0 && ooff + Cout <= out.size(3),
              "conv_geo: out must be contiguous NHWC (the input dtype) with room for the channel window");
  const int oH = out.size(1), oW = out.size(2);
  TORCH_CHECK(OSY >= 1 && OSX >= 1 && OOY >= 0 && OOX >= 0 && (Ho - 1) * OSY + OOY < oH &&
                  (Wo - 1) * OSX + OOX < oW,
              "conv_geo: output pixel map out of bounds");
  TORCH_CHECK(int64_t(B) * Ho * Wo < (int64_t(1) << 31) && out.numel() < (int64_t(1) << 31), "conv_geo: size");
  L.w = w.data_ptr();
  L.bias = bias ? bias->data_ptr<float>() : nullptr;
  L.B = B; L.H = Ho; L.W = Wo; L.KH = KH; L.KW = KW; L.PH = PH; L.PW = PW;
  L.Cout = Cout; L.Cout_pad = w.size(0); L.Ktot = w.size(2);
  L.f32 = f32 ? 1 : 0;
  const int epi = nscale ? EPI_NORM : 0;
  const NormX nx = norm_extras(nscale, bias, epi, Cout, "conv_geo");
  TORCH_CHECK(!relu || nscale, "conv_geo: relu goes with the EPI_NORM epilogue");
  L.epi = epi; L.scale = 1.f; L.hd = relu ? 1 : 0;
  L.chs = nx.chs;
  L.out = out.data_ptr(); L.ostr = out.size(3); L.ooff = ooff;
  L.tile = tile;
  L.geo = 1;
  L.Hi = Hi; L.Wi = Wi; L.SY = SY; L.SX = SX;
  L.oH = oH; L.oW = oW; L.OSY = OSY; L.OSX = OSX; L.OOY = OOY; L.OOX = OOX;
  TORCH_CHECK(rs::conv_launch(L, stream()), "conv_fused: tile ", L.tile, " is not instantiated for a ", KH, "x", KW,
              " kernel");
  RS_CHECK_LAUNCH();
}

void flow_encode(const Tensor& coords, const Tensor& w, const Tensor& bias, const Tensor& out, int64_t ooff,
                 const c10::optional<Tensor>& fout, int64_t foff) {
  TORCH_CHECK(coords.is_cuda() && coords.is_contiguous() && coords.scalar_type() == at::kFloat &&
                  coords.dim() == 4 && coords.size(1) == 2,
              "flow_encode: coords must be fp32 (B,2,H,W)");
  const int B = coords.size(0), H = coords.size(2), W = coords.size(3);
  const int Cout = bias.numel();
  TORCH_CHECK(Cout % 16 == 0, "flow_encode: Cout must be a multiple of 16");
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == at::kFloat && w.numel() == 98 * Cout,
              "flow_encode: w must be fp32 [49][2][Cout]");
  TORCH_CHECK(bias.is_cuda() && bias.scalar_type() == at::kFloat && bias.is_contiguous(), "flow_encode: bias fp32");
  const bool f32 = out.scalar_type() == at::kFloat;  // fp32 inference engine
  check_nhwc(out, B, H, W, "out", f32 ? at::kFloat : at::kBFloat16);
  TORCH_CHECK(ooff % 8 == 0 && out.size(3) % 8 == 0 && ooff + Cout <= out.size(3), "flow_encode: out window");
  void* fp = nullptr;
  int fstr = 0;
  if (fout) {
    check_nhwc(*fout, B, H, W, "fout", f32 ? at::kFloat : at::kBFloat16);
    TORCH_CHECK(foff >= 0 && foff + 2 <= fout->size(3), "flow_encode: fout window");
    fp = fout->data_ptr();
    fstr = fout->size(3);
  }
  const c10::DeviceGuard guard(coords.device());
  rs::flow_enc_launch(coords.data_ptr<float>(), B, H, W, w.data_ptr<float>(), bias.data_ptr<float>(), Cout,
                      out.data_ptr(), out.size(3), ooff, fp, fstr, foff, f32, stream());
  RS_CHECK_LAUNCH();
}

// Flow-head output conv (3x3, Cin in {128, 256} -> 2) with the coords epilogue:
// crd = src + bias + conv(x[..., xoff:xoff+Cin]) (src defaults to crd: in place).
// w: fp32 [2][3][3][Cin] (= conv2.weight.permute(0, 2, 3, 1)).
void flow_head(const Tensor& x, int64_t xoff, int64_t cin, const Tensor& w, const Tensor& bias, const Tensor& crd,
               const c10::optional<Tensor>& src) {
  TORCH_CHECK(cin == 128 || cin == 256, "flow_head: Cin must be 128 or 256");
  TORCH_CHECK(crd.is_cuda() && crd.is_contiguous() && crd.scalar_type() == at::kFloat && crd.dim() == 4 &&
                  crd.size(1) == 2,
              "flow_head: coords must be contiguous fp32 (B,2,H,W)");
  const int B = crd.size(0), H = crd.size(2), W = crd.size(3);
  const bool xf = x.scalar_type() == at::kFloat;  // fp32 inference engine
  check_nhwc(x, B, H, W, "x", xf ? at::kFloat : at::kBFloat16);
  const int vn = cin == 256 ? 4 : 2;  // channels per lane: aligned vector loads
  TORCH_CHECK(xoff >= 0 && xoff + cin <= x.size(3) && xoff % vn == 0 && x.size(3) % vn == 0,
              "flow_head: x channel window");
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == at::kFloat && w.numel() == 18 * cin,
              "flow_head: w must be fp32 [2][3][3][Cin]");
  TORCH_CHECK(bias.is_cuda() && bias.scalar_type() == at::kFloat && bias.numel() == 2, "flow_head: bias fp32 (2,)");
  if (src) TORCH_CHECK(src->sizes() == crd.sizes() && src->is_contiguous() && src->scalar_type() == at::kFloat,
                       "flow_head: src must match coords");
  const c10::DeviceGuard guard(crd.device());
  rs::flowhead_fwd_launch(x.data_ptr(), x.size(3), xoff, cin, w.data_ptr<float>(), bias.data_ptr<float>(), B, H, W,
                          crd.data_ptr<float>(), src ? src->data_ptr<float>() : crd.data_ptr<float>(), xf, stream());
  RS_CHECK_LAUNCH();
}

// Its input gradient through the hidden ReLU: out[..., ooff:ooff+Cin] = (act > 0) * conv^T(dflow).
void flow_head_dgrad(const Tensor& dflow, const Tensor& w, int64_t cin, const Tensor& act, int64_t aoff,
                     const Tensor& out, int64_t ooff) {
  TORCH_CHECK(cin == 128 || cin == 256, "flow_head_dgrad: Cin must be 128 or 256");
  TORCH_CHECK(dflow.is_cuda() && dflow.is_contiguous() && dflow.scalar_type() == at::kFloat && dflow.dim() == 4 &&
                  dflow.size(1) == 2,
              "flow_head_dgrad: dflow must be contiguous fp32 (B,2,H,W)");
  const int B = dflow.size(0), H = dflow.size(2), W = dflow.size(3);
  const bool f32 = out.scalar_type() == at::kFloat;  // fp32 training engine
  check_nhwc(act, B, H, W, "act", f32 ? at::kFloat : at::kBFloat16);
  check_nhwc(out, B, H, W, "out", f32 ? at::kFloat : at::kBFloat16);
  const int vn = cin == 256 ? 4 : 2;
  TORCH_CHECK(aoff >= 0 && aoff + cin <= act.size(3) && aoff % vn == 0 && act.size(3) % vn == 0,
              "flow_head_dgrad: act channel window");
  TORCH_CHECK(ooff >= 0 && ooff + cin <= out.size(3) && ooff % vn == 0 && out.size(3) % vn == 0,
              "flow_head_dgrad: out channel window");
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == at::kFloat && w.numel() == 18 * cin,
              "flow_head_dgrad: w must be fp32 [2][3][3][Cin]");
  const c10::DeviceGuard guard(dflow.device());
  rs::flowhead_dgrad_launch(dflow.data_ptr<float>(), w.data_ptr<float>(), cin, B, H, W, act.data_ptr(), act.size(3),
                            aoff, out.data_ptr(), out.size(3), ooff, f32, stream());
  RS_CHECK_LAUNCH();
}

// dW (fp32, [>=Cout][taps][Ktot], accumulated) += sum_p dY[p][yoff + co] X[p + tap][k]
// SY, SX > 1: a strided conv; the segments are on the INPUT grid (any Hi x Wi,
// X pixel = (y*SY + ky - KH/2, x*SX + kx - KW/2)), buffer-DMA kernel only.
void conv_wgrad_impl(const Tensor& dy, int64_t yoff, int64_t Cout, const std::vector<Tensor>& segs,
                     at::IntArrayRef seg_off, at::IntArrayRef seg_C, at::IntArrayRef seg_period, int64_t KH,
                     int64_t KW, const Tensor& dw, const c10::optional<Tensor>& db, int64_t bn128, int64_t SY,
                     int64_t SX) {
  TORCH_CHECK(dy.is_cuda() && dy.is_contiguous() && dy.dim() == 4 && dy.scalar_type() == at::kBFloat16,
              "conv_wgrad: dy must be contiguous bf16 NHWC");
  const int Bp = dy.size(0), H = dy.size(1), W = dy.size(2);
  const bool strided = SY != 1 || SX != 1;
  TORCH_CHECK(SY >= 1 && SX >= 1, "conv_wgrad: stride >= 1");
  const int Hi = strided ? segs.at(0).size(1) : H, Wi = strided ? segs.at(0).size(2) : W;
  static const int dma_env = [] {
    const char* e = getenv("RS_WGRAD_DMA");
    return e ? atoi(e) : 1;
  }();
  // the register-staged kernel reads whole BM-channel dY rows unguarded; the
  // DMA kernels read through a range-checked buffer resource (rows past the
  // tensor read as zero, channels >= Cout only feed discarded accumulators)
  const int bm = Cout > 64 ? 128 : 64;
  TORCH_CHECK(yoff >= 0 && yoff % 8 == 0 && yoff + (dma_env ? Cout : (Cout + bm - 1) / bm * bm) <= dy.size(3),
              "conv_wgrad: dy channel window out of bounds");
  TORCH_CHECK(bn128 >= 0 && bn128 <= 5, "conv_wgrad: tile variant 0..5");
  if (db) TORCH_CHECK(db->is_cuda() && db->scalar_type() == at::kFloat && db->numel() >= Cout, "conv_wgrad: db fp32");
  TORCH_CHECK(!segs.empty() && segs.size() <= 3 && seg_off.size() == segs.size() && seg_C.size() == segs.size() &&
                  seg_period.size() == segs.size(),
              "conv_wgrad: segment spec");
  rs::WgradLaunch L{};
  int Ktot = 0;
  for (size_t s = 0; s < 3; ++s) {
    if (s < segs.size()) {
      const Tensor& t = segs[s];
      TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.dim() == 4 && t.scalar_type() == at::kBFloat16 &&
                      t.size(1) == Hi && t.size(2) == Wi,
                  "conv_wgrad: segment must be contiguous bf16 NHWC with dy's spatial size (the input grid "
                  "when strided)");
      const int per = seg_period[s];
      TORCH_CHECK(per == t.size(0) * Hi * Wi && Bp % t.size(0) == 0,
                  "conv_wgrad: segment period must be its pixel count and its images divide dy's");
      const int C = seg_C[s], off = seg_off[s];
      TORCH_CHECK(C % 64 == 0 && off % 8 == 0 && off + C <= t.size(3), "conv_wgrad: segment window (C % 64)");
      L.seg_ptr[s] = static_cast<const at::BFloat16*>(t.data_ptr()) + off;
      L.seg_C[s] = C;
      L.seg_stride[s] = t.size(3);
      L.seg_period[s] = per;
      TORCH_CHECK(t.numel() * 2 < (int64_t(1) << 31), "conv_wgrad: segment tensor must be < 2 GiB");
      L.seg_bytes[s] = (unsigned)((t.numel() - off) * 2);
      Ktot += C;
    } else {
      L.seg_ptr[s] = L.seg_ptr[0];
      L.seg_C[s] = 64;
      L.seg_stride[s] = L.seg_stride[0];
      L.seg_period[s] = L.seg_period[0];
      L.seg_bytes[s] = L.seg_bytes[0];
    }
  }
  TORCH_CHECK(dw.is_cuda() && dw.is_contiguous() && dw.scalar_type() == at::kFloat && dw.dim() == 3 &&
                  dw.size(0) >= Cout && dw.size(1) == KH * KW && dw.size(2) == Ktot,
              "conv_wgrad: dw must be fp32 (>=Cout, taps, Ktot)");
  const c10::DeviceGuard guard(dy.device());
  L.dy = dy.data_ptr(); L.ystr = dy.size(3); L.yoff = yoff; L.Cout = Cout;
  TORCH_CHECK(dy.numel() * 2 < (int64_t(1) << 31), "conv_wgrad: dY tensor must be < 2 GiB");
  L.dy_bytes = (unsigned)(dy.numel() * 2);
  L.dma = dma_env;
  TORCH_CHECK(!strided || L.dma, "conv_wgrad: strided weight gradients need the buffer-DMA kernels");
  L.Hi = Hi; L.Wi = Wi; L.SY = SY; L.SX = SX;
  L.nseg = segs.size();
  L.Bp = Bp; L.H = H; L.W = W; L.KH = KH; L.KW = KW; L.Ktot = Ktot;
  L.dw = dw.data_ptr<float>();
  L.db = db ? db->data_ptr<float>() : nullptr;
  L.bn128 = bn128;
  L.part = nullptr;
  Tensor part;
  if (rs::deterministic()) {
    TORCH_CHECK(L.dma, "conv_wgrad: deterministic mode needs the buffer-DMA kernels (RS_WGRAD_DMA=1)");
    const int64_t n = int64_t(rs::wgrad_splits(L)) * (int64_t(Cout) * KH * KW * Ktot + Cout);
    part = at::empty({n}, dy.options().dtype(at::kFloat));
    L.part = part.data_ptr<float>();
  }
  rs::wgrad_launch(L, stream());
  RS_CHECK_LAUNCH();
}

void conv_wgrad(const Tensor& dy, int64_t yoff, int64_t Cout, const std::vector<Tensor>& segs,
                at::IntArrayRef seg_off, at::IntArrayRef seg_C, at::IntArrayRef seg_period, int64_t KH, int64_t KW,
                const Tensor& dw, const c10::optional<Tensor>& db, int64_t bn128) {
  conv_wgrad_impl(dy, yoff, Cout, segs, seg_off, seg_C, seg_period, KH, KW, dw, db, bn128, 1, 1);
}

void conv_wgrad_strided(const Tensor& dy, int64_t Cout, const std::vector<Tensor>& segs, at::IntArrayRef seg_off,
                        at::IntArrayRef seg_C, int64_t KH, int64_t KW, int64_t SY, int64_t SX, const Tensor& dw,
                        const c10::optional<Tensor>& db) {
  std::vector<int64_t> per;
  for (const auto& t : segs) per.push_back(t.size(0) * t.size(1) * t.size(2));
  conv_wgrad_impl(dy, 0, Cout, segs, seg_off, seg_C, per, KH, KW, dw, db, 0, SY, SX);
}

// Weight gradient of a stride-1 / pad-1 3x3 convolution on csrc/enc_wgrad.hip
// (halo tiles, all nine taps per block, deterministic partial reduction).
//   dy : NHWC bf16 [B, H, W, Cout] view (channels contiguous, pixels dense)
//   x  : NHWC bf16 [B, H, W, Cin] view
// returns dW fp32 [Cout, Cin, 3, 3] (the parameter layout)
static void check_nhwc_view(const Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.scalar_type() == at::kBFloat16, n, ": bf16 NHWC GPU tensor");
  TORCH_CHECK(t.stride(3) == 1 && t.stride(2) >= t.size(3) && t.stride(2) % 8 == 0 &&
                  t.stride(1) == t.size(2) * t.stride(2) && t.stride(0) == t.size(1) * t.stride(1),
              n, ": dense NHWC pixels with a channel stride % 8 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, n, ": 16-B aligned base");
  TORCH_CHECK(t.numel() / t.size(3) * t.stride(2) * 2 < (int64_t(1) << 31), n, ": too large for 32-bit offsets");
}

// Narrow-channel NHWC conv (csrc/sconv.hip; RAFT-small encoder inference):
//   x   : [B, Hi, Wi, Cin] bf16 / fp32 view (dense pixels, channel stride % 8 == 0)
//   w   : fp32 [Cout, KH, KW, Cin] contiguous;  bias: fp32 [Cout] or None
//   out : [B, Ho, Wo, >= yoff + Cout] same dtype as x, contiguous; out[..., yoff:yoff+Cout] =
//         [relu](conv(x) + bias) [then relu(. + res)]
void sconv(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, int64_t stride, int64_t pad,
           bool relu, const Tensor& out, int64_t yoff, const c10::optional<Tensor>& res) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat),
              "sconv: x bf16 / fp32 NHWC");
  const int B = x.size(0), Hi = x.size(1), Wi = x.size(2), Cin = x.size(3);
  TORCH_CHECK(x.stride(3) == 1 && x.stride(2) % 8 == 0 && x.stride(1) == Wi * x.stride(2) &&
                  x.stride(0) == Hi * x.stride(1) && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "sconv: x must be dense NHWC pixels with a channel stride % 8 == 0, 16-B aligned");
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == at::kFloat && w.dim() == 4 && w.size(3) == Cin,
              "sconv: w fp32 [Cout, KH, KW, Cin]");
  const int Cout = w.size(0), KH = w.size(1), KW = w.size(2);
  TORCH_CHECK(Cin % 8 == 0 && Cout % 8 == 0, "sconv: channel counts must be multiples of 8");
  TORCH_CHECK(std::min(4, Cout / 8) * 8 * KH * KW * Cin <= rs::sconv_max_weights(), "sconv: weight tile too large");
  TORCH_CHECK(stride >= 1 && pad >= 0, "sconv: geometry");
  const int Ho = (Hi + 2 * pad - KH) / stride + 1, Wo = (Wi + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.dim() == 4 && out.scalar_type() == x.scalar_type() &&
                  out.size(0) == B && out.size(1) == Ho && out.size(2) == Wo && yoff >= 0 && yoff % 8 == 0 &&
                  yoff + Cout <= out.size(3) && out.size(3) % 8 == 0,
              "sconv: out must be contiguous [B, Ho, Wo, C] with the window [yoff, yoff + Cout)");
  if (bias) TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kFloat && bias->numel() == Cout, "sconv: bias");
  if (res)
    TORCH_CHECK(res->is_cuda() && res->is_contiguous() && res->scalar_type() == x.scalar_type() && res->dim() == 4 &&
                    res->size(0) == B && res->size(1) == Ho && res->size(2) == Wo && res->size(3) == Cout,
                "sconv: residual must be contiguous [B, Ho, Wo, Cout]");
  const c10::DeviceGuard guard(x.device());
  rs::SconvLaunch L{};
  L.x = x.data_ptr(); L.xstr = x.stride(2); L.Cin = Cin; L.B = B; L.Hi = Hi; L.Wi = Wi;
  L.w = w.data_ptr<float>(); L.bias = bias ? bias->data_ptr<float>() : nullptr;
  L.y = out.data_ptr(); L.ystr = out.size(3); L.yoff = yoff; L.Cout = Cout;
  L.Ho = Ho; L.Wo = Wo; L.KH = KH; L.KW = KW; L.S = stride; L.P = pad; L.relu = relu ? 1 : 0;
  L.res = res ? res->data_ptr() : nullptr; L.rstr = Cout;
  L.f32 = x.scalar_type() == at::kFloat;
  rs::sconv_launch(L, stream());
  RS_CHECK_LAUNCH();
}

// Weight gradient of a narrow-channel conv (csrc/sconv_train.hip; RAFT-small
// encoder training): dw fp32 [Cout, KH, KW, Cin] = sum over pixels of
// dy (x) im2col(x); x / dy dense NHWC views of the same dtype (bf16 / fp32).
void sconv_wgrad(const Tensor& dy, const Tensor& x, int64_t KH, int64_t KW, int64_t stride, int64_t pad,
                 const Tensor& dw) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat),
              "sconv_wgrad: x bf16 / fp32 NHWC");
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.scalar_type() == x.scalar_type(), "sconv_wgrad: dy dtype");
  const int B = x.size(0), Hi = x.size(1), Wi = x.size(2), Cin = x.size(3);
  const int Ho = dy.size(1), Wo = dy.size(2), Cout = dy.size(3);
  TORCH_CHECK(x.stride(3) == 1 && x.stride(2) % 8 == 0 && x.stride(1) == Wi * x.stride(2) &&
                  x.stride(0) == Hi * x.stride(1) && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "sconv_wgrad: x must be dense NHWC pixels with a channel stride % 8 == 0, 16-B aligned");
  TORCH_CHECK(dy.stride(3) == 1 && dy.stride(1) == Wo * dy.stride(2) && dy.stride(0) == Ho * dy.stride(1) &&
                  dy.stride(2) % 4 == 0 && reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0 && Cout % 4 == 0,
              "sconv_wgrad: dy must be dense 16-B aligned NHWC pixels, channel stride % 4 == 0, Cout % 4 == 0");
  TORCH_CHECK(Cin % 8 == 0 && dy.size(0) == B && stride >= 1 && pad >= 0 && KH >= 1 && KW >= 1,
              "sconv_wgrad: shapes");
  TORCH_CHECK(Ho == (Hi + 2 * pad - KH) / stride + 1 && Wo == (Wi + 2 * pad - KW) / stride + 1,
              "sconv_wgrad: dy grid does not match the conv geometry");
  TORCH_CHECK(dw.is_cuda() && dw.is_contiguous() && dw.scalar_type() == at::kFloat &&
                  dw.numel() == (int64_t)Cout * KH * KW * Cin,
              "sconv_wgrad: dw fp32 [Cout, KH, KW, Cin]");
  const int OUT = Cout * KH * KW * Cin;
  int rows = 0;
  const int nblk = rs::sconv_wgrad_blocks(B, Ho, OUT, &rows);
  const c10::DeviceGuard guard(x.device());
  Tensor part = at::empty({(int64_t)nblk * OUT}, dw.options());
  rs::SconvWgradLaunch L{};
  L.x = x.data_ptr(); L.dy = dy.data_ptr(); L.xstr = x.stride(2); L.ystr = dy.stride(2);
  L.Cin = Cin; L.Cout = Cout; L.B = B; L.Hi = Hi; L.Wi = Wi; L.Ho = Ho; L.Wo = Wo;
  L.KH = KH; L.KW = KW; L.S = stride; L.P = pad; L.f32 = x.scalar_type() == at::kFloat;
  L.dw = dw.data_ptr<float>(); L.part = part.data_ptr<float>();
  rs::sconv_wgrad_launch(L, nblk, rows, stream());
  RS_CHECK_LAUNCH();
}

Tensor enc_wgrad(const Tensor& dy, const Tensor& x) {
  check_nhwc_view(dy, "enc_wgrad dy");
  check_nhwc_view(x, "enc_wgrad x");
  const int B = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3), Cout = dy.size(3);
  TORCH_CHECK(dy.size(0) == B && dy.size(1) == H && dy.size(2) == W, "enc_wgrad: dy / x shapes");
  TORCH_CHECK(Cin % 32 == 0 && Cout % 32 == 0 && Cin >= 64 && Cout >= 64 && Cin <= 512 && Cout <= 512,
              "enc_wgrad: channel counts must be multiples of 32, >= 64");
  const c10::DeviceGuard guard(x.device());
  rs::EncWgradLaunch L{};
  L.x = x.data_ptr();
  L.dy = dy.data_ptr();
  L.xstr = x.stride(2);
  L.ystr = dy.stride(2);
  L.x_bytes = (long)B * H * W * L.xstr * 2;
  L.dy_bytes = (long)B * H * W * L.ystr * 2;
  L.B = B; L.H = H; L.W = W; L.Cin = Cin; L.Cout = Cout;
  L.nsplit = rs::enc_wgrad_splits(B, H, W, Cin, Cout, &L.tpb);
  const int64_t nblk = int64_t(L.nsplit) * ((Cout + 63) / 64) * ((Cin + 63) / 64);
  Tensor part = at::empty({nblk * 64 * 9 * 64}, x.options().dtype(at::kFloat));
  // channels_last: the element order the reduce kernel writes (co, tap, ci)
  Tensor dw = at::empty({Cout, Cin, 3, 3}, x.options().dtype(at::kFloat).memory_format(at::MemoryFormat::ChannelsLast));
  L.part = part.data_ptr<float>();
  L.dw = dw.data_ptr<float>();
  rs::enc_wgrad_launch(L, stream());
  RS_CHECK_LAUNCH();
  return dw;
}

void colsum(const Tensor& dy, int64_t yoff, int64_t C, const Tensor& db) {
  TORCH_CHECK(dy.is_cuda() && dy.is_contiguous() && dy.scalar_type() == at::kBFloat16, "colsum: bf16 dy");
  TORCH_CHECK(yoff >= 0 && yoff + C <= dy.size(-1), "colsum: channel window");
  TORCH_CHECK(db.is_cuda() && db.scalar_type() == at::kFloat && db.numel() >= C, "colsum: fp32 db");
  const c10::DeviceGuard guard(dy.device());
  const int P = dy.numel() / dy.size(-1);
  Tensor part;
  if (rs::deterministic()) part = at::empty({int64_t(rs::colsum_blocks(P)) * C}, dy.options().dtype(at::kFloat));
  rs::colsum_launch(dy.data_ptr(), dy.size(-1), yoff, C, P, db.data_ptr<float>(),
                    part.defined() ? part.data_ptr<float>() : nullptr, stream());
  RS_CHECK_LAUNCH();
}

void flow_wgrad(const Tensor& coords, const Tensor& df, const Tensor& dw, const Tensor& db) {
  TORCH_CHECK(coords.is_cuda() && coords.is_contiguous() && coords.scalar_type() == at::kFloat && coords.dim() == 4 &&
                  coords.size(1) == 2,
              "flow_wgrad: coords fp32 (B',2,H,W)");
  const int Bp = coords.size(0), H = coords.size(2), W = coords.size(3);
  const bool f32 = df.scalar_type() == at::kFloat;  // fp32 training engine
  TORCH_CHECK(df.is_cuda() && df.is_contiguous() && (f32 || df.scalar_type() == at::kBFloat16) && df.dim() == 4 &&
                  df.size(0) == Bp && df.size(1) == H && df.size(2) == W,
              "flow_wgrad: df bf16 / fp32 (B',H,W,C)");
  const int Cout = db.numel();
  TORCH_CHECK(Cout <= df.size(3) && Cout <= 128 && dw.numel() == 98 * Cout && dw.scalar_type() == at::kFloat &&
                  db.scalar_type() == at::kFloat,
              "flow_wgrad: dw fp32 [49][2][Cout], db fp32 [Cout]");
  TORCH_CHECK(W <= 1024, "flow_wgrad: row width <= 1024 (LDS staging)");
  TORCH_CHECK(dw.is_contiguous() && db.is_contiguous(), "flow_wgrad: dw, db contiguous");
  const c10::DeviceGuard guard(coords.device());
  Tensor part;
  if (rs::deterministic())
    part = at::empty({int64_t(rs::flow_wgrad_blocks(Bp, H)) * 99 * Cout}, coords.options());
  rs::flow_wgrad_launch(coords.data_ptr<float>(), Bp, H, W, df.data_ptr(), df.size(3), Cout, dw.data_ptr<float>(),
                        db.data_ptr<float>(), part.defined() ? part.data_ptr<float>() : nullptr, f32, stream());
  RS_CHECK_LAUNCH();
}

// One ConvGRU pass backward through the gates (see csrc/conv.hip gru_gate_bwd_kernel).
void gru_gate_bwd(const Tensor& dh, const Tensor& z, const Tensor& q, const Tensor& h, int64_t hoff, const Tensor& dq,
                  const Tensor& dzr) {
  const int hd = z.size(-1);
  const int64_t P = z.numel() / hd;
  auto chk = [&](const Tensor& t, at::ScalarType dt, int minc, const char* n) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == dt && t.numel() / t.size(-1) == P &&
                    t.size(-1) >= minc,
                "gru_gate_bwd: ", n);
  };
  const bool f32 = z.scalar_type() == at::kFloat;  // fp32 training engine
  const at::ScalarType adt = f32 ? at::kFloat : at::kBFloat16;
  chk(dh, at::kFloat, hd, "dh (fp32)");
  chk(z, adt, hd, "z");
  chk(q, adt, hd, "q");
  chk(h, adt, hoff + hd, "h");
  chk(dq, adt, hd, "dq");
  chk(dzr, adt, hd, "dzr");
  const c10::DeviceGuard guard(z.device());
  rs::gru_gate_bwd_launch(dh.data_ptr<float>(), dh.size(-1), z.data_ptr(), hd, q.data_ptr(), q.size(-1), h.data_ptr(),
                          h.size(-1), hoff, dq.data_ptr(), dq.size(-1), dzr.data_ptr(), dzr.size(-1), P, hd, f32,
                          stream());
  RS_CHECK_LAUNCH();
}

// out = G[:, goff:goff+n] * (act[:, aoff:aoff+n] > 0) (zero-padded to out's width); G[:, goff:goff+nz] = 0
void relu_take(const Tensor& G, int64_t goff, int64_t n, int64_t nz, const Tensor& act, int64_t aoff, const Tensor& out) {
  const int64_t P = out.numel() / out.size(-1);
  TORCH_CHECK(G.is_cuda() && G.is_contiguous() && G.scalar_type() == at::kFloat && G.numel() / G.size(-1) == P &&
                  goff + std::max(n, nz) <= G.size(-1),
              "relu_take: G");
  const bool f32 = out.scalar_type() == at::kFloat;  // fp32 training engine
  const at::ScalarType adt = f32 ? at::kFloat : at::kBFloat16;
  TORCH_CHECK(act.is_contiguous() && act.scalar_type() == adt && act.numel() / act.size(-1) == P &&
                  aoff + n <= act.size(-1),
              "relu_take: act (the out dtype)");
  TORCH_CHECK(out.is_contiguous() && out.scalar_type() == adt && n <= out.size(-1), "relu_take: out");
  const c10::DeviceGuard guard(out.device());
  rs::relu_take_launch(G.data_ptr<float>(), G.size(-1), goff, n, nz, act.data_ptr(), act.size(-1), aoff, out.data_ptr(),
                       out.size(-1), P, f32, stream());
  RS_CHECK_LAUNCH();
}

int num_cus(int dev) {
  static int n[64] = {0};
  if (dev < 0 || dev >= 64) return 256;
  if (n[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    n[dev] = v;
  }
  return n[dev];
}

// Stride-1 3x3 'same' conv on the halo-tile kernel (csrc/enc_halo.hip):
// x NHWC (cin of its x.size(3) channels), w packed [Cout_pad][9][Ktot], y NHWC
// (cout of its y.size(3) channels), no bias.
void conv3x3_halo(const Tensor& x, const Tensor& w, const Tensor& y, int64_t cin, int64_t cout,
                  const c10::optional<Tensor>& nscale,
                  const c10::optional<Tensor>& nshift, const c10::optional<Tensor>& res, bool relu,
                  bool accumulate) {
  TORCH_CHECK(x.dim() == 4, "conv3x3_halo: x must be NHWC");
  const int B = x.size(0), H = x.size(1), W = x.size(2);
  check_nhwc(x, B, H, W, "conv3x3_halo: x");
  check_nhwc(y, B, H, W, "conv3x3_halo: y");
  TORCH_CHECK(rs::enc_halo_supported(cin, cout), "conv3x3_halo: unsupported channels ", cin, "->", cout);
  TORCH_CHECK(cin <= x.size(3) && x.size(3) % 8 == 0, "conv3x3_halo: x channels");
  TORCH_CHECK(cout <= y.size(3) && y.size(3) % 4 == 0, "conv3x3_halo: y channels");
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == at::kBFloat16 && w.dim() == 3 &&
                  w.size(0) >= cout && w.size(1) == 9 && w.size(2) >= cin && w.size(2) % 8 == 0,
              "conv3x3_halo: w must be packed [Cout_pad>=cout][9][Ktot>=cin] bf16");
  TORCH_CHECK(((uintptr_t)x.data_ptr() | (uintptr_t)w.data_ptr()) % 16 == 0 && (uintptr_t)y.data_ptr() % 8 == 0,
              "conv3x3_halo: alignment");
  TORCH_CHECK(x.numel() < (int64_t(1) << 31) && y.numel() < (int64_t(1) << 31), "conv3x3_halo: tensor too large");
  rs::EncEpi e;
  const NormX nx = norm_extras(nscale, nshift, nscale ? EPI_NORM : 0, cout, "conv3x3_halo");
  e.chs = nx.chs;
  e.shift = nscale ? nshift->data_ptr<float>() : nullptr;
  TORCH_CHECK(!relu || nscale, "conv3x3_halo: relu goes with nscale / nshift");
  TORCH_CHECK(!res || nscale, "conv3x3_halo: the residual goes with nscale / nshift");
  e.relu = relu ? 1 : 0;
  if (res) {
    check_nhwc(*res, B, H, W, "conv3x3_halo: res");
    TORCH_CHECK(cout <= res->size(3) && res->size(3) % 4 == 0 && (uintptr_t)res->data_ptr() % 8 == 0,
                "conv3x3_halo: res channels / alignment");
    e.res = static_cast<const uint16_t*>(res->data_ptr());
    e.rstr = res->size(3);
  }
  if (accumulate) {  // y += conv(x): the epilogue reads y as a plain (no ReLU) residual
    TORCH_CHECK(!res && !nscale, "conv3x3_halo: accumulate excludes res / nscale");
    e.res = static_cast<const uint16_t*>(y.data_ptr());
    e.rstr = y.size(3);
    e.res_relu = 0;
  }
  const c10::DeviceGuard guard(x.device());
  rs::enc_halo_launch(static_cast<const uint16_t*>(x.data_ptr()), x.size(3), static_cast<const uint16_t*>(w.data_ptr()),
                      w.size(2), static_cast<uint16_t*>(y.data_ptr()), y.size(3), B, H, W, cin, cout,
                      num_cus(x.get_device()), e, stream());
  RS_CHECK_LAUNCH();
}

// 7x7 / stride-2 / pad-3 stem conv, 3 -> Cout <= 64 (csrc/stem.hip).
//   x: NHWC image [B, Hi, Wi, 3] fp32 or bf16; w: packed [64][7][32] bf16 (k = kx*3 + ci;
//   fp32 output: the split [64][7][64] layout); out: NHWC [B, Ho, Wo, >= Cout] (bf16, or
//   fp32 -> the split-bf16 MFMA path); epi 0 (+ bias) or EPI_NORM (nscale with
//   bias = shift, relu).
void stem_conv(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, const Tensor& out, int64_t Cout,
               int64_t epi, const c10::optional<Tensor>& nscale, bool relu) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4 && x.size(3) == 3 &&
                  (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16),
              "stem_conv: x must be a contiguous NHWC [B,H,W,3] fp32 / bf16 image");
  const int B = x.size(0), Hi = x.size(1), Wi = x.size(2);
  const int Ho = (Hi + 6 - 7) / 2 + 1, Wo = (Wi + 6 - 7) / 2 + 1;
  const bool f32 = out.scalar_type() == at::kFloat;
  check_nhwc(out, B, Ho, Wo, "stem_conv: out", f32 ? at::kFloat : at::kBFloat16);
  TORCH_CHECK(Cout >= 1 && Cout <= 64 && Cout % 4 == 0 && out.size(3) >= Cout && out.size(3) % 4 == 0,
              "stem_conv: Cout must be a multiple of 4 in [4, 64]");
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == at::kBFloat16 && w.dim() == 3 &&
                  w.size(0) == 64 && w.size(1) == 7 && w.size(2) == (f32 ? 64 : 32),
              "stem_conv: packed weight must be bf16 [64][7][", f32 ? 64 : 32, "]");
  TORCH_CHECK(epi == 0 || epi == EPI_NORM, "stem_conv: epilogue 0 (bias) or EPI_NORM");
  if (bias)
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kFloat && bias->is_contiguous() &&
                    bias->numel() >= Cout, "stem_conv: bias fp32 (Cout,)");
  const NormX nx = norm_extras(nscale, bias, epi, Cout, "stem_conv");
  TORCH_CHECK(!relu || epi == EPI_NORM, "stem_conv: relu goes with EPI_NORM");
  TORCH_CHECK((uintptr_t)out.data_ptr() % 16 == 0, "stem_conv: out alignment");
  TORCH_CHECK(out.numel() < (int64_t(1) << 31) && x.numel() < (int64_t(1) << 31), "stem_conv: size");
  rs::StemLaunch L{};
  L.x = x.data_ptr(); L.x_bf16 = x.scalar_type() == at::kBFloat16;
  L.B = B; L.Hi = Hi; L.Wi = Wi; L.Ho = Ho; L.Wo = Wo;
  L.w = w.data_ptr(); L.bias = bias ? bias->data_ptr<float>() : nullptr;
  L.Cout = Cout; L.epi = epi; L.relu = relu ? 1 : 0;
  L.out = out.data_ptr(); L.ostr = out.size(3); L.ooff = 0;
  L.chs = nx.chs; L.f32 = f32 ? 1 : 0;
  const c10::DeviceGuard guard(x.device());
  rs::stem_launch(L, stream());
  RS_CHECK_LAUNCH();
}

// dW (fp32 [Cout][3][7][7]) of the stem conv from dy (NHWC bf16 [B, Ho, Wo, >= Cout],
// contiguous) and the image x: deterministic (per-block partials, ordered sum).
void stem_wgrad(const Tensor& x, const Tensor& dy, int64_t Cout, const Tensor& dw) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4 && x.size(3) == 3 &&
                  (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16),
              "stem_wgrad: x must be a contiguous NHWC [B,H,W,3] image");
  const int B = x.size(0), Hi = x.size(1), Wi = x.size(2);
  const int Ho = (Hi + 6 - 7) / 2 + 1, Wo = (Wi + 6 - 7) / 2 + 1;
  check_nhwc(dy, B, Ho, Wo, "stem_wgrad: dy");
  TORCH_CHECK(Cout >= 1 && Cout <= 64 && dy.size(3) >= Cout && dy.size(3) % 8 == 0 &&
                  (uintptr_t)dy.data_ptr() % 16 == 0, "stem_wgrad: dy channels / alignment");
  TORCH_CHECK(dw.is_cuda() && dw.is_contiguous() && dw.scalar_type() == at::kFloat && dw.numel() == Cout * 147,
              "stem_wgrad: dw must be fp32 [Cout][3][7][7]");
  int per = 0;
  const int nblk = rs::stem_wgrad_blocks(B, Ho, Wo, &per);
  const c10::DeviceGuard guard(x.device());
  Tensor part = at::empty({(int64_t)nblk * 64 * 224}, dw.options());
  rs::stem_wgrad_launch(x.data_ptr(), x.scalar_type() == at::kBFloat16, B, Hi, Wi, Ho, Wo,
                        static_cast<const uint16_t*>(dy.data_ptr()), dy.size(3), Cout, part.data_ptr<float>(), nblk,
                        per, dw.data_ptr<float>(), stream());
  RS_CHECK_LAUNCH();
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(raft_stir, m) {
  m.def("stem_conv(Tensor x, Tensor w, Tensor? bias, Tensor(a!) out, int Cout, int epi, Tensor? nscale=None, "
        "bool relu=False) -> ()");
  m.def("stem_wgrad(Tensor x, Tensor dy, int Cout, Tensor(a!) dw) -> ()");
  m.def("conv3x3_halo(Tensor x, Tensor w, Tensor(a!) y, int cin, int cout, "
        "Tensor? nscale=None, Tensor? nshift=None, Tensor? res=None, "
        "bool relu=False, bool accumulate=False) -> ()");
  m.def("conv_wgrad(Tensor dy, int yoff, int Cout, Tensor[] segs, int[] seg_off, int[] seg_C, int[] seg_period, "
        "int KH, int KW, Tensor(a!) dw, Tensor(b!)? db=None, int bn128=0) -> ()");
  m.def("flow_head(Tensor x, int xoff, int cin, Tensor w, Tensor bias, Tensor(a!) crd, Tensor? src) -> ()");
  m.def("flow_head_dgrad(Tensor dflow, Tensor w, int cin, Tensor act, int aoff, Tensor(a!) out, int ooff) -> ()");
  m.def("colsum(Tensor dy, int yoff, int C, Tensor(a!) db) -> ()");
  m.def("flow_wgrad(Tensor coords, Tensor df, Tensor(a!) dw, Tensor(b!) db) -> ()");
  m.def("conv_wgrad_strided(Tensor dy, int Cout, Tensor[] segs, int[] seg_off, int[] seg_C, int KH, int KW, "
        "int SY, int SX, Tensor(a!) dw, Tensor(b!)? db) -> ()");
  m.def("gru_gate_bwd(Tensor(a!) dh, Tensor z, Tensor q, Tensor h, int hoff, Tensor(b!) dq, Tensor(c!) dzr) -> ()");
  m.def("relu_take(Tensor(a!) G, int goff, int n, int nz, Tensor act, int aoff, Tensor(b!) out) -> ()");
  m.def("conv_fused(Tensor[] segs, int[] seg_off, int[] seg_C, Tensor w, Tensor? bias, int KH, int KW, "
        "int Cout, int epi, float scale, int hd, Tensor(a!) out, int ooff, Tensor(b!)? out2, int o2off, "
        "Tensor(c!)? out3, int o3off, Tensor? aux1, int a1off, Tensor? aux2, int a2off, int tile, "
        "Tensor? nscale=None) -> ()");
  m.def("enc_wgrad(Tensor dy, Tensor x) -> Tensor");
  m.def("sconv_wgrad(Tensor dy, Tensor x, int KH, int KW, int stride, int pad, Tensor(a!) dw) -> ()");
  m.def("sconv(Tensor x, Tensor w, Tensor? bias, int stride, int pad, bool relu, Tensor(a!) out, int yoff, "
        "Tensor? res) -> ()");
  m.def("conv_geo(Tensor[] segs, int[] seg_off, int[] seg_C, Tensor w, Tensor? bias, int KH, int KW, int PH, "
        "int PW, int SY, int SX, int Ho, int Wo, int Cout, Tensor(a!) out, int ooff, int OSY, int OSX, int OOY, "
        "int OOX, int tile, Tensor? nscale=None, bool relu=False) -> ()");
  m.def("flow_encode(Tensor coords, Tensor w, Tensor bias, Tensor(a!) out, int ooff, Tensor(b!)? fout, "
        "int foff) -> ()");
}

TORCH_LIBRARY_IMPL(raft_stir, CUDA, m) {
  m.impl("conv_fused", &conv_fused);
  m.impl("conv3x3_halo", &conv3x3_halo);
  m.impl("enc_wgrad", &enc_wgrad);
  m.impl("sconv_wgrad", &sconv_wgrad);
  m.impl("sconv", &sconv);
  m.impl("stem_conv", &stem_conv);
  m.impl("stem_wgrad", &stem_wgrad);
  m.impl("conv_geo", &conv_geo);
  m.impl("flow_encode", &flow_encode);
  m.impl("flow_head", &flow_head);
  m.impl("flow_head_dgrad", &flow_head_dgrad);
  m.impl("conv_wgrad", &conv_wgrad);
  m.impl("colsum", &colsum);
  m.impl("flow_wgrad", &flow_wgrad);
  m.impl("conv_wgrad_strided", &conv_wgrad_strided);
  m.impl("gru_gate_bwd", &gru_gate_bwd);
  m.impl("relu_take", &relu_take);
}
