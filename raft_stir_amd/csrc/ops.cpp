// Operator registration: torch.ops.raft_stir.*  (TORCH_LIBRARY, no pybind).
//
// Replaces reference alt_cuda_corr/correlation.cpp (pybind module with
// CHECK_CUDA/CHECK_CONTIGUOUS, launching on the legacy default stream).  Every
// op here validates shapes/dtypes/devices on the host BEFORE launching (a bad
// shape must never reach a kernel) and launches on PyTorch's current HIP
// stream, so the ops compose with torch streams and hipGraph capture.

#include <stdlib.h>
#include <atomic>
#include <ATen/ATen.h>
#include "host_common.h"
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <cmath>
#include <vector>

#include <hip/hip_runtime.h>

namespace rs {
// Deterministic mode (torch.ops.raft_stir.set_deterministic): the kernels that
// accumulate with fp32 atomics (weight / bias gradients, flow-encoder weight
// gradient) write per-split partials reduced in a fixed order instead, and the
// ops that have no such variant refuse to run.
static std::atomic<bool> g_deterministic{false};
bool deterministic() { return g_deterministic.load(std::memory_order_relaxed); }

void corr_volume_launch(const void* f1, const void* f2, bool bf16, int B, int N1, int H2, int W2,
                        int C, int levels, void* const* out, const int* Hs, const int* Ws, const int* Ss,
                        bool out_bf16, void* ws, float scale, hipStream_t stream);
void corr_lookup_fwd_launch(const void* const* pyr, bool pyr_bf16, const int* Hs, const int* Ws, const int* Ss,
                            int levels, const float* coords, int B, int H1, int W1, int r, void* out,
                            bool out_bf16, hipStream_t stream, int ostride);
void corr_lookup_bwd_launch(float* const* gpyr, const int* Hs, const int* Ws, const int* Ss, int levels,
                            const float* coords, int B, int H1, int W1, int r, const void* dout,
                            bool dout_bf16, hipStream_t stream, int dstride);
size_t corr_volume_split_ws(int B, int N1, int C, int levels, const int* Hs, const int* Ws);
int corr_bwd_pitch(int N2);
void upflow8_bwd_launch(const float* g, const float* ah, const float* aw, int NC, int H, int W, float* tmp,
                        float* out, hipStream_t stream);
size_t upflow8_cols_lds(int W);
void corr_bwd_gemm_launch(const void* G, const void* Gl, int Ep, const void* f1, const void* f1l, const void* f2,
                          const void* f2l, int B, int N1, int N2, int C, void* df1, void* df2, hipStream_t stream);
void pyr_grad_fold_launch(float* const* gpyr, const int* Hs, const int* Ws, const int* Ss, int levels, long rows,
                          float scale, hipStream_t stream, void* out_bf16 = nullptr, int opitch = 0,
                          void* out_lo = nullptr);
void wpack_gather_launch(const int* code, long long n, const long long* tab, void* out, bool out_bf16,
                         const long long* lo, const long long* hi, const float* s, int nr, hipStream_t stream);
void split_bf16_launch(const float* x, long n, uint16_t* hi, uint16_t* lo, hipStream_t s);
bool corr_otf_supported_channels(int C);
void corr_otf_fwd_launch(const void* f1, const void* const* f2, const int* Hs, const int* Ws,
                         int levels, bool fm_bf16, const float* coords, int B, int H1, int W1, int C,
                         int r, float scale, void* out, bool out_bf16, hipStream_t stream);
void corr_otf_bwd_launch(const void* f1, const void* const* f2, const int* Hs, const int* Ws,
                         int levels, bool fm_bf16, const float* coords, int B, int H1, int W1, int C,
                         int r, float scale, const void* dout, bool dout_bf16, float* df1,
                         float* const* df2, bool det, float* const* df2f, unsigned* fxs, hipStream_t stream);
void convex_up_fwd_launch(const float* flow, const void* mask, bool mask_bf16, int N, int H, int W,
                          float* out, hipStream_t stream);
void convex_up_bwd_launch(const float* flow, const void* mask, bool mask_bf16, const void* dup,
                          bool dup_bf16, int N, int H, int W, void* dmask, int dpitch, float* dflow,
                          float* partial, hipStream_t stream);
void ctx_act_launch(bool bf, const void* cn, long P, int hd, int cd, void* hx, int hxp, void* inp, int ip,
                    hipStream_t s);
void ctx_act_bwd_launch(bool bf, const float* G, int gp, const void* hx, int hxp, const void* inp, int ip, long P,
                        int hd, int cd, void* dcn, hipStream_t s);
void gru_gate_zr_launch(bool bf, const void* zr, const void* h, const void* x, long P, int hd,
                        int cin, void* z, void* r, void* rhx, hipStream_t s);
void gru_gate_q_launch(bool bf, const void* q, const void* z, const void* h, long P, int hd,
                       void* hn, void* qt, hipStream_t s);
void gru_bwd_q_launch(bool bf, const void* dhn, bool dhn_bf, const void* z, const void* h,
                      const void* qt, long P, int hd, void* dq, void* dzr, float* dh,
                      hipStream_t s);
void gru_bwd_r_launch(bool bf, const void* drhx, const void* h, const void* r, long P, int hd,
                      int cin, void* dzr, hipStream_t s);
void gru_bwd_fin_launch(bool bf, const float* dhd, const void* drhx, const void* r,
                        const void* dhx, long P, int hd, int cin, void* dh, void* dx,
                        hipStream_t s);
}  // namespace rs

namespace {

using at::Tensor;

hipStream_t cur_stream() { return rs::current_stream(); }

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous (got strides ", t.strides(), ")");
}
void check_dtype(const Tensor& t, std::initializer_list<at::ScalarType> ok, const char* name) {
  for (auto s : ok)
    if (t.scalar_type() == s) return;
  TORCH_CHECK(false, name, " has unsupported dtype ", t.scalar_type());
}
bool is_bf16(const Tensor& t) { return t.scalar_type() == at::kBFloat16; }

// Pooled sizes with floor semantics (avg_pool2d(2,2) applied l times).
void level_sizes(int H, int W, int levels, int* Hs, int* Ws) {
  for (int l = 0; l < levels; ++l) {
    Hs[l] = H;
    Ws[l] = W;
    H /= 2;
    W /= 2;
  }
}

// ---------------------------------------------------------------- corr volume
// Pyramid levels are (B, N1, H_l, W_l) views whose (b, i) rows start at a
// padded pitch S_l = round_up(H_l*W_l, 64) elements (128-B aligned rows for the
// flat volume kernel's whole-line stores); fp32, or bf16 when out_bf16.
// RS_CORR_F32_SPLIT=0: the exact-fp32 MFMA kernel (mfma_f32_16x16x4f32) for fp32 maps instead
static bool split_f32_volume() {
  static const bool on = [] {
    const char* e = getenv("RS_CORR_F32_SPLIT");
    return !(e && e[0] == '0');
  }();
  return on;
}

std::vector<Tensor> corr_volume(const Tensor& f1, const Tensor& f2, int64_t levels, double scale, bool out_bf16) {
  check_gpu(f1, "f1");
  check_gpu(f2, "f2");
  check_dtype(f1, {at::kFloat, at::kBFloat16}, "f1");
  TORCH_CHECK(f1.scalar_type() == f2.scalar_type(), "f1/f2 dtype mismatch");
  TORCH_CHECK(f1.dim() == 3 && f2.dim() == 4, "f1 must be (B,N1,C), f2 (B,H2,W2,C)");
  TORCH_CHECK(levels >= 1 && levels <= 4, "levels must be in [1,4]");
  const int B = f1.size(0), N1 = f1.size(1), C = f1.size(2);
  const int H2 = f2.size(1), W2 = f2.size(2);
  TORCH_CHECK(f2.size(0) == B && f2.size(3) == C, "f1/f2 batch/channel mismatch");
  TORCH_CHECK(C % (is_bf16(f1) ? 64 : 32) == 0, "channels must be a multiple of 64 (bf16) / 32");
  const c10::DeviceGuard guard(f1.device());
  int Hs[4], Ws[4];
  level_sizes(H2, W2, levels, Hs, Ws);
  for (int l = 0; l < levels; ++l) TORCH_CHECK(Hs[l] > 0 && Ws[l] > 0, "pyramid level ", l, " is empty");
  TORCH_CHECK(!out_bf16 || is_bf16(f1), "corr_volume: a bf16 pyramid needs bf16 feature maps");
  std::vector<Tensor> outs;
  void* ptrs[4];
  int Ss[4];
  const auto odt = out_bf16 ? at::kBFloat16 : at::kFloat;
  for (int l = 0; l < levels; ++l) {
    Ss[l] = (Hs[l] * Ws[l] + 63) / 64 * 64;
    Tensor store = at::empty({(int64_t)B * N1 * Ss[l]}, f1.options().dtype(odt));
    outs.push_back(store.as_strided({B, N1, Hs[l], Ws[l]}, {(int64_t)N1 * Ss[l], Ss[l], Ws[l], 1}));
    ptrs[l] = store.data_ptr();
  }
  Tensor ws;
  if (is_bf16(f1) && levels > 1) {
    int64_t n = 0;
    for (int l = 1; l < levels; ++l) n += (int64_t)B * Hs[l] * Ws[l] * C;
    ws = at::empty({n}, f1.options());
  } else if (!is_bf16(f1) && split_f32_volume() && (3 * C) % 64 == 0 && f1.is_contiguous() && f2.is_contiguous()) {
    // fp32 maps: split-bf16 operands on the flat MFMA GEMM (csrc/corr_volume.hip split3_kernel)
    ws = at::empty({(int64_t)rs::corr_volume_split_ws(B, N1, C, levels, Hs, Ws) / 2}, f1.options().dtype(at::kBFloat16));
  }
  rs::corr_volume_launch(f1.data_ptr(), f2.data_ptr(), is_bf16(f1), B, N1, H2, W2, C, levels, ptrs,
                         Hs, Ws, Ss, out_bf16, ws.defined() ? ws.data_ptr() : nullptr, (float)scale, cur_stream());
  RS_CHECK_LAUNCH();
  return outs;
}

// Pyramid level l: (B, N1, H_l, W_l) with unit x stride, row stride W_l and a
// (b, i) row pitch S_l >= H_l*W_l (corr_volume pads it; plain contiguous tensors
// have S_l = H_l*W_l).  Every level one dtype: fp32 (gradients: always) or bf16.
void check_pyr(const std::vector<Tensor>& pyr, int B, int N1, int* Hs, int* Ws, int* Ss, bool allow_bf16 = false) {
  TORCH_CHECK(!pyr.empty() && pyr.size() <= 4, "pyramid must have 1..4 levels");
  for (size_t l = 0; l < pyr.size(); ++l) {
    TORCH_CHECK(pyr[l].is_cuda(), "pyramid level must be a GPU tensor");  // rows may be padded (strides below)
    if (allow_bf16) check_dtype(pyr[l], {at::kFloat, at::kBFloat16}, "pyramid level");
    else check_dtype(pyr[l], {at::kFloat}, "pyramid level");
    TORCH_CHECK(pyr[l].scalar_type() == pyr[0].scalar_type(), "pyramid levels must share one dtype");
    TORCH_CHECK(pyr[l].dim() == 4 && pyr[l].size(0) == B && pyr[l].size(1) == N1,
                "pyramid level ", l, " must be (B, H1*W1, H_l, W_l)");
    Hs[l] = pyr[l].size(2);
    Ws[l] = pyr[l].size(3);
    Ss[l] = pyr[l].stride(1);
    TORCH_CHECK(pyr[l].stride(3) == 1 && pyr[l].stride(2) == Ws[l] && Ss[l] >= Hs[l] * Ws[l] &&
                    pyr[l].stride(0) == (int64_t)N1 * Ss[l],
                "pyramid level ", l, ": rows must be dense (pitch >= H*W)");
  }
}

void check_coords(const Tensor& coords) {
  check_gpu(coords, "coords");
  check_dtype(coords, {at::kFloat}, "coords");
  TORCH_CHECK(coords.dim() == 4 && coords.size(1) == 2, "coords must be (B,2,H,W)");
}

// ---------------------------------------------------------------- lookup
Tensor corr_lookup(const std::vector<Tensor>& pyr, const Tensor& coords, int64_t radius,
                   bool out_bf16) {
  check_coords(coords);
  const int B = coords.size(0), H1 = coords.size(2), W1 = coords.size(3);
  int Hs[4], Ws[4], Ss[4];
  check_pyr(pyr, B, H1 * W1, Hs, Ws, Ss, true);
  TORCH_CHECK(radius >= 0 && radius <= 4, "radius must be in [0,4]");
  const c10::DeviceGuard guard(coords.device());
  const int levels = pyr.size();
  const int D = 2 * radius + 1;
  Tensor out = at::empty({B, H1, W1, levels * D * D},
                         coords.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  const void* ptrs[4];
  for (int l = 0; l < levels; ++l) ptrs[l] = pyr[l].data_ptr();
  rs::corr_lookup_fwd_launch(ptrs, is_bf16(pyr[0]), Hs, Ws, Ss, levels, coords.data_ptr<float>(), B, H1, W1,
                             radius, out.data_ptr(), out_bf16, cur_stream(), 0);
  RS_CHECK_LAUNCH();
  return out;
}

// Lookup into a preallocated channels-last buffer whose rows may be wider than
// levels*(2r+1)^2 (K-aligned for the fused conv); the padding is zeroed.
void corr_lookup_into(const std::vector<Tensor>& pyr, const Tensor& coords, int64_t radius,
                      const Tensor& out) {
  check_coords(coords);
  const int B = coords.size(0), H1 = coords.size(2), W1 = coords.size(3);
  int Hs[4], Ws[4], Ss[4];
  check_pyr(pyr, B, H1 * W1, Hs, Ws, Ss, true);
  TORCH_CHECK(radius >= 0 && radius <= 4, "radius must be in [0,4]");
  const int levels = pyr.size();
  const int D = 2 * radius + 1;
  check_gpu(out, "out");
  check_dtype(out, {at::kFloat, at::kBFloat16}, "out");
  TORCH_CHECK(out.dim() == 4 && out.size(0) == B && out.size(1) == H1 && out.size(2) == W1 &&
                  out.size(3) >= levels * D * D,
              "out must be (B,H1,W1,>=levels*(2r+1)^2)");
  const c10::DeviceGuard guard(coords.device());
  const void* ptrs[4];
  for (int l = 0; l < levels; ++l) ptrs[l] = pyr[l].data_ptr();
  rs::corr_lookup_fwd_launch(ptrs, is_bf16(pyr[0]), Hs, Ws, Ss, levels, coords.data_ptr<float>(), B, H1, W1,
                             radius, out.data_ptr(), is_bf16(out), cur_stream(), out.size(3));
  RS_CHECK_LAUNCH();
}

void corr_lookup_backward(const std::vector<Tensor>& gpyr, const Tensor& coords, int64_t radius,
                          const Tensor& dout) {
  check_coords(coords);
  const int B = coords.size(0), H1 = coords.size(2), W1 = coords.size(3);
  int Hs[4], Ws[4], Ss[4];
  check_pyr(gpyr, B, H1 * W1, Hs, Ws, Ss);
  const int levels = gpyr.size();
  const int D = 2 * radius + 1;
  check_gpu(dout, "dout");
  check_dtype(dout, {at::kFloat, at::kBFloat16}, "dout");
  TORCH_CHECK(dout.dim() == 4 && dout.size(0) == B && dout.size(1) == H1 && dout.size(2) == W1 &&
                  dout.size(3) >= levels * D * D,
              "dout must be (B,H1,W1,>=levels*(2r+1)^2) (rows may be K-padded)");
  const c10::DeviceGuard guard(coords.device());
  float* ptrs[4];
  for (int l = 0; l < levels; ++l) ptrs[l] = gpyr[l].data_ptr<float>();
  rs::corr_lookup_bwd_launch(ptrs, Hs, Ws, Ss, levels, coords.data_ptr<float>(), B, H1, W1, radius,
                             dout.data_ptr(), is_bf16(dout), cur_stream(), dout.size(3));
  RS_CHECK_LAUNCH();
}

void pyr_grad_fold(const std::vector<Tensor>& gpyr, double scale) {
  TORCH_CHECK(!gpyr.empty() && gpyr.size() <= 4, "pyramid must have 1..4 levels");
  const int B = gpyr[0].size(0), N1 = gpyr[0].size(1);
  int Hs[4], Ws[4], Ss[4];
  check_pyr(gpyr, B, N1, Hs, Ws, Ss);
  const c10::DeviceGuard guard(gpyr[0].device());
  float* ptrs[4];
  for (size_t l = 0; l < gpyr.size(); ++l) ptrs[l] = gpyr[l].data_ptr<float>();
  rs::pyr_grad_fold_launch(ptrs, Hs, Ws, Ss, gpyr.size(), (long)B * N1, (float)scale, cur_stream());
  RS_CHECK_LAUNCH();
}

// Same fold, written as bf16 into `out` (B, N1, H0, W0) instead of in place:
// the operand of the bf16 fmap-gradient GEMMs.
void pyr_grad_fold_bf16(const std::vector<Tensor>& gpyr, double scale, const Tensor& out) {
  TORCH_CHECK(!gpyr.empty() && gpyr.size() <= 4, "pyramid must have 1..4 levels");
  const int B = gpyr[0].size(0), N1 = gpyr[0].size(1);
  int Hs[4], Ws[4], Ss[4];
  check_pyr(gpyr, B, N1, Hs, Ws, Ss);
  check_gpu(out, "out");
  check_dtype(out, {at::kBFloat16}, "out");
  TORCH_CHECK(out.is_contiguous() && out.numel() == gpyr[0].numel(), "pyr_grad_fold_bf16: out shape");
  const c10::DeviceGuard guard(gpyr[0].device());
  float* ptrs[4];
  for (size_t l = 0; l < gpyr.size(); ++l) ptrs[l] = gpyr[l].data_ptr<float>();
  rs::pyr_grad_fold_launch(ptrs, Hs, Ws, Ss, gpyr.size(), (long)B * N1, (float)scale, cur_stream(), out.data_ptr());
  RS_CHECK_LAUNCH();
}

// Volume backward (csrc/corr_bwd.hip): the gradient pyramid folded once into
// a bf16 level-0 gradient G (rows padded to a multiple of 64 with zeros), then
// both feature-gradient GEMMs (df1 = G f2, df2 = G^T f1) in one MFMA launch.
// bf16 features -> bf16 gradients; fp32 features -> fp32 gradients through
// split-bf16 operands (G and the features as hi + lo pairs, three K passes).
// C % 128 == 0; deterministic (no atomics).
std::vector<Tensor> corr_volume_backward(const std::vector<Tensor>& gpyr, const Tensor& f1, const Tensor& f2,
                                         double scale) {
  check_gpu(f1, "f1");
  check_gpu(f2, "f2");
  check_dtype(f1, {at::kBFloat16, at::kFloat}, "f1");
  TORCH_CHECK(f2.scalar_type() == f1.scalar_type(), "corr_volume_backward: f1 / f2 dtypes differ");
  const bool split = f1.scalar_type() == at::kFloat;
  TORCH_CHECK(f1.dim() == 3 && f1.is_contiguous(), "corr_volume_backward: f1 must be contiguous (B, N1, C)");
  TORCH_CHECK(f2.dim() == 4 && f2.is_contiguous(), "corr_volume_backward: f2 must be contiguous (B, H2, W2, C)");
  const int B = f1.size(0), N1 = f1.size(1), C = f1.size(2);
  TORCH_CHECK(C % 128 == 0, "corr_volume_backward: feature channels must be a multiple of 128");
  TORCH_CHECK(f2.size(0) == B && f2.size(3) == C, "corr_volume_backward: f1 / f2 shapes");
  int Hs[4], Ws[4], Ss[4];
  check_pyr(gpyr, B, N1, Hs, Ws, Ss);
  TORCH_CHECK(Hs[0] == f2.size(1) && Ws[0] == f2.size(2), "corr_volume_backward: level 0 must be f2's grid");
  const int N2 = Hs[0] * Ws[0];
  const int Ep = rs::corr_bwd_pitch(N2);
  int64_t coarse = 0;
  for (size_t l = 1; l < gpyr.size(); ++l) coarse += (int64_t)Hs[l] * Ws[l];
  const bool rowfold = Ep <= 6144 && coarse <= 4096;
  // the row fold (<= 6144 cells; the only one with a split output) or, for
  // larger bf16 grids, the quad fold (16-B aligned level-0 rows)
  TORCH_CHECK(rowfold || (!split && Ss[0] % 4 == 0 && (uintptr_t)gpyr[0].data_ptr() % 16 == 0),
              "corr_volume_backward: grids over 6144 cells need bf16 features and 16-B aligned level-0 rows");
  TORCH_CHECK((int64_t)B * N1 * Ep * 2 < (int64_t(1) << 31) && (int64_t)B * std::max(N1, N2) * C * 2 < (int64_t(1) << 31),
              "corr_volume_backward: operands must be < 2 GiB");
  const c10::DeviceGuard guard(f1.device());
  auto bo = f1.options().dtype(at::kBFloat16);
  Tensor G = at::empty({(int64_t)B * N1, Ep}, bo);
  Tensor Gl = split ? at::empty({(int64_t)B * N1, Ep}, bo) : Tensor();
  float* ptrs[4];
  for (size_t l = 0; l < gpyr.size(); ++l) ptrs[l] = gpyr[l].data_ptr<float>();
  rs::pyr_grad_fold_launch(ptrs, Hs, Ws, Ss, gpyr.size(), (long)B * N1, (float)scale, cur_stream(), G.data_ptr(), Ep,
                           split ? Gl.data_ptr() : nullptr);
  RS_CHECK_LAUNCH();
  // df1 and df2 as the two halves of one buffer when they have the same size
  // (the feature encoder ran both images as one batch: the caller can then
  // hand the whole buffer back as that batch's gradient, no concatenation)
  Tensor df1, df2;
  if (f1.numel() == f2.numel()) {
    Tensor both = at::empty({2, f1.numel()}, f1.options());
    df1 = both[0].view(f1.sizes());
    df2 = both[1].view(f2.sizes());
  } else {
    df1 = at::empty_like(f1);
    df2 = at::empty_like(f2);
  }
  if (split) {
    TORCH_CHECK((uintptr_t)f1.data_ptr() % 16 == 0 && (uintptr_t)f2.data_ptr() % 16 == 0,
                "corr_volume_backward: fp32 features must be 16-B aligned");
    Tensor h1 = at::empty(f1.sizes(), bo), l1 = at::empty(f1.sizes(), bo);
    Tensor h2 = at::empty(f2.sizes(), bo), l2 = at::empty(f2.sizes(), bo);
    rs::split_bf16_launch(f1.data_ptr<float>(), f1.numel(), reinterpret_cast<uint16_t*>(h1.data_ptr()),
                          reinterpret_cast<uint16_t*>(l1.data_ptr()), cur_stream());
    rs::split_bf16_launch(f2.data_ptr<float>(), f2.numel(), reinterpret_cast<uint16_t*>(h2.data_ptr()),
                          reinterpret_cast<uint16_t*>(l2.data_ptr()), cur_stream());
    RS_CHECK_LAUNCH();
    rs::corr_bwd_gemm_launch(G.data_ptr(), Gl.data_ptr(), Ep, h1.data_ptr(), l1.data_ptr(), h2.data_ptr(),
                             l2.data_ptr(), B, N1, N2, C, df1.data_ptr(), df2.data_ptr(), cur_stream());
  } else {
    rs::corr_bwd_gemm_launch(G.data_ptr(), nullptr, Ep, f1.data_ptr(), nullptr, f2.data_ptr(), nullptr, B, N1, N2, C,
                             df1.data_ptr(), df2.data_ptr(), cur_stream());
  }
  RS_CHECK_LAUNCH();
  return {df1, df2};
}

// ---------------------------------------------------------------- on-the-fly corr
void check_otf(const Tensor& f1, const std::vector<Tensor>& f2, const Tensor& coords, int* Hs,
               int* Ws) {
  check_gpu(f1, "f1");
  check_dtype(f1, {at::kFloat, at::kBFloat16}, "f1");
  check_coords(coords);
  TORCH_CHECK(f1.dim() == 4, "f1 must be (B,H1,W1,C)");
  const int B = f1.size(0), C = f1.size(3);
  TORCH_CHECK(coords.size(0) == B && coords.size(2) == f1.size(1) && coords.size(3) == f1.size(2),
              "coords/f1 shape mismatch");
  TORCH_CHECK(rs::corr_otf_supported_channels(C), "on-the-fly corr: unsupported channel count ", C);
  TORCH_CHECK(!f2.empty() && f2.size() <= 4, "f2 pyramid must have 1..4 levels");
  for (size_t l = 0; l < f2.size(); ++l) {
    check_gpu(f2[l], "f2 level");
    TORCH_CHECK(f2[l].scalar_type() == f1.scalar_type(), "f2/f1 dtype mismatch");
    TORCH_CHECK(f2[l].dim() == 4 && f2[l].size(0) == B && f2[l].size(3) == C,
                "f2 level must be (B,H_l,W_l,C)");
    Hs[l] = f2[l].size(1);
    Ws[l] = f2[l].size(2);
  }
}

Tensor corr_otf(const Tensor& f1, const std::vector<Tensor>& f2, const Tensor& coords,
                int64_t radius, double scale, bool out_bf16) {
  int Hs[4], Ws[4];
  check_otf(f1, f2, coords, Hs, Ws);
  TORCH_CHECK(radius >= 0 && radius <= 4, "radius must be in [0,4]");
  const c10::DeviceGuard guard(f1.device());
  const int B = f1.size(0), H1 = f1.size(1), W1 = f1.size(2), C = f1.size(3);
  const int levels = f2.size(), D = 2 * radius + 1;
  Tensor out = at::empty({B, H1, W1, levels * D * D},
                         f1.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  const void* p[4];
  for (int l = 0; l < levels; ++l) p[l] = f2[l].data_ptr();
  rs::corr_otf_fwd_launch(f1.data_ptr(), p, Hs, Ws, levels, is_bf16(f1), coords.data_ptr<float>(),
                          B, H1, W1, C, radius, (float)scale, out.data_ptr(), out_bf16,
                          cur_stream());
  RS_CHECK_LAUNCH();
  return out;
}

std::vector<Tensor> corr_otf_backward(const Tensor& f1, const std::vector<Tensor>& f2,
                                      const Tensor& coords, int64_t radius, double scale,
                                      const Tensor& dout) {
  int Hs[4], Ws[4];
  check_otf(f1, f2, coords, Hs, Ws);
  const c10::DeviceGuard guard(f1.device());
  const int B = f1.size(0), H1 = f1.size(1), W1 = f1.size(2), C = f1.size(3);
  const int levels = f2.size(), D = 2 * radius + 1;
  // deterministic mode: df2 accumulates in 32.32 fixed point with int64 atomics (order-independent)
  const bool det = rs::deterministic();
  check_gpu(dout, "dout");
  TORCH_CHECK(dout.dim() == 4 && dout.size(0) == B && dout.size(1) == H1 && dout.size(2) == W1 &&
                  dout.size(3) == levels * D * D,
              "dout must be (B,H1,W1,levels*(2r+1)^2)");
  std::vector<Tensor> res;
  Tensor df1 = at::empty({B, H1, W1, C}, f1.options().dtype(at::kFloat));
  res.push_back(df1);
  const void* p[4];
  float* d[4];
  float* df[4];
  std::vector<Tensor> fx;
  for (int l = 0; l < levels; ++l) {
    p[l] = f2[l].data_ptr();
    if (det) {
      res.push_back(at::empty({B, Hs[l], Ws[l], C}, f1.options().dtype(at::kFloat)));
      fx.push_back(at::zeros({B, Hs[l], Ws[l], C}, f1.options().dtype(at::kLong)));
      d[l] = reinterpret_cast<float*>(fx.back().data_ptr<int64_t>());
      df[l] = res.back().data_ptr<float>();
    } else {
      res.push_back(at::zeros({B, Hs[l], Ws[l], C}, f1.options().dtype(at::kFloat)));
      d[l] = df[l] = res.back().data_ptr<float>();
    }
  }
  Tensor fxs;  // deterministic mode: max|dout|, max|f1|, non-finite flag (the fixed-point scale)
  if (det) fxs = at::zeros({4}, f1.options().dtype(at::kInt));
  rs::corr_otf_bwd_launch(f1.data_ptr(), p, Hs, Ws, levels, is_bf16(f1), coords.data_ptr<float>(),
                          B, H1, W1, C, radius, (float)scale, dout.data_ptr(), is_bf16(dout),
                          df1.data_ptr<float>(), d, det, df,
                          det ? reinterpret_cast<unsigned*>(fxs.data_ptr<int>()) : nullptr, cur_stream());
  RS_CHECK_LAUNCH();
  return res;
}

// ---------------------------------------------------------------- convex upsample
Tensor convex_upsample(const Tensor& flow, const Tensor& mask) {
  check_gpu(flow, "flow");
  check_dtype(flow, {at::kFloat}, "flow");
  check_gpu(mask, "mask");
  check_dtype(mask, {at::kFloat, at::kBFloat16}, "mask");
  TORCH_CHECK(flow.dim() == 4 && flow.size(1) == 2, "flow must be (N,2,H,W)");
  const int N = flow.size(0), H = flow.size(2), W = flow.size(3);
  TORCH_CHECK(mask.dim() == 4 && mask.size(0) == N && mask.size(1) == H && mask.size(2) == W &&
                  mask.size(3) == 576,
              "mask must be channels-last (N,H,W,576)");
  // the kernel reads 8 mask channels / writes 8 output floats per vector access
  TORCH_CHECK(flow.is_contiguous() && mask.is_contiguous() && (reinterpret_cast<uintptr_t>(mask.data_ptr()) & 15) == 0,
              "convex_upsample: contiguous flow and 16-byte aligned contiguous mask required");
  const c10::DeviceGuard guard(flow.device());
  Tensor out = at::empty({N, 2, 8 * H, 8 * W}, flow.options());
  rs::convex_up_fwd_launch(flow.data_ptr<float>(), mask.data_ptr(), is_bf16(mask), N, H, W,
                           out.data_ptr<float>(), cur_stream());
  RS_CHECK_LAUNCH();
  return out;
}

// Adjoint of the x8 bilinear (align_corners) upsampling: g [N, C, 8H, 8W] fp32,
// ah [8H, H], aw [8W, W] fp32 interpolation matrices -> [N, C, H, W] fp32 (x 8)
Tensor upflow8_backward(const Tensor& g, const Tensor& ah, const Tensor& aw) {
  check_gpu(g, "g");
  check_dtype(g, {at::kFloat}, "g");
  TORCH_CHECK(g.dim() == 4 && g.is_contiguous() && g.size(2) % 8 == 0 && g.size(3) % 8 == 0,
              "upflow8_backward: g must be contiguous (N, C, 8H, 8W)");
  const int H = g.size(2) / 8, W = g.size(3) / 8;
  TORCH_CHECK(ah.is_cuda() && ah.is_contiguous() && ah.scalar_type() == at::kFloat && ah.size(0) == 8 * H &&
                  ah.size(1) == H && aw.is_cuda() && aw.is_contiguous() && aw.scalar_type() == at::kFloat &&
                  aw.size(0) == 8 * W && aw.size(1) == W,
              "upflow8_backward: interpolation matrices [8H, H] / [8W, W] fp32");
  TORCH_CHECK(rs::upflow8_cols_lds(W) <= 65536, "upflow8_backward: width ", W, " exceeds the column pass's LDS");
  const c10::DeviceGuard guard(g.device());
  Tensor out = at::empty({g.size(0), g.size(1), H, W}, g.options());
  Tensor tmp = at::empty({g.size(0) * g.size(1) * 8 * H * W}, g.options());
  rs::upflow8_bwd_launch(g.data_ptr<float>(), ah.data_ptr<float>(), aw.data_ptr<float>(), g.size(0) * g.size(1), H, W,
                         tmp.data_ptr<float>(), out.data_ptr<float>(), cur_stream());
  RS_CHECK_LAUNCH();
  return out;
}

// dmask_out: optional (N,H,W,Cp) buffer (Cp >= 576, Cp % 8 == 0, the mask's dtype) the mask
// gradient is written into (channels 0..575; the rest untouched) -- e.g. the fused engine's
// padded d_mask, without a copy
std::vector<Tensor> convex_upsample_backward(const Tensor& flow, const Tensor& mask,
                                             const Tensor& dup, const c10::optional<Tensor>& dmask_out) {
  check_gpu(flow, "flow");
  check_gpu(mask, "mask");
  check_gpu(dup, "grad");
  check_dtype(dup, {at::kFloat, at::kBFloat16}, "grad");
  const int N = flow.size(0), H = flow.size(2), W = flow.size(3);
  TORCH_CHECK(mask.dim() == 4 && mask.size(3) == 576, "mask must be (N,H,W,576)");
  TORCH_CHECK(dup.dim() == 4 && dup.size(0) == N && dup.size(1) == 2 && dup.size(2) == 8 * H &&
                  dup.size(3) == 8 * W,
              "grad must be (N,2,8H,8W)");
  TORCH_CHECK(flow.is_contiguous() && mask.is_contiguous() && dup.is_contiguous() &&
                  mask.size(0) == N && mask.size(1) == H && mask.size(2) == W &&
                  ((reinterpret_cast<uintptr_t>(mask.data_ptr()) | reinterpret_cast<uintptr_t>(dup.data_ptr())) & 15) == 0,
              "convex_upsample_backward: contiguous, 16-byte aligned operands required");
  const c10::DeviceGuard guard(flow.device());
  Tensor dflow = at::empty_like(flow);
  Tensor dmask;
  if (dmask_out) {
    dmask = *dmask_out;
    TORCH_CHECK(dmask.is_cuda() && dmask.is_contiguous() && dmask.scalar_type() == mask.scalar_type() &&
                    dmask.dim() == 4 && dmask.size(0) == N && dmask.size(1) == H && dmask.size(2) == W &&
                    dmask.size(3) >= 576 && dmask.size(3) % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(dmask.data_ptr()) & 15) == 0,
                "convex_upsample_backward: dmask_out must be a contiguous, aligned (N,H,W,>=576) buffer of the mask's dtype");
  } else {
    dmask = at::empty_like(mask);
  }
  Tensor partial = at::empty({(int64_t)N * H * W * 18}, flow.options());
  rs::convex_up_bwd_launch(flow.data_ptr<float>(), mask.data_ptr(), is_bf16(mask), dup.data_ptr(),
                           is_bf16(dup), N, H, W, dmask.data_ptr(), (int)dmask.size(3), dflow.data_ptr<float>(),
                           partial.data_ptr<float>(), cur_stream());
  RS_CHECK_LAUNCH();
  return {dflow, dmask};
}

// ---------------------------------------------------------------- GRU gates
// All inputs are NHWC-contiguous, viewed as (P, channels).
int64_t pixels(const Tensor& t) { return t.numel() / t.size(-1); }

// cn: (B,H,W,hd+cd) contiguous; hx: (B,H,W,>=hd) contiguous; inp: (B,H,W,cd)
// with unit channel stride and evenly strided pixel rows (contiguous, or a
// channel window of a wider NHWC buffer: the inference engine's hx slots);
// all of cn's dtype
bool rows_view(const Tensor& t) {
  return t.stride(3) == 1 && t.stride(2) >= t.size(3) && t.stride(1) == t.size(2) * t.stride(2) &&
         t.stride(0) == t.size(1) * t.stride(1);
}

void context_act(const Tensor& cn, const Tensor& hx, const Tensor& inp, int64_t hd) {
  check_gpu(cn, "cn");
  check_dtype(cn, {at::kFloat, at::kBFloat16}, "cn");
  TORCH_CHECK(cn.dim() == 4 && hx.dim() == 4 && inp.dim() == 4 && cn.is_contiguous() && hx.is_contiguous() &&
                  rows_view(inp) && hx.scalar_type() == cn.scalar_type() && inp.scalar_type() == cn.scalar_type(),
              "context_act: NHWC tensors of one dtype (inp: evenly strided pixel rows)");
  const int64_t cd = cn.size(3) - hd;
  TORCH_CHECK(hd > 0 && cd > 0 && hx.size(3) >= hd && inp.size(3) == cd && hx.sizes().slice(0, 3) == cn.sizes().slice(0, 3) &&
                  inp.sizes().slice(0, 3) == cn.sizes().slice(0, 3),
              "context_act: shapes");
  const c10::DeviceGuard guard(cn.device());
  const long P = cn.size(0) * cn.size(1) * cn.size(2);
  rs::ctx_act_launch(is_bf16(cn), cn.data_ptr(), P, (int)hd, (int)cd, hx.data_ptr(), (int)hx.size(3), inp.data_ptr(),
                     (int)inp.stride(2), cur_stream());
  RS_CHECK_LAUNCH();
}

// G: (B,H,W,gp) fp32 gradient rows [d h | d inp | ...]; hx / inp as context_act left them
Tensor context_act_backward(const Tensor& G, const Tensor& hx, const Tensor& inp, int64_t hd) {
  check_gpu(G, "G");
  check_dtype(G, {at::kFloat}, "G");
  TORCH_CHECK(G.dim() == 4 && hx.dim() == 4 && inp.dim() == 4 && G.is_contiguous() && hx.is_contiguous() &&
                  inp.is_contiguous() && hx.scalar_type() == inp.scalar_type(),
              "context_act_backward: contiguous NHWC tensors");
  const int64_t cd = inp.size(3);
  TORCH_CHECK(hd > 0 && G.size(3) >= hd + cd && hx.size(3) >= hd && hx.sizes().slice(0, 3) == G.sizes().slice(0, 3) &&
                  inp.sizes().slice(0, 3) == G.sizes().slice(0, 3),
              "context_act_backward: shapes");
  const c10::DeviceGuard guard(G.device());
  Tensor dcn = at::empty({G.size(0), G.size(1), G.size(2), hd + cd}, hx.options());
  const long P = G.size(0) * G.size(1) * G.size(2);
  rs::ctx_act_bwd_launch(is_bf16(hx), G.data_ptr<float>(), (int)G.size(3), hx.data_ptr(), (int)hx.size(3),
                         inp.data_ptr(), (int)cd, P, (int)hd, (int)cd, dcn.data_ptr(), cur_stream());
  RS_CHECK_LAUNCH();
  return dcn;
}

std::vector<Tensor> gru_gate_zr(const Tensor& zr, const Tensor& h, const Tensor& x) {
  check_gpu(zr, "zr");
  check_gpu(h, "h");
  check_gpu(x, "x");
  check_dtype(h, {at::kFloat, at::kBFloat16}, "h");
  TORCH_CHECK(zr.scalar_type() == h.scalar_type() && x.scalar_type() == h.scalar_type(),
              "gru_gate_zr: dtype mismatch");
  const int hd = h.size(-1), cin = x.size(-1);
  const int64_t P = pixels(h);
  TORCH_CHECK(zr.size(-1) == 2 * hd && pixels(zr) == P && pixels(x) == P, "gru_gate_zr: shapes");
  const c10::DeviceGuard guard(h.device());
  auto sz = h.sizes().vec();
  Tensor z = at::empty_like(h), r = at::empty_like(h);
  sz.back() = hd + cin;
  Tensor rhx = at::empty(sz, h.options());
  rs::gru_gate_zr_launch(is_bf16(h), zr.data_ptr(), h.data_ptr(), x.data_ptr(), P, hd, cin,
                         z.data_ptr(), r.data_ptr(), rhx.data_ptr(), cur_stream());
  RS_CHECK_LAUNCH();
  return {z, r, rhx};
}

std::vector<Tensor> gru_gate_q(const Tensor& q, const Tensor& z, const Tensor& h) {
  check_gpu(q, "q");
  check_gpu(z, "z");
  check_gpu(h, "h");
  TORCH_CHECK(q.sizes() == h.sizes() && z.sizes() == h.sizes(), "gru_gate_q: shapes");
  TORCH_CHECK(q.scalar_type() == h.scalar_type() && z.scalar_type() == h.scalar_type(),
              "gru_gate_q: dtype mismatch");
  const c10::DeviceGuard guard(h.device());
  Tensor hn = at::empty_like(h), qt = at::empty_like(h);
  rs::gru_gate_q_launch(is_bf16(h), q.data_ptr(), z.data_ptr(), h.data_ptr(), pixels(h),
                        h.size(-1), hn.data_ptr(), qt.data_ptr(), cur_stream());
  RS_CHECK_LAUNCH();
  return {hn, qt};
}

std::vector<Tensor> gru_bwd_q(const Tensor& dhn, const Tensor& z, const Tensor& h,
                              const Tensor& qt) {
  check_gpu(dhn, "dhn");
  check_gpu(z, "z");
  check_gpu(h, "h");
  check_gpu(qt, "qt");
  TORCH_CHECK(dhn.sizes() == h.sizes() && z.sizes() == h.sizes() && qt.sizes() == h.sizes(),
              "gru_bwd_q: shapes");
  const c10::DeviceGuard guard(h.device());
  const int hd = h.size(-1);
  const int64_t P = pixels(h);
  auto sz = h.sizes().vec();
  Tensor dq = at::empty_like(h);
  sz.back() = 2 * hd;
  Tensor dzr = at::empty(sz, h.options());
  Tensor dh = at::empty(h.sizes(), h.options().dtype(at::kFloat));
  rs::gru_bwd_q_launch(is_bf16(h), dhn.data_ptr(), is_bf16(dhn), z.data_ptr(), h.data_ptr(),
                       qt.data_ptr(), P, hd, dq.data_ptr(), dzr.data_ptr(), dh.data_ptr<float>(),
                       cur_stream());
  RS_CHECK_LAUNCH();
  return {dq, dzr, dh};
}

void gru_bwd_r(const Tensor& drhx, const Tensor& h, const Tensor& r, const Tensor& dzr) {
  check_gpu(drhx, "drhx");
  check_gpu(h, "h");
  check_gpu(r, "r");
  check_gpu(dzr, "dzr");
  const int hd = h.size(-1), cin = drhx.size(-1) - hd;
  const int64_t P = pixels(h);
  TORCH_CHECK(pixels(drhx) == P && dzr.size(-1) == 2 * hd && pixels(dzr) == P, "gru_bwd_r: shapes");
  TORCH_CHECK(drhx.scalar_type() == h.scalar_type() && dzr.scalar_type() == h.scalar_type(),
              "gru_bwd_r: dtype mismatch");
  const c10::DeviceGuard guard(h.device());
  rs::gru_bwd_r_launch(is_bf16(h), drhx.data_ptr(), h.data_ptr(), r.data_ptr(), P, hd, cin,
                       dzr.data_ptr(), cur_stream());
  RS_CHECK_LAUNCH();
}

std::vector<Tensor> gru_bwd_fin(const Tensor& dhd, const Tensor& drhx, const Tensor& r,
                                const Tensor& dhx) {
  check_gpu(dhd, "dhd");
  check_gpu(drhx, "drhx");
  check_gpu(r, "r");
  check_gpu(dhx, "dhx");
  check_dtype(dhd, {at::kFloat}, "dhd");
  const int hd = r.size(-1), cin = drhx.size(-1) - hd;
  const int64_t P = pixels(r);
  TORCH_CHECK(pixels(drhx) == P && dhx.sizes() == drhx.sizes() && dhd.sizes() == r.sizes(),
              "gru_bwd_fin: shapes");
  TORCH_CHECK(drhx.scalar_type() == r.scalar_type() && dhx.scalar_type() == r.scalar_type(),
              "gru_bwd_fin: dtype mismatch");
  const c10::DeviceGuard guard(r.device());
  auto sz = r.sizes().vec();
  Tensor dh = at::empty_like(r);
  sz.back() = cin;
  Tensor dx = at::empty(sz, r.options());
  rs::gru_bwd_fin_launch(is_bf16(r), dhd.data_ptr<float>(), drhx.data_ptr(), r.data_ptr(),
                         dhx.data_ptr(), P, hd, cin, dh.data_ptr(), dx.data_ptr(), cur_stream());
  RS_CHECK_LAUNCH();
  return {dh, dx};
}

void set_deterministic(bool on) { rs::g_deterministic.store(on); }
bool is_deterministic() { return rs::deterministic(); }

}  // namespace

// Packed-weight gather (csrc/wpack.hip): out[i] = scale * source[code[i]] with
// code = (source row << 24) | logical index (-1: zero); tab int64 [nsrc][10]
// = (data_ptr, is_bf16, size[4], stride[4]) of the sources (host-built, on
// the device); ranges: up to 4 [lo, hi) output ranges multiplied by rs[k].
void wpack_gather(const Tensor& code, const Tensor& tab, const Tensor& out, at::IntArrayRef rlo,
                  at::IntArrayRef rhi, at::ArrayRef<double> rs_) {
  check_gpu(code, "code");
  check_gpu(tab, "tab");
  check_gpu(out, "out");
  TORCH_CHECK(code.scalar_type() == at::kInt && code.dim() == 1, "wpack_gather: code must be int32 [n]");
  TORCH_CHECK(tab.scalar_type() == at::kLong && tab.dim() == 2 && tab.size(1) == 10 && tab.size(0) <= 128,
              "wpack_gather: tab must be int64 [<=128][10]");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "wpack_gather: out bf16/fp32");
  TORCH_CHECK(out.numel() == code.numel(), "wpack_gather: out / code size");
  TORCH_CHECK(rlo.size() == rhi.size() && rlo.size() == rs_.size() && rlo.size() <= 4, "wpack_gather: ranges");
  long long lo[4], hi[4];
  float sc[4];
  for (size_t r = 0; r < rlo.size(); ++r) {
    lo[r] = rlo[r];
    hi[r] = rhi[r];
    sc[r] = (float)rs_[r];
  }
  const c10::DeviceGuard guard(out.device());
  rs::wpack_gather_launch(code.data_ptr<int>(), code.numel(), reinterpret_cast<const long long*>(tab.data_ptr<int64_t>()), out.data_ptr(),
                          out.scalar_type() == at::kBFloat16, lo, hi, sc, (int)rlo.size(), cur_stream());
  RS_CHECK_LAUNCH();
}

// fp32 -> (hi, lo) bf16 with hi = bf16(x), lo = bf16(x - hi) (csrc/split.hip)
std::vector<Tensor> split_bf16(const Tensor& x) {
  check_gpu(x, "x");
  check_dtype(x, {at::kFloat}, "x");
  TORCH_CHECK(x.is_contiguous(), "split_bf16: x must be contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "split_bf16: x must be 16-byte aligned");
  const c10::DeviceGuard guard(x.device());
  Tensor hi = at::empty(x.sizes(), x.options().dtype(at::kBFloat16));
  Tensor lo = at::empty(x.sizes(), x.options().dtype(at::kBFloat16));
  if (x.numel() > 0)
    rs::split_bf16_launch(x.data_ptr<float>(), x.numel(), reinterpret_cast<uint16_t*>(hi.data_ptr()),
                          reinterpret_cast<uint16_t*>(lo.data_ptr()), cur_stream());
  RS_CHECK_LAUNCH();
  return {hi, lo};
}

TORCH_LIBRARY(raft_stir, m) {
  m.def("wpack_gather(Tensor code, Tensor tab, Tensor(a!) out, int[] rlo, int[] rhi, float[] rs) -> ()");
  m.def("set_deterministic(bool on) -> ()", &set_deterministic);
  m.def("is_deterministic() -> bool", &is_deterministic);
  m.def("corr_volume(Tensor f1, Tensor f2, int levels, float scale, bool out_bf16=False) -> Tensor[]");
  m.def("corr_lookup(Tensor[] pyr, Tensor coords, int radius, bool out_bf16) -> Tensor");
  m.def("corr_lookup_into(Tensor[] pyr, Tensor coords, int radius, Tensor(a!) out) -> ()");
  m.def("corr_lookup_backward(Tensor(a!)[] gpyr, Tensor coords, int radius, Tensor dout) -> ()");
  m.def("pyr_grad_fold(Tensor(a!)[] gpyr, float scale) -> ()");
  m.def("pyr_grad_fold_bf16(Tensor[] gpyr, float scale, Tensor(a!) out) -> ()");
  m.def("corr_volume_backward(Tensor[] gpyr, Tensor f1, Tensor f2, float scale) -> Tensor[]");
  m.def("split_bf16(Tensor x) -> Tensor[]");
  m.def("corr_otf(Tensor f1, Tensor[] f2, Tensor coords, int radius, float scale, bool out_bf16) -> Tensor");
  m.def("corr_otf_backward(Tensor f1, Tensor[] f2, Tensor coords, int radius, float scale, Tensor dout) -> Tensor[]");
  m.def("convex_upsample(Tensor flow, Tensor mask) -> Tensor");
  m.def("convex_upsample_backward(Tensor flow, Tensor mask, Tensor grad, Tensor(a!)? dmask_out=None) -> Tensor[]");
  m.def("upflow8_backward(Tensor g, Tensor ah, Tensor aw) -> Tensor");
  m.def("context_act(Tensor cn, Tensor(a!) hx, Tensor(b!) inp, int hd) -> ()");
  m.def("context_act_backward(Tensor G, Tensor hx, Tensor inp, int hd) -> Tensor");
  m.def("gru_gate_zr(Tensor zr, Tensor h, Tensor x) -> Tensor[]");
  m.def("gru_gate_q(Tensor q, Tensor z, Tensor h) -> Tensor[]");
  m.def("gru_bwd_q(Tensor dhn, Tensor z, Tensor h, Tensor qt) -> Tensor[]");
  m.def("gru_bwd_r(Tensor drhx, Tensor h, Tensor r, Tensor(a!) dzr) -> ()");
  m.def("gru_bwd_fin(Tensor dhd, Tensor drhx, Tensor r, Tensor dhx) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(raft_stir, CUDA, m) {
  m.impl("wpack_gather", &wpack_gather);
  m.impl("corr_volume", &corr_volume);
  m.impl("corr_lookup", &corr_lookup);
  m.impl("corr_lookup_into", &corr_lookup_into);
  m.impl("corr_lookup_backward", &corr_lookup_backward);
  m.impl("pyr_grad_fold", &pyr_grad_fold);
  m.impl("pyr_grad_fold_bf16", &pyr_grad_fold_bf16);
  m.impl("corr_volume_backward", &corr_volume_backward);
  m.impl("split_bf16", &split_bf16);
  m.impl("corr_otf", &corr_otf);
  m.impl("corr_otf_backward", &corr_otf_backward);
  m.impl("convex_upsample", &convex_upsample);
  m.impl("convex_upsample_backward", &convex_upsample_backward);
  m.impl("upflow8_backward", &upflow8_backward);
  m.impl("context_act", &context_act);
  m.impl("context_act_backward", &context_act_backward);
  m.impl("gru_gate_zr", &gru_gate_zr);
  m.impl("gru_gate_q", &gru_gate_q);
  m.impl("gru_bwd_q", &gru_bwd_q);
  m.impl("gru_bwd_r", &gru_bwd_r);
  m.impl("gru_bwd_fin", &gru_bwd_fin);
}
