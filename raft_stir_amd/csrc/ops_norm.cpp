// torch.ops.raft_stir.norm_* : fused NHWC normalisation + activation (csrc/norm.hip).
#include <ATen/ATen.h>
#include "host_common.h"
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>

namespace rs {
int norm_ws_floats(int B, int P, int C, bool bf16, bool stats);
void norm_set_reduce_blocks(int n);
void norm_stats_launch(bool bf16, const void* x, int B, int P, int C, int G, float eps, float* ws,
                       float* mean, float* rstd, float* rm, float* rv, long long* nbt, const float* rbias,
                       float mom, float unb, hipStream_t s);
void norm_fwd_launch(bool bf16, const void* x, const void* res, const float* mean,
                     const float* rstd, const float* gamma, const float* beta, int B, int P, int C,
                     int G, bool relu, void* y, const float* const* rnorm, hipStream_t s);
void norm_bwd_launch(bool bf16, const void* x, const void* dy, const void* res, const float* mean,
                     const float* rstd, const float* gamma, const float* beta, int B, int P, int C,
                     int G, bool relu, bool batch_stats, float* ws, float* s1, float* s2, void* dx,
                     void* dres, const void* dy2, const float* const* rnorm, float* ws2, float* rs1,
                     float* rs2, hipStream_t s);
}  // namespace rs

namespace {
using at::Tensor;

hipStream_t stream() { return rs::current_stream(); }

// x: (B, H, W, C) contiguous (an NCHW-shaped channels_last tensor is passed as
// its NHWC permute by the Python side).
void check_x(const Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4, "norm: x must be contiguous (B,H,W,C) on GPU");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "norm: x must be fp32/bf16");
  const int64_t C = x.size(3);
  const int vn = x.scalar_type() == at::kBFloat16 ? 8 : 4;
  TORCH_CHECK(C % vn == 0 && C / vn <= 256, "norm: channel count ", C, " unsupported");
}

void check_like(const c10::optional<Tensor>& t, const Tensor& x, const char* n) {
  if (!t) return;
  TORCH_CHECK(t->sizes() == x.sizes() && t->scalar_type() == x.scalar_type() && t->is_contiguous(),
              "norm: ", n, " must match x");
}

void check_param(const c10::optional<Tensor>& t, int64_t C, const char* n) {
  if (!t) return;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() == C && t->is_contiguous(),
              "norm: ", n, " must be fp32 (C,)");
}

const float* fptr(const c10::optional<Tensor>& t) { return t ? t->data_ptr<float>() : nullptr; }

// running_mean / running_var / nbt (+ bias, the producing conv's bias folded
// into the statistics): the train-mode BatchNorm running update, fused into
// the statistics launch (batch statistics only).
std::vector<Tensor> norm_stats(const Tensor& x, bool per_sample, double eps, const c10::optional<Tensor>& rmean,
                               const c10::optional<Tensor>& rvar, const c10::optional<Tensor>& nbt,
                               const c10::optional<Tensor>& bias, double momentum, int64_t n) {
  check_x(x);
  const c10::DeviceGuard g(x.device());
  const int B = x.size(0), P = x.size(1) * x.size(2), C = x.size(3);
  const int G = per_sample ? B : 1;
  const bool bf = x.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bool(rmean) == bool(rvar) && (!rmean || !per_sample), "norm_stats: running stats need batch statistics");
  check_param(rmean, C, "running_mean");
  check_param(rvar, C, "running_var");
  check_param(bias, C, "bias");
  if (nbt) TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1, "norm_stats: nbt");
  auto fo = x.options().dtype(at::kFloat);
  Tensor ws = at::empty({rs::norm_ws_floats(B, P, C, bf, true)}, fo);
  Tensor mean = at::empty({G, C}, fo), rstd = at::empty({G, C}, fo);
  const float unb = n > 1 ? (float)((double)n / (double)(n - 1)) : 1.f;
  rs::norm_stats_launch(bf, x.data_ptr(), B, P, C, G, (float)eps, ws.data_ptr<float>(), mean.data_ptr<float>(),
                        rstd.data_ptr<float>(), rmean ? rmean->data_ptr<float>() : nullptr, rvar ? rvar->data_ptr<float>() : nullptr,
                        nbt ? reinterpret_cast<long long*>(nbt->data_ptr<int64_t>()) : nullptr, fptr(bias),
                        (float)momentum, unb, stream());
  RS_CHECK_LAUNCH();
  return {mean, rstd};
}

// rmean / rrstd (+ rgamma / rbeta): the residual is a RAW tensor normalised
// on the fly (no ReLU on it) -- the downsample shortcut's norm inside the
// block's output pass (models/fused_encoder.py)
struct RNorm {
  const float* p[4] = {nullptr, nullptr, nullptr, nullptr};
  bool on = false;
};

RNorm rnorm_args(const c10::optional<Tensor>& rmean, const c10::optional<Tensor>& rrstd,
                 const c10::optional<Tensor>& rgamma, const c10::optional<Tensor>& rbeta, const Tensor& mean,
                 const c10::optional<Tensor>& res, int64_t C) {
  RNorm r;
  TORCH_CHECK(bool(rmean) == bool(rrstd), "norm: rmean / rrstd come together");
  if (!rmean) return r;
  TORCH_CHECK(bool(res), "norm: an affine residual needs res");
  TORCH_CHECK(rmean->sizes() == mean.sizes() && rrstd->sizes() == mean.sizes() && rmean->is_contiguous() &&
                  rrstd->is_contiguous() && rmean->scalar_type() == at::kFloat && rrstd->scalar_type() == at::kFloat,
              "norm: residual statistics must match the main statistics' shape");
  check_param(rgamma, C, "rgamma");
  check_param(rbeta, C, "rbeta");
  r.p[0] = rmean->data_ptr<float>();
  r.p[1] = rrstd->data_ptr<float>();
  r.p[2] = fptr(rgamma);
  r.p[3] = fptr(rbeta);
  r.on = true;
  return r;
}

Tensor norm_act(const Tensor& x, const Tensor& mean, const Tensor& rstd,
                const c10::optional<Tensor>& gamma, const c10::optional<Tensor>& beta,
                const c10::optional<Tensor>& res, bool relu, const c10::optional<Tensor>& rmean,
                const c10::optional<Tensor>& rrstd, const c10::optional<Tensor>& rgamma,
                const c10::optional<Tensor>& rbeta) {
  check_x(x);
  const int B = x.size(0), P = x.size(1) * x.size(2), C = x.size(3);
  const int G = mean.size(0);
  TORCH_CHECK(mean.is_contiguous() && rstd.is_contiguous() && mean.numel() == (int64_t)G * C &&
                  rstd.numel() == (int64_t)G * C && (G == 1 || G == B),
              "norm_act: stats shape");
  check_param(gamma, C, "gamma");
  check_param(beta, C, "beta");
  check_like(res, x, "residual");
  const RNorm rn = rnorm_args(rmean, rrstd, rgamma, rbeta, mean, res, C);
  const c10::DeviceGuard g(x.device());
  Tensor y = at::empty_like(x);
  rs::norm_fwd_launch(x.scalar_type() == at::kBFloat16, x.data_ptr(), res ? res->data_ptr() : nullptr,
                      mean.data_ptr<float>(), rstd.data_ptr<float>(), fptr(gamma), fptr(beta), B, P, C,
                      G, relu, y.data_ptr(), rn.on ? rn.p : nullptr, stream());
  RS_CHECK_LAUNCH();
  return y;
}

// returns dx, dres (empty if no residual), s1 (= dbeta per group), s2 (= dgamma per group),
// and the (2, G, C) buffer s1 / s2 are views of.
// batch_stats=false: the statistics were constants (BatchNorm in eval mode), so
// dx = gamma * rstd * g without the mean/variance terms.
// dy2: a second upstream gradient added on the fly (the skip path's).  With
// an affine residual (rmean ...) dres is the gradient of the RAW residual
// through its normalisation, and a sixth output holds its (2, G, C) sums.
std::vector<Tensor> norm_act_backward(const Tensor& dy, const Tensor& x, const Tensor& mean,
                                      const Tensor& rstd, const c10::optional<Tensor>& gamma,
                                      const c10::optional<Tensor>& beta,
                                      const c10::optional<Tensor>& res, bool relu,
                                      bool batch_stats, const c10::optional<Tensor>& dy2,
                                      const c10::optional<Tensor>& rmean, const c10::optional<Tensor>& rrstd,
                                      const c10::optional<Tensor>& rgamma, const c10::optional<Tensor>& rbeta) {
  check_x(x);
  check_like(dy, x, "grad");
  check_like(dy2, x, "second grad");
  check_like(res, x, "residual");
  TORCH_CHECK(!rmean || batch_stats, "norm_act_backward: an affine residual needs batch statistics");
  const int B = x.size(0), P = x.size(1) * x.size(2), C = x.size(3);
  const int G = mean.size(0);
  TORCH_CHECK(mean.numel() == (int64_t)G * C && rstd.numel() == (int64_t)G * C && (G == 1 || G == B),
              "norm_act_backward: stats shape");
  check_param(gamma, C, "gamma");
  check_param(beta, C, "beta");
  const c10::DeviceGuard g(x.device());
  const bool bf = x.scalar_type() == at::kBFloat16;
  auto fo = x.options().dtype(at::kFloat);
  Tensor ws = at::empty({rs::norm_ws_floats(B, P, C, bf, false)}, fo);
  // s1 / s2 are the two halves of one (2, G, C) buffer: the per-channel sums
  // over groups (dbeta, dgamma) are then ONE reduction (ops/norm.py)
  Tensor s12 = at::empty({2, G, C}, fo);
  Tensor s1 = s12.select(0, 0), s2 = s12.select(0, 1);
  Tensor dx = at::empty_like(x);
  Tensor dres = res ? at::empty_like(x) : at::empty({0}, x.options());
  const RNorm rn = rnorm_args(rmean, rrstd, rgamma, rbeta, mean, res, C);
  Tensor ws2, r12;
  if (rn.on) {
    ws2 = at::empty_like(ws);
    r12 = at::empty({2, G, C}, fo);
  }
  rs::norm_bwd_launch(bf, x.data_ptr(), dy.data_ptr(), res ? res->data_ptr() : nullptr,
                      mean.data_ptr<float>(), rstd.data_ptr<float>(), fptr(gamma), fptr(beta), B, P, C,
                      G, relu, batch_stats, ws.data_ptr<float>(), s1.data_ptr<float>(),
                      s2.data_ptr<float>(), dx.data_ptr(), res ? dres.data_ptr() : nullptr,
                      dy2 ? dy2->data_ptr() : nullptr, rn.on ? rn.p : nullptr,
                      rn.on ? ws2.data_ptr<float>() : nullptr, rn.on ? r12.data_ptr<float>() : nullptr,
                      rn.on ? r12.data_ptr<float>() + (int64_t)G * C : nullptr, stream());
  RS_CHECK_LAUNCH();
  if (rn.on) return {dx, dres, s1, s2, s12, r12};
  return {dx, dres, s1, s2, s12};
}

void norm_set_reduce_blocks_op(int64_t n) { rs::norm_set_reduce_blocks((int)n); }

}  // namespace

TORCH_LIBRARY_FRAGMENT(raft_stir, m) {
  m.def("norm_set_reduce_blocks(int n) -> ()", &norm_set_reduce_blocks_op);
  m.def("norm_stats(Tensor x, bool per_sample, float eps, Tensor(a!)? running_mean=None, "
        "Tensor(b!)? running_var=None, Tensor(c!)? nbt=None, Tensor? bias=None, float momentum=0.1, int n=0) -> Tensor[]");
  m.def("norm_act(Tensor x, Tensor mean, Tensor rstd, Tensor? gamma, Tensor? beta, Tensor? res, bool relu, "
        "Tensor? rmean=None, Tensor? rrstd=None, Tensor? rgamma=None, Tensor? rbeta=None) -> Tensor");
  m.def("norm_act_backward(Tensor dy, Tensor x, Tensor mean, Tensor rstd, Tensor? gamma, Tensor? beta, Tensor? res, "
        "bool relu, bool batch_stats, Tensor? dy2=None, Tensor? rmean=None, Tensor? rrstd=None, "
        "Tensor? rgamma=None, Tensor? rbeta=None) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(raft_stir, CUDA, m) {
  m.impl("norm_stats", &norm_stats);
  m.impl("norm_act", &norm_act);
  m.impl("norm_act_backward", &norm_act_backward);
}
