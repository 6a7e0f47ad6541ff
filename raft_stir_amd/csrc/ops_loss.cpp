// torch.ops.raft_stir.seq_loss / seq_loss_backward (csrc/loss.hip).
#include <ATen/ATen.h>
#include "host_common.h"
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>

namespace rs {
void seq_loss_fwd_launch(const float* preds, const float* gt, const float* valid, int N, int B, long HW,
                         float gamma, float max_flow, float* partial, int nblocks, float* out, hipStream_t s);
int seq_loss_blocks(long P);
int seq_loss_partials(long P);
void seq_loss_bwd_launch(const float* preds, const float* gt, const float* valid, int N, int B, long HW,
                         float gamma, float max_flow, const float* gout, float* grad, hipStream_t s);
}  // namespace rs

namespace {
using at::Tensor;

hipStream_t stream() { return rs::current_stream(); }

void check(const Tensor& preds, const Tensor& gt, const Tensor& valid) {
  TORCH_CHECK(preds.is_cuda() && gt.is_cuda() && valid.is_cuda(), "seq_loss: GPU tensors expected");
  TORCH_CHECK(preds.scalar_type() == at::kFloat && gt.scalar_type() == at::kFloat &&
                  valid.scalar_type() == at::kFloat,
              "seq_loss: fp32 preds / gt / valid expected");
  TORCH_CHECK(preds.is_contiguous() && gt.is_contiguous() && valid.is_contiguous(),
              "seq_loss: contiguous tensors expected");
  TORCH_CHECK(gt.dim() == 4 && gt.size(1) == 2, "seq_loss: gt must be (B,2,H,W)");
  TORCH_CHECK(preds.dim() == 5 && preds.size(1) == gt.size(0) && preds.size(2) == 2 &&
                  preds.size(3) == gt.size(2) && preds.size(4) == gt.size(3),
              "seq_loss: preds must be (N,B,2,H,W) matching gt");
  TORCH_CHECK(valid.dim() == 3 && valid.size(0) == gt.size(0) && valid.size(1) == gt.size(2) &&
                  valid.size(2) == gt.size(3),
              "seq_loss: valid must be (B,H,W)");
}

// returns (loss, metrics): metrics = [EPE, 1 px, 3 px, 5 px] of the last prediction over the valid pixels
std::vector<Tensor> seq_loss(const Tensor& preds, const Tensor& gt, const Tensor& valid, double gamma,
                             double max_flow) {
  check(preds, gt, valid);
  const c10::DeviceGuard guard(preds.device());
  const int N = preds.size(0), B = gt.size(0);
  const long HW = (long)gt.size(2) * gt.size(3);
  const int nb = rs::seq_loss_blocks((long)B * HW);
  Tensor partial = at::empty({rs::seq_loss_partials((long)B * HW)}, gt.options());
  Tensor out = at::empty({5}, gt.options());
  rs::seq_loss_fwd_launch(preds.data_ptr<float>(), gt.data_ptr<float>(), valid.data_ptr<float>(), N, B, HW,
                          (float)gamma, (float)max_flow, partial.data_ptr<float>(), nb, out.data_ptr<float>(),
                          stream());
  RS_CHECK_LAUNCH();
  return {out.select(0, 0), out.narrow(0, 1, 4)};
}

Tensor seq_loss_backward(const Tensor& grad_out, const Tensor& preds, const Tensor& gt, const Tensor& valid,
                         double gamma, double max_flow) {
  check(preds, gt, valid);
  TORCH_CHECK(grad_out.is_cuda() && grad_out.numel() == 1 && grad_out.scalar_type() == at::kFloat,
              "seq_loss_backward: scalar fp32 grad expected");
  const c10::DeviceGuard guard(preds.device());
  const int N = preds.size(0), B = gt.size(0);
  const long HW = (long)gt.size(2) * gt.size(3);
  Tensor grad = at::empty_like(preds);
  Tensor go = grad_out.contiguous();
  rs::seq_loss_bwd_launch(preds.data_ptr<float>(), gt.data_ptr<float>(), valid.data_ptr<float>(), N, B, HW,
                          (float)gamma, (float)max_flow, go.data_ptr<float>(), grad.data_ptr<float>(), stream());
  RS_CHECK_LAUNCH();
  return grad;
}
}  // namespace

TORCH_LIBRARY_FRAGMENT(raft_stir, m) {
  m.def("seq_loss(Tensor preds, Tensor gt, Tensor valid, float gamma, float max_flow) -> Tensor[]");
  m.def("seq_loss_backward(Tensor grad, Tensor preds, Tensor gt, Tensor valid, float gamma, float max_flow) "
        "-> Tensor");
}

TORCH_LIBRARY_IMPL(raft_stir, CUDA, m) {
  m.impl("seq_loss", &seq_loss);
  m.impl("seq_loss_backward", &seq_loss_backward);
}
