// torch.ops.raft_stir.clip_adamw_ : gradient clipping + AdamW over a whole
// parameter list in two launches per 96-tensor group (csrc/optim.hip).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <cmath>
#include <vector>

#include "host_common.h"
#include "optim.h"

namespace rs {
void clip_adamw_launch(const optim::TList* groups, int ngroups, long long total_blocks, float* partial, float* m,
                       float* v, const float* lr_dev, float lr, float beta1, float beta2, float eps, float wd,
                       float max_norm, bool clip, float* state, float* norm_out, hipStream_t s);
}  // namespace rs

namespace {
using at::Tensor;

// params / grads: fp32 device tensors of identical shape and dense strides
// (pairwise); moff[i]: flat offset of params[i]'s moments in exp_avg /
// exp_avg_sq; partial: fp32 scratch of >= sum over groups of ceil(numel / CH)
// floats; state: fp32 (completed steps, pending flag) -- see sumsq_kernel.
// max_norm <= 0: no clipping.  Returns ||grads|| (fp32, 0-dim); a non-finite
// norm leaves every parameter and moment unchanged.
Tensor clip_adamw(at::TensorList params, at::TensorList grads, const Tensor& exp_avg, const Tensor& exp_avg_sq,
                  const Tensor& partial, at::IntArrayRef moff, const c10::optional<Tensor>& lr_t, double lr,
                  double beta1, double beta2, double eps, double weight_decay, double max_norm, const Tensor& state) {
  TORCH_CHECK(params.size() == grads.size() && params.size() == moff.size() && !params.empty(),
              "clip_adamw_: params, grads and moff must have one entry per parameter");
  const auto dev = params[0].device();
  TORCH_CHECK(state.numel() == 2, "clip_adamw_: state must hold (steps, pending flag)");
  for (const Tensor* t : {&exp_avg, &exp_avg_sq, &partial, &state})
    TORCH_CHECK(t->device() == dev && t->scalar_type() == at::kFloat && t->is_contiguous(),
                "clip_adamw_: moments and scratch must be contiguous fp32 on the parameters' device");
  if (lr_t) TORCH_CHECK(lr_t->device() == dev && lr_t->scalar_type() == at::kFloat && lr_t->numel() == 1,
                        "clip_adamw_: lr tensor must be a one-element fp32 tensor on the device");
  const c10::DeviceGuard guard(dev);
  std::vector<rs::optim::TList> groups;
  long long pblocks = 0;
  for (size_t i = 0; i < params.size(); ++i) {
    const Tensor& p = params[i];
    const Tensor& g = grads[i];
    TORCH_CHECK(p.is_cuda() && p.device() == dev && p.scalar_type() == at::kFloat, "clip_adamw_: fp32 device params");
    TORCH_CHECK(g.device() == dev && g.scalar_type() == at::kFloat && g.sizes() == p.sizes() &&
                    g.strides() == p.strides() && p.is_non_overlapping_and_dense(),
                "clip_adamw_: grad ", i, " must match its parameter's dtype, shape and dense strides");
    TORCH_CHECK(moff[i] >= 0 && moff[i] + p.numel() <= exp_avg.numel() && exp_avg_sq.numel() == exp_avg.numel(),
                "clip_adamw_: moment offset out of range for parameter ", i);
    if (groups.empty() || groups.back().n == rs::optim::MAXT) {
      if (!groups.empty()) pblocks += (groups.back().off[groups.back().n] + rs::optim::CH - 1) / rs::optim::CH;
      groups.emplace_back();
      rs::optim::TList& L = groups.back();
      L.n = 0;
      L.off[0] = 0;
      L.pbase = (int)pblocks;
    }
    rs::optim::TList& L = groups.back();
    L.p[L.n] = p.data_ptr<float>();
    L.g[L.n] = const_cast<float*>(g.data_ptr<float>());
    L.moff[L.n] = moff[i];
    L.off[L.n + 1] = L.off[L.n] + p.numel();
    ++L.n;
  }
  pblocks += (groups.back().off[groups.back().n] + rs::optim::CH - 1) / rs::optim::CH;
  TORCH_CHECK(partial.numel() >= pblocks, "clip_adamw_: partial scratch needs ", pblocks, " floats");
  Tensor norm = at::empty({}, exp_avg.options());
  rs::clip_adamw_launch(groups.data(), (int)groups.size(), pblocks, partial.data_ptr<float>(),
                        exp_avg.data_ptr<float>(), exp_avg_sq.data_ptr<float>(),
                        lr_t ? lr_t->data_ptr<float>() : nullptr, (float)lr, (float)beta1, (float)beta2, (float)eps,
                        (float)weight_decay, (float)max_norm, max_norm > 0, state.data_ptr<float>(),
                        norm.data_ptr<float>(), rs::current_stream());
  RS_CHECK_LAUNCH();
  return norm;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(raft_stir, m) {
  m.def("clip_adamw_(Tensor(a!)[] params, Tensor[] grads, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, "
        "Tensor(d!) partial, int[] moff, Tensor? lr_t, float lr, float beta1, float beta2, float eps, "
        "float weight_decay, float max_norm, Tensor(e!) state) -> Tensor");
}

TORCH_LIBRARY_IMPL(raft_stir, CUDA, m) { m.impl("clip_adamw_", &clip_adamw); }
