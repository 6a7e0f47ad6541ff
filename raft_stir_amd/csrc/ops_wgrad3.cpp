// torch.ops.raft_stir.wgrad_v3: the all-taps, split-K weight gradient of a
// stride-1 conv over a batched image stack (csrc/wgrad_v3.hip).  Same operand
// conventions as conv_wgrad (ops_conv.cpp): dY an NHWC bf16 [NI, H, W, *]
// buffer read at channels [yoff, yoff + Cout), X up to three NHWC bf16
// segments (64-channel multiples) whose images repeat over the stack with
// period seg_period pixels; dW (fp32 [>= Cout][KH*KW][Ktot]) and db
// (fp32 [Cout]) are accumulated into.  Deterministic: per-split partials
// reduced in a fixed order.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include "host_common.h"

namespace rs {
struct Wgrad3Launch {
  const void* dy;
  int ystr, yoff, Cout;
  unsigned dy_bytes;
  const void* seg_ptr[3];
  int seg_C[3], seg_stride[3], seg_imgs[3];
  unsigned seg_bytes[3];
  int nseg;
  int NI, H, W, KH, KW, Ktot;
  float* dw;
  float* db;
  float* part;
  int bm;
  int nsplit;
};
int wgrad3_splits(int NI, int H, int W, int KH, int Cout, int Ktot, int bm);
long wgrad3_workspace(int Cout, int Ktot, int KH, int KW, int bm, int nsplit);
void wgrad3_launch(const Wgrad3Launch& L, hipStream_t stream);
}  // namespace rs

namespace {
using at::Tensor;

void wgrad_v3(const Tensor& dy, int64_t yoff, int64_t Cout, const std::vector<Tensor>& segs,
              at::IntArrayRef seg_off, at::IntArrayRef seg_C, at::IntArrayRef seg_period, int64_t KH, int64_t KW,
              const Tensor& dw, const c10::optional<Tensor>& db, int64_t bm) {
  TORCH_CHECK(dy.is_cuda() && dy.is_contiguous() && dy.dim() == 4 && dy.scalar_type() == at::kBFloat16,
              "wgrad_v3: dy must be contiguous bf16 NHWC");
  TORCH_CHECK((KH == 3 && KW == 3) || (KH == 1 && KW == 5) || (KH == 5 && KW == 1),
              "wgrad_v3: 3x3, 1x5 and 5x1 kernels only");
  TORCH_CHECK(bm == 64 || bm == 128, "wgrad_v3: bm must be 64 or 128");
  const int NI = dy.size(0), H = dy.size(1), W = dy.size(2);
  // dY rows are read through a range-checked buffer: channels past Cout only feed discarded rows
  TORCH_CHECK(yoff >= 0 && yoff % 8 == 0 && Cout > 0 && yoff + Cout <= dy.size(3),
              "wgrad_v3: dy channel window out of bounds");
  TORCH_CHECK(dy.numel() * 2 < (int64_t(1) << 31), "wgrad_v3: dY tensor must be < 2 GiB");
  TORCH_CHECK(!segs.empty() && segs.size() <= 3 && seg_off.size() == segs.size() && seg_C.size() == segs.size() &&
                  seg_period.size() == segs.size(),
              "wgrad_v3: segment spec");
  rs::Wgrad3Launch L{};
  int Ktot = 0;
  for (size_t s = 0; s < segs.size(); ++s) {
    const Tensor& t = segs[s];
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.dim() == 4 && t.scalar_type() == at::kBFloat16 &&
                    t.size(1) == H && t.size(2) == W,
                "wgrad_v3: segment must be contiguous bf16 NHWC with dy's spatial size");
    TORCH_CHECK(seg_period[s] == t.size(0) * H * W && NI % t.size(0) == 0,
                "wgrad_v3: segment period must be its pixel count and its images divide dy's");
    const int C = seg_C[s], off = seg_off[s];
    TORCH_CHECK(C % 64 == 0 && off % 8 == 0 && off + C <= t.size(3), "wgrad_v3: segment window (C % 64)");
    TORCH_CHECK(t.numel() * 2 < (int64_t(1) << 31), "wgrad_v3: segment tensor must be < 2 GiB");
    L.seg_ptr[s] = static_cast<const at::BFloat16*>(t.data_ptr()) + off;
    L.seg_C[s] = C;
    L.seg_stride[s] = t.size(3);
    L.seg_imgs[s] = t.size(0);
    L.seg_bytes[s] = (unsigned)((t.numel() - off) * 2);
    Ktot += C;
  }
  TORCH_CHECK(dw.is_cuda() && dw.is_contiguous() && dw.scalar_type() == at::kFloat && dw.dim() == 3 &&
                  dw.size(0) >= Cout && dw.size(1) == KH * KW && dw.size(2) == Ktot,
              "wgrad_v3: dw must be fp32 (>=Cout, taps, Ktot)");
  if (db) TORCH_CHECK(db->is_cuda() && db->is_contiguous() && db->scalar_type() == at::kFloat && db->numel() >= Cout,
                      "wgrad_v3: db fp32 (Cout,)");
  // the reduction adds rows [0, Cout) of a [round_up(Cout, bm)][taps][Ktot] partial into dw: rows past
  // dw.size(0) are never touched; partial rows >= Cout are discarded
  const c10::DeviceGuard guard(dy.device());
  L.dy = dy.data_ptr(); L.ystr = dy.size(3); L.yoff = yoff; L.Cout = Cout;
  L.dy_bytes = (unsigned)(dy.numel() * 2);
  L.nseg = segs.size();
  L.NI = NI; L.H = H; L.W = W; L.KH = KH; L.KW = KW; L.Ktot = Ktot;
  L.dw = dw.data_ptr<float>();
  L.db = db ? db->data_ptr<float>() : nullptr;
  L.bm = bm;
  L.nsplit = rs::wgrad3_splits(NI, H, W, KH, Cout, Ktot, bm);
  Tensor part = at::empty({rs::wgrad3_workspace(Cout, Ktot, KH, KW, bm, L.nsplit)}, dy.options().dtype(at::kFloat));
  L.part = part.data_ptr<float>();
  rs::wgrad3_launch(L, rs::current_stream());
  RS_CHECK_LAUNCH();
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(raft_stir, m) {
  m.def("wgrad_v3(Tensor dy, int yoff, int Cout, Tensor[] segs, int[] seg_off, int[] seg_C, int[] seg_period, "
        "int KH, int KW, Tensor(a!) dw, Tensor(b!)? db, int bm) -> ()");
}
TORCH_LIBRARY_IMPL(raft_stir, CUDA, m) { m.impl("wgrad_v3", &wgrad_v3); }
