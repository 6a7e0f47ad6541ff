"""Wall time of the first (cold: MIOpen solution search) and steady training steps."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from raft_stir_amd.config import make_args  # noqa: E402
from raft_stir_amd.data.synthetic import make_batch  # noqa: E402
from raft_stir_amd.models import RAFT  # noqa: E402
from raft_stir_amd.train.loss import sequence_loss  # noqa: E402

dev = torch.device("cuda")
m = RAFT(make_args(mixed_precision=True)).to(dev).to(memory_format=torch.channels_last).train()
opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
i1, i2, flow, valid = make_batch(8, 368, 496, seed=0, device=dev)
ts = []
for it in range(8):
    torch.cuda.synchronize()
    t0 = time.time()
    preds = m(i1, i2, iters=12)
    loss, _ = sequence_loss(preds, flow, valid, 0.8, sync_metrics=False)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    ts.append((time.time() - t0) * 1e3)
print(os.environ.get("TAG", ""), "first %.0f ms, second %.0f ms, steady %.1f ms" % (ts[0], ts[1], sum(ts[3:]) / 5),
      flush=True)
