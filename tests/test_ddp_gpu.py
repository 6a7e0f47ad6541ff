"""Data parallelism around the fused training engine on the GPU.

1. RCCL (``nccl`` backend) on one MI355X: a world of one, DDP wrapped with
   ``force=True`` so the real DDP + packed-gradient path runs -- the fused
   engine, DeferGrads, the side streams, ``gradient_as_bucket_view`` and the
   engine's packed all-reduce issued from the weight-gradient stream.  Under
   deterministic mode (runtime/determinism.py) the gradients must be BITWISE
   equal to an un-wrapped replica's, and the issue order must show the overlap:
   the packed update-block all-reduce and the first DDP bucket are issued
   BEFORE the encoder backward has produced its last gradient.
2. Two ranks on one GPU over gloo (RCCL needs one GPU per rank): per-rank
   batch 1 must reproduce a single process that runs the same two batch-1
   backward passes and accumulates them (the same per-sample launches, so
   only the fp32 reduction order differs: <= 1e-5 relative, deterministic
   mode), with BatchNorm frozen on both, and the two replicas must be bitwise
   identical after the step; and match ONE batch-2 single-process pass
   within 3e-2 (batch equivalence; different launches and bf16 roundings).

Reference semantics: /root/reference/train.py:138 (DataParallel over --gpus).
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

COMMON = r'''
import os, sys, torch
sys.path.insert(0, os.environ["ROOT"])
import torch.distributed as dist
from raft_stir_amd.config import make_args
from raft_stir_amd.models import RAFT
from raft_stir_amd.data.synthetic import make_batch
from raft_stir_amd.train.loss import sequence_loss
from raft_stir_amd.parallel import dist as rd

def flat_grads(m):
    return torch.cat([p.grad.detach().float().flatten() for p in m.parameters()])

def new_model(dev, state=None):
    torch.manual_seed(0)
    m = RAFT(make_args(mixed_precision=True)).to(dev).to(memory_format=torch.channels_last).train()
    if state is not None:
        m.load_state_dict(state)
    m.freeze_bn()
    return m
'''

NCCL_WORKER = COMMON + r'''
from raft_stir_amd.runtime.determinism import set_deterministic
set_deterministic(True)
info = rd.init_distributed(backend="nccl", force=True)
assert dist.get_backend() == "nccl"
dev = torch.device("cuda", 0)
m = new_model(dev)
ref = new_model(dev, m.state_dict())
ddp = rd.wrap_ddp(m, device=dev, force=True)
eng = m._train_engine()
assert eng.grad_group is not None, "packed update-block all-reduce not attached"
trace = []
eng.trace = trace
enc_ids = {id(p): n for n, p in m.named_parameters() if not n.startswith("update_block")}
for n, p in m.named_parameters():
    if id(p) in enc_ids:
        p.register_post_accumulate_grad_hook(lambda p, n=n: trace.append(("enc_grad", n)))
def hook(state, bucket):
    trace.append(("ddp_bucket", bucket.index()))
    fut = dist.all_reduce(bucket.buffer(), async_op=True).get_future()
    return fut.then(lambda f: f.value()[0])
ddp.register_comm_hook(None, hook)
i1, i2, fl, v = make_batch(2, 192, 256, seed=7, device=dev)
for step in range(2):  # step 0 builds DDP's buckets; step 1 is the steady state
    trace.clear()
    m.zero_grad(set_to_none=True)
    loss, _ = sequence_loss(ddp(i1, i2, iters=4), fl, v, 0.8, sync_metrics=False)
    loss.backward()
torch.cuda.synchronize()
ref.zero_grad(set_to_none=True)
l2, _ = sequence_loss(ref(i1, i2, iters=4), fl, v, 0.8, sync_metrics=False)
l2.backward()
g1, g2 = flat_grads(m), flat_grads(ref)
rel = ((g1 - g2).norm() / g2.norm()).item()
ub = [i for i, (n, p) in enumerate(m.named_parameters()) if n.startswith("update_block")]
ps = list(m.parameters())
gu1 = torch.cat([ps[i].grad.float().flatten() for i in ub])
gu2 = torch.cat([list(ref.parameters())[i].grad.float().flatten() for i in ub])
relu = ((gu1 - gu2).norm() / gu2.norm()).item()
kinds = [k for k, _ in trace]
print("TRACE", kinds.count("packed_allreduce"), kinds.count("ddp_bucket"), kinds.count("enc_grad"))
last_enc = max(i for i, k in enumerate(kinds) if k == "enc_grad")
print("ORDER", kinds.index("packed_allreduce"), kinds.index("ddp_bucket"), last_enc)
print("REL", rel, relu, torch.isfinite(g1).all().item())
print("BITWISE", torch.equal(g1, g2))
rd.shutdown()
'''

GLOO_WORKER = COMMON + r'''
from raft_stir_amd.runtime.determinism import set_deterministic
set_deterministic(True)
info = rd.init_distributed(backend="gloo")
dev = torch.device("cuda", 0)
m = new_model(dev)
ref = new_model(dev, m.state_dict())
ddp = rd.wrap_ddp(m, device=dev)
i1, i2, fl, v = make_batch(2, 192, 256, seed=7, device=dev)
r = info.rank
loss, _ = sequence_loss(ddp(i1[r:r+1], i2[r:r+1], iters=4), fl[r:r+1], v[r:r+1], 0.8, sync_metrics=False)
loss.backward()
torch.save(flat_grads(m).cpu(), os.environ["OUT"] + f"/rank{r}.pt")
if r == 0:
    # the same two per-sample passes in one process, accumulated, then averaged like DDP
    for k in range(2):
        l2, _ = sequence_loss(ref(i1[k:k+1], i2[k:k+1], iters=4), fl[k:k+1], v[k:k+1], 0.8, sync_metrics=False)
        l2.backward()
    torch.save((flat_grads(ref) / 2).cpu(), os.environ["OUT"] + "/single.pt")
    # and ONE batch-2 pass of a fresh replica (batch equivalence: the mean loss
    # over the global batch, as the reference's DataParallel computes it)
    ref2 = new_model(dev, m.state_dict())
    l3, _ = sequence_loss(ref2(i1, i2, iters=4), fl, v, 0.8, sync_metrics=False)
    l3.backward()
    torch.save(flat_grads(ref2).cpu(), os.environ["OUT"] + "/batched.pt")
    print("PACKED", m._train_engine().grad_group is not None)
rd.shutdown()
'''


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(tmp_path):
    env = dict(os.environ, ROOT=ROOT, OUT=str(tmp_path))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    return env


def _val(out, tag):
    return [l.split()[1:] for l in out.splitlines() if l.startswith(tag)][-1]


def test_ddp_nccl_fused_engine_world1(cuda, tmp_path):
    script = tmp_path / "n.py"
    script.write_text(NCCL_WORKER)
    env = _env(tmp_path)
    env.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    n_packed, n_bucket, n_enc = map(int, _val(r.stdout, "TRACE"))
    assert n_packed == 1 and n_bucket >= 2 and n_enc > 0
    i_packed, i_bucket, i_last_enc = map(int, _val(r.stdout, "ORDER"))
    # overlap: both reductions are issued while the encoder backward is still producing gradients
    assert i_packed < i_last_enc and i_bucket < i_last_enc
    rel, relu, finite = _val(r.stdout, "REL")
    assert finite == "True"
    # same weights, same inputs, deterministic kernels, a world of one: bitwise
    assert _val(r.stdout, "BITWISE") == ["True"], (rel, relu)


def test_ddp_two_ranks_match_single_process(cuda, tmp_path):
    script = tmp_path / "w.py"
    script.write_text(GLOO_WORKER)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(script)]
    r = subprocess.run(cmd, env=_env(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert _val(r.stdout, "PACKED") == ["True"]
    a = torch.load(tmp_path / "rank0.pt", weights_only=True)
    b = torch.load(tmp_path / "rank1.pt", weights_only=True)
    s = torch.load(tmp_path / "single.pt", weights_only=True)
    assert torch.equal(a, b)  # all-reduced gradients -> identical replicas
    assert torch.isfinite(a).all()
    rel = ((a - s).norm() / s.norm()).item()
    # identical per-sample launches: only the order of the two-term fp32 sums differs
    assert rel < 1e-5, rel
    # batch equivalence vs one batch-2 process: different launches (batch-2
    # tiles, bf16 rounding of batched activations), same math
    bt = torch.load(tmp_path / "batched.pt", weights_only=True)
    relb = ((a - bt).norm() / bt.norm()).item()
    assert relb < 3e-2, relb
