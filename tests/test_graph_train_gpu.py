"""Whole-step hipGraph training (runtime/graph.py GraphedTrainStep, the
one-GPU ``bench.py --train-graph`` path): the graphed replays -- fused
engine on its HIP streams, loss, backward, clip, capturable AdamW, weight
repacking recorded in the graph -- must follow the eager step's loss
trajectory from the same initialisation (same batches; only the fp32
atomic-scatter order differs), and the weights must move.
Reference step: /root/reference/train.py:162-183.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import copy, os, sys, argparse, torch
sys.path.insert(0, os.environ["ROOT"])
from raft_stir_amd.config import make_args
from raft_stir_amd.models import RAFT
from raft_stir_amd.data.synthetic import DevicePool
from raft_stir_amd.train.loss import sequence_loss
from raft_stir_amd.train.optim import fetch_optimizer
from raft_stir_amd.runtime.graph import GraphedTrainStep
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m_e = RAFT(make_args(mixed_precision=True, small=os.environ.get("SMALL") == "1")).to(dev).to(
    memory_format=torch.channels_last).train()
m_g = copy.deepcopy(m_e)
targs = argparse.Namespace(lr=2e-4, wdecay=1e-4, epsilon=1e-8, num_steps=1000)
loss_fn = lambda p, f, v: sequence_loss(p, f, v, gamma=0.8, sync_metrics=False)[0]
pool = DevicePool(4, 2, 192, 256, dev, seed=0)
batches = [pool.next() for _ in range(4)]
w0 = torch.cat([p.detach().float().flatten() for p in m_g.parameters()])

opt_g, sch_g = fetch_optimizer(targs, m_g, capturable=True)
gs = GraphedTrainStep(m_g, opt_g, loss_fn, batches[0], clip=1.0, warmup=3, iters=6)
# the constructor's 3 eager warm-up steps advanced m_g: mirror them on the eager replica
opt_e, sch_e = fetch_optimizer(targs, m_e)
def estep(b):
    opt_e.zero_grad(set_to_none=True)
    loss = loss_fn(m_e(b[0], b[1], iters=6), b[2], b[3])
    loss.backward()
    torch.nn.utils.clip_grad_norm_(m_e.parameters(), 1.0)
    opt_e.step()
    return loss.detach()
for _ in range(3):
    estep(batches[0])
le, lg = [], []
for i in range(8):
    if i == 4:
        # a model registered AFTER the capture (ADVICE r2: its packed layouts must
        # not move or free the storage the captured repack reads)
        m_x = copy.deepcopy(m_e)
        with torch.no_grad():
            m_x(batches[0][0], batches[0][1], iters=2)
        import gc; gc.collect()
        torch.cuda.empty_cache()
    b = batches[i % 4]
    le.append(float(estep(b)))
    lg.append(float(gs.step(b)))
torch.cuda.synchronize()
w1 = torch.cat([p.detach().float().flatten() for p in m_g.parameters()])
print("LOSSES", " ".join(f"{a:.5f},{b:.5f}" for a, b in zip(le, lg)))
print("MOVED", float((w1 - w0).norm()))
# eager inference after graphed steps sees the weights the replays wrote:
# equal to a fresh model holding the same values (fresh packs)
m_g.eval(); m_f = copy.deepcopy(m_g).eval()
with torch.no_grad():
    a = m_g(batches[1][0], batches[1][1], iters=4, test_mode=True)[1]
    bb = m_f(batches[1][0], batches[1][1], iters=4, test_mode=True)[1]
print("EVALDIFF", float((a - bb).abs().max()), float(bb.abs().max()))
'''


@pytest.mark.parametrize("small", [False, True])  # (RAFT-small: bench.py's default training step)
def test_graphed_train_step_tracks_eager(cuda, tmp_path, small):
    script = tmp_path / "g.py"
    script.write_text(WORKER)
    env = dict(os.environ, ROOT=ROOT, SMALL="1" if small else "0")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("LOSSES")][-1]
    pairs = [tuple(map(float, t.split(","))) for t in line.split()[1:]]
    assert len(pairs) == 8
    for e, g in pairs:
        assert abs(e - g) <= 0.05 * abs(e) + 1e-3, pairs
    moved = float([l for l in r.stdout.splitlines() if l.startswith("MOVED")][-1].split()[1])
    assert moved > 0
    d, ref = map(float, [l for l in r.stdout.splitlines() if l.startswith("EVALDIFF")][-1].split()[1:])
    assert d <= 1e-3 * max(ref, 1.0), (d, ref)
