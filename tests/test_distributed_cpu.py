"""Data parallelism without a cluster: multi-process DDP over
gloo on the CPU, launched exactly like the GPU job (torch.distributed.run,
127.0.0.1 rendezvous).  Two ranks with per-rank batch 1 must end with the
same weights as one process with the global batch 2 (same samples: the
sampler shards one global permutation), which pins gradient averaging,
sampler sharding and rank-0 checkpointing."""
import os
import socket
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--device", "cpu", "--stage", "synthetic", "--small", "--iters", "2", "--image_size", "128", "128",
        "--batch_size", "2", "--num_workers", "0", "--lr", "0.0004", "--wdecay", "0.0001",
        "--synthetic_length", "8", "--sum_freq", "2", "--val_freq", "1000", "--num_steps", "3"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _env():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["OMP_NUM_THREADS"] = "2"
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def test_ddp_gloo_matches_single_process(tmp_path):
    single = ARGS + ["--name", "s", "--ckpt_dir", str(tmp_path / "s"), "--log_dir", str(tmp_path / "ls")]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "train.py")] + single, env=_env(),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    multi = ARGS + ["--name", "m", "--ckpt_dir", str(tmp_path / "m"), "--log_dir", str(tmp_path / "lm")]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "train.py")] + multi
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    a = torch.load(tmp_path / "s" / "s.pth", weights_only=True)
    b = torch.load(tmp_path / "m" / "m.pth", weights_only=True)
    assert a.keys() == b.keys()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    torch.manual_seed(1234)
    init = RAFT(make_args(small=True)).state_dict()
    keys = [k for k in a if a[k].is_floating_point()]
    diff = torch.cat([(a[k] - b[k]).flatten() for k in keys])
    moved = torch.cat([(a[k] - init[k[len("module."):]]).flatten() for k in keys])
    assert moved.norm() > 0
    assert (diff.norm() / moved.norm()).item() < 0.05


def test_ddp_gradient_allreduce_exact(tmp_path):
    """Per-rank batch-1 gradients averaged by DDP == batch-2 gradients of one process."""
    script = tmp_path / "g.py"
    script.write_text(
        "import torch\n"
        "from raft_stir_amd.parallel import dist as d\n"
        "from raft_stir_amd.config import make_args\n"
        "from raft_stir_amd.models import RAFT\n"
        "from raft_stir_amd.data.synthetic import make_batch\n"
        "from raft_stir_amd.train.loss import sequence_loss\n"
        "info = d.init_distributed(backend='gloo')\n"
        "torch.manual_seed(0)\n"
        "m = RAFT(make_args(small=True)).train()\n"
        "ref = RAFT(make_args(small=True)).train(); ref.load_state_dict(m.state_dict())\n"
        "i1, i2, fl, v = make_batch(2, 128, 128, seed=5)\n"
        "ddp = d.wrap_ddp(m)\n"
        "r = info.rank\n"
        "loss, _ = sequence_loss(ddp(i1[r:r+1], i2[r:r+1], iters=2), fl[r:r+1], v[r:r+1], 0.8)\n"
        "loss.backward()\n"
        "if info.is_main:\n"
        "    l2, _ = sequence_loss(ref(i1, i2, iters=2), fl, v, 0.8)\n"
        "    l2.backward()\n"
        "    g1 = torch.cat([p.grad.flatten() for p in m.parameters()])\n"
        "    g2 = torch.cat([p.grad.flatten() for p in ref.parameters()])\n"
        "    print('REL', ((g1 - g2).norm() / g2.norm()).item())\n"
        "d.shutdown()\n")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(script)]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rel = float([l for l in r.stdout.splitlines() if l.startswith("REL")][-1].split()[1])
    assert rel < 1e-5, rel


def test_collective_helpers_gloo(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(
        "import torch, json\n"
        "from raft_stir_amd.parallel import dist as d\n"
        "info = d.init_distributed(backend='gloo')\n"
        "m = d.reduce_metrics({'a': torch.tensor(float(info.rank)), 'b': 2.0 * info.rank})\n"
        "mx = d.all_reduce_max(float(info.rank + 1))\n"
        "d.barrier()\n"
        "if info.is_main: print(json.dumps({'m': m, 'mx': mx, 'ws': info.world_size}))\n"
        "d.shutdown()\n")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(script)]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["ws"] == 3 and out["mx"] == 3.0
    assert abs(out["m"]["a"] - 1.0) < 1e-9 and abs(out["m"]["b"] - 2.0) < 1e-9


def _ckpt_rel(a, b, init):
    keys = [k for k in a if a[k].is_floating_point()]
    diff = torch.cat([(a[k] - b[k]).flatten() for k in keys])
    moved = torch.cat([(a[k] - init[k[len("module."):] if k.startswith("module.") else k]).flatten() for k in keys])
    assert moved.norm() > 0
    return (diff.norm() / moved.norm()).item()


def test_spawn_worker_three_ranks_matches_single_process(tmp_path):
    """train.py --gpus 0 1 2 without a launcher: main() spawns one process per
    rank (_spawn_worker, 127.0.0.1 rendezvous) -- here as three gloo CPU ranks
    (RS_SPAWN_CPU=1) with per-rank batch 1 against one process with the global
    batch 3 on the same samples."""
    args = [a if a != "2" or i == 0 or ARGS[i - 1] != "--batch_size" else "3" for i, a in enumerate(ARGS)]
    assert args[args.index("--batch_size") + 1] == "3"
    single = args + ["--name", "s", "--ckpt_dir", str(tmp_path / "s"), "--log_dir", str(tmp_path / "ls")]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "train.py")] + single, env=_env(),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env = _env()
    env["RS_SPAWN_CPU"] = "1"
    multi = args + ["--gpus", "0", "1", "2", "--name", "m", "--ckpt_dir", str(tmp_path / "m"),
                    "--log_dir", str(tmp_path / "lm")]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "train.py")] + multi, env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    a = torch.load(tmp_path / "s" / "s.pth", weights_only=True)
    b = torch.load(tmp_path / "m" / "m.pth", weights_only=True)
    assert a.keys() == b.keys()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    torch.manual_seed(1234)
    init = RAFT(make_args(small=True)).state_dict()
    assert _ckpt_rel(a, b, init) < 0.05


def test_packed_update_allreduce_four_ranks(tmp_path):
    """The fused engine's data-parallel contract at world size 4 (gloo):
    wrap_ddp(packed_update_grads=True) replicates the update-block parameters
    from rank 0, makes DDP ignore them and attaches the packed all-reduce;
    reduce_packed averages a packed gradient buffer over the ranks; a step the
    fused engine cannot take refuses to run; the encoder gradients still go
    through DDP's buckets (averaged) while the ignored update-block gradients
    stay rank-local."""
    script = tmp_path / "p.py"
    script.write_text(
        "import json, torch\n"
        "from raft_stir_amd.parallel import dist as d\n"
        "from raft_stir_amd.config import make_args\n"
        "from raft_stir_amd.models import RAFT\n"
        "from raft_stir_amd.data.synthetic import make_batch\n"
        "from raft_stir_amd.train.loss import sequence_loss\n"
        "info = d.init_distributed(backend='gloo')\n"
        "r, ws = info.rank, info.world_size\n"
        "torch.manual_seed(100 + r)  # different init per rank: the broadcast must fix it\n"
        "m = RAFT(make_args(small=True)).train()\n"
        "ddp = d.wrap_ddp(m, packed_update_grads=True)\n"
        "eng = m._train_engine()\n"
        "upd = torch.cat([p.detach().flatten() for p in eng.params])\n"
        "g = torch.arange(1000, dtype=torch.float32) * (r + 1)\n"
        "eng.reduce_packed(g)\n"
        "i1, i2, fl, v = make_batch(ws, 128, 128, seed=3)\n"
        "try:\n"
        "    m(i1[r:r+1], i2[r:r+1], iters=2)  # CPU step: not the fused engine -> must refuse\n"
        "    guard = False\n"
        "except RuntimeError:\n"
        "    guard = True\n"
        "eng.grad_group = None  # (CPU: the stock update block; DDP still ignores its parameters)\n"
        "loss, _ = sequence_loss(ddp(i1[r:r+1], i2[r:r+1], iters=2), fl[r:r+1], v[r:r+1], 0.8)\n"
        "loss.backward()\n"
        "ids = {id(p) for p in eng.params}\n"
        "enc = torch.cat([p.grad.flatten() for p in m.parameters() if id(p) not in ids and p.grad is not None])\n"
        "ug = torch.cat([p.grad.flatten() for p in eng.params if p.grad is not None])\n"
        "out = {}\n"
        "for name, t in (('upd', upd), ('enc', enc), ('ug', ug)):\n"
        "    lst = [torch.zeros_like(t) for _ in range(ws)]\n"
        "    torch.distributed.all_gather(lst, t)\n"
        "    out[name] = max((x - lst[0]).abs().max().item() for x in lst)\n"
        "out['packed'] = (g - torch.arange(1000, dtype=torch.float32) * (ws + 1) / 2).abs().max().item()\n"
        "out['ws'] = ws\n"
        "out['guard'] = guard\n"
        "if info.is_main: print(json.dumps(out))\n"
        "d.shutdown()\n")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(script)]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["ws"] == 4
    assert out["guard"]               # an ineligible step refuses instead of skipping the reduction
    assert out["upd"] == 0.0          # update-block parameters replicated from rank 0
    assert out["packed"] < 1e-3       # packed buffer averaged over the four ranks
    assert out["enc"] < 1e-6          # encoder gradients all-reduced by DDP
    assert out["ug"] > 1e-6           # ignored update-block gradients left rank-local
