"""bench.py driver contract on the CPU (gloo ranks): ``--gpus N`` started
without a launcher must spawn N ranks itself (torch.distributed.run as a child
process), time the step on every rank and print ONE JSON line from rank 0
with the whole-job value and ``n_gpus``/``parallelism`` = N."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--device", "cpu", "--steps", "2", "--warmup", "1", "--batch", "1", "--size", "128", "128",
        "--iters", "2"]


def _run(extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + ARGS + extra, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON line (rank 0)
    return json.loads(lines[0])


def test_bench_spawns_ranks_for_gpus_n():
    out = _run(["--gpus", "2"])
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 2
    assert out["steps"] == 2 and out["warmup"] == 1
    assert out["value"] > 0 and out["final_loss"] == out["final_loss"]  # finite
    # whole-job value: global pairs / the slowest rank's time
    assert abs(out["value"] - 2 * 2 / (out["ms_per_step"] * 2 / 1000.0)) / out["value"] < 0.01


def test_bench_single_rank_default():
    out = _run([])
    assert out["n_gpus"] == 1 and out["config"]["parallelism"] == "dp1"
