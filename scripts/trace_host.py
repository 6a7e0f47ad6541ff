#!/usr/bin/env python
"""Why is the GPU idle inside a training step?  Joins a rocprofv3 kernel trace
with its HIP runtime-API trace (``--kernel-trace --hip-runtime-trace``) and,
for one steady-state step, reports:

* every fully idle GPU interval > ``--min-us`` (no kernel on any queue) and
  every main-queue gap > ``--min-us``, with the host API calls that were
  running during it (summed per function) and the launch lag of the kernel
  that ends it (kernel start - end of its launch call: ~0 means the host
  launched it just in time, i.e. the gap is host time);
* the per-function totals of blocking calls (synchronize, malloc, free,
  event sync) inside the step.

    python scripts/trace_host.py DIR   (the rocprofv3 -d directory)
"""
import argparse
import collections
import csv
import glob
import os


def load(d, pat):
    rows = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-us", type=float, default=80.0)
    a = ap.parse_args()
    ks = load(a.dir, "*kernel_trace.csv")
    api = load(a.dir, "*hip_api_trace.csv")
    T = lambda r: (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    ks.sort(key=lambda r: T(r)[0])
    # steady-state step: between the last two optimizer (FusedAdam) kernel groups
    idx = [i for i, r in enumerate(ks) if ("FusedAdam" in r["Kernel_Name"] or "adamw_kernel" in r["Kernel_Name"])]
    groups = []
    for i in idx:
        if groups and i - groups[-1][-1] <= 2:
            groups[-1].append(i)
        else:
            groups.append([i])
    s0, s1 = groups[-2][-1] + 1, groups[-1][-1] + 1
    step = ks[s0:s1]
    t0, t1 = T(step[0])[0], max(T(r)[1] for r in step)
    print(f"step {(t1 - t0) / 1e6:.3f} ms, {len(step)} kernels")
    launch_end = {}
    for r in api:
        cid = r.get("Correlation_Id")
        if cid:
            launch_end[cid] = T(r)[1]
    api_in = [r for r in api if T(r)[1] >= t0 and T(r)[0] <= t1]
    main_tid = collections.Counter(r["Thread_Id"] for r in api_in).most_common(1)[0][0]
    host = sorted((r for r in api_in if r["Thread_Id"] == main_tid), key=lambda r: T(r)[0])

    def calls_in(s, e):
        c = collections.defaultdict(float)
        n = collections.Counter()
        for r in host:
            a_, b_ = T(r)
            if b_ < s or a_ > e:
                continue
            c[r["Function"]] += (min(b_, e) - max(a_, s)) / 1e3
            n[r["Function"]] += 1
        return ", ".join(f"{k} {v:.0f}us/{n[k]}" for k, v in sorted(c.items(), key=lambda x: -x[1])[:5])

    def lag(r):
        le = launch_end.get(r.get("Correlation_Id"))
        return (T(r)[0] - le) / 1e3 if le else float("nan")

    # fully idle intervals
    iv = sorted(T(r) + (r,) for r in step)
    idle, ce, last = [], iv[0][1], iv[0][2]
    for s, e, r in iv[1:]:
        if s > ce and s - ce > a.min_us * 1e3:
            idle.append((ce, s, last, r))
        if e > ce:
            ce, last = e, r
    tot = sum(s - e for e, s, _, _ in idle) / 1e6
    print(f"fully idle intervals > {a.min_us:.0f} us: {len(idle)}, {tot:.3f} ms")
    for e, s, prev, nxt in idle:
        print(f"  at {(e - t0) / 1e6:7.3f} ms idle {(s - e) / 1e3:6.0f} us | before: {prev['Kernel_Name'][:40]} | "
              f"after: {nxt['Kernel_Name'][:40]} (launch lag {lag(nxt):.0f} us) | host: {calls_in(e, s)}")
    qs = collections.Counter(r["Queue_Id"] for r in step)
    mq = [r for r in step if r["Queue_Id"] == qs.most_common(1)[0][0]]
    gaps = [(T(x)[1], T(y)[0], y) for x, y in zip(mq, mq[1:]) if T(y)[0] - T(x)[1] > a.min_us * 1e3]
    print(f"main-queue gaps > {a.min_us:.0f} us: {len(gaps)}, {sum(s - e for e, s, _ in gaps) / 1e6:.3f} ms")
    for e, s, y in gaps:
        other = [r for r in step if r["Queue_Id"] != y["Queue_Id"] and T(r)[1] > e and T(r)[0] < s]
        busy = sum(min(T(r)[1], s) - max(T(r)[0], e) for r in other) / 1e3
        print(f"  at {(e - t0) / 1e6:7.3f} ms gap {(s - e) / 1e3:6.0f} us (other queues busy {busy:5.0f} us) | next: "
              f"{y['Kernel_Name'][:40]} (launch lag {lag(y):.0f} us) | host: {calls_in(e, s)}")
    blocking = collections.defaultdict(float)
    nb = collections.Counter()
    for r in host:
        f = r["Function"]
        if any(k in f for k in ("Synchronize", "Malloc", "Free", "Query", "Wait")):
            blocking[f] += (T(r)[1] - T(r)[0]) / 1e3
            nb[f] += 1
    print("host calls that can block, inside the step:")
    for f, v in sorted(blocking.items(), key=lambda x: -x[1])[:12]:
        print(f"  {f:40s} {v:8.0f} us  {nb[f]}x")
    lags = [lag(r) for r in step if lag(r) == lag(r)]
    lags.sort()
    if lags:
        print(f"launch lag over the step's kernels: median {lags[len(lags) // 2]:.0f} us, "
              f"p10 {lags[len(lags) // 10]:.0f} us, min {lags[0]:.0f} us (small = host-bound)")


if __name__ == "__main__":
    main()
