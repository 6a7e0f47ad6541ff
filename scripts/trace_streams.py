#!/usr/bin/env python
"""Stream-level summary of one training step from a rocprofv3 kernel trace:
per-queue busy time, GPU-idle time, and the main-queue gaps (what the other
queues run while the main stream waits).

    python scripts/trace_streams.py gpurun_out/trace/train_kernel_trace.csv.gz [A_ms B_ms]

Steps are delimited by the optimizer kernel; TRACE_ANCHOR=<kernel substring>
(with TRACE_GROUP=<max index distance inside one anchor group>) delimits
them by another kernel instead (scripts/bench_encoders.py: stem_fwd, 60).

With A_ms B_ms: also list every kernel of the step that starts in [A, B] ms
(queue, stream, start, duration) -- what each queue runs around a gap.
"""
import collections
import csv
import gzip
import os
import sys

TOP = 25


def main(path, window=None):
    op = gzip.open if path.endswith(".gz") else open
    rows = list(csv.DictReader(op(path, "rt")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    anchor = os.environ.get("TRACE_ANCHOR")  # e.g. "stem_fwd": steps delimited by this kernel's groups
    if anchor:
        idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
        idx = [i - 1 for i in idx]  # the step ends just before the anchor group
    else:
        idx = [i for i, r in enumerate(rows) if ("FusedAdam" in r["Kernel_Name"] or "adamw_kernel" in r["Kernel_Name"])]
    groups = []
    gap = int(os.environ.get("TRACE_GROUP", "2"))
    for i in idx:
        if groups and i - groups[-1][-1] <= gap:
            groups[-1].append(i)
        else:
            groups.append([i])
    s0, s1 = groups[-2][-1] + 1, groups[-1][-1] + 1
    step = rows[s0:s1]
    T = lambda r: (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    t0 = min(T(r)[0] for r in step)
    t1 = max(T(r)[1] for r in step)
    byq, cnt = collections.defaultdict(float), collections.Counter()
    for r in step:
        s, e = T(r)
        byq[r["Queue_Id"]] += (e - s) / 1e6
        cnt[r["Queue_Id"]] += 1
    iv = sorted(T(r) for r in step)
    busy, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"step {(t1 - t0) / 1e6:.3f} ms, {len(step)} kernels, GPU busy {busy / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e6:.3f} ms")
    for q in sorted(byq):
        print(f"  queue {q}: {cnt[q]} kernels, {byq[q]:.3f} ms busy")
    main = max(byq, key=byq.get)
    mq = [r for r in step if r["Queue_Id"] == main]
    gaps = []
    for a, b in zip(mq, mq[1:]):
        g = T(b)[0] - T(a)[1]
        if g > 100000:
            gaps.append(((T(a)[1] - t0) / 1e6, g / 1e6, b["Kernel_Name"][:60]))
    print(f"main-queue gaps > 100 us: {len(gaps)}, {sum(g[1] for g in gaps):.3f} ms")
    for g in gaps:
        print(f"  at {g[0]:7.3f} ms: {g[1]:6.3f} ms idle, then {g[2]}")
    # timeline: per 0.5 ms bin, each queue's busy fraction and its longest kernel there
    BIN = 500000
    nb = (t1 - t0) // BIN + 1
    qs = sorted(byq, key=byq.get, reverse=True)
    occ = {q: [0.0] * nb for q in qs}
    top = {q: [("", 0)] * nb for q in qs}
    for r in step:
        s, e = T(r)
        q = r["Queue_Id"]
        for bi in range((s - t0) // BIN, (e - t0) // BIN + 1):
            lo, hi = max(s, t0 + bi * BIN), min(e, t0 + (bi + 1) * BIN)
            if hi > lo:
                occ[q][bi] += (hi - lo) / BIN
                if hi - lo > top[q][bi][1]:
                    top[q][bi] = (r["Kernel_Name"].replace("void ", "").split("(")[0].split("<")[0][-28:], hi - lo)
    print("timeline (0.5 ms bins): busy % per queue [" + ", ".join(qs) + "] and the main queue's longest kernel")
    for bi in range(nb):
        print(f"  {bi * 0.5:5.1f} ms  " + " ".join(f"{100 * min(occ[q][bi], 1):4.0f}" for q in qs) + "   "
              + " | ".join(top[q][bi][0] for q in qs))
    # per-queue kernel families (template arguments kept: tiles differ)
    for q in sorted(byq, key=byq.get, reverse=True):
        fam, n = collections.defaultdict(float), collections.Counter()
        for r in step:
            if r["Queue_Id"] == q:
                s, e = T(r)
                k = r["Kernel_Name"].replace("void ", "").split("(")[0][:70]
                fam[k] += (e - s) / 1e6
                n[k] += 1
        print(f"queue {q} top kernels:")
        for k in sorted(fam, key=fam.get, reverse=True)[:TOP]:
            print(f"  {fam[k]:7.3f} ms {n[k]:4d}x  {k}")
    if window:
        a, b = window
        print(f"kernels starting in [{a}, {b}] ms (queue / stream, start, duration):")
        for r in step:
            s, e = T(r)
            if a <= (s - t0) / 1e6 <= b:
                print(f"  q{r['Queue_Id']} s{r.get('Stream_Id', '?')} {(s - t0) / 1e6:8.3f} {(e - s) / 1e3:8.1f} us  "
                      + r["Kernel_Name"].replace("void ", "")[:90])


if __name__ == "__main__":
    main(sys.argv[1], (float(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else None)
