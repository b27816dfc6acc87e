"""Overlap analysis of a rocprofv3 --kernel-trace CSV (one bench step or more):
span, device-busy time (union of kernel intervals), summed kernel time, mean
concurrency, and per kernel family: calls, summed time, and the busy time during
which that family was the ONLY thing running (what removing it would save at most).

  python tools/trace_overlap.py gpurun_out/r04c/c1_kernel_trace.csv [--last-ms 20]
"""
import argparse
import csv
import re
from collections import defaultdict


def family(name: str) -> str:
    m = re.search(r"::(\w+?)(?:<|\()", name)
    if m:
        return m.group(1)
    return name.split("(")[0][:40]


def union_len(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last-ms", type=float, default=0.0, help="only the last N ms of the trace")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
           r.get("Queue_Id", r.get("Stream_Id", ""))) for r in rows]
    ks.sort()
    if a.last_ms > 0:
        end = max(k[1] for k in ks)
        ks = [k for k in ks if k[0] >= end - a.last_ms * 1e6]
    t0, t1 = ks[0][0], max(k[1] for k in ks)
    span = t1 - t0
    busy = union_len([(s, e) for s, e, _, _ in ks])
    summ = sum(e - s for s, e, _, _ in ks)
    print(f"kernels {len(ks)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms ({busy / span * 100:.1f} %)  "
          f"sum {summ / 1e6:.3f} ms  mean concurrency while busy {summ / max(busy, 1):.2f}  "
          f"queues {len(set(k[3] for k in ks))}")
    # exclusive time per family: sweep the event list
    ev = []
    for s, e, n, _ in ks:
        ev.append((s, 1, family(n)))
        ev.append((e, -1, family(n)))
    ev.sort()
    active = defaultdict(int)
    excl = defaultdict(int)
    last = ev[0][0]
    for t, d, f in ev:
        live = [k for k, v in active.items() if v > 0]
        if len(live) == 1 and sum(active.values()) == 1:
            excl[live[0]] += t - last
        active[f] += d
        last = t
    fam = defaultdict(lambda: [0, 0])
    for s, e, n, _ in ks:
        fam[family(n)][0] += 1
        fam[family(n)][1] += e - s
    print(f"{'family':34s} {'calls':>6s} {'sum ms':>8s} {'avg us':>8s} {'alone ms':>9s}")
    for f, (c, t) in sorted(fam.items(), key=lambda x: -x[1][1]):
        print(f"{f:34s} {c:6d} {t / 1e6:8.3f} {t / c / 1e3:8.1f} {excl[f] / 1e6:9.3f}")


if __name__ == "__main__":
    main()
