"""Per-iteration timeline of a rocprofv3 kernel trace (--kernel-trace --output-format csv).

Usage: python tools/timeline.py <dir with *kernel_trace.csv> [--anchor k_gemm_nn_gram] [--iters 100]

Takes the window that starts at the launch of the anchor kernel `iters` occurrences before
its last one and ends at the end of the trace, and prints for each kernel name the launch
count, total and mean duration, and the idle time on the GPU right before it (the gap from
the previous kernel's end to its start: launch latency, host waits, dependent collectives).
Test/analysis tooling only.
"""
import argparse
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--anchor", default="k_gemm_nn_gram")
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit("no kernel_trace.csv under " + a.dir)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    anchors = [i for i, r in enumerate(rows) if a.anchor in r[2]]
    if len(anchors) < a.iters:
        sys.exit(f"only {len(anchors)} launches of {a.anchor}")
    i0 = anchors[-a.iters]
    win = rows[i0:]
    t0, t1 = win[0][0], max(r[1] for r in win)
    busy = defaultdict(float)
    cnt = defaultdict(int)
    gap = defaultdict(float)
    prev_end = None
    for s, e, n in win:
        busy[n] += (e - s) * 1e-3
        cnt[n] += 1
        if prev_end is not None:
            gap[n] += max(0, s - prev_end) * 1e-3
        prev_end = e if prev_end is None else max(prev_end, e)
    span = (t1 - t0) * 1e-3
    tot_busy = sum(busy.values())
    tot_gap = sum(gap.values())
    it = a.iters
    print(f"window: {len(win)} kernels, {span:.1f} us = {span / it:.1f} us per {a.anchor} "
          f"({1e6 / (span / it):.1f} per s); busy {tot_busy / it:.1f} us, idle {tot_gap / it:.1f} us per iteration")
    print(f"{'kernel':60s} {'n/it':>6s} {'us/it':>8s} {'mean us':>8s} {'idle before/it':>14s}")
    for n in sorted(busy, key=lambda n: -busy[n]):
        print(f"{n:60s} {cnt[n] / it:6.2f} {busy[n] / it:8.1f} {busy[n] / cnt[n]:8.2f} {gap[n] / it:14.2f}")


if __name__ == "__main__":
    main()
