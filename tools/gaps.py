"""Idle gaps between consecutive dispatches on one queue, from a rocprofv3
kernel trace (`--kernel-trace`, csv): for each (previous kernel -> next
kernel) pair, the count and the median / mean gap in microseconds between the
previous dispatch's end and the next one's start (overlapping dispatches,
e.g. from other queues, give negative gaps and are skipped).

usage: python tools/gaps.py <prof dir or *_kernel_trace.csv> [--min-us 0] [--max-us 1000]
"""
import csv
import re
import statistics
import sys
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    return re.sub(r"<[^>]*>", "", name.split("(")[0].replace("dqdk::", "").replace("void ", "")).strip()


def main():
    src = Path(sys.argv[1])
    files = [src] if src.is_file() else sorted(src.glob("**/*kernel_trace.csv"))
    lo = float(sys.argv[sys.argv.index("--min-us") + 1]) if "--min-us" in sys.argv else 0.0
    hi = float(sys.argv[sys.argv.index("--max-us") + 1]) if "--max-us" in sys.argv else 1000.0
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((r.get("Queue_Id", "0"), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             short(r["Kernel_Name"])))
    by_q = defaultdict(list)
    for q, s, e, n in rows:
        by_q[q].append((s, e, n))
    gaps = defaultdict(list)
    for q, ds in by_q.items():
        ds.sort()
        for (s0, e0, n0), (s1, e1, n1) in zip(ds, ds[1:]):
            g = (s1 - e0) / 1e3
            if lo <= g <= hi:
                gaps[(n0, n1)].append(g)
    for (a, b), g in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
        print(f"{a:28s} -> {b:28s} n={len(g):5d} median={statistics.median(g):7.2f} us mean={statistics.mean(g):7.2f} us")


if __name__ == "__main__":
    main()
