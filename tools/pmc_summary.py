"""Summarise rocprofv3 PMC passes (tools/pmc.sh) per kernel: mean per dispatch.

Read bytes: with the request-size pass (TCC_EA0_RDREQ_{32B,64B,128B}_sum),
exactly 32 / 64 / 128 B per request of each size (`hbm_read_bytes_by_size`,
used as `hbm_read_bytes_corrected`); FETCH_SIZE's own expression counts
128-B requests through TCC_BUBBLE, which on gfx950 misses them, so it is
also kept doubled as MI355X_MICROARCH.md prescribes for wide coalesced
reads (`hbm_read_bytes_fetch_x2`).  The two agree within 0.1 % for this
path's kernels, whose reads leave L2 as 128-B requests (r06w); the exact
form also holds where requests are 32 or 64 B.  FETCH_SIZE / WRITE_SIZE are
in KB.

usage: python tools/pmc_summary.py <pmc dir> [<summary.json> <workload key>]
The workload key is the one bench.py looks up: "<frame_len>:<csum|nocsum>:<frames>".
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


def load(d: Path):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(d.glob("p*/**/*counter_collection.csv")):
        with open(f) as fh:
            rows = list(csv.DictReader(fh))
        per = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in rows:
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            names[key] = r["Kernel_Name"]
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        for key, cs in per.items():
            for c, v in cs.items():
                acc[names[key]][c].append(v)
    return acc


def summarise(d: Path) -> dict:
    out = {}
    for k, cs in load(d).items():
        short = re.sub(r"<[^>]*>", "", k.split("(")[0].replace("dqdk::", "").replace("void ", "")).strip()
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in m:
            m["hbm_read_bytes_fetch_x2"] = m["FETCH_SIZE"] * 1024 * 2
            m["hbm_read_bytes_corrected"] = m["hbm_read_bytes_fetch_x2"]
        sz = ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")
        if all(c in m for c in sz):
            m["hbm_read_bytes_by_size"] = 32 * m[sz[0]] + 64 * m[sz[1]] + 128 * m[sz[2]]
            if "TCC_EA0_RDREQ_sum" in m:  # requests of none of the three sizes (expected 0)
                m["rdreq_unsized"] = m["TCC_EA0_RDREQ_sum"] - m[sz[0]] - m[sz[1]] - m[sz[2]]
            m["hbm_read_bytes_corrected"] = m["hbm_read_bytes_by_size"]
        if "WRITE_SIZE" in m:
            m["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_bytes_per_launch"] = m["hbm_read_bytes_corrected"] + m["hbm_write_bytes"]
        out[short] = m
    return out


def main():
    d = Path(sys.argv[1])
    out = summarise(d)
    for k, m in sorted(out.items()):
        if k.startswith("__amd"):
            continue
        print(k)
        for c, v in sorted(m.items()):
            print(f"   {c:32s} {v:16.4g}")
    if len(sys.argv) > 3:
        p = Path(sys.argv[2])
        allw = json.loads(p.read_text()) if p.exists() else {}
        allw[sys.argv[3]] = {k: v for k, v in out.items() if k.startswith("rx_")}
        p.write_text(json.dumps(allw, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
