#!/usr/bin/env python3
"""Print value + per-kernel ms of an A/B directory (tools/ab_run.sh output)."""
import glob
import json
import sys

for f in sorted(glob.glob(f"gpurun_out/ab_{sys.argv[1]}/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "ERR", e)
        continue
    ks = " ".join(f"{k[3:]}={v['ms_per_batch']:.4f}" for k, v in d["kernels"].items() if v["ms_per_batch"] > 0.003)
    print(f"{f.split('/')[-1][:-5]:14s} {d['value']:8.2f} {ks}")
