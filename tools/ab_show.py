"""Print per-kernel times of an A/B run (tools/ab_run.sh)."""
import json
import sys
from pathlib import Path

for f in sorted(Path(sys.argv[1]).glob("*.json")):
    try:
        d = json.loads(f.read_text())
    except Exception as e:  # noqa: BLE001
        print(f.name, "ERR", e)
        continue
    ks = {k: v["avg_ms"] for k, v in d["kernels"].items() if v["avg_ms"] > 0.01}
    print(f"{f.stem:24s} {d['value']:9.2f}", " ".join(f"{k[3:]}={v:.4f}" for k, v in ks.items()))
