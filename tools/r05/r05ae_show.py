#!/usr/bin/env python3
"""Per-dispatch view of call r05ae's PMC passes: every rx_decode_fused
dispatch in order with its duration and counters (pass 1: UTCL1 translation
miss rate, mean TCP -> TCC read latency; pass 2: UTCL2 busy share, mean
TCC -> memory read queue level)."""
import csv
import json
import sys
from collections import OrderedDict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r05ae"
out = {}
for p in ("p1", "p2"):
    rows = OrderedDict()
    with open(f"{d}/{p}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            if "rx_decode_fused" not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            e = rows.setdefault(k, {"us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
            e[r["Counter_Name"]] = float(r["Counter_Value"])
    lst = []
    for k, e in rows.items():
        if p == "p1":
            e["utcl1_miss_rate"] = e["TCP_UTCL1_TRANSLATION_MISS_sum"] / max(e["TCP_UTCL1_REQUEST_sum"], 1)
            e["tcp_tcc_lat"] = e["TCP_TCC_READ_REQ_LATENCY_sum"] / max(e["TCP_TCC_READ_REQ_sum"], 1)
        else:
            e["utcl2_busy"] = e["GRBM_UTCL2_BUSY"] / max(e["GRBM_GUI_ACTIVE"], 1)
            e["ea_rd_level"] = e["TCC_EA0_RDREQ_LEVEL_sum"] / max(e["TCC_EA0_RDREQ_sum"], 1)
        lst.append(dict(dispatch=k, **e))
    out[p] = lst
    for e in lst:
        extra = (f"miss {e['utcl1_miss_rate']:.4f} lat {e['tcp_tcc_lat']:.0f}" if p == "p1"
                 else f"utcl2 {e['utcl2_busy']:.3f} ealevel {e['ea_rd_level']:.1f}")
        print(p, e["dispatch"], f"{e['us']:.0f} us", extra)
    try:
        line = json.loads(open(f"{d}/{p}.json").read().strip().splitlines()[-1])
        print(p, "probe", line.get("staging_probe"))
    except Exception as ex:  # noqa: BLE001
        print(p, "no bench line", ex)
json.dump(out, open(f"{d}/summary.json", "w"), indent=1)
