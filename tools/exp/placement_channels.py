"""Summarise a placement_pmc.py run under `rocprofv3 --pmc ... --output-format json`: the last
2 * reps K2 dispatches (fast set first), every counter per TCC instance (8 XCDs x 16 channels,
records in the order of the counter's `instances` list), as totals, per-XCD and per-channel
sums and the spread over the 128 instances.

    python tools/exp/placement_channels.py <results.json> <reps> [out.json]"""
import json
import sys

import numpy as np


def main():
    d = json.load(open(sys.argv[1]))
    reps = int(sys.argv[2])
    t = d["rocprofiler-sdk-tool"][0]
    names = {c["id"]["handle"]: c["name"] for c in t["counters"]}
    dims = {c["name"]: [(x["dimensions"][0]["index"], x["dimensions"][1]["index"]) for x in c["instances"]]
            for c in t["counters"]}
    k2 = [r for r in t["callback_records"]["counter_collection"]
          if r["dispatch_data"]["dispatch_info"]["grid_size"]["x"] == 262144]
    out = {"dispatches": []}
    for i, r in enumerate(k2[-2 * reps:]):
        vals = {}
        for rec in r["records"]:
            vals.setdefault(names[rec["counter_id"]["handle"]], []).append(rec["value"])
        row = {"set": "fast" if i < reps else "slow",
               "ms": round((r["dispatch_data"]["end_timestamp"] - r["dispatch_data"]["start_timestamp"]) / 1e6, 4)}
        for nm, v in vals.items():
            v = np.asarray(v, np.float64)
            grid = np.zeros((8, 16))
            for (inst, xcc), x in zip(dims[nm], v):
                grid[xcc, inst] += x
            row[nm] = {"total": float(v.sum()), "min": float(v.min()), "max": float(v.max()),
                       "cv": float(v.std() / v.mean()) if v.mean() else None,
                       "per_xcc": grid.sum(1).round(1).tolist(), "per_channel": grid.sum(0).round(1).tolist()}
        out["dispatches"].append(row)
    s = json.dumps(out)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s)
    for row in out["dispatches"]:
        print(row["set"], row["ms"], {k: (round(v["total"] / 1e6, 3), round(v["cv"], 4) if v["cv"] else None)
                                      for k, v in row.items() if isinstance(v, dict)})


if __name__ == "__main__":
    main()
