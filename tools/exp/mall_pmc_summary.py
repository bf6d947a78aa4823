"""Summarize tools/exp/mall_pmc.sh: FETCH_SIZE (KB, x2 gfx950 wide-load correction) per step of
K1 (l1_*) and of K2's kernels, per (group size, arrangement).  The measurement steps are the
last 3 of each process (mall_groups.py --one G I 3).
    python tools/exp/mall_pmc_summary.py gpurun_out/<tag>"""
import csv
import glob
import json
import os
import sys


def main(root):
    for d in sorted(glob.glob(os.path.join(root, "g*_i*"))):
        if not os.path.isdir(d):
            continue
        f = glob.glob(os.path.join(d, "**", "p_counter_collection.csv"), recursive=True)[0]
        k1 = k2 = mean = 0.0
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "FETCH_SIZE":
                continue
            name, v = r["Kernel_Name"], 2.0 * float(r["Counter_Value"]) * 1024
            if "l1_" in name:
                k1 += v
            elif "mean" in name:
                mean += v
            elif "anonymous namespace" in name:
                k2 += v
        G, I = os.path.basename(d)[1:].split("_i")
        x_group = int(G) * (1 << 20) * 4
        print(json.dumps({"group_clients": int(G), "arrangement": "interleaved" if I == "1" else "separate",
                          "steps": 3, "k1_fetch_GB_per_step": round(k1 / 3 / 1e9, 3),
                          "k2_fetch_GB_per_step": round(k2 / 3 / 1e9, 3), "mean_fetch_GB_per_step": round(mean / 3 / 1e9, 3),
                          "x_GB": round(1024 * (1 << 20) * 4 / 1e9, 3), "group_x_MiB": x_group >> 20}))


if __name__ == "__main__":
    main(sys.argv[1])
