"""Per-kernel averages of every PMC counter found under a rocprofv3 output directory.
    python tools/pmc_table.py <dir> [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys


def main(root, *subs):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if subs and not any(s in name for s in subs):
                continue
            acc[name[:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main(*sys.argv[1:])
