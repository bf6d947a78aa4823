"""Print the kernel timeline of the second-to-last call that starts with a given kernel from a
rocprofv3 kernel trace (start / end / duration in us relative to that kernel, queue id).
    python tools/trace_timeline.py <s_kernel_trace.csv> [first-kernel-substring] [count]"""
import csv
import sys


def main(path, first="l1_partial", count=60):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    s = idx[-2] if len(idx) > 1 else idx[-1]
    t0 = int(rows[s]["Start_Timestamp"])
    for r in rows[s:s + count]:
        a = (int(r["Start_Timestamp"]) - t0) / 1e3
        b = (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"{a:9.1f} {b:9.1f} {b - a:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:60]}")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]), *([int(sys.argv[3])] if len(sys.argv) > 3 else []))
