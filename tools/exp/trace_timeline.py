"""Print one call's dispatch timeline from a rocprofv3 --kernel-trace CSV.

    python tools/exp/trace_timeline.py <kernel_trace.csv> <first-kernel substring> [nth-from-last]

The call is the span from the nth-from-last (default 2) dispatch whose name contains the
substring to the next one; times in microseconds from the span's first start."""
import csv
import re
import sys


def main():
    path, marker = sys.argv[1], sys.argv[2]
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    s = idx[-back]
    e = idx[-back + 1] if back > 1 else len(rows)
    t0 = int(rows[s]["Start_Timestamp"])
    for r in rows[s:e]:
        n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0][:44]
        st = (int(r["Start_Timestamp"]) - t0) / 1e3
        en = (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"{n:46s} q{r['Queue_Id']:>3s} {st:9.1f} {en:9.1f} {en - st:8.1f}")


if __name__ == "__main__":
    main()
