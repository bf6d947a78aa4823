"""Summarise a tools/profile_round.sh output dir into profiles/: kernel stats CSV copy and
pmc_<tag>.json with per-launch HBM bytes for the quantize kernel (gfx950 correction:
FETCH_SIZE reads half the bytes of wide coalesced streaming loads -> x2; MI355X_MICROARCH.md)."""
import csv, glob, json, os, shutil, sys
src, tag = sys.argv[1], sys.argv[2]
pipeline = sys.argv[3] if len(sys.argv) > 3 else "codes"
# quantize_stream_kernel<WQ, WC, CVEC, NIB> instance used by each bench pipeline
VARIANT = {"q": "<true, false, true, false>", "codes": "<true, true, true, false>",
           "encode": "<false, true, true, false>", "codes4": "<true, true, true, true>"}
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)
st = glob.glob(os.path.join(src, "stats", "**", "*kernel_stats.csv"), recursive=True)
if st:
    shutil.copy(st[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
# The bench probes its output placement before warmup (extra K2 launches on candidate
# buffers, pipeline.py), so the stats average mixes those in; the timed steps are the LAST
# launches of each kernel.  Per-kernel averages over the last `steps` dispatches, from the
# same pass's per-dispatch trace:
STEPS = int(os.environ.get("PROFILE_STEPS", "10"))
tr = glob.glob(os.path.join(src, "stats", "**", "*kernel_trace.csv"), recursive=True)
timed = {}
if tr:
    per = {}
    for r in csv.DictReader(open(tr[0])):
        per.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k, v in per.items():
        last = v[-STEPS:]
        timed[k[:100]] = {"calls_total": len(v), "timed_calls": len(last), "avg_ms_timed": sum(last) / len(last) / 1e6,
                          "avg_ms_all": sum(v) / len(v) / 1e6}
    json.dump({"tag": tag, "steps": STEPS, "kernels": timed}, open(os.path.join(prof, f"{tag}_kernel_timed.json"), "w"),
              indent=1)
def per_kernel(kind, counter):
    fs = glob.glob(os.path.join(src, kind, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for r in csv.DictReader(open(fs[0])):
        if r["Counter_Name"] != counter:
            continue
        vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return vals
fetch, write = per_kernel("fetch", "FETCH_SIZE"), per_kernel("write", "WRITE_SIZE")
out = {"tag": tag, "d": 1 << 20, "clients": 1024, "pipeline": pipeline, "units": "bytes per launch",
       "method": "rocprofv3 --kernel-trace --pmc, one counter per pass; FETCH_SIZE (KB) x2 (gfx950 wide-load correction) + WRITE_SIZE (KB), x1024",
       "kernels": {}}
for k in fetch:
    f = sum(fetch[k]) / len(fetch[k]); w = sum(write.get(k, [0])) / max(1, len(write.get(k, [0])))
    out["kernels"][k[:80]] = {"fetch_kb_raw": f, "write_kb": w, "hbm_bytes": (2 * f + w) * 1024}
    if "quantize_stream_kernel" in k and VARIANT[pipeline] in k:
        out["quantize_bytes_per_launch"] = (2 * f + w) * 1024
        out["quantize_kernel"] = k[:120]
sq = glob.glob(os.path.join(src, "sq", "**", "*counter_collection.csv"), recursive=True)
if sq:
    agg = {}
    for r in csv.DictReader(open(sq[0])):
        if "quantize_stream_kernel" in r["Kernel_Name"] and VARIANT[pipeline] in r["Kernel_Name"]:
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out["quantize_sq"] = {c: sum(v) / len(v) for c, v in agg.items()}
json.dump(out, open(os.path.join(prof, f"pmc_{tag}.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))
