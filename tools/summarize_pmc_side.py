"""Per-kernel HBM bytes of a side path (biased / EDEN / QUIC-FL batch) from the passes of
tools/pmc_sidepaths.sh, against each kernel's pass floor (algorithmic bytes).

    python tools/summarize_pmc_side.py OUTDIR/biased biased TAG   ->  profiles/pmc_TAG_biased.json

FETCH_SIZE counts half the bytes of 16-byte-per-lane streaming reads on gfx950
(MI355X_MICROARCH.md): `fetch_bytes_x2` applies that correction, `fetch_bytes_raw` does not;
for kernels whose loads are narrower (gathers, 4-byte lanes) the raw figure is the closer one.
"""
import csv
import glob
import json
import os
import sys

D, N = 1 << 20, 1024
# kernel-name substring -> (pass floor in bytes per launch, what it reads/writes)
FLOORS = {
    "biased": [
        ("l1_partial_kernel<true, (anonymous namespace)::AbsOp", 4 * D * N, "KB1: read x"),
        ("l1_partial_kernel<true, (anonymous namespace)::RezKHistOp", 4 * D * N, "KB2: read x (k' and digit 1)"),
        ("rez_compact_kernel", 4 * D * N, "KB4b: read x (bucket keys; round 4 only)"),
        ("rez_output_fine_kernel", 8 * D * N, "KB6f: read x, write q, list the threshold bin (round 5)"),
        ("rez_output_kernel", 8 * D * N, "KB6: read x, write q (all clients over its two launches)"),
        ("rez_tiecount_kernel", 0, "KB5: ambiguous clients only"),
    ],
    "eden": [
        ("fwht_low4096_kernel<1", 8 * D * N, "sender low pass: read x, write"),
        ("fwht_high256_kernel<true, false>", 8 * D * N, "sender high pass: read, write"),
        ("eden_norm", 4 * D * N, "norm: read"),
        ("fwht_low4096_kernel<3", 8 * D * N, "bins + receiver's first pass: read, write"),
        ("fwht_high256_kernel<true, true>", 8 * D * N, "receiver high pass: read, write"),
    ],
    "quicfl": [
        ("fwht_low4096_kernel<1", 8 * D * N, "sender low pass"),
        ("fwht_high256_kernel", 8 * D * N, "sender high pass / receiver passes"),
        ("eden_norm", 4 * D * N, "norm"),
        ("quicfl_send_wave_kernel", (4 + 1 + 1 + 1 + 1) * D * N,
         "KQ1: read rot, h (write + read), X u8, mask (exact values ~0.4 %)"),
        ("quicfl_recv_wave_kernel", (1 + 1 + 4) * D * N, "KQ2: read X, mask, write f32"),
    ],
}


def per_kernel(root, counter):
    vals = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return vals


def main(src, path, tag):
    fetch = per_kernel(os.path.join(src, "fetch"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "write"), "WRITE_SIZE")
    out = {"tag": tag, "path": path, "d": D, "clients": N, "units": "bytes per launch (mean over launches)",
           "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE in separate passes (KB); "
                     "fetch_bytes_x2 = 2 x FETCH_SIZE (gfx950 wide-load correction)", "kernels": {}}
    for k in sorted(fetch):
        f = sum(fetch[k]) / len(fetch[k]) * 1024
        w = sum(write.get(k, [0.0])) / max(1, len(write.get(k, []))) * 1024
        e = {"launches": len(fetch[k]), "fetch_bytes_raw": f, "fetch_bytes_x2": 2 * f, "write_bytes": w}
        for sub, floor, what in FLOORS.get(path, []):
            if sub in k and floor:
                e.update({"pass_floor_bytes": floor, "what": what,
                          "ratio_x2": round((2 * f + w) / floor, 3), "ratio_raw": round((f + w) / floor, 3)})
                break
        out["kernels"][k[:110]] = e
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                       f"pmc_{tag}_{path}.json")
    json.dump(out, open(dst, "w"), indent=1)
    for k, e in out["kernels"].items():
        if e["fetch_bytes_raw"] + e["write_bytes"] > 1e8:
            print(f"{k[:70]:70s} x{e['launches']:3d} fetch2 {e['fetch_bytes_x2'] / 1e9:7.3f} GB  "
                  f"write {e['write_bytes'] / 1e9:7.3f} GB  ratio {e.get('ratio_x2', '-')}")


if __name__ == "__main__":
    main(*sys.argv[1:])
