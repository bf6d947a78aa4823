"""Collate the config-C4 NMSE curves (d = 2^22, 50 instances, tools/nmse_curves.py outputs under
profiles/) into one summary: per distribution the driver's own user grid (ND:43 and
Lognormal_dist.py:43: arange(1, 102, 5); Laplace_dist.py:43, Gamma_dist.py:40,
Bernoulli_dist.py:44: arange(1, 101, 5)), the avg / max script NMSE of every scheme and rate
on it, the run time, and a compact table.  A run over the 21-point grid holds the 20-point
driver grid as its first 20 rows (same streams: the counts are drawn in order), and its 21st
row (n = 101) is kept apart as `beyond_driver_grid`.

    python tools/c4_summary.py profiles/r6*_nmse_curves_d4194304_*_i50.json > profiles/r6_c4_summary.json"""
import json
import sys

DRIVER_USERS = {"normal": list(range(1, 102, 5)), "lognormal": list(range(1, 102, 5)),
                "laplace": list(range(1, 101, 5)), "gamma": list(range(1, 101, 5)),
                "bernoulli": list(range(1, 101, 5))}


def main():
    out = {"config": "C4: d = 2^22, 50 instances, the drivers' seeds (np.random.seed(42), torch.manual_seed(42)), "
                     "schemes in the drivers' call order (EDEN, unbiased, biased, QUIC-FL; DRIVE / Kashin / Scalar "
                     "not built, so the torch stream is that of a driver calling only these)",
           "quicfl_tables": "synthetic sender tables (tests/golden/quicfl_tables.py; the published ones are absent "
                            "from the reference) with the reference's receiver tables",
           "nmse": "script NMSE (ND:155: ||est - emp||^2 / (num_trials * sum||v||^2 * n)), avg and max over instances",
           "distributions": {}}
    table = []
    for path in sys.argv[1:]:
        r = json.load(open(path))
        for key, v in r["curves"].items():
            dist, sc, rate = key.split("/")
            grid = DRIVER_USERS[dist]
            users = v["users"]
            idx = [users.index(u) for u in grid]
            d = out["distributions"].setdefault(dist, {"users": grid, "instances": r["instances"], "source": path,
                                                       "timing_s": r.get("timing", {}).get(dist), "curves": {}})
            e = {"avg": [v["avg"][i] for i in idx], "max": [v["max"][i] for i in idx]}
            extra = [u for u in users if u not in grid]
            if extra:
                e["beyond_driver_grid"] = {str(u): {"avg": v["avg"][users.index(u)], "max": v["max"][users.index(u)]}
                                           for u in extra}
            d["curves"][f"{sc}/{rate}"] = e
            if sc == "unbiased" or rate == "R1":
                pick = [1, 11, 51, grid[-1]]
                table.append({"dist": dist, "scheme": f"{sc} {rate}",
                              **{f"n={u}": round(e["avg"][grid.index(u)], 12) for u in pick}})
    out["table_avg"] = table
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
