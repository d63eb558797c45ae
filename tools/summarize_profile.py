#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into the files committed under profiles/.

    python tools/summarize_profile.py --trace DIR/r1_kernel_trace.csv --stats DIR/r1_kernel_stats.csv \
        [--fetch pmc/fetch_counter_collection.csv --write pmc/write_counter_collection.csv] --tag r01

Writes profiles/<tag>_kernel_stats.csv (copy), profiles/<tag>_gemm_by_shape.txt (per tile/grid:
launches, average µs) and, with PMC files, profiles/<tag>_pmc_gemm.json: average HBM bytes per GEMM
launch = (2·FETCH_SIZE + WRITE_SIZE)·1024 (gfx950: FETCH_SIZE reports half of a wide coalesced read,
MI355X_MICROARCH.md §HBM).
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def gemm_key(name, grid_threads):
    tmpl = name.split("<", 1)[1].split(">", 1)[0] if "<" in name else name
    return f"gemm<{tmpl}> grid={int(grid_threads) // 256}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--stats", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--tag", default="r01")
    args = ap.parse_args()
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(args.stats, os.path.join(out, f"{args.tag}_kernel_stats.csv"))

    by = collections.defaultdict(list)
    total = 0
    for r in csv.DictReader(open(args.trace)):
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        total += d
        if "gemm_" in r["Kernel_Name"] and "_kernel" in r["Kernel_Name"]:
            by[gemm_key(r["Kernel_Name"], r["Grid_Size_X"])].append(d)
    g_tot = sum(sum(v) for v in by.values())
    lines = [f"# rocprofv3 --kernel-trace: GEMM launches by tile config and grid ({args.tag})",
             f"# all kernels: {total / 1e6:.1f} ms; GEMM kernels: {g_tot / 1e6:.1f} ms "
             f"({100 * g_tot / max(1, total):.1f} %), {sum(len(v) for v in by.values())} launches, "
             f"avg {g_tot / max(1, sum(len(v) for v in by.values())) / 1e3:.1f} us"]
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"{k:48s} launches={len(v):6d} avg_us={sum(v) / len(v) / 1e3:9.1f} "
                     f"share={100 * sum(v) / g_tot:5.1f}%")
    open(os.path.join(out, f"{args.tag}_gemm_by_shape.txt"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))

    if args.fetch and args.write:
        def load(fn, ctr):
            vals = collections.defaultdict(list)
            for r in csv.DictReader(open(fn)):
                if r["Counter_Name"] == ctr and "gemm_" in r["Kernel_Name"] and "_kernel" in r["Kernel_Name"]:
                    vals[gemm_key(r["Kernel_Name"], r["Grid_Size"])].append(float(r["Counter_Value"]))
            return vals
        f, w = load(args.fetch, "FETCH_SIZE"), load(args.write, "WRITE_SIZE")
        # per kernel (template + grid): HBM bytes per launch from the counter passes; the class
        # average weights each kernel by its launch count in the TRACED update (the counter passes
        # may sample fewer minibatch steps), so it has the mix of bench.py's roofline
        per = {}
        for k in f:
            if k in w and f[k] and w[k]:
                per[k] = (2 * sum(f[k]) / len(f[k]) + sum(w[k]) / len(w[k])) * 1024
        cnt = {k: len(v) for k, v in by.items() if k in per}
        tot = sum(cnt.values())
        dom = max(by, key=lambda k: sum(by[k]))
        res = {"launches_traced": tot,
               "hbm_bytes_per_launch": sum(per[k] * c for k, c in cnt.items()) / max(1, tot),
               "dominant": {"kernel": dom, "hbm_bytes_per_launch": per.get(dom),
                            "avg_us": sum(by[dom]) / len(by[dom]) / 1e3, "launches": len(by[dom])},
               "by_kernel": {k: {"hbm_bytes_per_launch": per[k], "launches_in_update": cnt[k],
                                 "pmc_samples": len(f[k])} for k in sorted(cnt, key=lambda k: -cnt[k])},
               "note": "(2*FETCH_SIZE + WRITE_SIZE)*1024 per GEMM launch (gfx950: FETCH_SIZE reports half of a "
                       "wide coalesced read), separate --pmc passes per counter; class average weighted by the "
                       "traced serial update's launch counts (a pair launch counts once, as in bench.py)"}
        json.dump(res, open(os.path.join(out, f"{args.tag}_pmc_gemm.json"), "w"), indent=1)
        print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
