#!/usr/bin/env python3
"""BASELINE.md §3 rows from one box's bench lines: tools/results_table.py DIR_A DIR_B prints the markdown
rows (DIR_A: r04_final_a.sh's bench.json = C4; DIR_B: r04_final_b.sh's per-config lines)."""
import json
import os
import sys


def row(name, gpus, path, note=""):
    if not os.path.exists(path):
        return f"| {name} | {gpus} | — | — | — | — | — | — | — |"
    lines = [ln for ln in open(path) if ln.startswith("{")]     # RCCL may print a banner first
    d = json.loads(lines[-1])
    ms = d["ms_per_step"]
    rf = d.get("roofline", {})
    cb = d.get("cpu_baseline") or {}
    cpu = cb.get("value")
    allc = (cb.get("all_cores") or {}).get("value")
    cpu_s = f"{cpu:,.0f} / {allc:,.0f} env-steps/s" if cpu and allc else ("—" if not cpu else f"{cpu:,.0f}")
    ratio = f"{d['value'] / cpu:,.0f}×" if cpu else "—"
    mb = d.get("minibatch_steps_per_sec")
    frac = rf.get("frac")
    return (f"| {name} | {gpus} | {1000 / ms:.3g} ({ms:,.1f} ms) | {d['value']:,.0f} | "
            f"{mb:,.0f} | {frac:.3f} of {rf.get('peak', 0):.0f} {rf.get('unit', '')} | {note} | {cpu_s} | {ratio} |")


def main():
    a, b = sys.argv[1], sys.argv[2]
    print(row("C2", 1, os.path.join(b, "c2.json"), "—"))
    print(row("C3", 1, os.path.join(b, "c3.json"), "—"))
    print(row("C3, B = 64", 1, os.path.join(b, "c3b64.json"), "—"))
    print(row("C4", 1, os.path.join(a, "bench.json"), "1.00"))
    print(row("C4 G = 8 shard (rank 0, emulated)", "1 of 8", os.path.join(b, "shard8.json"),
              "unmeasured on hardware (N = 2…8 runs are the driver's)"))
    print(row("C4, B = 64", 1, os.path.join(b, "c4b64.json"), "—"))
    print(row("C5 per-rank shard (bf16)", "1 of 8", os.path.join(b, "c5.json"), "unmeasured on hardware"))


if __name__ == "__main__":
    main()
