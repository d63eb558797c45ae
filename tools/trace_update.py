#!/usr/bin/env python3
"""Per-kernel breakdown of the LAST PPO update in a rocprofv3 --kernel-trace CSV.

    python tools/trace_update.py gpurun_out/prof/run_kernel_trace.csv [--top 30]
"""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--top", type=int, default=30)
args = ap.parse_args()
rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
# the last update: from the GAE's V(state) forward (every layer, m = N) with its copies and fills,
# next_value_map_kernel, the own-row forward of V(next_state), the scan, then the minibatch loops
# (round 5: the window used to start `layers` rows before next_value_map_kernel and missed the first
# forward GEMMs and copies of the GAE)
anchor = [i for i, r in enumerate(rows) if "next_value_map" in r["Kernel_Name"] or "gae_block" in r["Kernel_Name"]]
j = anchor[-1] if anchor else len(rows) - 1
# walk back over the GAE's forward GEMMs and its copies / fills (a rollout or the previous update's
# Adam ends the walk)
while j > 0 and any(t in rows[j - 1]["Kernel_Name"] for t in ("gemm", "rocclr", "fill", "copy")):
    j -= 1
# … up to its last Adam launch (a bench run's rollout measurement may follow the update)
end = max((i for i in range(j, len(rows)) if "adam" in rows[i]["Kernel_Name"]), default=len(rows) - 1)
last = rows[j:end + 1]
t0, t1 = int(last[0]["Start_Timestamp"]), int(last[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last)
print(f"update span {(t1 - t0) / 1e6:.2f} ms, kernel busy {busy / 1e6:.2f} ms, {len(last)} launches")
agg = collections.defaultdict(lambda: [0, 0])
for r in last:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:72]
    key = f"{n} g={int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}"
    agg[key][0] += 1
    agg[key][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
    print(f"{v[1] / 1e6:8.2f} ms {100 * v[1] / busy:5.1f}% {v[0]:5d} x {v[1] / v[0] / 1e3:8.1f} us  {k}")
