#!/usr/bin/env python3
"""One line per bench log: ms per update, the GEMM class rate, the dominant template and the per-shape
averages (µs) — for reading A/B runs.   python tools/bench_brief.py gpurun_out/TAG/*.log"""
import json
import sys

for path in sys.argv[1:]:
    lines = [ln for ln in open(path, errors="replace") if ln.startswith("{")]
    if not lines:
        print(f"{path}: no JSON line")
        continue
    d = json.loads(lines[-1])
    rf = d.get("roofline") or {}
    dom = rf.get("dominant") or {}
    shapes = " ".join(f"{s['op']}:{s['m']}x{s['n']}x{s['l']}={s['avg_us']:.1f}" for s in rf.get("by_shape", [])[:8])
    comm = d.get("comm")
    print(f"{path}: {d['ms_per_step']:.2f} ms/update  class {rf.get('frac', 0):.3f}  dominant {dom.get('op')} "
          f"{dom.get('frac', 0):.3f} ({dom.get('avg_us', 0):.1f} us)  serial {rf.get('serial_update_ms', 0):.1f} ms"
          + (f"  comm {comm['us_per_minibatch_step']:.1f} us/step [{comm['mode'][:24]}]" if comm else ""))
    print(f"    {shapes}")
