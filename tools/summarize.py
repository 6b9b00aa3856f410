#!/usr/bin/env python3
"""Print the key numbers of a gpurun_out/ session: bench lines and rocprofv3 kernel stats."""
import csv
import glob
import json
import os
import sys

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(os.path.join(OUT, "bench*.log"))):
    L = [l for l in open(f) if l.startswith("{")]
    if not L:
        print(f, "no line")
        continue
    d = json.loads(L[-1])
    print(os.path.basename(f), f"value={d['value'] / 1e6:.1f}M ms/step={d['ms_per_step']} k={d.get('kernels_ms_per_step')}")
    if d.get("roofline"):
        r = d["roofline"]
        print("   roofline", r["kernel"], r["frac"], "launch_us", r["kernel_avg_launch_us"], "pipeline", r["pipeline"]["frac"])
    for k in ("host_path", "c4_frame", "bird"):
        if d.get(k):
            print("  ", k, d[k].get("ms_per_frame"))
    if d.get("hamming"):
        print("   hamming", d["hamming"]["matches_per_s"] / 1e12, "T/s mfma frac", (d["hamming"].get("mfma_i8") or d["hamming"].get("mfma_fp4") or {}).get("frac"))
    if d.get("cpu_baseline"):
        c = d["cpu_baseline"]
        print("   cpu", c["value"], c["cores"], c.get("host_estimate_value"), "speedup", d.get("speedup_vs_cpu_allcore"),
              d.get("speedup_vs_cpu_host_estimate"))
for f in sorted(glob.glob(os.path.join(OUT, "prof*", "run_kernel_stats.csv"))):
    print(f)
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        n = n[:n.index("(")] if "(" in n else n
        print(f"   {n[-32:]:32s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs']) / 1e3:9.2f} "
              f"min_us={float(r['MinNs']) / 1e3:9.2f} max_us={float(r['MaxNs']) / 1e3:9.2f}")
