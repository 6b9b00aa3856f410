#!/usr/bin/env python3
"""Summarise tools/ham_prof.sh: per-launch kernel durations of the Hamming leg from the rocprofv3 kernel
trace, the bench line's own HIP-event figure, SQ / MFMA counters and HBM bytes per launch, and the
FP4 MFMA roofline fraction recomputed from the trace.

  ops per launch = 512 x sum over the 255 pairs of n_query x n_train    (32 x 32 pairs x K = 256 bits x 2 = 512
                   ops per pair; bench.py `hamming.mfma_fp4`)
  frac           = ops per launch / (mean k_top2_mfma + mean k_top2b_merge duration in the trace: one launch is
                   the top-2 kernel and, when the trains are sliced, the merge after it on the same stream) / 10 PF
Counter sections are per dispatch; rocprofv3 serialises dispatches while it counts.

FETCH_SIZE is doubled (gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md §HBM); WRITE_SIZE
is taken as is.  Usage: python3 tools/ham_report.py gpurun_out/ham > report.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

PEAK_FP4_OPS = 10.0e15  # dense fp4 (e2m1) MFMA: 4x the bf16 rate (2.5 PF dense), MI355X_MICROARCH.md §Matrix cores
KERNELS = ("k_top2_mfma", "k_top2b_merge")


def kname(s):
    for k in KERNELS:
        if re.search(r"\b" + k + r"\b", s) or (k + "<") in s or (k + "(") in s:
            return k
    return None


def trace(d):
    fn = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    dur = defaultdict(list)
    for row in csv.DictReader(open(fn[0])):
        k = kname(row["Kernel_Name"])
        if k:
            dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    return dur, fn[0]


def counters(d):
    fn = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for row in csv.DictReader(open(fn[0])):
        k = kname(row["Kernel_Name"])
        if not k:
            continue
        per[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[k].add(row["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in per.items()}, {k: len(v) for k, v in disp.items()}


def bench_line(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def main(root):
    line = bench_line(os.path.join(root, "bench.log"))
    ham = line["hamming"]
    mkey, peak = "mfma_fp4", PEAK_FP4_OPS
    ops = ham[mkey]["achieved_ops_per_s"] * ham["kernel_avg_us"] * 1e-6   # 512 x evals per launch
    dur, tfile = trace(os.path.join(root, "trace"))
    mean = {k: sum(v) / len(v) for k, v in dur.items()}
    t_launch = sum(mean.values())
    out = {"bench_line_hamming": ham, "ops_per_launch": ops, "trace_file": os.path.relpath(tfile, root),
           "trace_dispatches": {k: len(v) for k, v in dur.items()},
           "trace_mean_us_per_dispatch": {k: round(v, 3) for k, v in mean.items()},
           "trace_launch_us": round(t_launch, 3),
           "mfma_form": mkey, "peak_ops_per_s": peak,
           "frac_from_trace": round(ops / (t_launch * 1e-6) / peak, 4),
           "frac_bench_line": ham[mkey]["frac"]}
    sq, n = counters(os.path.join(root, "sq"))
    sq2, _ = counters(os.path.join(root, "sq2"))
    for k in sq:
        sq[k].update(sq2.get(k, {}))
    out["sq_per_dispatch"] = {k: {c: round(v) for c, v in sorted(cs.items())} for k, cs in sq.items()}
    out["sq_dispatches"] = n
    t = sq.get("k_top2_mfma")
    if t:
        # MFMA pipe cycles summed over SIMDs / (SIMDs x busy cycles of the kernel): the matrix cores' duty
        # cycle; GRBM_GUI_ACTIVE / 8 XCDs / wall = the effective clock
        w = mean.get("k_top2_mfma", 0) * 1e-6 * len(dur.get("k_top2_mfma", [])) / max(1, n.get("k_top2_mfma", 1))
        out["top2_mfma"] = {
            "mfma_insts": t.get("SQ_INSTS_MFMA"), "valu_insts": t.get("SQ_INSTS_VALU"),
            "valu_per_mfma": round(t["SQ_INSTS_VALU"] / t["SQ_INSTS_MFMA"], 3) if t.get("SQ_INSTS_MFMA") else None,
            "mfma_busy_frac": (round(t["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * t["GRBM_GUI_ACTIVE"] / 8), 4)
                               if t.get("GRBM_GUI_ACTIVE") else None),
            "effective_clock_ghz": round(t["GRBM_GUI_ACTIVE"] / 8 / w / 1e9, 3) if w and t.get("GRBM_GUI_ACTIVE") else None,
        }
    fetch, _ = counters(os.path.join(root, "fetch"))
    write, _ = counters(os.path.join(root, "write"))
    out["hbm_bytes_per_dispatch"] = {k: {"fetch_corrected": round(2 * fetch.get(k, {}).get("FETCH_SIZE", 0) * 1024),
                                       "write": round(write.get(k, {}).get("WRITE_SIZE", 0) * 1024)}
                                   for k in set(fetch) | set(write)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ham")
