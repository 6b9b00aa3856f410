#!/usr/bin/env python3
"""Summarise tools/ham_prof.sh: per-launch kernel durations of the Hamming leg from the rocprofv3 kernel
trace, the bench line's own HIP-event figure, SQ / MFMA counters and HBM bytes per launch, and the
MFMA-i8 roofline fraction recomputed from the trace.

  ops per launch = 512 x sum over the 255 pairs of n_query x n_train    (32 x 32 pairs x K = 256 bits x 2 = 512
                   ops per pair; bench.py `hamming.mfma_i8`, or `mfma_fp4` for the e2m1 form)
  frac           = ops per launch / (leg wall time in the trace: the launch's first kernel start to its last
                   kernel end, expansion and top-2 chunks overlapping on two streams) / the form's dense peak
Counter sections are per dispatch (one chunk); rocprofv3 serialises dispatches while it counts.

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

PEAK_I8_OPS = 5.0e15   # dense int8 MFMA: 2x the bf16 rate (2.5 PF dense), MI355X_MICROARCH.md §Matrix cores
PEAK_FP4_OPS = 10.0e15  # dense fp4 (e2m1) MFMA: 4x the bf16 rate (ORBGPU_TOP2 'f')
KERNELS = ("k_expand_pm1", "k_expand_fp4", "k_top2_mfma", "k_top2b_merge")


def kname(s):
    for k in KERNELS:
        if re.search(r"\b" + k + r"\b", s) or (k + "<") in s or (k + "(") in s:
            return k
    return None


def trace(d):
    fn = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    dur = defaultdict(list)
    spans = []
    for row in csv.DictReader(open(fn[0])):
        k = kname(row["Kernel_Name"])
        if k:
            t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            dur[k].append((t1 - t0) / 1e3)
            spans.append((t0, t1))
    return dur, fn[0], sorted(spans)


def leg_spans(spans, legs):
    """Wall time (us) of each Hamming leg launch: its kernels (expansion chunks on the side stream, top-2 chunks
    on the launch stream, which overlap) from the first start to the last end."""
    per = len(spans) // legs
    return [(max(e for _, e in spans[i * per:(i + 1) * per]) - spans[i * per][0]) / 1e3 for i in range(legs)]


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
    mkey = "mfma_fp4" if "mfma_fp4" in ham else "mfma_i8"
    peak = PEAK_FP4_OPS if mkey == "mfma_fp4" else PEAK_I8_OPS
    ops = ham[mkey]["achieved_ops_per_s"] * ham["kernel_avg_us"] * 1e-6   # 512 x evals per launch
    dur, tfile, spans = trace(os.path.join(root, "trace"))
    legs = int(os.environ.get("HAM_LEGS", "21"))   # bench.py's Hamming leg: one warm launch + max(2, steps) timed
    ls = leg_spans(spans, legs)[1:]                # the warm launch dropped
    t_launch = sum(ls) / len(ls)
    mean = {k: sum(v) / len(v) for k, v in dur.items()}
    out = {"bench_line_hamming": ham, "ops_per_launch": ops, "trace_file": os.path.relpath(tfile, root),
           "trace_dispatches": {k: len(v) for k, v in dur.items()},
           "trace_mean_us_per_dispatch": {k: round(v, 3) for k, v in mean.items()},
           "trace_leg_us": round(t_launch, 3),
           "trace_leg_note": "per launch of orb_hamming_top2_frames_device: first kernel start to last kernel end "
                             "(expansion chunks on the second stream overlap the top-2 chunks)",
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
