#!/usr/bin/env python3
"""Turn tools/pmc.sh's rocprofv3 counter CSVs into HBM bytes per launch (profiles/pmc_traffic.json).

FETCH_SIZE / WRITE_SIZE are in KiB (MI355X_MICROARCH.md / cdna_hip_programming.md:
hbm_bytes = (FETCH_SIZE + WRITE_SIZE) * 1024).  On gfx950 FETCH_SIZE under-reports wide streaming
reads by 2x and other widths are uncalibrated, so tools/pmc_calib.hip streams known byte counts
with 1-, 4- and 16-byte lanes; the correction factor of each width is known_bytes / counter_bytes.
liborbgpu's kernels read with 4-byte lanes (k_fast ROI staging, k_resize dword stores, k_describe
window loads) plus byte gathers (k_resize taps), so the report gives the raw counter bytes and the
value corrected with the dword-width factor ("corrected").

Usage: python3 tools/pmc_report.py gpurun_out/pmc > report.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

SHORT = {"k_fast": "fast", "k_fast_wave": "fast", "k_resize": "resize", "k_resize_tiled": "resize",
         "k_octree": "octree", "k_describe": "describe", "k_top2_mfma": "hamming", "k_top2b_merge": "hamming_merge",
         "k_stereo": "stereo", "k_stereo_cut": "stereo_cut", "k_calib_read_u8": "calib_read_u8",
         "k_calib_read_u32": "calib_read_u32", "k_calib_read_u128": "calib_read_u128",
         "k_calib_write_u32": "calib_write_u32"}


def short_name(kname):
    m = re.search(r"(k_[A-Za-z0-9_]+)\s*\(", kname) or re.search(r"(k_[A-Za-z0-9_]+)", kname)
    return SHORT.get(m.group(1), m.group(1)) if m else None


def load(dirpath, counter):
    """{kernel: [value per dispatch]} for one counter from a rocprofv3 csv output directory."""
    per = defaultdict(lambda: defaultdict(float))   # kernel -> dispatch -> value
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection*.csv"), recursive=True)
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                k = short_name(row.get("Kernel_Name", ""))
                if k is None:
                    continue
                did = row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(per[k]))
                per[k][did] += float(row["Counter_Value"])
    return {k: list(v.values()) for k, v in per.items()}, files


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    calib_read = 512 << 20
    calib_write = 256 << 20
    out = {"unit_note": "counters in KiB -> bytes x1024; per launch = mean over dispatches",
           # the bench configuration the passes ran (tools/pmc.sh: C3 unless BENCH_ARGS names another); bench.py
           # attaches the figures only to a line of the same configuration
           "workload": os.environ.get("PMC_WORKLOAD", "c3"),
           "calibration": {}, "raw_bytes_per_launch": {}, "per_launch_bytes": {}}
    fr, ffiles = load(os.path.join(root, "calib_FETCH_SIZE"), "FETCH_SIZE")
    wr, wfiles = load(os.path.join(root, "calib_WRITE_SIZE"), "WRITE_SIZE")
    if not ffiles or not wfiles:
        out["error"] = "no counter_collection csv found under " + root
        print(json.dumps(out, indent=1))
        return
    factors = {}
    for width in ("u8", "u32", "u128"):
        v = fr.get("calib_read_" + width)
        if v:
            got = sum(v) / len(v) * 1024
            factors["read_" + width] = calib_read / got if got else None
            out["calibration"]["read_" + width] = {"known_bytes": calib_read, "counter_bytes": got,
                                                   "factor": factors["read_" + width]}
    v = wr.get("calib_write_u32")
    if v:
        got = sum(v) / len(v) * 1024
        factors["write_u32"] = calib_write / got if got else None
        out["calibration"]["write_u32"] = {"known_bytes": calib_write, "counter_bytes": got,
                                           "factor": factors["write_u32"]}
    bf, _ = load(os.path.join(root, "bench_FETCH_SIZE"), "FETCH_SIZE")
    bw, _ = load(os.path.join(root, "bench_WRITE_SIZE"), "WRITE_SIZE")
    rf = factors.get("read_u32") or 1.0
    wf = factors.get("write_u32") or 1.0
    for k in sorted(set(bf) | set(bw)):
        if k.startswith("calib"):
            continue
        fb = sum(bf.get(k, [0])) / max(1, len(bf.get(k, []))) * 1024
        wb = sum(bw.get(k, [0])) / max(1, len(bw.get(k, []))) * 1024
        out["raw_bytes_per_launch"][k] = {"fetch": fb, "write": wb, "dispatches": len(bf.get(k, []))}
        out["per_launch_bytes"][k] = fb * rf + wb * wf
    # SQ issue counters per launch (VALU roofline; SQ_*_CYCLES are quad-cycles)
    out["sq_per_launch"] = {}
    for fn in glob.glob(os.path.join(root, "bench_SQ", "**", "*counter_collection*.csv"), recursive=True):
        acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
        with open(fn) as f:
            for row in csv.DictReader(f):
                k = short_name(row.get("Kernel_Name", ""))
                if k is None:
                    continue
                acc[k][row["Counter_Name"]][row.get("Dispatch_Id", "0")] += float(row["Counter_Value"])
        for k, cs in acc.items():
            out["sq_per_launch"][k] = {c: sum(d.values()) / len(d) for c, d in cs.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
