#!/usr/bin/env python3
"""Copy the summaries of a tools/gpu_round.sh run from gpurun_out/ into profiles/<round>/ (tracked).

Usage: python3 tools/collect_profiles.py r02 v1
Writes profiles/r02/v1_<bench|bench_c2|bench_c5>.json (the JSON lines), v1_kernel_stats.csv (rocprofv3
--kernel-trace --stats of the timed loop, two batches in flight), v1_kernel_stats_serial.csv (the same
loop one batch at a time: the per-launch durations the bench's roofline pass measures), v1_pytest_gpu.txt
and, when PMC passes ran, v1_pmc.json, refreshing profiles/pmc_traffic.json (read by bench.py for
roofline.traffic / roofline.valu), stamped with the git commit the measured code came from.
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def main():
    rnd, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(prof, exist_ok=True)
    commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                            text=True).stdout.strip()
    dirty = subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--", "orb-slam-birdview_amd", "include"],
                           capture_output=True, text=True).stdout.strip()
    if dirty:
        commit += "+dirty"
    main_line = None
    for name in ("bench", "bench_driver_form", "bench_c2", "bench_c5", "bench_c5b1"):
        p = os.path.join(OUT, name + ".log")
        if not os.path.exists(p):
            continue
        lines = [l for l in open(p).read().splitlines() if l.startswith("{")]
        if lines:
            with open(os.path.join(prof, f"{tag}_{name}.json"), "w") as f:
                f.write(lines[-1] + "\n")
            if name == "bench":
                main_line = json.loads(lines[-1])
    for src, dst in (("prof", "kernel_stats.csv"), ("prof_serial", "kernel_stats_serial.csv")):
        p = os.path.join(OUT, src, "run_kernel_stats.csv")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(prof, f"{tag}_{dst}"))
    if os.path.exists(os.path.join(OUT, "pytest_gpu.log")):
        shutil.copy(os.path.join(OUT, "pytest_gpu.log"), os.path.join(prof, f"{tag}_pytest_gpu.txt"))
    rep = os.path.join(OUT, "pmc", "report.json")
    if os.path.exists(rep) and main_line:
        d = json.load(open(rep))
        d["commit"] = commit
        d["batch_frames_per_launch"] = main_line["config"]["batch_per_gpu"]
        d["config"] = "C3 1280x720, 2000 features, bench.py --steps 3 --warmup 1 --only-extract --no-profile-pass"
        d["method"] = ("tools/pmc.sh: rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | SQ_* --kernel-trace (separate "
                       "passes); tools/pmc_calib.hip known-byte streams give the per-width factor")
        for path in (os.path.join(prof, f"{tag}_pmc.json"), os.path.join(ROOT, "profiles", "pmc_traffic.json")):
            with open(path, "w") as f:
                json.dump(d, f, indent=1)
    # roofline.frac reproduced from the committed serial trace: the dominant kernel's mean duration over
    # the timed launches only (the trace also holds the warm-up launches, whose clocks are still ramping)
    tr = os.path.join(OUT, "prof_serial", "run_kernel_trace.csv")
    if os.path.exists(tr) and main_line and main_line.get("roofline"):
        import csv
        rl = main_line["roofline"]
        kname = {"fast": "k_fast_wave", "describe": "k_describe", "resize": "k_resize", "octree": "k_octree"}[rl["kernel"]]
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                for r in sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
                if kname in r["Kernel_Name"]]
        warm = int(os.environ.get("SERIAL_WARMUP", "20"))
        timed = durs[warm:] if len(durs) > warm else durs
        mean_us = sum(timed) / len(timed) / 1e3
        ach = rl["algorithmic_bytes_per_launch"] / (mean_us * 1e-6) / 1e9
        chk = {"kernel": kname, "trace": f"{tag}_kernel_stats_serial.csv / run_kernel_trace.csv (prof_serial)",
               "launches": len(durs), "warmup_launches_dropped": len(durs) - len(timed),
               "mean_us_timed": round(mean_us, 2), "mean_us_all": round(sum(durs) / len(durs) / 1e3, 2),
               "algorithmic_bytes_per_launch": rl["algorithmic_bytes_per_launch"],
               "achieved_GBs_from_trace": round(ach, 1), "frac_from_trace": round(ach / rl["peak"], 4),
               "bench_line": {"kernel_avg_launch_us": rl["kernel_avg_launch_us"], "frac": rl["frac"]}}
        with open(os.path.join(prof, f"{tag}_roofline_check.json"), "w") as f:
            json.dump(chk, f, indent=1)
        shutil.copy(tr, os.path.join(prof, f"{tag}_kernel_trace_serial.csv"))
    print("collected", rnd, tag, "commit", commit)


if __name__ == "__main__":
    main()
