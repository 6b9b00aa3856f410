#!/usr/bin/env python3
"""Copy the summaries of a tools/gpu_round.sh run from gpurun_out/ into profiles/ (tracked).

Usage: python3 tools/collect_profiles.py <tag>   e.g. r01_v3
Writes profiles/<tag>_bench.json, <tag>_kernel_stats.csv, <tag>_pytest_gpu.log, <tag>_pmc.json and
refreshes profiles/pmc_traffic.json (read by bench.py for roofline.traffic / roofline.valu), stamped
with the git commit the measured code came from.
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def main():
    tag = sys.argv[1]
    commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                            text=True).stdout.strip()
    dirty = subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--", "orb-slam-birdview_amd", "include"],
                           capture_output=True, text=True).stdout.strip()
    if dirty:
        commit += "+dirty"
    lines = [l for l in open(os.path.join(OUT, "bench.log")).read().splitlines() if l.startswith("{")]
    with open(os.path.join(PROF, f"{tag}_bench.json"), "w") as f:
        f.write(lines[-1] + "\n")
    shutil.copy(os.path.join(OUT, "prof", "run_kernel_stats.csv"), os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    shutil.copy(os.path.join(OUT, "pytest_gpu.log"), os.path.join(PROF, f"{tag}_pytest_gpu.log"))
    rep = os.path.join(OUT, "pmc", "report.json")
    if os.path.exists(rep):
        d = json.load(open(rep))
        d["commit"] = commit
        d["batch_frames_per_launch"] = json.loads(lines[-1])["config"]["batch_per_gpu"]
        d["config"] = "C3 1280x720, 2000 features, bench.py --steps 3 --warmup 1 --no-cpu"
        d["method"] = ("tools/pmc.sh: rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | SQ_* --kernel-trace (separate "
                       "passes); tools/pmc_calib.hip known-byte streams give the per-width factor")
        for name in (f"{tag}_pmc.json", "pmc_traffic.json"):
            with open(os.path.join(PROF, name), "w") as f:
                json.dump(d, f, indent=1)
    print("collected", tag, "commit", commit)


if __name__ == "__main__":
    main()
