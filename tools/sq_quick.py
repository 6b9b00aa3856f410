#!/usr/bin/env python3
"""Per-kernel mean SQ counters per launch from one rocprofv3 --pmc pass (tools/sq_quick.sh)."""
import csv
import glob
import sys
from collections import defaultdict

KERNELS = {"k_fast_wave": "fast", "k_describe": "describe", "k_resize_tiled": "resize", "k_octree": "octree",
           "k_expand_pm1": "expand_pm1", "k_top2_mfma": "top2_mfma", "k_top2b_merge": "top2b_merge"}


def main(d):
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for row in csv.DictReader(open(path)):
        name = next((v for k, v in KERNELS.items() if k in row["Kernel_Name"]), None)
        if not name:
            continue
        acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[name].add(row["Dispatch_Id"])
    for name, c in acc.items():
        n = len(disp[name])
        print(name, "dispatches", n, {k: round(v / n / 1e6, 3) for k, v in sorted(c.items())}, "(M per launch)")


if __name__ == "__main__":
    main(sys.argv[1])
