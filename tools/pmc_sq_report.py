#!/usr/bin/env python3
"""Per-kernel SQ counter summary (mean per dispatch) from tools/pmc_sq.sh output."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_report import short_name  # noqa: E402
import csv  # noqa: E402
from collections import defaultdict  # noqa: E402


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_sq"
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for fn in glob.glob(os.path.join(root, "**", "*counter_collection*.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                k = short_name(row.get("Kernel_Name", ""))
                if k is None:
                    continue
                acc[k][row["Counter_Name"]][row.get("Dispatch_Id", "0")] += float(row["Counter_Value"])
    out = {k: {c: sum(d.values()) / len(d) for c, d in v.items()} for k, v in acc.items()}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
