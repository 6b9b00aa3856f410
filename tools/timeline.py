#!/usr/bin/env python3
"""Print one frame's GPU timeline from a rocprofv3 kernel (+ memory-copy) trace CSV directory:
kernel / copy name, start offset, duration and the gap before it (us).
Usage: python3 tools/timeline.py gpurun_out/hp [frame_index_from_end]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ev = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:]))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
ev.sort()
# frames start at a resize launch preceded by a copy: split at copies followed by the first resize
starts = [i for i, e in enumerate(ev) if e[2].startswith("copy") and (i == 0 or not ev[i - 1][2].startswith("copy"))]
i0 = starts[-back] if len(starts) >= back else 0
i1 = starts[-back + 1] if back > 1 else len(ev)
t0 = ev[i0][0]
prev = t0
for s, e, n in ev[i0:i1]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap {(s - prev) / 1e3:6.1f}  {n}")
    prev = e
print(f"total {(ev[i1 - 1][1] - t0) / 1e3:.1f} us")
