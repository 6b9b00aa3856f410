#!/usr/bin/env python3
"""Static instruction count of k_fast_wave<48> per phase, from the disassembly (CPU, no GPU).

Builds extract_kernels.hip to assembly with -DORBGPU_ISA_MARKS=1 (the kernel's phase stamps become assembly comments:
no instruction, only a scheduling boundary), then counts the instructions between the marks by class.  Phases (the
ORBGPU_STAMP numbers): 0 -> 6 ROI store (widening into the 16-bit tile); 1 -> 2 prefilter + survivor compaction;
2 -> 3 exact arc strength of the survivors; 3 -> 4 NMS + emission + the minThFAST pass's reset; 4 -> 5 the count
store; before 0: cell setup and the next cell's ROI loads.  Static counts are per code copy (the kernel unrolls its
two cells per wave, so most phases appear twice); the dynamic count per cell is the PMC's (SQ_INSTS_VALU per launch
/ cells), which weights each phase by its trip count (prefilter row rounds, survivor chunks, the minThFAST pass)."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "orb-slam-birdview_amd")


def main():
    flags = subprocess.run(["make", "-s", "-C", PKG, "--no-print-directory", "print-flags-extract_kernels"],
                           capture_output=True, text=True, check=True).stdout.split()
    out = "/tmp/orbgpu_fast_marks.s"
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-DORBGPU_ISA_MARKS=1", "--cuda-device-only", "-S",
                    os.path.join(PKG, "csrc", "extract_kernels.hip"), "-o", out], check=True, capture_output=True)
    txt = open(out).read()
    name = next(m.group(1) for m in re.finditer(r"^(_ZN6orbgpu11k_fast_waveILi48E\S*):", txt, re.M))
    body = txt[txt.index(name + ":"):txt.index(".Lfunc_end", txt.index(name + ":"))]
    seg = "setup"
    counts = collections.defaultdict(collections.Counter)
    order = []
    for line in body.split("\n"):
        m = re.search(r";ORBGPU_MARK (\d+)", line)
        if m:
            seg = {"0": "ROI store", "6": "after ROI store", "1": "cell body start", "2": "arc strength",
                   "3": "NMS + emit + minTh reset", "4": "count store", "5": "tail"}[m.group(1)]
            seg = {"cell body start": "prefilter + compaction"}.get(seg, seg)
            if seg not in order:
                order.append(seg)
            continue
        t = line.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":") or not line.startswith("\t"):
            continue
        op = t.split()[0]
        cls = ("VALU" if op.startswith("v_") else "SALU" if op.startswith("s_") and not op.startswith(("s_waitcnt", "s_load", "s_buffer"))
               else "LDS" if op.startswith("ds_") else "VMEM" if op.startswith(("buffer_", "global_", "flat_")) else
               "SMEM" if op.startswith(("s_load", "s_buffer")) else "wait" if op.startswith("s_waitcnt") else "other")
        counts[seg][cls] += 1
    if "setup" not in order:
        order.insert(0, "setup")
    print(f"{'phase':28s} {'VALU':>6s} {'SALU':>6s} {'LDS':>5s} {'VMEM':>5s} {'SMEM':>5s} {'wait':>5s}")
    tot = collections.Counter()
    for sname in order:
        c = counts[sname]
        tot.update(c)
        print(f"{sname:28s} {c['VALU']:6d} {c['SALU']:6d} {c['LDS']:5d} {c['VMEM']:5d} {c['SMEM']:5d} {c['wait']:5d}")
    print(f"{'total':28s} {tot['VALU']:6d} {tot['SALU']:6d} {tot['LDS']:5d} {tot['VMEM']:5d} {tot['SMEM']:5d} {tot['wait']:5d}")


if __name__ == "__main__":
    sys.exit(main())
