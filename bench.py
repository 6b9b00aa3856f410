#!/usr/bin/env python3
"""ORB front-end throughput on MI355X — BASELINE.json metric:
"ORB features/sec per GPU (1280x720, 2000 kp, 8 levels) + Hamming matches/sec".

One step = one batched pass of the extraction hot path (pyramid -> per-cell FAST+NMS ->
DistributeOctTree -> IC angle + Gaussian + rBRIEF) over `--batch` synthetic frames already resident in
HBM, on each GPU.  Frames shard across GPUs (one process per GPU, no data-path collective); value =
keypoints produced by all ranks / max-over-ranks time of the K timed steps.

Configs (BASELINE.json):
  c3 (default)  1280x720, 2000 features, B = 256 frames per GPU per step, weak scaling
  c2            640x480, 1000 features, B = 256 per GPU, weak scaling
  c5            BASELINE config 5: ONE 8-frame batch of 1280x720 @ 4000 features per step, sharded over the
                N GPUs (8/N frames each), strong scaling
  c4 is a leg of every run (`c4_frame`): left / right / bird 1280x720 streams, each on its own GPU when
  the process sees >= 3 devices (stereo pyramid + descriptors moved over xGMI), else all on one.

Multi-GPU: `python bench.py --gpus N` spawns N ranks itself (before any GPU call) when WORLD_SIZE is
unset; under torch.distributed.run the ranks come from the environment and must number --gpus.

Also on the same line:
  roofline      dominant kernel's algorithmic bytes per launch / its HIP-event-timed duration (events on
                liborbgpu's own stream, a separate pass of the same steps); PMC traffic from profiles/
  cpu_baseline  the oracle restatement of ORBextractor (oracle/, kind "port") rebuilt -march=native on
                the box, rank 0 at N=1 only: single thread (5 warm-up + 50 timed frames, median, per-stage
                times) and frame-parallel on every CPU this process may use
  hamming       all-pairs top-2 Hamming between consecutive frames' descriptors on the matrix cores (the
                brute-force SearchByBoW inner loop), matches/s = distance evaluations per second, its FP4
                MFMA fraction, and the restated CPU loops beside it

Usage: python bench.py [--gpus N --steps K --warmup W --batch B --config c3|c2|c5 --no-cpu --only-extract]
"""
import argparse
import json
import os
import platform
import resource
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))

METRIC = "ORB features/sec per GPU (1280×720, 2000 kp, 8 levels) + Hamming matches/sec"
CONFIGS = {   # BASELINE.json configs; C3 is the headline single-GPU workload
    "c2": dict(w=640, h=480, nfeatures=1000, batch=256, scaling="weak",
               name="C2 640x480 synthetic, 1000 features, 8 levels"),
    "c3": dict(w=1280, h=720, nfeatures=2000, batch=256, scaling="weak",
               name="C3 1280x720 KITTI-style synthetic, 2000 features, 8 levels"),
    # C5's 8-frame step (1 frame per GPU at N = 8) is latency-bound: four batches in flight, one per
    # hardware queue (GPU_MAX_HW_QUEUES = 4), measured 370 vs 290 M features/s at B = 8 and 131 vs 78 at
    # B = 1 against two; C2 / C3 batches of 256 peak at two
    "c5": dict(w=1280, h=720, nfeatures=4000, global_batch=8, scaling="strong", pipelines=4,
               name="C5 8-frame batch of 1280x720 synthetic, 4000 features each, sharded over the GPUs"),
}
PEAK_HBM_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec
PEAK_FP4_OPS = 10.0e15           # MI355X_MICROARCH.md: FP4 (e2m1) MFMA = 4x the dense BF16 rate per clock
MIN_WARMUP_S = 0.3                # extraction warm-up floor (seconds of steps) before the timed loop
KNAMES = ["resize", "fast", "octree", "describe", "hamming", "stereo", "flow"]   # ORB_K_* order


# ---------------------------------------------------------------- distributed plumbing
def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def dist_init(world):
    if world <= 1:
        return None
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo")   # timing reductions only: the data path has no collective
    return dist


def barrier(dist):
    if dist is not None:
        dist.barrier()


def reduce_max_sum(dist, tmax, vsum):
    """Max of tmax and sum of vsum over ranks."""
    if dist is None:
        return tmax, vsum
    import torch
    t = torch.tensor([tmax], dtype=torch.float64)
    v = torch.tensor([vsum], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(v, op=dist.ReduceOp.SUM)
    return float(t.item()), float(v.item())


def gather(dist, obj):
    if dist is None:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def frame_range(rank, batch):
    """Synthetic frame indices of a rank: each GPU extracts its own distinct frames."""
    return rank * batch, batch


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn(nranks, argv):
    """`--gpus N` without a launcher: start N rank processes of this script (one per GPU, env rendezvous on
    127.0.0.1) before this process touches the GPU, and exit with the first failing rank's status."""
    port = free_port()
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks), LOCAL_WORLD_SIZE=str(nranks),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        rc = rc or c
    return rc


# ---------------------------------------------------------------- algorithmic bytes
def level_sizes(w, h, nl=8, sf=1.2):
    import numpy as np
    s = [np.float32(1.0)]
    for _ in range(1, nl):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(sf))))
    return [(int(np.rint(np.float32(w) * (np.float32(1) / x))), int(np.rint(np.float32(h) * (np.float32(1) / x))))
            for x in s]


def fast_cells(w, h):
    """FAST cells per frame: the reference's grid per level, nCols x nRows with nCols = (w_l - 32) / 30
    (ORBextractor.cc:773-787: minBorder 16, W = 30)."""
    return sum(((a - 32) // 30) * ((b - 32) // 30) for a, b in level_sizes(w, h))


def algorithmic_bytes(w, h, kps_per_frame, cands_per_frame):
    """Per-frame compulsory bytes by kernel."""
    lv = level_sizes(w, h)
    P = [a * b for a, b in lv]
    Ptot = sum(P)
    K = kps_per_frame
    C = cands_per_frame
    return {
        "resize": sum(P[:-1]) + sum(P[1:]),          # read level l-1, write level l
        "fast": Ptot + 4 * C,                         # read every level once, write packed candidates
        "octree": 4 * C + 4 * K,                      # read candidates, write survivors
        "describe": K * (43 * 43 + 28 + 32),          # 43x43 window per keypoint, KeyPoint + descriptor out
        "pipeline": 3 * Ptot + 1321 * K,              # SURVEY §8d B_extract = 3P + 1321K
        "flow": 3 * Ptot + 1321 * K,                  # the dataflow launch (small batches) runs the whole pipeline
    }


PEAK_VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9   # 256 CUs x 4 SIMD-32 x 2.4 GHz (MI355X_MICROARCH.md)
# Measured VALU issue ceiling of the integer VOP3 / VOP3P class these kernels are made of (v_perm,
# v_alignbyte, v_pk_*_u16, v_min3/max3, v_dot4/dot2, v_mul_u32_u24, v_max_i32): 4.33 cycles per wave64
# instruction per SIMD at the 2.4 GHz nominal clock, 8 waves per SIMD (tools/valu_rate.hip,
# profiles/r02/valu_rate.txt); v_add_u32 / v_add_f32 / v_fma_f32 issue at 2.5.
VALU_INT_CYCLES = 4.33
VALU_INT_CEIL = 256 * 4 * 2.4e9 / VALU_INT_CYCLES   # wave64 instructions per second, whole chip


def read_pmc(kernel, batch, workload):
    """(HBM bytes per launch, VALU instructions per launch, source) of `kernel` from the rocprofv3 PMC
    summary (tools/pmc.sh -> profiles/pmc_traffic.json), scaled to `batch` frames per launch, or Nones
    when the summary was collected on another configuration (its "workload", C3 when absent)."""
    path = os.environ.get("ORBGPU_PMC_JSON") or os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except Exception:
        return None, None, None
    if d.get("workload", "c3") != workload:
        return None, None, None
    k = batch / float(d.get("batch_frames_per_launch", batch) or batch)
    sq = d.get("sq_per_launch", {}).get(kernel, {})
    tb, vi = d.get("per_launch_bytes", {}).get(kernel), sq.get("SQ_INSTS_VALU")
    return (tb * k if tb is not None else None), (vi * k if vi is not None else None), d.get("commit", "this session")


# ---------------------------------------------------------------- CPU baseline (oracle, rank 0, N=1)
def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def cpu_budget():
    """CPUs this process may run on: its affinity mask, capped by a cgroup CPU quota if one is set
    (os.cpu_count() shows the whole host on the GPU box)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        pass
    return (min(aff, quota) if quota else aff), aff, quota


_ORACLE = None


def oracle_native():
    """The oracle rebuilt -march=native on this host (the reference's own flag, CMakeLists.txt:10-11), in a
    temporary directory; falls back to the in-tree x86-64-v3 build if the compile fails."""
    global _ORACLE
    if _ORACLE is not None:
        return _ORACLE
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle   # test infrastructure: used ONLY as the timed CPU baseline here
    import tempfile
    out = os.path.join(tempfile.gettempdir(), f"orbgpu_oracle_native_{os.getpid()}", "liborb_oracle.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    try:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "MARCH=native", f"OUT={out}"], check=True,
                       timeout=300, capture_output=True)
        oracle.use_library(out)
        oracle.BUILD = "-O3 -march=native -ffp-contract=off (built on this host)"
    except Exception as e:   # keep the baseline, say which build it is
        oracle.BUILD = f"-O3 -march=x86-64-v3 (in-tree; native rebuild failed: {type(e).__name__})"
    oracle.lib()
    _ORACLE = oracle
    return oracle


def cpu_baseline(cfg, frames_np):
    import numpy as np
    oracle = oracle_native()
    cores, aff, quota = cpu_budget()
    nf = cfg["nfeatures"]
    frames = np.ascontiguousarray(frames_np[:16])
    fm, stages, kps1 = oracle.bench_single(frames, nf, warmup=5, timed=50)
    med = float(np.median(fm))
    single = kps1 / 50 / (med / 1e3)
    total = max(16 * cores, 256)
    secs, kpsN = oracle.bench_parallel(frames, nf, cores, 1, total)
    allcore = kpsN / secs
    out = {"value": round(allcore, 1), "unit": "features/s", "cores": cores, "kind": "port",
           "frames_per_s": round(total / secs, 2),
           "single_thread_value": round(single, 1), "single_thread_median_ms_per_frame": round(med, 3),
           "single_thread_stage_ms_per_frame": {k: round(v / 50, 3) for k, v in stages.items()},
           "cpu_model": cpu_model(), "affinity_cpus": aff, "cgroup_quota_cpus": quota, "host_cpus": os.cpu_count(),
           "build": oracle.BUILD,
           "sample": f"single thread: 5 warm-up + 50 timed frames (median); frame-parallel: {cores} threads x 1 "
                     f"warm-up frame, then {total} frames ({len(frames)} distinct {cfg['w']}x{cfg['h']}, {nf} "
                     f"features); oracle/orb_oracle.cpp (restated CPU baseline, not OpenCV)"}
    if aff > cores:   # a CPU quota caps this process below the host's CPUs: state the full-host estimate too
        out["host_estimate_value"] = round(allcore / cores * aff, 1)
        out["host_estimate_note"] = f"measured {cores}-thread rate scaled to the {aff} CPUs of the affinity mask"
    return out


def hamming_cpu(ex, B, oracle):
    """Restated DescriptorDistance + SearchByBoW selection (ORBmatcher.cc:159-288, 1647-1663) on the
    same consecutive-frame pairs, single thread and every usable CPU."""
    import numpy as np
    cores, _, _ = cpu_budget()
    npairs = min(8, B - 1)
    counts = ex.counts()[:npairs + 1].astype(np.int32)
    desc = np.zeros((npairs + 1, ex.kp_cap, 32), np.uint8)
    ang = np.zeros((npairs + 1, ex.kp_cap), np.float32)
    for f in range(npairs + 1):
        k, d = ex.results(f)
        desc[f, :len(d)] = d
        ang[f, :len(k)] = k["angle"]
    qf, tf = np.arange(npairs), np.arange(1, npairs + 1)
    res = {}
    for mode, name in ((1, "bruteforce_top2"), (0, "search_by_bow_single_node")):
        s1, ev = oracle.bench_hamming(desc, ang, counts, qf, tf, mode, 1, 1)
        sN, _ = oracle.bench_hamming(desc, ang, counts, qf, tf, mode, cores, max(1, (2 * cores) // npairs))
        itN = max(1, (2 * cores) // npairs)
        res[name] = {"single_thread_matches_per_s": round(ev / s1, 1), "allcore_matches_per_s": round(ev * itN / sN, 1),
                     "cores": cores}
    res["note"] = (f"{npairs} consecutive-frame pairs (~{int(counts.mean())} descriptors each); matches/s = nq*nt "
                   f"distance evaluations per second; SearchByBoW skips already-matched frame features, so its "
                   f"nominal rate is an upper bound of the work it does; {oracle.BUILD}")
    return res


# ---------------------------------------------------------------- C4: three streams, one GPU each
def c4_leg(cfg, frames, first, dist, rank, world, local):
    """Per tracking frame (Frame.cc:124-127, 320-342, 662-836): ORBextractor on the rectified left and right
    images concurrently (the reference's two std::threads), the birdview cv::ORB stream at the same time,
    then ComputeStereoMatches on the left GPU and the bird(t) x bird(t-1) all-pairs Hamming top-2 on the
    bird GPU.  Host images in and results out (the drop-in caller's boundary).  With >= 3 GPUs visible,
    left / right / bird each get a GPU (rank 0 runs the leg while the other ranks wait)."""
    import numpy as np
    import orbgpu
    from orbgpu.synth import bench_frames, synth_bird_mask, synth_stereo_right
    ndev = orbgpu.device_count()
    if world > 1 and rank != 0:
        barrier(dist)
        return None
    devs = (0, 1, 2) if ndev >= 3 else (local, local, local)
    w, h, nf = 1280, 720, 2000   # BASELINE C4: three 1280x720 streams, 2000 features
    if frames.shape[1:] != (h, w) or len(frames) < 17:
        frames = bench_frames(w, h, 17, first=first)
    exl = orbgpu.ORBextractor(nf, 1.2, 8, 20, 7, device=devs[0])
    exr = orbgpu.ORBextractor(nf, 1.2, 8, 20, 7, device=devs[1])
    bo = orbgpu.BirdORB(2000, device=devs[2])
    mt = orbgpu.ORBmatcher(0.7, True, device=devs[2])
    nc4 = min(16, len(frames) - 1)
    lefts = [np.ascontiguousarray(frames[i]) for i in range(nc4 + 1)]
    rights = [synth_stereo_right(lefts[i], first + i) for i in range(nc4 + 1)]
    bmask = synth_bird_mask(w, h, first)
    birds = [np.ascontiguousarray(frames[(i + nc4 // 2) % len(frames)]) for i in range(nc4 + 1)]

    def c4_frame(i, prev_desc):
        out = {}

        def run(key, fn):
            out[key] = fn()
        th = [threading.Thread(target=run, args=("l", lambda: exl(lefts[i]))),
              threading.Thread(target=run, args=("r", lambda: exr(rights[i]))),
              threading.Thread(target=run, args=("b", lambda: bo.extract(birds[i], bmask)))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        (kl, dl), (kr, dr), (kb, db) = out["l"], out["r"], out["b"]
        _u, _d, nst = orbgpu.compute_stereo_matches(exl, exr, kl, dl, kr, dr, 0.54, 0.54 * 721.5)
        nm = 0
        if prev_desc is not None and len(db) and len(prev_desc):
            dist_, _idx, _nv = mt.hamming_topk(db, prev_desc, 2)
            nm = int((dist_[:, 0] <= 50).sum())
        return db, len(kl) + len(kr), nst, len(kb), nm
    prev = None
    for i in range(3):   # warm-up: graph capture, allocations, the host threads' first HIP calls
        prev, _, _, _, _ = c4_frame(i % (nc4 + 1), prev)
    tc0 = time.perf_counter()
    tot = [0, 0, 0, 0]
    per = []
    for i in range(1, nc4 + 1):
        t = time.perf_counter()
        prev, a, b_, c_, d_ = c4_frame(i, prev)
        per.append(time.perf_counter() - t)
        tot = [tot[0] + a, tot[1] + b_, tot[2] + c_, tot[3] + d_]
    tc1 = time.perf_counter()
    for o in (exl, exr, bo):
        o.close()
    if world > 1:
        barrier(dist)
    return {"ms_per_frame": round((tc1 - tc0) / nc4 * 1e3, 3), "frames_per_s": round(nc4 / (tc1 - tc0), 1),
            "ms_per_frame_median": round(float(np.median(per)) * 1e3, 3),
            "devices": {"left": devs[0], "right": devs[1], "bird": devs[2]},
            "stereo_keypoints_per_frame": tot[0] // nc4, "left_with_depth_per_frame": tot[1] // nc4,
            "bird_keypoints_per_frame": tot[2] // nc4, "bird_matches_le_th_low_per_frame": tot[3] // nc4,
            "note": "host images: left + right ORBextractor and the birdview cv::ORB + cornerSubPix concurrently "
                    "(one host thread per stream), then ComputeStereoMatches (right pyramid over xGMI when on "
                    "another GPU) and bird(t) x bird(t-1) Hamming top-2; synchronous per tracking frame"}


# ---------------------------------------------------------------- main
def matcher_leg(img, w, h, nf, device):
    """Per-call latency of SearchByBoW (KF,F) / (KF,KF), SearchForTriangulation, SearchForInitialization
    and Frame::ComputeBoW on two C3 frames (the second shifted by (2, 3) px), FeatureVectors from a
    synthetic ORBvoc-sized vocabulary (k = 10, L = 6, levelsup 4), GPU adapter vs oracle CPU loop."""
    import tempfile
    import numpy as np
    from orbgpu.synth import write_synth_vocab_large
    exe = os.path.join(ROOT, "tools", "matcher_latency")
    if not os.path.exists(exe):
        return {"error": "tools/matcher_latency not built"}
    tmp = tempfile.mkdtemp(prefix="orbgpu_matcher_")
    raw, voc = os.path.join(tmp, "frames.raw"), os.path.join(tmp, "voc.bin")
    try:
        from orbgpu.synth import synth_stereo_right
        a = np.ascontiguousarray(img)
        b = np.ascontiguousarray(np.roll(a, (2, 3), axis=(0, 1)))
        sr = np.ascontiguousarray(synth_stereo_right(a, 0))   # a rectified right view of `a` (ComputeStereoMatches)
        with open(raw, "wb") as f:
            f.write(a.tobytes() + b.tobytes() + a.tobytes() + sr.tobytes())
        write_synth_vocab_large(voc, 10, 6)
        r = subprocess.run([exe, raw, str(w), str(h), str(nf), voc, "50", "10"], capture_output=True, text=True,
                           timeout=300, env=dict(os.environ, ORBGPU_DEVICE=str(device)))
        if r.returncode not in (0, 1) or not r.stdout.strip():
            return {"error": f"rc {r.returncode}: {r.stderr.strip()[-300:]}"}
        out = json.loads(r.stdout.strip().splitlines()[-1])
        out["note"] = ("median us per call, one call per frame / keyframe pair as Tracking.cc:1029-1032, "
                       "LoopClosing.cc:265, LocalMapping.cc:278, Tracking.cc:738-739, Frame.cc:562-569 and Frame.cc:141 make them "
                       "(the _x10 entries: a caller's loop over 10 keyframes as one batched call against 10 runs of the CPU loop -- "
                       "SearchByBoW_KF_F_x10 Tracking.cc:1931-1938, SearchByBoW_KF_KF_x10 LoopClosing.cc:252-265, "
                       "SearchForTriangulation_x10 LocalMapping.cc:247-278); "
                       "GPU = adapter/ORBmatcher_gpu.cc (host inputs, upload + kernels + host replay), CPU = the "
                       "oracle's restatement of each body, single thread, same inputs; outputs compared equal")
        return out
    finally:
        for p in (raw, voc):
            if os.path.exists(p):
                os.unlink(p)
        os.rmdir(tmp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 timed steps after 20 warm-up ones (≈ 0.2 s at C3): 20 steps after 3 read 2-3 % low
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=0, help="frames per step per GPU (default: the config's)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-hamming", action="store_true")
    ap.add_argument("--no-stereo", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--no-bird", action="store_true")
    ap.add_argument("--no-c4", action="store_true")
    ap.add_argument("--no-profile-pass", action="store_true",
                    help="skip the per-kernel HIP-event pass (a rocprofv3 trace then holds only the timed launches)")
    ap.add_argument("--no-matcher", action="store_true", help="skip the per-call ORBmatcher / ComputeBoW leg")
    ap.add_argument("--only-extract", action="store_true", help="the extraction steps only (no other leg)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher plumbing only (tests/test_dist_cpu.py): ranks, rendezvous, reductions, the rank-0 "
                         "line; no GPU is touched")
    ap.add_argument("--pipelines", type=int, default=int(os.environ.get("ORBGPU_BENCH_PIPELINES", "0")),
                    help="batches in flight: consecutive steps alternate over this many extractor contexts "
                         "(own stream and buffers each), so one batch's latency-bound phases overlap another's "
                         "(default: the config's, 2 for C2/C3, 4 for C5)")
    args = ap.parse_args()
    if args.pipelines <= 0:
        args.pipelines = CONFIGS[args.config].get("pipelines", 2)
    if args.only_extract:
        args.no_cpu = args.no_hamming = args.no_stereo = args.no_host_path = args.no_bird = args.no_c4 = True
        args.no_matcher = True

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(args.gpus, sys.argv[1:]))   # before anything touches the GPU
    rank, world, local = dist_env()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    dist = dist_init(world)
    if args.dry_run:
        tmax, total = reduce_max_sum(dist, 1.0 + rank, 100.0 * (rank + 1))
        ranks = gather(dist, {"rank": rank, "device": local, "host": socket.gethostname()})
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "value": total / tmax, "ranks": ranks}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    if os.environ.get("ORBGPU_BENCH_ONE_DEVICE") == "1":   # rehearsal of the N-rank path on a 1-GPU box
        local = 0
    import numpy as np
    import orbgpu
    from orbgpu.synth import bench_frames

    cfg = CONFIGS[args.config]
    w, h, nf = cfg["w"], cfg["h"], cfg["nfeatures"]
    if cfg["scaling"] == "strong":   # C5: one global batch sharded over the ranks
        G = cfg["global_batch"]
        if G % world:
            raise SystemExit(f"bench.py: config {args.config} shards {G} frames; --gpus must divide it")
        B = args.batch or G // world
        first = rank * B
    else:
        B = args.batch or cfg["batch"]
        first, _ = frame_range(rank, B)
    frames = bench_frames(w, h, B, first=first)
    ex = orbgpu.BatchExtractor(nf, w, h, B, device=local)
    ex.upload(frames)                         # inputs resident in HBM before timing
    exs = [ex]
    for _ in range(1, max(1, args.pipelines)):
        e2 = orbgpu.BatchExtractor(nf, w, h, B, device=local)
        e2.upload(frames)
        exs.append(e2)

    def sync():
        for e in exs:
            e.sync()

    for _ in range(args.warmup):
        for e in exs:
            e.launch()
    sync()
    # then at least MIN_WARMUP_S of steps in all: a short --warmup left the timed loop 2-3 % below its steady rate
    # (clocks and queues still settling); the line reports both counts
    warm_run, tw0 = args.warmup, time.perf_counter()
    while time.perf_counter() - tw0 < MIN_WARMUP_S:
        for e in exs:
            e.launch()
        sync()
        warm_run += 1
    kps_per_step = int(ex.counts().sum())
    assert all(int(e.counts().sum()) == kps_per_step for e in exs)

    # timed region: graph replays only; step s runs on context s mod pipelines
    barrier(dist)
    sync()
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    for st in range(args.steps):
        exs[st % len(exs)].launch()
    sync()
    t1 = time.perf_counter()
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    # host cores this rank kept busy during the timed steps (host utilisation beside the 1->N curve)
    host_busy = ((ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)) / max(t1 - t0, 1e-9)
    barrier(dist)
    local_time = t1 - t0
    _, host_busy_sum = reduce_max_sum(dist, 0.0, host_busy)
    tmax, total_kps = reduce_max_sum(dist, local_time, float(kps_per_step * args.steps))
    _, total_frames = reduce_max_sum(dist, 0.0, float(B * args.steps))
    ranks = gather(dist, {"rank": rank, "device": local, "host": socket.gethostname(),
                          "frames_per_step": B, "first_frame": first, "keypoints_per_step": kps_per_step,
                          "seconds": round(local_time, 6)})

    # per-kernel breakdown (HIP events on the library's stream) from a separate pass of the same steps
    kms = None
    if not args.no_profile_pass:
        ex.profile(True)
        for _ in range(args.steps):
            ex.launch()
        sync()
        kms, klaunch = ex.profile_read()
        ex.profile(False)

    # ---- Hamming: all-pairs top-2 between consecutive frames' descriptors (device-resident, one
    # launch for all B-1 pairs: orb_hamming_top2_frames_device on the matrix cores)
    ham = None
    if not args.no_hamming and B >= 2:
        counts = ex.counts()
        L = orbgpu._lib.lib()
        pairs = B - 1
        qf, tf = np.arange(pairs, dtype=np.int32), np.arange(1, B, dtype=np.int32)
        dbest = [ex._alloc(pairs * ex.kp_cap * 4) for _ in range(3)]

        def ham_step():
            ex.hamming_top2_frames(qf, tf, *dbest)
        for _ in range(3):   # warm-up: the pair list's upload (re-sent only when it changes), the scratch arena
            ham_step()
        sync()
        hs = max(2, args.steps)
        # timed launches without the profiling markers (each marker creates and records a HIP event on the host)
        barrier(dist)
        th0 = time.perf_counter()
        for _ in range(hs):
            ham_step()
        sync()
        th1 = time.perf_counter()
        # kernel time: HIP events on the library's stream, a separate pass of the same launches
        ex.profile(True)
        for _ in range(hs):
            ham_step()
        sync()
        hms, hl = ex.profile_read()
        ex.profile(False)
        for p in dbest:
            L.orb_device_free(ex.h, p)
        evals_step = float(sum(int(counts[a]) * int(counts[b]) for a, b in zip(qf, tf)))
        evals = evals_step * hs
        htmax, hevals = reduce_max_sum(dist, th1 - th0, evals)
        kt = hms[4] / 1e3 / max(hl[4], 1)
        ham = {"matches_per_s": round(hevals / htmax, 1),
               "queries_per_s": round(hevals / float(np.mean(counts)) / htmax, 1),
               "pair": f"frame f vs f+1 descriptors (~{int(np.mean(counts))} each), {pairs} pairs per launch",
               "us_per_launch_wall": round((th1 - th0) / hs * 1e6, 2),
               "kernel_avg_us": round(kt * 1e6, 2),
               # k_top2_mfma: 512 MFMA ops per distance (a 32 x 32 tile over K = 256 bits x 2 per MAC) on the +-4
               # e2m1 form, against the dense FP4 peak
               "mfma_fp4": ({"achieved_ops_per_s": round(512.0 * evals_step / kt, 1), "peak_ops_per_s": PEAK_FP4_OPS,
                             "frac": round(512.0 * evals_step / kt / PEAK_FP4_OPS, 4)} if kt > 0 else None),
               "kernel_hbm_gbs": round((32.0 * 2 * float(counts.sum()) + 12 * float(counts.sum())) / kt / 1e9, 2)
               if kt > 0 else None}
        if rank == 0 and world == 1 and not args.no_cpu:
            ham["cpu_baseline"] = hamming_cpu(ex, B, oracle_native())

    # ---- roofline of the dominant kernel (per-step algorithmic bytes / per-step kernel time)
    per_frame_kps = kps_per_step / B
    cands_per_frame = 0   # FAST survivors of frame 0 (all levels), from the debug view of the last batch
    for l in range(8):
        n = orbgpu._lib.lib().orb_debug_candidates(ex.h, 0, l, None, 0)
        cands_per_frame += (-n - 1) if n < 0 else n
    ab = algorithmic_bytes(w, h, per_frame_kps, cands_per_frame)
    roofline, ms_per_step_k = None, None
    if kms is not None:
        steps = args.steps
        # (a small batch runs as one dataflow launch, ORB_K_FLOW: then that is the only extraction kernel)
        ms_per_step_k = {KNAMES[i]: kms[i] / steps for i in (0, 1, 2, 3, 6) if klaunch[i] > 0}
        dom = max(ms_per_step_k, key=ms_per_step_k.get)
        dom_bytes = ab[dom] * B
        dom_s = ms_per_step_k[dom] / 1e3
        achieved = dom_bytes / dom_s / 1e9
        launches_per_step = klaunch[KNAMES.index(dom)] / steps
        traffic, valu_insts, pmc_src = read_pmc(dom, B, args.config)
        sum_k_s = sum(ms_per_step_k.values()) / 1e3
        launch_s = dom_s / launches_per_step
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(achieved / PEAK_HBM_GBS, 5),
                    "traffic": (round(traffic) if traffic is not None else None),   # HBM bytes per launch (PMC)
                    "algorithmic_bytes_per_launch": int(ab[dom] * B / launches_per_step),
                    "algorithmic_bytes_per_frame": int(ab[dom]), "launches_per_step": launches_per_step,
                    "kernel_avg_launch_us": round(launch_s * 1e6, 2),
                    # the kernel's real limiter is VALU issue: PMC SQ_INSTS_VALU per launch / launch time, against
                    # the measured issue ceiling of the integer instruction class it is made of
                    "valu": ({"achieved_wave_insts_per_s": round(valu_insts / launch_s, 1),
                              "ceiling_wave_insts_per_s": round(VALU_INT_CEIL, 1),
                              "frac": round(valu_insts / launch_s / VALU_INT_CEIL, 4),
                              "ceiling": "measured: 4.33 cycles per wave64 integer VOP3/VOP3P instruction per SIMD "
                                         "(tools/valu_rate.hip, profiles/r02/valu_rate.txt)",
                              "dual_rate_frac": round(valu_insts * 64 / launch_s / PEAK_VALU_LANE_OPS, 4),
                              "valu_insts_per_launch": valu_insts,
                              "valu_insts_per_cell": (round(valu_insts / (fast_cells(w, h) * B / launches_per_step), 1)
                                                      if dom == "fast" else None),
                              "pmc_source": pmc_src}
                             if valu_insts else None),
                    "pipeline": {"bytes_per_frame": int(ab["pipeline"]),
                                 "achieved": round(ab["pipeline"] * B / sum_k_s / 1e9, 2),
                                 "frac": round(ab["pipeline"] * B / sum_k_s / 1e9 / PEAK_HBM_GBS, 5)}}

    # ---- Frame::ComputeStereoMatches on the GPU (BASELINE C4's stereo leg): a
    # separate batch of rectified synthetic pairs (frames 2p, 2p+1) extracted once, then the stereo
    # kernels timed alone over all pairs per launch (pyramids and keypoints resident in HBM)
    stereo = None
    if not args.no_stereo:
        from orbgpu.synth import synth_stereo_right
        npairs = max(1, B // 4)
        sf = []
        for i in range(npairs):
            left = frames[i % len(frames)]
            sf += [left, synth_stereo_right(left, first + i)]
        sx = orbgpu.BatchExtractor(nf, w, h, 2 * npairs, device=local)
        sx.upload(np.stack(sf))
        sx.launch()
        sx.sync()
        cap = sx.kp_cap
        du, dd, dn = sx._alloc(npairs * cap * 4), sx._alloc(npairs * cap * 4), sx._alloc(npairs * 4)
        mb, mbf = 0.54, 0.54 * 721.5   # KITTI-like baseline (m) and baseline * fx
        sx.stereo(npairs, mb, mbf, du, dd, dn)
        sx.sync()
        sx.profile(True)
        ss = max(2, args.steps)
        barrier(dist)
        ts0 = time.perf_counter()
        for _ in range(ss):
            sx.stereo(npairs, mb, mbf, du, dd, dn)
        sx.sync()
        ts1 = time.perf_counter()
        sms, sl = sx.profile_read()
        sx.profile(False)
        nmatched = np.zeros(npairs, np.int32)
        orbgpu._lib.check(orbgpu._lib.lib().orb_memcpy_d2h(sx.h, nmatched.ctypes.data, dn, nmatched.nbytes))
        stmax, spairs = reduce_max_sum(dist, ts1 - ts0, float(npairs * ss))
        st_k = sms[5] / 1e3 / max(sl[5], 1)
        stereo = {"pairs_per_s": round(spairs / stmax, 1), "pairs_per_launch": npairs,
                  "kernel_avg_us": round(st_k * 1e6, 2),
                  "left_keypoints_with_depth_per_pair": round(float(nmatched.mean()), 1),
                  "note": "stereo kernels only (k_stereo + k_stereo_cut), inputs resident; "
                          "synthetic rectified pairs, disparity 0-64 px per 16-row band"}
        for ptr in (du, dd, dn):
            orbgpu._lib.lib().orb_device_free(sx.h, ptr)
        sx.close()

    # ---- the reference's own boundary: ORBextractor::operator() on a HOST image (orb_extract: H2D
    # of the frame, the same kernels, D2H of keypoints + descriptors, synchronous per frame, one
    # context) — the PCIe-inclusive per-frame rate a drop-in caller sees.  Never the headline value.
    host_path = None
    if not args.no_host_path:
        hx = orbgpu.ORBextractor(nf, 1.2, 8, 20, 7, device=local)
        nh = min(32, len(frames))
        hx(frames[0])
        hx(frames[1 % len(frames)])
        t0h = time.perf_counter()
        nkp = 0
        for i in range(nh):
            k_, d_ = hx(frames[i])
            nkp += len(k_)
        t1h = time.perf_counter()
        py_ms = (t1h - t0h) / nh * 1e3
        hx.close()
        # the same boundary through the C++ mirror (ORB_SLAM2::ORBextractor::operator(), as Frame::ExtractORB
        # calls it), timed in a child process: the drop-in caller's latency without Python overhead
        cpp = None
        exe = os.path.join(ROOT, "tools", "host_latency")
        if os.path.exists(exe):
            import tempfile
            nfr = min(16, len(frames))
            with tempfile.NamedTemporaryFile(suffix=".raw", delete=False) as tf:
                for i in range(nfr):
                    tf.write(np.ascontiguousarray(frames[i]).tobytes())
                raw = tf.name
            try:
                r = subprocess.run([exe, raw, str(w), str(h), str(nfr), str(nf), "200", str(local)],
                                   capture_output=True, text=True, timeout=120)
                if r.returncode == 0:
                    cpp = json.loads(r.stdout.strip().splitlines()[-1])
            finally:
                os.unlink(raw)
        ms = cpp["ms_per_frame_median"] if cpp else py_ms
        host_path = {"frames_per_s": round(1e3 / ms, 1), "features_per_s": round(per_frame_kps * 1e3 / ms, 1),
                     "ms_per_frame": round(ms, 4), "caller": "C++ mirror (tools/host_latency)" if cpp else "python",
                     "cpp": cpp, "python_ms_per_frame": round(py_ms, 4),
                     "note": "ORBextractor::operator() per host frame: pageable upload, direct launches (two-launch "
                             "pyramid), outputs written by the kernels into pinned memory, one frame in flight, "
                             "median of 200"}

    # ---- the ORBmatcher drop-ins per call (SURVEY 8(a) rows a9-a13 at the reference's granularity: one call
    # per frame / keyframe pair) and Frame::ComputeBoW, through the reference-signature adapter, against
    # the oracle's single-thread CPU loops on the same inputs (tools/matcher_latency.cc; rank 0 at N = 1)
    matcher = matcher_c2 = None
    if rank == 0 and world == 1 and not args.no_matcher:
        matcher = matcher_leg(frames[0], w, h, nf, local)
        if (w, h, nf) != (640, 480, 1000):
            # and at the reference's TUM size (C2, Examples/Monocular/TUM1.yaml:30-43), where a call is a few us of CPU
            # work, so the GPU's per-call fixed cost (one upload, the launches, one synchronisation) shows
            matcher_c2 = matcher_leg(bench_frames(640, 480, 1, first=first)[0], 640, 480, 1000, local)

    # ---- birdview stream (BASELINE C4's bird stream): Frame.cc:320-342 fused on one
    # device-resident image + mask per call (orb_bird_extract_device); synchronous per frame (the host
    # selection, libstdc++ nth_element as the reference, sits mid-pipeline)
    bird = None
    if not args.no_bird:
        from orbgpu.synth import synth_bird_mask
        L = orbgpu._lib.lib()
        bimg = np.ascontiguousarray(frames[0])
        bmask = synth_bird_mask(w, h, first)
        di, dm = ex._alloc(w * h), ex._alloc(w * h)
        orbgpu._lib.check(L.orb_memcpy_h2d(ex.h, di, bimg.ctypes.data, w * h))
        orbgpu._lib.check(L.orb_memcpy_h2d(ex.h, dm, bmask.ctypes.data, w * h))
        bo = orbgpu.BirdORB(2000, device=local)
        bo.extract_device(di, w, h, dm)
        nb = max(4, args.steps)
        barrier(dist)
        tb0 = time.perf_counter()
        nbk = 0
        for _ in range(nb):
            kb, _db = bo.extract_device(di, w, h, dm)
            nbk += len(kb)
        tb1 = time.perf_counter()
        btmax, bframes = reduce_max_sum(dist, tb1 - tb0, float(nb))
        bird = {"frames_per_s": round(bframes / btmax, 1), "features_per_s": round(bframes / btmax * nbk / nb, 1),
                "ms_per_frame": round((tb1 - tb0) / nb * 1e3, 3), "keypoints_per_frame": nbk // nb,
                "note": "cv::ORB(2000) masked detect + cornerSubPix + compute (Frame.cc:320-342), image and "
                        "mask resident, keypoints + descriptors downloaded per frame"}
        if rank == 0 and world == 1 and not args.no_cpu:
            oracle = oracle_native()
            ob = oracle.OracleCvORB(2000)
            ob.extract(bimg, bmask)
            tc0 = time.perf_counter()
            for _ in range(3):
                ob.extract(bimg, bmask)
            tc1 = time.perf_counter()
            bird["cpu_single_thread_ms_per_frame"] = round((tc1 - tc0) / 3 * 1e3, 2)
            bird["cpu_kind"] = "port (oracle/cvorb_oracle.inc, scalar restatement of OpenCV 3.2 ORB)"
        bo.close()
        for ptr in (di, dm):
            L.orb_device_free(ex.h, ptr)

    c4 = None
    if not args.no_c4:
        c4 = c4_leg(cfg, frames, first, dist, rank, world, local)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(cfg, frames[:16])

    if rank == 0:
        value = total_kps / tmax
        out = {"metric": METRIC, "value": round(value, 1), "unit": "features/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "warmup_steps_run": warm_run, "ms_per_step": round(tmax / args.steps * 1e3, 4), "higher_is_better": True,
               "scaling": cfg["scaling"], "vs_baseline": None, "dtype": "u8", "data": "synthetic",
               "config": {"workload": cfg["name"], "width": w, "height": h, "nfeatures": nf, "nlevels": 8,
                          "scale_factor": 1.2, "ini_th_fast": 20, "min_th_fast": 7, "batch_per_gpu": B,
                          "global_batch": B * world, "parallelism": f"frame-sharded x{world} (no collective)",
                          "batches_in_flight": len(exs)},
               "ranks": ranks,
               "frames_per_s": round(total_frames / tmax, 1),
               "host_cores_busy": round(host_busy_sum, 3),   # all ranks' processes, timed region
               "keypoints_per_frame": round(per_frame_kps, 1),
               "kernels_ms_per_step": ({k: round(v, 4) for k, v in ms_per_step_k.items()} if ms_per_step_k else None),
               "roofline": roofline, "cpu_baseline": cpu, "hamming": ham, "stereo": stereo,
               "bird": bird, "c4_frame": c4, "host_path": host_path, "matcher": matcher, "matcher_c2": matcher_c2}
        if cpu:
            out["speedup_vs_cpu_allcore"] = round(value / cpu["value"], 2)
            if "host_estimate_value" in cpu:
                out["speedup_vs_cpu_host_estimate"] = round(value / cpu["host_estimate_value"], 2)
        print(json.dumps(out), flush=True)
    for e in exs:
        e.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
