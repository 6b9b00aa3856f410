"""Python simulation of the GPU's table-in-list-order DistributeOctTree (k_octree), checked against
the oracle's std::list restatement.  Design validation only (CPU)."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from orbgpu.synth import synth_frame  # noqa: E402


def f32(x):
    return float(np.float32(x))


def quadrant(x, y, r):
    x0, x1, y0, y1 = r
    hx, hy = (x1 - x0 + 1) >> 1, (y1 - y0 + 1) >> 1
    return (1 if x >= x0 + hx else 0) | (2 if y >= y0 + hy else 0)


def child(r, q):
    x0, x1, y0, y1 = r
    hx, hy = (x1 - x0 + 1) >> 1, (y1 - y0 + 1) >> 1
    xm, ym = x0 + hx, y0 + hy
    return ((xm if q & 1 else x0), (x1 if q & 1 else xm), (ym if q & 2 else y0), (y1 if q & 2 else ym))


def octree(cands, W, H, N):
    nIni = int(round(f32(np.float32(W) / np.float32(H))))
    hX = np.float32(np.float32(W) / np.float32(nIni))
    rects = [(int(np.float32(hX * np.float32(t))), int(np.float32(hX * np.float32(t + 1))), 0, H) for t in range(nIni)]
    knode = [min(int(np.float32(np.float32(x) / hX)), nIni - 1) for x, y, s in cands]
    cnt = [0] * nIni
    for t in knode:
        cnt[t] += 1
    remap, table = {}, []
    for t in range(nIni):
        if cnt[t] > 0:
            remap[t] = len(table)
            table.append([rects[t], cnt[t], -1 - t])
    knode = [remap[t] for t in knode]
    S = len(table)
    nextSeq = 0
    phase = 1
    while True:
        prev = S
        quad = [[0] * 4 for _ in range(S)]
        for i, (x, y, s) in enumerate(cands):
            t = knode[i]
            if table[t][1] > 1:
                quad[t][quadrant(x, y, table[t][0])] += 1
        if phase == 1:
            order = [t for t in range(S) if table[t][1] > 1]
        else:
            srt = sorted([t for t in range(S) if table[t][1] > 1], key=lambda t: (table[t][1], table[t][2]),
                         reverse=True)
            order = []
            size = S
            for t in srt:
                order.append(t)
                size += sum(1 for q in range(4) if quad[t][q] > 0) - 1
                if size >= N:
                    break
        rank = {t: r for r, t in enumerate(order)}
        nch = [sum(1 for q in range(4) if quad[t][q] > 0) for t in order]
        P = np.concatenate([[0], np.cumsum(nch)]).astype(int) if order else np.array([0])
        CH = int(P[-1]) if order else 0
        new = [None] * (CH + S - len(order))
        info = {}
        pos = CH
        for t in range(S):
            if t not in rank:
                new[pos] = table[t]
                info[t] = pos
                pos += 1
        big = 0
        for r, t in enumerate(order):
            mask = sum((1 << q) for q in range(4) if quad[t][q] > 0)
            start = CH - P[r] - nch[r]
            for q in range(4):
                if mask & (1 << q):
                    p = start + bin(mask >> (q + 1)).count("1")
                    new[p] = [child(table[t][0], q), quad[t][q], nextSeq + P[r] + bin(mask & ((1 << q) - 1)).count("1")]
                    big += quad[t][q] > 1
            info[t] = (start, mask)
        for i, (x, y, s) in enumerate(cands):
            t = knode[i]
            if t in rank:
                start, mask = info[t]
                q = quadrant(x, y, table[t][0])
                knode[i] = start + bin(mask >> (q + 1)).count("1")
            else:
                knode[i] = info[t]
        nextSeq += CH
        table = new
        S = len(table)
        if S >= N or S == prev:
            break
        if phase == 1 and S + big * 3 > N:
            phase = 2
    best = [None] * S
    for i, (x, y, s) in enumerate(cands):
        t = knode[i]
        if best[t] is None or s > cands[best[t]][2]:
            best[t] = i
    return [cands[best[t]] for t in range(S)]


def check(w, h, nfeat, idx, kind="scene"):
    img = synth_frame(w, h, idx, kind)
    o = oracle.OracleExtractor(nfeat)
    o.run(img)
    tabs = o.tables()
    ok = True
    for l in range(8):
        lv = o.level(l)
        W = lv.shape[1] - 19 + 3 - 16
        H = lv.shape[0] - 19 + 3 - 16
        c = [tuple(map(int, r)) for r in o.candidates(l)]
        res = octree(c, W, H, int(tabs["n_per_level"][l]))
        ref = o.level_keypoints(l)
        refl = [(int(k["x"]) - 16, int(k["y"]) - 16, int(k["response"])) for k in ref]
        if res != refl:
            ok = False
            print(f"level {l}: MISMATCH sim {len(res)} oracle {len(refl)}")
    print(w, h, nfeat, idx, kind, "OK" if ok else "FAIL")
    return ok


if __name__ == "__main__":
    allok = True
    for args in [(320, 240, 500, 0), (640, 480, 1000, 0), (640, 480, 1000, 1), (1280, 720, 2000, 0),
                 (640, 480, 1000, 3, "noise"), (1280, 720, 4000, 5), (640, 480, 100, 2), (640, 480, 5000, 7)]:
        allok &= check(*args)
    print("ALL OK" if allok else "FAIL")
