"""Deterministic synthetic gray frames for parity tests and the bench.

Frame `idx` is seeded with splitmix64(0x5EED0000 + idx):
  * bilinear value-noise background on a 16-px lattice, lattice values U[40, 215];
  * 300 opaque axis-aligned rectangles then 100 filled circles (painter's order),
    intensity U[0, 255];
  * per-pixel integer noise U[-3, 3], clamped to [0, 255].
This gives corners on rectangle vertices plus texture, so most FAST cells pass iniThFAST.
Edge frames: `flat` (constant 128, zero keypoints) and `noise` (pure U[0,255], maximum
candidate count, stresses the octree).  Stereo right frames are the left frame shifted by a
seeded per-row-band disparity in [0, 64].

Counter-based splitmix64: draw k of a stream with seed s is mix64(s + (k+1)*GOLDEN), which is
exactly the k-th output of the sequential splitmix64 generator, vectorised with numpy.
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


class SplitMix64:
    def __init__(self, seed):
        self.seed = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
        self.k = 0

    def draw(self, n):
        with np.errstate(over="ignore"):
            ks = np.arange(self.k + 1, self.k + 1 + n, dtype=np.uint64)
            out = _mix64(self.seed + ks * GOLDEN)
        self.k += n
        return out

    def uniform_int(self, lo, hi, n):
        """n integers uniform in [lo, hi] (inclusive)."""
        span = np.uint64(hi - lo + 1)
        return (self.draw(n) % span).astype(np.int64) + lo


def synth_frame(w, h, idx=0, kind="scene"):
    """Return a (h, w) uint8 frame."""
    rng = SplitMix64(0x5EED0000 + idx)
    if kind == "flat":
        return np.full((h, w), 128, np.uint8)
    if kind == "noise":
        return rng.uniform_int(0, 255, w * h).astype(np.uint8).reshape(h, w)
    if kind != "scene":
        raise ValueError(kind)
    cell = 16
    gw, gh = w // cell + 2, h // cell + 2
    lat = rng.uniform_int(40, 215, gw * gh).reshape(gh, gw).astype(np.int64)
    ys, xs = np.mgrid[0:h, 0:w]
    gx, gy = xs // cell, ys // cell
    fx, fy = xs % cell, ys % cell
    top = lat[gy, gx] * (cell - fx) + lat[gy, gx + 1] * fx
    bot = lat[gy + 1, gx] * (cell - fx) + lat[gy + 1, gx + 1] * fx
    img = (top * (cell - fy) + bot * fy + (cell * cell) // 2) // (cell * cell)
    rect = rng.uniform_int(0, 1 << 30, 300 * 5).reshape(300, 5)
    for x0, y0, rw, rh, val in rect:
        x0 %= w
        y0 %= h
        rw = 4 + rw % max(1, w // 8)
        rh = 4 + rh % max(1, h // 8)
        img[y0:y0 + rh, x0:x0 + rw] = val % 256
    circ = rng.uniform_int(0, 1 << 30, 100 * 4).reshape(100, 4)
    rmax = max(4, min(w, h) // 16)
    for cx, cy, r, val in circ:
        cx %= w
        cy %= h
        r = 3 + r % rmax
        y0, y1 = max(0, cy - r), min(h, cy + r + 1)
        x0, x1 = max(0, cx - r), min(w, cx + r + 1)
        yy, xx = np.mgrid[y0:y1, x0:x1]
        m = (xx - cx) ** 2 + (yy - cy) ** 2 <= r * r
        img[y0:y1, x0:x1][m] = val % 256
    noise = rng.uniform_int(-3, 3, w * h).reshape(h, w)
    return np.clip(img + noise, 0, 255).astype(np.uint8)


def synth_stereo_right(left, idx=0, max_disp=64):
    """Right view: left shifted by a seeded disparity per 16-row band (edge-replicated)."""
    h, w = left.shape
    rng = SplitMix64(0x5EED8000 + idx)
    bands = (h + 15) // 16
    disp = rng.uniform_int(0, max_disp, bands)
    right = np.empty_like(left)
    for b in range(bands):
        d = int(disp[b])
        rows = slice(16 * b, min(h, 16 * b + 16))
        right[rows, :w - d] = left[rows, d:]
        right[rows, w - d:] = left[rows, w - 1:w]
    return right


def synth_bird_mask(w, h, idx=0):
    """Birdview validity mask (0 / 255), like mono_fisheye.cc's ConvertMaskBirdview output: the
    four corners outside the fisheye coverage are zero (quarter ellipses), plus a seeded zero band."""
    rng = SplitMix64(0xB1D00000 + idx)
    yy, xx = np.mgrid[0:h, 0:w]
    m = np.full((h, w), 255, np.uint8)
    rx, ry = w * 0.22, h * 0.22
    for cx, cy in ((0, 0), (w - 1, 0), (0, h - 1), (w - 1, h - 1)):
        m[((xx - cx) / rx) ** 2 + ((yy - cy) / ry) ** 2 < 1.0] = 0
    r = rng.draw(2)
    y0 = int(r[0] % np.uint64(max(h - 8, 1)))
    m[y0:y0 + 2 + int(r[1] % np.uint64(6)), :] = 0
    return m


def synth_batch(w, h, n, first=0, kind="scene"):
    return np.stack([synth_frame(w, h, first + i, kind) for i in range(n)])


def bench_frames(w, h, count, first=0, distinct=64):
    """The bench's batch (bench.py): `distinct` seeded frames first .. first+distinct-1 (the generator
    costs ~0.1 s per 1280x720 frame), then circularly shifted copies by (7k, 13k) px, k = 1, 2, ..., so
    every frame of the batch is a distinct image that is fully processed."""
    base = synth_batch(w, h, min(count, distinct), first=first)
    reps = [base] + [np.roll(base, (7 * k, 13 * k), axis=(1, 2)) for k in range(1, (count + len(base) - 1) // len(base))]
    return np.ascontiguousarray(np.concatenate(reps)[:count])


def write_synth_vocab(path, k=10, L=3, seed=0, scoring=0, weighting=0, stop_frac=0.05):
    """Write a synthetic DBoW2 ORB vocabulary in ORBvoc.bin's binary format
    (TemplatedVocabulary::saveToBinaryFile, TemplatedVocabulary.h:1512-1531): a complete k-ary tree of
    depth L, nodes numbered breadth-first (children of a node consecutive, as DBoW2's k-means build
    numbers them), each child descriptor = its parent's with ~1/4 of the bits flipped, leaf weights
    U(0.1, 3) with `stop_frac` of them 0 (stopped words).  The real ORBvoc.bin is not in the
    container; tests and the bench use this instead.  Returns (nb_nodes, nwords)."""
    import struct
    rng = np.random.default_rng(seed)
    desc = [rng.integers(0, 256, 32, dtype=np.uint8)]   # root (not stored)
    parent = [0]
    level = [0]
    frontier = [0]
    for lv in range(1, L + 1):
        nxt = []
        for p in frontier:
            for _ in range(k):
                flip = rng.random(256) < 0.25
                bits = np.unpackbits(desc[p]) ^ flip.astype(np.uint8)
                desc.append(np.packbits(bits))
                parent.append(p)
                level.append(lv)
                nxt.append(len(desc) - 1)
        frontier = nxt
    nb_nodes = len(desc)
    with open(path, "wb") as f:
        f.write(struct.pack("<6i", nb_nodes, 4 + 32 + 4 + 1, k, L, scoring, weighting))
        nwords = 0
        for i in range(1, nb_nodes):
            leaf = level[i] == L
            w = 0.0
            if leaf:
                nwords += 1
                w = 0.0 if rng.random() < stop_frac else float(rng.uniform(0.1, 3.0))
            f.write(struct.pack("<i", parent[i]) + desc[i].tobytes() + struct.pack("<f", w) + bytes([1 if leaf else 0]))
    return nb_nodes, nwords


def write_synth_vocab_large(path, k=10, L=6, seed=0, stop_frac=0.05):
    """write_synth_vocab's tree and file format, generated level by level with numpy: for the
    ORBvoc.bin-sized k = 10, L = 6 tree (1,111,111 nodes, 10^6 words) the per-node loop would take
    minutes.  Each child = its parent with every bit flipped with probability 1/4 (the AND of two
    random bytes per byte); TF-IDF weighting, L1 scoring (ORBvoc.bin's own).  Returns (nb_nodes, nwords)."""
    import struct
    rng = np.random.default_rng(seed)
    rec = np.dtype([("parent", "<i4"), ("desc", "u1", 32), ("weight", "<f4"), ("leaf", "u1")])
    nb_nodes = 1 + sum(k ** lv for lv in range(1, L + 1))
    nwords = k ** L
    with open(path, "wb") as f:
        f.write(struct.pack("<6i", nb_nodes, 4 + 32 + 4 + 1, k, L, 0, 0))
        parent_desc = rng.integers(0, 256, (1, 32), dtype=np.uint8)   # root (not stored)
        first_id = 0                                                   # id of the first node of the parent level
        for lv in range(1, L + 1):
            n = k ** lv
            pd = np.repeat(parent_desc, k, axis=0)
            flip = rng.integers(0, 256, (n, 32), dtype=np.uint8) & rng.integers(0, 256, (n, 32), dtype=np.uint8)
            r = np.zeros(n, rec)
            r["parent"] = first_id + np.arange(n) // k
            r["desc"] = pd ^ flip
            if lv == L:
                w = rng.uniform(0.1, 3.0, n).astype(np.float32)
                w[rng.random(n) < stop_frac] = 0.0
                r["weight"] = w
                r["leaf"] = 1
            f.write(r.tobytes())
            first_id = 1 + sum(k ** j for j in range(1, lv))   # ids of this level: children numbered breadth-first
            parent_desc = r["desc"]
    return nb_nodes, nwords


def fisheye_driver_frame(keep_mask, idx=0):
    """The mono_fisheye driver's image path (Examples/Monocular/mono_fisheye.cc:102-116) over a seeded
    synthetic frame of the camera's size: applyMask (:202-212, pixels whose mask pixel has G > 250 set to 0;
    `keep_mask` is the (1208, 1920) bool array of pixels that stay), crop Rect(0, 0, 1900, 800) (:111-113),
    then cv::resize(..., Size(0, 0), 0.5, 0.5) (:116).  For an exact 2x2 downscale OpenCV's INTER_LINEAR
    switches to the INTER_AREA fast path, the rounded mean (a + b + c + d + 2) >> 2.  The frame is
    synthesised gray (the driver's colour image is converted to gray later, in Tracking), so only the
    geometry and the mask are the driver's.  Returns (950x400 image, 950x400 keep mask as 0 / 255: a
    pixel stays when at least two of its four source pixels stay)."""
    h, w = keep_mask.shape
    img = synth_frame(w, h, idx)
    img = np.where(keep_mask, img, 0).astype(np.uint8)
    img = img[:800, :1900].astype(np.int32)
    km = keep_mask[:800, :1900].astype(np.int32)
    out = (img[0::2, 0::2] + img[0::2, 1::2] + img[1::2, 0::2] + img[1::2, 1::2] + 2) >> 2
    kq = km[0::2, 0::2] + km[0::2, 1::2] + km[1::2, 0::2] + km[1::2, 1::2]
    return np.ascontiguousarray(out.astype(np.uint8)), np.where(kq >= 2, 255, 0).astype(np.uint8)
