// liborbgpu host side: context, geometry, device buffers, and the extractor entry points of the C-ABI
// (include/orbgpu.h).  Matcher entry points live in matcher.hip.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "orbgpu_ctx.h"

namespace orbgpu {

thread_local std::string g_last_error;

void set_error(const char* what, hipError_t e) {
    char buf[512];
    if (e != hipSuccess) std::snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    else std::snprintf(buf, sizeof buf, "%s", what);
    g_last_error = buf;
}

/* ---------------- ORBextractor tables (ORBextractor.cc:410-470) ---------------- */
static inline int round_half_even(float v) { return (int)std::nearbyint(v); }   // cvRound(float)
static inline int round_half_even(double v) { return (int)std::nearbyint(v); }  // cvRound(double)

void compute_tables(Ctx* c) {
    const int nl = c->p.nlevels;
    const double sf = (double)c->p.scaleFactor;   // ORBextractor.h:98 keeps scaleFactor as double
    c->scale[0] = 1.0f;
    c->sigma2[0] = 1.0f;
    for (int i = 1; i < nl; i++) {
        c->scale[i] = (float)(c->scale[i - 1] * sf);
        c->sigma2[i] = c->scale[i] * c->scale[i];
    }
    for (int i = 0; i < nl; i++) {
        c->inv_scale[i] = 1.0f / c->scale[i];
        c->inv_sigma2[i] = 1.0f / c->sigma2[i];
    }
    const float factor = (float)(1.0f / sf);
    float ndesired = c->p.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nl));
    int sum = 0;
    for (int l = 0; l < nl - 1; l++) {
        c->n_per_level[l] = round_half_even(ndesired);
        sum += c->n_per_level[l];
        ndesired *= factor;
    }
    c->n_per_level[nl - 1] = std::max(c->p.nfeatures - sum, 0);
    // umax: pre-computed ends of the rows of the circular patch (:454-469)
    const int hp = kHalfPatch;
    int v, v0, vmax = (int)std::floor(hp * std::sqrt(2.f) / 2 + 1);
    int vmin = (int)std::ceil(hp * std::sqrt(2.f) / 2);
    const double hp2 = hp * hp;
    for (v = 0; v <= vmax; ++v) c->umax[v] = round_half_even(std::sqrt(hp2 - v * v));
    for (v = hp, v0 = 0; v >= vmin; --v) {
        while (c->umax[v0] == c->umax[v0 + 1]) ++v0;
        c->umax[v] = v0;
        ++v0;
    }
    // k_describe carries this table as the packed constant 0x3689ABCDDEEEFFFF (4 bits per row)
    unsigned long long packed = 0;
    for (int i = 0; i < 16; i++) packed |= (unsigned long long)c->umax[i] << (4 * i);
    c->umax_ok = packed == 0x3689ABCDDEEEFFFFull;
    // Gaussian 7x7 sigma 2: getGaussianKernel(7, 2, CV_32F) -> convertTo(CV_32S, 256)
    float cf[7];
    double s = 0;
    for (int i = 0; i < 7; i++) {
        const double x = i - 3.0;
        cf[i] = (float)std::exp(-0.5 / (2.0 * 2.0) * x * x);
        s += cf[i];
    }
    s = 1. / s;
    for (int i = 0; i < 7; i++) cf[i] = (float)(cf[i] * s);
    for (int i = 0; i < 7; i++) c->gk[i] = round_half_even(cf[i] * 256.f);
}

/* ---------------- per-image-size geometry ---------------- */
void resize_coefs(int sw, int dw, std::vector<ResizeCoef>& out, bool vertical) {
    // OpenCV 3.2 resize INTER_LINEAR coefficient setup (imgwarp.cpp)
    const double scale = 1. / ((double)dw / sw);
    for (int d = 0; d < dw; d++) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int s0 = (int)std::floor(f);
        f -= s0;
        if (!vertical) {
            if (s0 < 0) { f = 0; s0 = 0; }
            if (s0 + 1 >= sw && s0 >= sw - 1) { f = 0; s0 = sw - 1; }
        }
        ResizeCoef rc;
        auto sat_short = [](int x) { return std::min(std::max(x, -32768), 32767); };
        rc.c0 = sat_short(round_half_even((1.f - f) * 2048));
        rc.c1 = sat_short(round_half_even(f * 2048));
        rc.s0 = std::min(std::max(s0, 0), sw - 1);
        rc.s1 = std::min(std::max(s0 + 1, 0), sw - 1);
        out.push_back(rc);
    }
}

int build_geometry(Ctx* c, int W, int H, Geom& g, std::vector<ResizeCoef>& coefs, int* rcoef_off) {
    std::memset(&g, 0, sizeof g);
    const int nl = c->p.nlevels;
    g.nlevels = nl;
    g.W = W;
    g.H = H;
    g.iniTh = std::min(std::max(c->p.iniThFAST, 0), 255);
    g.minTh = std::min(std::max(c->p.minThFAST, 0), 255);
    g.variant = c->p.variant;
    for (int i = 0; i < 16; i++) g.umax[i] = c->umax[i];
    for (int i = 0; i < 7; i++) g.gk[i] = c->gk[i];
    for (int sh = 0; sh < 4; sh++)   // k_describe's MFMA tap fragments (Geom::desc_taps)
        for (int tc = 0; tc < kDescTapTiles; tc++)
            for (int l = 0; l < 64; l++) {
                uint8_t b[16];
                for (int e = 0; e < 16; e++) {
                    const int t = 16 * (l >> 4) + e - sh - (16 * tc + (l & 15));
                    b[e] = (uint8_t)(t >= 0 && t <= 6 ? c->gk[t] : 0);
                }
                std::memcpy(&g.desc_taps[(sh * kDescTapTiles + tc) * 64 + l], b, 16);
            }
    long long pyr = 0;
    int cells = 0, cand = 0, kpc = 0, maxN = 0, maxNini = 0, maxLevelCand = 0;
    coefs.clear();
    for (int l = 0; l < nl; l++) {
        LevelGeom& L = g.L[l];
        L.w = round_half_even((float)W * c->inv_scale[l]);   // ComputePyramid :1112
        L.h = round_half_even((float)H * c->inv_scale[l]);
        L.pitch = (L.w + 63) & ~63;
        if (l > 0) {
            L.pyr_off = pyr;
            pyr += (long long)L.pitch * L.h;
            rcoef_off[l] = (int)coefs.size();
            resize_coefs(g.L[l - 1].w, L.w, coefs, false);
            resize_coefs(g.L[l - 1].h, L.h, coefs, true);
            // k_resize_tiled<TH> stages each tile's source span in a fixed LDS tile: check it fits
            const ResizeCoef* cx = &coefs[rcoef_off[l]];
            const ResizeCoef* cy = cx + L.w;
            bool xfits = true;
            for (int x0 = 0; x0 < L.w && xfits; x0 += kRsTileW) {
                const int x1 = std::min(x0 + kRsTileW, L.w) - 1;
                xfits = cx[x1].s1 - (cx[x0].s0 & ~15) + 1 <= kRsPitch;   // 16-byte aligned span start
            }
            L.rs_tiled = 0;
            int span_rows[3] = {0, 0, 0};   // the largest source span of a tile, per tile height
            for (int i = 0; i < 3 && xfits; i++) {
                const int th = 16 << i;
                bool fits = true;
                for (int y0 = 0; y0 < L.h && fits; y0 += th) {
                    const int y1 = std::min(y0 + th, L.h) - 1;
                    span_rows[i] = std::max(span_rows[i], cy[y1].s1 - cy[y0].s0 + 1);
                    fits = cy[y1].s1 - cy[y0].s0 + 1 <= rs_rows(th);
                }
                if (fits) L.rs_tiled |= 1 << i;
            }
            // the LDS source tile is sized to the tile height the launch uses (32 rows when they fit)
            L.rs_span_rows = (L.rs_tiled & 2) ? span_rows[1] : span_rows[0];
            // and the staging loop to the tile with the most 16-byte source chunks (the aligned-source path)
            L.rs_chunks = 0;
            if (L.rs_tiled & 3) {
                const int th = (L.rs_tiled & 2) ? 32 : 16;
                int nq_max = 0, nr_max = 0;
                for (int x0 = 0; x0 < L.w; x0 += kRsTileW) {
                    const int x1 = std::min(x0 + kRsTileW, L.w) - 1;
                    nq_max = std::max(nq_max, ((cx[x1].s1 - (cx[x0].s0 & ~15)) >> 4) + 1);
                }
                for (int y0 = 0; y0 < L.h; y0 += th) {
                    const int y1 = std::min(y0 + th, L.h) - 1;
                    nr_max = std::max(nr_max, cy[y1].s1 - cy[y0].s0 + 1);
                }
                L.rs_chunks = nq_max * nr_max;
            }
        }
        L.maxBX = L.w - kEdgeThreshold + 3;
        L.maxBY = L.h - kEdgeThreshold + 3;
        const float width = (float)(L.maxBX - kMinBorder), height = (float)(L.maxBY - kMinBorder);
        L.nCols = (int)(width / 30.f);
        L.nRows = (int)(height / 30.f);
        if (L.nCols <= 0 || L.nRows <= 0 || L.w < 2 || L.h < 2) return ORB_ERR_GEOMETRY;
        L.wCell = (int)std::ceil(width / L.nCols);
        L.hCell = (int)std::ceil(height / L.nRows);
        if (L.wCell + 6 > kFastMaxRoi || L.hCell + 6 > kFastMaxRoi) return ORB_ERR_GEOMETRY;
        L.cell_base = cells;
        cells += L.nCols * L.nRows;
        L.cell_cap = ((L.wCell + 1) / 2) * ((L.hCell + 1) / 2);
        L.cand_base = cand;
        L.cand_cap = L.cell_cap * L.nCols * L.nRows;
        cand += L.cand_cap;
        maxLevelCand = std::max(maxLevelCand, L.cand_cap);
        L.nfeat = c->n_per_level[l];
        L.nIni = (int)std::round(width / (float)(L.maxBY - kMinBorder));   // DistributeOctTree :543
        if (L.nIni <= 0) return ORB_ERR_GEOMETRY;                          // reference divides by zero
        L.hX = width / L.nIni;
        L.kp_cap = std::max(L.nfeat + 3, 4 * L.nIni) + 4;
        L.kp_base = kpc;
        kpc += L.kp_cap;
        maxN = std::max(maxN, L.nfeat);
        maxNini = std::max(maxNini, L.nIni);
        L.scale = c->scale[l];
        L.patch_size = (float)(int)(kPatchSize * c->scale[l]);
    }
    if (W > kMaxDim || H > kMaxDim) return ORB_ERR_GEOMETRY;
    g.ncells = cells;
    g.ncand = cand;
    g.nkpcap = kpc;
    g.pyr_bytes = (pyr + 255) & ~255LL;
    g.max_level_cand = maxLevelCand;
    int nc = std::max(maxN + 8, 4 * maxNini + 8);
    nc = (nc + 63) & ~63;
    g.node_cap = nc;
    fast_wave_layout(g);
    if (g.fast_wave_bytes > 64 * 1024 || octree_lds_bytes(nc) > 160 * 1024) return ORB_ERR_GEOMETRY;
    return ORB_OK;
}

/* ---------------- buffers ---------------- */
template <class T>
static hipError_t grow(T*& p, size_t& cap, size_t need) {
    if (need <= cap && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc((void**)&p, std::max<size_t>(need, 256) * sizeof(T));
    if (e == hipSuccess) cap = std::max<size_t>(need, 256);
    return e;
}

/* The few-launch pyramid's plan (k_pyramid_chain): the levels in segments of up to kChainSeg, one
 * launch each, every level of a segment computed from the segment's base level (the frame, or the
 * previous segment's last level).  Per level l output tiles of 64 x 32 (32 x 16 for the third and later
 * levels of a segment, so a tile's recomputed chain stays short), and for each tile the region of every
 * level base .. l-1 its pixels depend on, walked back through the resize coefficient tables (monotone:
 * a region's span is its end columns' / rows' source indices).  Regions above the base start at a
 * multiple of 4 and span a multiple of 4 columns; the base region is clipped to the level. */
static void build_chain(const Geom& g, const std::vector<ResizeCoef>& coefs, const int* off, std::vector<ChainJob>& jobs,
                        ChainPlan& plan, int first_base, int seg_len) {
    jobs.clear();
    plan = ChainPlan{};
    const int nl = g.nlevels;
    if (nl < 2 || first_base >= nl - 1) return;
    auto r4 = [](int x) { return (x + 3) & ~3; };
    for (int base = first_base; base < nl - 1; base += seg_len) {
        const int top = std::min(base + seg_len, nl - 1);
        ChainSegment sg;
        sg.job0 = (int)jobs.size();
        int bufb = 0, coefe = 0;
        for (int l = base + 1; l <= top; l++) {
            const int TW = l - base <= 2 ? 64 : 32, TH = l - base <= 2 ? 32 : 16;
            const int wl = g.L[l].w, hl = g.L[l].h;
            for (int y0 = 0; y0 < hl; y0 += TH)
                for (int x0 = 0; x0 < wl; x0 += TW) {
                    ChainJob J;
                    std::memset(&J, 0, sizeof J);
                    J.level = l;
                    J.base = base;
                    J.reg[l] = make_int4(x0, r4(std::min(x0 + TW, wl)), y0, std::min(y0 + TH, hl));
                    int ce = 0;
                    for (int k = l; k > base; k--) {
                        const int4 R = J.reg[k];
                        const ResizeCoef* cx = &coefs[off[k]];
                        const ResizeCoef* cy = cx + g.L[k].w;
                        const int sx0 = cx[R.x].s0, sx1 = cx[std::min(R.y, g.L[k].w) - 1].s1 + 1;
                        const int sy0 = cy[R.z].s0, sy1 = cy[R.w - 1].s1 + 1;
                        J.reg[k - 1] = make_int4(sx0 & ~3, k - 1 > base ? r4(sx1) : std::min(sx1, g.L[k - 1].w), sy0, sy1);
                        ce += (R.y - R.x) + (R.w - R.z);
                    }
                    for (int k = base; k < l; k++) {
                        const int4 R = J.reg[k];
                        bufb = std::max(bufb, r4(R.y - R.x) * (R.w - R.z));
                    }
                    coefe = std::max(coefe, ce);
                    jobs.push_back(J);
                }
        }
        sg.njobs = (int)jobs.size() - sg.job0;
        sg.buf_bytes = (bufb + 15) & ~15;
        sg.coef_entries = coefe;
        sg.lds_bytes = 2 * sg.buf_bytes + 16 * coefe;
        if (sg.lds_bytes > 64 * 1024) {   // wide images keep the per-level launches
            jobs.clear();
            plan = ChainPlan{};
            return;
        }
        plan.seg[plan.nseg++] = sg;
    }
    plan.first_base = first_base;
}

int Ctx::ensure_geometry(int W, int H) {
    if (have_geom && geom.W == W && geom.H == H) return ORB_OK;
    Geom g;
    std::vector<ResizeCoef> coefs;
    int off[ORBGPU_MAX_LEVELS] = {0};
    int st = build_geometry(this, W, H, g, coefs, off);
    if (st != ORB_OK) {
        set_error("image too small or too large for the configured pyramid", hipSuccess);
        return st;
    }
    hipError_t e;
    if ((e = grow(d_geom, geom_cap, 1)) != hipSuccess) return set_error("hipMalloc geom", e), ORB_ERR_NOMEM;
    if ((e = grow(d_rcoef, rcoef_cap, coefs.size())) != hipSuccess) return set_error("hipMalloc coef", e), ORB_ERR_NOMEM;
    std::vector<CellDesc> cells;
    build_cells(g, cells);
    if ((e = grow(d_cells, cells_cap, cells.size())) != hipSuccess) return set_error("hipMalloc cells", e), ORB_ERR_NOMEM;
    if ((e = hipMemcpyAsync(d_cells, cells.data(), cells.size() * sizeof(CellDesc), hipMemcpyHostToDevice, stream)) !=
        hipSuccess)
        return set_error("upload cells", e), ORB_ERR_HIP;
    if ((e = hipMemcpyAsync(d_geom, &g, sizeof g, hipMemcpyHostToDevice, stream)) != hipSuccess)
        return set_error("upload geom", e), ORB_ERR_HIP;
    if ((e = hipMemcpyAsync(d_rcoef, coefs.data(), coefs.size() * sizeof(ResizeCoef), hipMemcpyHostToDevice,
                            stream)) != hipSuccess)
        return set_error("upload coefs", e), ORB_ERR_HIP;
    // the host path's plan (one frame in flight: levels 1..7 from the frame in segments of kChainSeg) and, for
    // small batches, levels 1..kSmallChainBase per level and the rest from that level in one segment
    ChainPlan cplan, cplan2;
    for (int which = 0; which < 2; which++) {
        std::vector<ChainJob> cjobs;
        ChainPlan& pl = which ? cplan2 : cplan;
        if (which == 1 && kSmallChainBase <= 0) break;
        build_chain(g, coefs, off, cjobs, pl, which ? kSmallChainBase : 0, which ? ORBGPU_MAX_LEVELS : kChainSeg);
        if (!pl.nseg) continue;
        ChainJob*& dj = which ? d_chain2 : d_chain;
        size_t& cap = which ? chain2_cap : chain_cap;
        if ((e = grow(dj, cap, cjobs.size())) != hipSuccess) return set_error("hipMalloc chain", e), ORB_ERR_NOMEM;
        if ((e = hipMemcpyAsync(dj, cjobs.data(), cjobs.size() * sizeof(ChainJob), hipMemcpyHostToDevice, stream)) !=
            hipSuccess)
            return set_error("upload chain", e), ORB_ERR_HIP;
        if (which == 0) chain_jobs_host = cjobs;
    }
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return set_error("sync", e), ORB_ERR_HIP;
    geom = g;
    chain = cplan;
    chain_small = cplan2;
    std::memcpy(rcoef_off, off, sizeof off);
    have_geom = true;
    ++geom_serial;
    return ORB_OK;
}

int Ctx::ensure_frames(int nframes) {
    const Geom& g = geom;
    hipError_t e;
    const bool fresh_err = d_err == nullptr;
    const size_t nl = g.nlevels;
    if ((e = grow(d_pyr, pyr_cap, (size_t)nframes * g.pyr_bytes)) != hipSuccess ||
        (e = grow(d_cands, cands_cap, (size_t)nframes * g.ncand)) != hipSuccess ||
        (e = grow(d_candFirst, candfirst_cap, (size_t)nframes * g.ncells * kCandRec)) != hipSuccess ||
        (e = grow(d_keys, keys_cap, (size_t)nframes * nl * g.max_level_cand)) != hipSuccess ||
        (e = grow(d_knode, knode_cap, (size_t)nframes * nl * g.max_level_cand)) != hipSuccess ||
        (e = grow(d_lvlKps, lvlkps_cap, (size_t)nframes * g.nkpcap)) != hipSuccess ||
        (e = grow(d_lvlCount, lvlc_cap, (size_t)nframes * nl)) != hipSuccess ||
        (e = grow(d_err, err_cap, 2)) != hipSuccess) {
        set_error("device allocation for the extractor", e);
        return ORB_ERR_NOMEM;
    }
    if (fast_stamps && (e = grow(d_stamps, stamps_cap, (size_t)nframes * (g.ncells * 8 + g.nlevels * 32 + g.nkpcap * 8))) != hipSuccess)
        return set_error("stamps", e), ORB_ERR_NOMEM;
    // the overflow flag is read by orb_sync even before the first extraction (every extraction zeroes
    // it in its first kernel)
    if (fresh_err && (e = hipMemsetAsync(d_err, 0, 2 * sizeof(int), stream)) != hipSuccess)
        return set_error("memset", e), ORB_ERR_HIP;
    return ORB_OK;
}

// The dataflow launch's plan for this geometry and frame count (built on the host, uploaded once per change); false
// flow_ok: the geometry does not take it (the per-kernel launches run).  Counters are zeroed here once and re-zeroed
// by every launch's last workgroup.
int Ctx::ensure_flow(int nframes) {
    if (flow_ok && flow_serial == geom_serial && flow.nframes == nframes) return ORB_OK;
    flow_ok = false;
    std::vector<FlowTask> tasks;
    FlowPlan pl;
    const int blocks = std::min(num_cu, flow_blocks > 0 ? flow_blocks : kFlowDefaultBlocks * nframes);
    // per-level resize tasks; ORBGPU_FLOW_CHAIN=1: chain-job pyramid tasks (each tile's region chain from the segment
    // base, as k_pyramid_chain), measured slower at one frame, both forms in tests/test_gpu_flow.py
    const char* fc = std::getenv("ORBGPU_FLOW_CHAIN");
    const bool use_chain = chain.nseg > 0 && fc && fc[0] == '1';
    if (!build_flow(geom, nframes, blocks, use_chain ? &chain : nullptr, &chain_jobs_host, tasks, pl)) return ORB_OK;
    flow_chain_plan = use_chain ? chain : ChainPlan{};
    hipError_t e;
    // (a launch queued earlier may still read the old task table or counters)
    if ((tasks.size() > flow_cap || (size_t)pl.nctr > flow_ctr_cap) && (e = hipStreamSynchronize(stream)) != hipSuccess)
        return set_error("sync", e), ORB_ERR_HIP;
    if ((e = grow(d_flow, flow_cap, tasks.size())) != hipSuccess) return set_error("hipMalloc flow tasks", e), ORB_ERR_NOMEM;
    const bool fresh = (size_t)pl.nctr > flow_ctr_cap || !d_flow_ctr;
    if ((e = grow(d_flow_ctr, flow_ctr_cap, (size_t)pl.nctr)) != hipSuccess)
        return set_error("hipMalloc flow counters", e), ORB_ERR_NOMEM;
    if (fresh && (e = hipMemsetAsync(d_flow_ctr, 0, flow_ctr_cap * sizeof(int), stream)) != hipSuccess)
        return set_error("memset flow counters", e), ORB_ERR_HIP;
    if ((e = hipMemcpyAsync(d_flow, tasks.data(), tasks.size() * sizeof(FlowTask), hipMemcpyHostToDevice, stream)) !=
        hipSuccess)
        return set_error("upload flow tasks", e), ORB_ERR_HIP;
    if (flow_stamps && (e = grow(d_flow_stamps, flow_stamps_cap, (size_t)pl.ntasks * 4)) != hipSuccess)
        return set_error("hipMalloc flow stamps", e), ORB_ERR_NOMEM;
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return set_error("sync", e), ORB_ERR_HIP;
    flow = pl;
    flow_serial = geom_serial;
    flow_ok = true;
    return ORB_OK;
}

ExtractBuffers Ctx::buffers() const {
    ExtractBuffers b;
    b.d_geom = d_geom;
    b.d_rcoef = d_rcoef;
    b.d_cells = d_cells;
    std::memcpy(b.rcoef_off, rcoef_off, sizeof rcoef_off);
    b.d_chain = d_chain;
    b.chain = chain;
    b.d_pyr = d_pyr;
    b.d_cands = d_cands;
    b.d_candFirst = d_candFirst;
    b.d_keys = d_keys;
    b.d_knode = d_knode;
    b.d_lvlKps = d_lvlKps;
    b.d_lvlCount = d_lvlCount;
    b.d_err = d_err;
    b.zero_err = 1;
    b.err_host = nullptr;
    b.d_stamps = fast_stamps ? d_stamps : nullptr;
    b.fork_s2 = nullptr;
    b.ev_fork = b.ev_join = nullptr;
    b.d_flow = nullptr;
    b.d_flow_ctr = nullptr;
    b.flow_chain = ChainPlan{};
    b.d_flow_args = nullptr;
    b.d_flow_stamps = nullptr;
    return b;
}

void Ctx::marker(void* user, int id, int begin, hipStream_t s) {
    Ctx* c = (Ctx*)user;
    if (!c->prof_on) return;
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return;
    (void)hipEventRecord(ev, s);
    if (begin) c->prof_open[id] = ev;
    else c->prof_pairs.push_back({id, c->prof_open[id], ev});
}

int Ctx::run_extract(const uint8_t* d_frames, int nframes, long long frame_pitch, int row_stride, orb_keypoint* d_kps,
                     uint8_t* d_desc, int* d_counts, int kp_cap, int* err, bool latency, int* err_host) {
    hipError_t e;
    ExtractBuffers bufs = buffers();
    if (err) bufs.d_err = err;
    bufs.err_host = err_host;
    // the few-launch pyramid trades redundant work for fewer dependent launches: the whole plan pays for one
    // frame in flight (the host path); batches of a frame or two (C5 at one frame per GPU) take the small plan
    if (!latency) {
        bufs.chain = chain_small;
        bufs.d_chain = d_chain2;
    }
    // small batches: the dataflow launch (stamps are per-kernel diagnostics: the per-kernel launches)
    if (!latency && nframes <= flow_max_frames && !fast_stamps) {
        const int st = ensure_flow(nframes);
        if (st != ORB_OK) return st;
        if (flow_ok) {
            bufs.d_flow = d_flow;
            bufs.d_flow_ctr = d_flow_ctr;
            bufs.flow = flow;
            bufs.flow_chain = flow_chain_plan;
            bufs.d_chain = d_chain;   // (the chain tasks' jobs: the host-path plan, levels from the frame)
            // the kernel reads its arguments from device memory: uploaded when they differ from the last call's
            // (stream-ordered behind the launches still reading the old ones; a pageable copy of 0.2 KB returns once
            // the runtime has staged it)
            if (!d_flow_args && (e = hipMalloc((void**)&d_flow_args, sizeof(FlowArgs))) != hipSuccess)
                return set_error("hipMalloc flow args", e), ORB_ERR_NOMEM;
            bufs.d_flow_stamps = flow_stamps ? d_flow_stamps : nullptr;
            const FlowArgs A = flow_args(bufs, d_frames, frame_pitch, row_stride, nframes, d_kps, d_desc, d_counts, kp_cap);
            if (std::memcmp(&A, &h_flow_args, sizeof A) != 0 || !flow_args_valid) {
                if ((e = hipMemcpyAsync(d_flow_args, &A, sizeof A, hipMemcpyHostToDevice, stream)) != hipSuccess) {
                    flow_args_valid = false;
                    return set_error("upload flow args", e), ORB_ERR_HIP;
                }
                h_flow_args = A;
                flow_args_valid = true;
            }
            bufs.d_flow_args = d_flow_args;
        }
    }
    // one frame in flight (ORBGPU_FORK=1): level 0's FAST -> octree on a second stream beside the pyramid
    if (latency && fork && !prof_on && !fast_stamps && geom.nlevels > 1) {
        hipError_t fe = hipSuccess;
        if (!stream2 && (fe = hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking)) != hipSuccess)
            return set_error("second stream", fe), ORB_ERR_HIP;
        if (!ev_fork && (fe = hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming)) != hipSuccess)
            return set_error("fork event", fe), ORB_ERR_HIP;
        if (!ev_join && (fe = hipEventCreateWithFlags(&ev_join, hipEventDisableTiming)) != hipSuccess)
            return set_error("join event", fe), ORB_ERR_HIP;
        bufs.fork_s2 = stream2;
        bufs.ev_fork = ev_fork;
        bufs.ev_join = ev_join;
    }
    // one frame in flight (the host path): direct launches measured faster than a graph replay (the first
    // kernel is dispatched as soon as it is launched, while the host submits the rest)
    if (use_graph && !prof_on && !fast_stamps && !latency) {
        // HIP graph replay: one submission per batch instead of 10 launches; captured on the first batch
        // with a given set of buffers / arguments and re-instantiated when any of them changes
        const std::array<uintptr_t, 24> key = {
            (uintptr_t)d_frames, (uintptr_t)nframes, (uintptr_t)frame_pitch, (uintptr_t)row_stride, (uintptr_t)d_kps,
            (uintptr_t)d_desc, (uintptr_t)d_counts, (uintptr_t)kp_cap, (uintptr_t)geom.W, (uintptr_t)geom.H,
            (uintptr_t)geom_serial, (uintptr_t)d_geom, (uintptr_t)d_rcoef, (uintptr_t)d_cells, (uintptr_t)d_pyr,
            (uintptr_t)d_cands, (uintptr_t)d_candFirst, (uintptr_t)d_keys, (uintptr_t)d_knode, (uintptr_t)d_lvlKps,
            (uintptr_t)d_lvlCount, (uintptr_t)bufs.d_err, (uintptr_t)stream,
            (uintptr_t)bufs.chain.nseg ^ ((uintptr_t)err_host << 4) ^ ((uintptr_t)(bufs.fork_s2 != nullptr) << 3) ^
                ((uintptr_t)bufs.d_flow << 8) ^ ((uintptr_t)bufs.flow.ntasks << 1) ^ ((uintptr_t)bufs.flow.blocks << 20)};
        if (!gexec || key != gkey) {
            if (gexec) (void)hipGraphExecDestroy(gexec);
            if (graph) (void)hipGraphDestroy(graph);
            gexec = nullptr;
            graph = nullptr;
            if ((e = hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal)) != hipSuccess)
                return set_error("graph capture", e), ORB_ERR_HIP;
            // the overflow flag is zeroed by the FAST kernel (no separate memset node)
            hipError_t le = launch_extract(geom, bufs, d_frames, frame_pitch, row_stride, nframes, d_kps, d_desc,
                                           d_counts, kp_cap, stream, nullptr, nullptr);
            hipGraph_t gr = nullptr;
            e = hipStreamEndCapture(stream, &gr);
            if (le != hipSuccess || e != hipSuccess) {
                if (gr) (void)hipGraphDestroy(gr);
                return set_error("graph capture", le != hipSuccess ? le : e), ORB_ERR_HIP;
            }
            if ((e = hipGraphInstantiate(&gexec, gr, nullptr, nullptr, 0)) != hipSuccess) {
                (void)hipGraphDestroy(gr);
                gexec = nullptr;
                return set_error("graph instantiate", e), ORB_ERR_HIP;
            }
            graph = gr;
            gkey = key;
        }
        if ((e = hipGraphLaunch(gexec, stream)) != hipSuccess) return set_error("graph launch", e), ORB_ERR_HIP;
    } else {   // ORBGPU_GRAPH=0, per-kernel profiling or stamps: direct launches (same kernels, same order)
        e = launch_extract(geom, bufs, d_frames, frame_pitch, row_stride, nframes, d_kps, d_desc, d_counts, kp_cap,
                           stream, &Ctx::marker, this);
        if (e != hipSuccess) return set_error("kernel launch", e), ORB_ERR_HIP;
    }
    last_frames = d_frames;
    last_frame_pitch = frame_pitch;
    last_row_stride = row_stride;
    last_nframes = nframes;
    last_kps = d_kps;
    last_desc = d_desc;
    last_counts = d_counts;
    last_kp_cap = kp_cap;
    level_cache_valid = 0;
    return ORB_OK;
}

}  // namespace orbgpu

using namespace orbgpu;

#define CTX_GUARD(ctx)                                                              \
    if (!(ctx)) {                                                                   \
        set_error("NULL context", hipSuccess);                                      \
        return ORB_ERR_ARG;                                                         \
    }                                                                               \
    {                                                                               \
        hipError_t _e = hipSetDevice((ctx)->device);                                \
        if (_e != hipSuccess) return set_error("hipSetDevice", _e), ORB_ERR_HIP;    \
    }

extern "C" {

int orb_abi_version(void) { return ORBGPU_ABI_VERSION; }
const char* orb_last_error(void) { return g_last_error.c_str(); }

int orb_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

orb_ctx* orb_create(const orb_params* p, int* status) {
    auto fail = [&](int st) -> orb_ctx* {
        if (status) *status = st;
        return nullptr;
    };
    if (!p || p->nlevels < 1 || p->nlevels > ORBGPU_MAX_LEVELS || p->nfeatures < 0 || !(p->scaleFactor > 1.0f)) {
        set_error("invalid orb_params", hipSuccess);
        return fail(ORB_ERR_ARG);
    }
    if (p->variant & ~ORB_VARIANT_MASK) {
        set_error("invalid orb_params.variant (unknown ORB_VARIANT_* bits)", hipSuccess);
        return fail(ORB_ERR_ARG);
    }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || p->device < 0 || p->device >= ndev) {
        set_error("no HIP device (liborbgpu has no CPU fallback)", e);
        return fail(ORB_ERR_HIP);
    }
    if ((e = hipSetDevice(p->device)) != hipSuccess) return set_error("hipSetDevice", e), fail(ORB_ERR_HIP);
    Ctx* c = new (std::nothrow) Ctx();
    if (!c) return fail(ORB_ERR_NOMEM);
    c->p = *p;
    c->device = p->device;
    if (hipDeviceGetAttribute(&c->num_cu, hipDeviceAttributeMultiprocessorCount, p->device) != hipSuccess ||
        c->num_cu < 1)
        c->num_cu = 256;
    // diagnostics only (tests/test_gpu_extract.py checks both leave the results unchanged):
    // ORBGPU_FAST_STAMPS=1 records kernel phase timestamps, ORBGPU_GRAPH=0 launches without graph replay
    if (const char* e = std::getenv("ORBGPU_FAST_STAMPS")) c->fast_stamps = e[0] == '1';
    if (const char* ev = std::getenv("ORBGPU_GRAPH")) c->use_graph = ev[0] != '0';
    // ORBGPU_STEREO_STAGE=1: orb_compute_stereo_matches stages the right side as for a peer device
    if (const char* ev = std::getenv("ORBGPU_STEREO_STAGE")) c->stereo_stage = ev[0] == '1';
    if (const char* ev = std::getenv("ORBGPU_FORK")) c->fork = ev[0] != '0';
    if (const char* ev = std::getenv("ORBGPU_UPLOAD")) c->upload_stream = ev[0] != '0';
    // ORBGPU_FLOW=1: batches of one or two frames take the dataflow launch (A/B and parity of both forms);
    // ORBGPU_FLOW_BLOCKS=n: its workgroups
    if (const char* ev = std::getenv("ORBGPU_FLOW")) c->flow_max_frames = ev[0] == '0' ? 0 : 2;
    if (const char* ev = std::getenv("ORBGPU_FLOW_BLOCKS")) c->flow_blocks = std::atoi(ev);
    if (const char* ev = std::getenv("ORBGPU_FLOW_STAMPS")) c->flow_stamps = ev[0] == '1';
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) {
        delete c;
        set_error("hipStreamCreate", e);
        return fail(ORB_ERR_HIP);
    }

    compute_tables(c);
    if (!c->umax_ok) {
        orb_destroy(reinterpret_cast<orb_ctx*>(c));
        set_error("internal: umax table differs from the kernel's packed constant", hipSuccess);
        return fail(ORB_ERR_INTERNAL);
    }
    if (p->max_width > 0 && p->max_height > 0) {
        int st = c->ensure_geometry(p->max_width, p->max_height);
        if (st == ORB_OK) st = c->ensure_frames(std::max(1, p->max_batch));
        if (st != ORB_OK) {
            orb_destroy(reinterpret_cast<orb_ctx*>(c));
            return fail(st);
        }
    }
    if (status) *status = ORB_OK;
    return reinterpret_cast<orb_ctx*>(c);
}

void orb_destroy(orb_ctx* h) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto& pr : c->prof_pairs) {
        (void)hipEventDestroy(pr.b);
        (void)hipEventDestroy(pr.e);
    }
    void* bufs[] = {c->d_flow, c->d_flow_ctr, c->d_flow_args, c->d_flow_stamps, c->d_cells, c->d_stamps, c->d_geom, c->d_rcoef, c->d_chain, c->d_chain2, c->d_pyr, c->d_cands, c->d_candFirst, c->d_keys, c->d_knode,
                    c->d_lvlKps, c->d_lvlCount, c->d_err, c->d_in,
                    c->d_scratch, c->d_peer, c->d_pairs};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (c->h_pinned) (void)hipHostFree(c->h_pinned);
    if (c->h_mstage) (void)hipHostFree(c->h_mstage);
    if (c->h_img) (void)hipHostFree(c->h_img);
    if (c->h_flags) (void)hipHostFree(c->h_flags);
    for (int i = 0; i < 2; i++) {
        if (c->h_pairs[i]) (void)hipHostFree(c->h_pairs[i]);
        if (c->pairs_ev[i]) (void)hipEventDestroy(c->pairs_ev[i]);
    }
    if (c->gexec) (void)hipGraphExecDestroy(c->gexec);
    if (c->graph) (void)hipGraphDestroy(c->graph);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    delete c;
}

int orb_scale_tables(const orb_ctx* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                     int* n_per_level, int* umax16) {
    const Ctx* c = reinterpret_cast<const Ctx*>(h);
    if (!c) return ORB_ERR_ARG;
    const int nl = c->p.nlevels;
    for (int i = 0; i < nl; i++) {
        if (scale) scale[i] = c->scale[i];
        if (inv_scale) inv_scale[i] = c->inv_scale[i];
        if (sigma2) sigma2[i] = c->sigma2[i];
        if (inv_sigma2) inv_sigma2[i] = c->inv_sigma2[i];
        if (n_per_level) n_per_level[i] = c->n_per_level[i];
    }
    if (umax16)
        for (int i = 0; i < 16; i++) umax16[i] = c->umax[i];
    return ORB_OK;
}

int orb_batch_kp_cap(orb_ctx* h, int w, int hgt) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    int st = c->ensure_geometry(w, hgt);
    if (st != ORB_OK) return st;
    return c->geom.nkpcap;
}

int orb_extract_batch_device(orb_ctx* h, const uint8_t* d_frames, int nframes, int w, int hgt, size_t frame_pitch,
                             size_t row_stride, orb_keypoint* d_kps, uint8_t* d_desc, int* d_counts, int kp_cap) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    if (!d_frames || nframes <= 0 || !d_kps || !d_desc || !d_counts || row_stride < (size_t)w ||
        row_stride >= (size_t)1 << 24)   // kernels form row offsets with 24-bit multiplies
        return set_error("orb_extract_batch_device: bad arguments", hipSuccess), ORB_ERR_ARG;
    int st = c->ensure_geometry(w, hgt);
    if (st != ORB_OK) return st;
    if (kp_cap < c->geom.nkpcap) {
        set_error("kp_cap smaller than orb_batch_kp_cap()", hipSuccess);
        return ORB_ERR_CAPACITY;
    }
    if ((st = c->ensure_frames(nframes)) != ORB_OK) return st;
    return c->run_extract(d_frames, nframes, (long long)frame_pitch, (int)row_stride, d_kps, d_desc, d_counts, kp_cap);
}

int orb_sync(orb_ctx* h) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return set_error("hipStreamSynchronize", e), ORB_ERR_HIP;
    int err[2] = {0, 0};
    if (c->d_err && (e = hipMemcpy(err, c->d_err, sizeof err, hipMemcpyDeviceToHost)) != hipSuccess)
        return set_error("read error flag", e), ORB_ERR_HIP;
    if (err[0] | err[1]) {
        set_error((err[1] & 4) ? "dataflow launch: a task's wait timed out (outputs invalid)"
                               : "octree node table overflow (raise nfeatures capacity)", hipSuccess);
        return ORB_ERR_INTERNAL;
    }
    return ORB_OK;
}

int orb_extract(orb_ctx* h, const uint8_t* img, int w, int hgt, size_t stride, orb_keypoint* kps, int cap, int* n,
                uint8_t* desc) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    if (!img || w <= 0 || hgt <= 0) return ORB_OK;   // _image.empty(): outputs untouched (:1046-1047)
    if (!n || stride < (size_t)w) return set_error("orb_extract: bad arguments", hipSuccess), ORB_ERR_ARG;
    int st = c->ensure_geometry(w, hgt);
    if (st != ORB_OK) return st;
    if ((st = c->ensure_frames(1)) != ORB_OK) return st;
    hipError_t e;
    const size_t pitch = ((size_t)w + 63) & ~(size_t)63;
    const int kcap = c->geom.nkpcap;
    const size_t kbytes = ((size_t)kcap * sizeof(orb_keypoint) + 63) & ~(size_t)63;   // descriptors 64-B aligned
    const size_t need = 16 + kbytes + (size_t)kcap * 32;
    if ((e = grow(c->d_in, c->in_cap, pitch * hgt)) != hipSuccess) return set_error("device allocation", e), ORB_ERR_NOMEM;
    // every allocation before the first launch: with the streamed upload the upload kernel queued below polls for
    // the host copy that follows it, so nothing in between may block on the stream (hipHostFree / hipFree do)
    if (need > c->pinned_cap) {
        if (c->h_pinned) (void)hipHostFree(c->h_pinned);
        c->h_pinned = nullptr;
        c->pinned_cap = 0;
        // mapped + coherent (fine-grained) explicitly: k_describe stores the outputs straight into this block and
        // the host reads them after hipStreamSynchronize, with no D2H copy in between
        if ((e = hipHostMalloc(&c->h_pinned, need, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
            return set_error("pinned staging", e), ORB_ERR_NOMEM;
        c->pinned_cap = need;
    }
    constexpr int kBands = 16;   // (h_flags[kBands .. 63]: [63] = the upload kernel's timeout flag)
    const int band_rows = (hgt + kBands - 1) / kBands, nbands = (hgt + band_rows - 1) / band_rows;
    if (c->upload_stream) {
        if (pitch * hgt > c->himg_cap) {
            if (c->h_img) (void)hipHostFree(c->h_img);
            c->h_img = nullptr;
            c->himg_cap = 0;
            if ((e = hipHostMalloc((void**)&c->h_img, pitch * hgt, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
                return set_error("pinned image staging", e), ORB_ERR_NOMEM;
            c->himg_cap = pitch * hgt;
        }
        if (!c->h_flags) {
            if ((e = hipHostMalloc((void**)&c->h_flags, 64 * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent)) !=
                hipSuccess)
                return set_error("pinned upload flags", e), ORB_ERR_NOMEM;
            std::memset(c->h_flags, 0, 64 * sizeof(uint32_t));
        }
        if (++c->upload_seq == 0) c->upload_seq = 1;   // (flags start at 0)
        // the upload kernel first; the host copy raising the band flags follows (below), then the extraction launches
        if ((e = launch_upload_stream(c->h_img, c->h_flags, c->upload_seq, c->d_in, (int)pitch, hgt, nbands, band_rows,
                                      c->h_flags + 63, c->stream)) != hipSuccess)
            return set_error("upload kernel", e), ORB_ERR_HIP;
    } else {
        // pageable 2-D upload (measured faster than a host copy into pinned staging + one DMA: 0.149 vs 0.168
        // ms per C3 frame end to end, tools/host_latency; profiles/r03/latency_probe_upload.json)
        if ((e = hipMemcpy2DAsync(c->d_in, pitch, img, stride, w, hgt, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
            return set_error("upload image", e), ORB_ERR_HIP;
    }
    // output block [count | overflow flag | 8 B pad | keypoints | descriptors] in pinned, host-coherent
    // memory: k_describe writes the keypoints, descriptors and count straight into it (and copies the
    // octree's overflow flag), so no download follows the kernels
    uint8_t* hp = static_cast<uint8_t*>(c->h_pinned);
    int* hcnt = reinterpret_cast<int*>(hp);
    orb_keypoint* hk = reinterpret_cast<orb_keypoint*>(hp + 16);
    uint8_t* hd = hp + 16 + kbytes;
    if (c->upload_stream) {
        // the host half of the streamed upload, band by band, each band's flag raised after its bytes (x86 stores
        // are ordered; the release store keeps the compiler from sinking the copy past it).  Before the extraction
        // launches: the upload kernel pulls each band over PCIe while the host copies the next
        for (int b = 0; b < nbands; b++) {
            const int r0 = b * band_rows, r1 = std::min(hgt, r0 + band_rows);
            for (int r = r0; r < r1; r++) std::memcpy(c->h_img + (size_t)r * pitch, img + (size_t)r * stride, (size_t)w);
            __atomic_store_n(c->h_flags + b, c->upload_seq, __ATOMIC_RELEASE);
        }
    }
    st = c->run_extract(c->d_in, 1, (long long)pitch * hgt, (int)pitch, hk, hd, hcnt, kcap, nullptr, true, hcnt + 1);
    if (st != ORB_OK) return st;
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return set_error("extract", e), ORB_ERR_HIP;
    if (c->upload_stream && __atomic_load_n(c->h_flags + 63, __ATOMIC_ACQUIRE)) {
        c->h_flags[63] = 0;
        return set_error("streamed image upload timed out", hipSuccess), ORB_ERR_INTERNAL;
    }
    if (hcnt[1]) {
        set_error("octree node table overflow (raise nfeatures capacity)", hipSuccess);
        return ORB_ERR_INTERNAL;
    }
    const int nk = hcnt[0];
    if (nk > cap || !kps || !desc) {
        *n = nk;
        set_error("orb_extract: output capacity too small", hipSuccess);
        return ORB_ERR_CAPACITY;
    }
    if (nk > 0) {
        std::memcpy(kps, hk, (size_t)nk * sizeof(orb_keypoint));
        std::memcpy(desc, hd, (size_t)nk * 32);
    }
    *n = nk;
    return ORB_OK;
}

static int level_view(Ctx* c, int frame, int level, uint8_t* dst, int* w, int* hgt) {
    if (!c->have_geom || frame < 0 || frame >= c->last_nframes || level < 0 || level >= c->geom.nlevels)
        return set_error("no such level/frame", hipSuccess), ORB_ERR_ARG;
    const LevelGeom& L = c->geom.L[level];
    *w = L.w;
    *hgt = L.h;
    if (!dst) return ORB_OK;
    hipError_t e;
    if (level == 0)
        e = hipMemcpy2DAsync(dst, L.w, c->last_frames + frame * c->last_frame_pitch, c->last_row_stride, L.w, L.h,
                             hipMemcpyDeviceToHost, c->stream);
    else
        e = hipMemcpy2DAsync(dst, L.w, c->d_pyr + frame * c->geom.pyr_bytes + L.pyr_off, L.pitch, L.w, L.h,
                             hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return set_error("download level", e), ORB_ERR_HIP;
    return ORB_OK;
}

int orb_get_level(orb_ctx* h, int level, const uint8_t** data, int* w, int* hgt, size_t* stride) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    if (!data || !w || !hgt) return ORB_ERR_ARG;
    int lw, lh;
    int st = level_view(c, 0, level, nullptr, &lw, &lh);
    if (st != ORB_OK) return st;
    if (!(c->level_cache_valid & (1u << level))) {
        c->level_host[level].resize((size_t)lw * lh);
        if ((st = level_view(c, 0, level, c->level_host[level].data(), &lw, &lh)) != ORB_OK) return st;
        c->level_cache_valid |= 1u << level;
    }
    *data = c->level_host[level].data();
    *w = lw;
    *hgt = lh;
    if (stride) *stride = (size_t)lw;
    return ORB_OK;
}

int orb_debug_fast_stamps(orb_ctx* h, uint64_t* out, int cap) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    if (c->flow_stamps && c->d_flow_stamps) {   // the dataflow launch's per-task stamps
        const int n = std::min((int)c->flow_stamps_cap, cap);
        hipError_t e = hipMemcpy(out, c->d_flow_stamps, (size_t)n * 8, hipMemcpyDeviceToHost);
        return e == hipSuccess ? n : ORB_ERR_HIP;
    }
    if (!c->fast_stamps || !c->d_stamps) return 0;
    const int n = std::min((int)c->stamps_cap, cap);
    hipError_t e = hipMemcpy(out, c->d_stamps, (size_t)n * 8, hipMemcpyDeviceToHost);
    return e == hipSuccess ? n : ORB_ERR_HIP;
}

int orb_debug_sincosf(orb_ctx* h, const float* x, int n, float* s, float* c) {
    Ctx* ctx = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(ctx);
    if (n < 0 || (n > 0 && (!x || !s || !c))) return set_error("orb_debug_sincosf: bad arguments", hipSuccess), ORB_ERR_ARG;
    if (n == 0) return ORB_OK;
    float* d = nullptr;
    hipError_t e = hipMalloc((void**)&d, (size_t)n * 12);
    if (e != hipSuccess) return set_error("hipMalloc", e), ORB_ERR_NOMEM;
    if ((e = hipMemcpyAsync(d, x, (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream)) == hipSuccess &&
        (e = launch_debug_sincosf(d, n, d + n, d + 2 * (size_t)n, ctx->stream)) == hipSuccess &&
        (e = hipMemcpyAsync(s, d + n, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream)) == hipSuccess &&
        (e = hipMemcpyAsync(c, d + 2 * (size_t)n, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream)) == hipSuccess)
        e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(d);
    return e == hipSuccess ? ORB_OK : (set_error("orb_debug_sincosf", e), ORB_ERR_HIP);
}

int orb_debug_level_image(orb_ctx* h, int frame, int level, uint8_t* out, int* w, int* hgt) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    return level_view(c, frame, level, out, w, hgt);
}

int orb_debug_candidates(orb_ctx* h, int frame, int level, int* out, int cap) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    if (!c->have_geom || frame < 0 || frame >= c->last_nframes || level < 0 || level >= c->geom.nlevels)
        return ORB_ERR_ARG;
    const LevelGeom& L = c->geom.L[level];
    const int ncl = L.nCols * L.nRows;
    std::vector<uint32_t> slots((size_t)L.cand_cap), rec((size_t)ncl * kCandRec);   // [count | first corners]
    hipError_t e;
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess ||
        (e = hipMemcpy(rec.data(), c->d_candFirst + ((size_t)frame * c->geom.ncells + L.cell_base) * kCandRec,
                       rec.size() * sizeof(uint32_t), hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(slots.data(), c->d_cands + (size_t)frame * c->geom.ncand + L.cand_base,
                       slots.size() * sizeof(uint32_t), hipMemcpyDeviceToHost)) != hipSuccess)
        return set_error("download candidates", e), ORB_ERR_HIP;
    int n = 0;
    for (int i = 0; i < ncl; i++)
        for (int k = 0; k < (int)rec[(size_t)i * kCandRec]; k++) {
            const uint32_t v = k < kCandFirst ? rec[(size_t)i * kCandRec + 1 + k] : slots[(size_t)i * L.cell_cap + k];
            if (n < cap && out) {
                out[3 * n] = v & 0xFFF;
                out[3 * n + 1] = (v >> 12) & 0xFFF;
                out[3 * n + 2] = v >> 24;
            }
            n++;
        }
    return n > cap ? -n - 1 : n;
}

int orb_debug_level_keypoints(orb_ctx* h, int frame, int level, int* out, int cap) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    if (!c->have_geom || frame < 0 || frame >= c->last_nframes || level < 0 || level >= c->geom.nlevels)
        return ORB_ERR_ARG;
    const LevelGeom& L = c->geom.L[level];
    int n = 0;
    std::vector<uint32_t> v((size_t)L.kp_cap);
    hipError_t e;
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess ||
        (e = hipMemcpy(&n, c->d_lvlCount + (size_t)frame * c->geom.nlevels + level, sizeof(int),
                       hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(v.data(), c->d_lvlKps + (size_t)frame * c->geom.nkpcap + L.kp_base, v.size() * 4,
                       hipMemcpyDeviceToHost)) != hipSuccess)
        return set_error("download level keypoints", e), ORB_ERR_HIP;
    if (n > cap) return -n - 1;
    for (int i = 0; i < n; i++) {
        out[3 * i] = v[i] & 0xFFF;
        out[3 * i + 1] = (v[i] >> 12) & 0xFFF;
        out[3 * i + 2] = v[i] >> 24;
    }
    return n;
}

void* orb_device_alloc(orb_ctx* h, size_t bytes) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    if (!c || hipSetDevice(c->device) != hipSuccess) return nullptr;
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 1);
    if (e != hipSuccess) {
        set_error("hipMalloc", e);
        return nullptr;
    }
    return p;
}

int orb_device_free(orb_ctx* h, void* p) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    hipError_t e = hipFree(p);
    return e == hipSuccess ? ORB_OK : (set_error("hipFree", e), ORB_ERR_HIP);
}

int orb_memcpy_h2d(orb_ctx* h, void* dst, const void* src, size_t bytes) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return e == hipSuccess ? ORB_OK : (set_error("h2d", e), ORB_ERR_HIP);
}

int orb_memcpy_d2h(orb_ctx* h, void* dst, const void* src, size_t bytes) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return e == hipSuccess ? ORB_OK : (set_error("d2h", e), ORB_ERR_HIP);
}

int orb_memset_device(orb_ctx* h, void* dst, int value, size_t bytes) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    hipError_t e = hipMemsetAsync(dst, value, bytes, c->stream);
    return e == hipSuccess ? ORB_OK : (set_error("memset", e), ORB_ERR_HIP);
}

int orb_profile_enable(orb_ctx* h, int on) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    (void)hipStreamSynchronize(c->stream);
    for (auto& pr : c->prof_pairs) {
        (void)hipEventDestroy(pr.b);
        (void)hipEventDestroy(pr.e);
    }
    c->prof_pairs.clear();
    c->prof_on = on != 0;
    return ORB_OK;
}

int orb_profile_read(orb_ctx* h, double* ms_total, int* launches) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return set_error("sync", e), ORB_ERR_HIP;
    for (int k = 0; k < ORB_K_COUNT; k++) {
        if (ms_total) ms_total[k] = 0;
        if (launches) launches[k] = 0;
    }
    for (auto& pr : c->prof_pairs) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, pr.b, pr.e) != hipSuccess) continue;
        if (ms_total) ms_total[pr.id] += ms;
        if (launches) launches[pr.id] += 1;
    }
    return ORB_OK;
}

}  // extern "C"
