// cista_abi.hip -- C ABI (include/cista_lstc.h) of the MI355X CISTA-LSTC hot path:
// parameter packing, workspace carving, per-layer launch configuration and the per-frame
// schedule of CistaLSTCNet.forward (reference e2v/e2v_model.py:41-90).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "../../include/cista_lstc.h"
#include "cista_kernels.hpp"
#include "cista_backward.hpp"

using namespace cista;

namespace {

constexpr size_t ALIGN = 256;
inline size_t align_up(size_t x) { return (x + ALIGN - 1) & ~(ALIGN - 1); }

// ---------------------------------------------------------------------------------------
// packed parameter blob layout
// ---------------------------------------------------------------------------------------
enum ConvId { CV_W0, CV_P0, CV_GATES, CV_OUTG, CV_D, CV_P, CV_DG, CV_LSTM, CV_UP, CV_IN, CV_UP4, CV_COUNT };

struct ConvShape { int cout, cin, G; };

ConvShape conv_shape(int id, int C) {
    switch (id) {
        case CV_W0: return {C, C, 1};
        case CV_P0: return {2 * C, C, 1};
        case CV_GATES: return {4 * C, 3 * C, 2};     // (in, forget)           base_layers.py:58
        case CV_OUTG: return {2 * C, 4 * C, 1};
        case CV_D: return {C, 2 * C, 1};
        case CV_P: return {2 * C, C, 1};
        case CV_DG: return {C, 2 * C, 1};
        case CV_LSTM: return {4 * C, 2 * C, 4};      // (in, remember, out, cell) base_layers.py:116
        case CV_IN: return {C, 32, 1};               // composed input stage + W0 over the s2d input
        case CV_UP4: return {4 * C, C, 1};           // phase-decomposed upsample conv (4 phases x C)
        default: return {C, C, 1};                   // CV_UP
    }
}

struct Layout {
    size_t wp[CV_COUNT], bp[CV_COUNT], sc[CV_COUNT];
    size_t dwp[CV_COUNT], dbp[CV_COUNT];   // dgrad B fragments (flipped, transposed) + zero bias
    size_t wE, wI, bIn, wF, bF, lambda, wC, bC, wS, bS, wU4, bU4;
    size_t w4p, b4p;                       // W0 dgrad as a four-phase conv (pack_w0phase_kernel)
    size_t wsp;                            // weight |max| partials of the pack (weight_absmax_kernel)
    size_t total;
};

Layout make_layout(const cista_config &cfg) {
    Layout L;
    const int C = cfg.base_channels, nb = cfg.num_bins;
    size_t off = 0;
    for (int i = 0; i < CV_COUNT; ++i) {
        const ConvShape s = conv_shape(i, C);
        L.wp[i] = off;
        off = align_up(off + (size_t)(s.cin / 32) * 9 * (s.cout / 16) * 2 * 64 * 16);
        L.bp[i] = off;
        off = align_up(off + (size_t)s.cout * 4);
        L.sc[i] = off;
        off = align_up(off + 8);
    }
    for (int i = 0; i < CV_COUNT; ++i) {
        const ConvShape s = conv_shape(i, C);
        L.dwp[i] = off;
        off = align_up(off + (size_t)(s.cout / 32) * 9 * (s.cin / 16) * 2 * 64 * 16);
        L.dbp[i] = off;
        off = align_up(off + (size_t)s.cin * 4);
    }
    L.wE = off; off = align_up(off + (size_t)nb * 9 * (C / 2) * 4);
    L.wI = off; off = align_up(off + (size_t)9 * (C / 2) * 4);
    L.bIn = off; off = align_up(off + (size_t)C * 4);
    L.wF = off; off = align_up(off + (size_t)9 * C * 4);
    L.bF = off; off = align_up(off + 4);
    L.lambda = off; off = align_up(off + (size_t)2 * C * 4);
    L.wC = off; off = align_up(off + (size_t)9 * 25 * (nb + 1) * C * 4);   // fused input + W0
    L.bC = off; off = align_up(off + (size_t)C * 4);
    L.wS = off; off = align_up(off + (size_t)C * 32 * 9 * 4);            // CV_IN, reference layout
    L.bS = off; off = align_up(off + (size_t)C * 4);
    L.wU4 = off; off = align_up(off + (size_t)4 * C * C * 9 * 4);        // CV_UP4, reference layout
    L.bU4 = off; off = align_up(off + (size_t)4 * C * 4);
    L.w4p = off; off = align_up(off + (size_t)(C / 32) * 9 * (4 * C / 16) * 2 * 64 * 16);
    L.b4p = off; off = align_up(off + (size_t)4 * C * 4);
    L.wsp = off; off = align_up(off + (size_t)CV_COUNT * WS_PARTS * 4);
    L.total = off;
    return L;
}

bool cfg_ok(const cista_config *cfg) {
    return cfg && cfg->base_channels > 0 && cfg->depth >= 0 && cfg->num_bins >= 1;
}
bool cfg_supported(const cista_config *cfg) { return cfg->base_channels % 32 == 0; }

template <class T> inline const T *blob(const void *p, size_t off) {
    return reinterpret_cast<const T *>(static_cast<const char *>(p) + off);
}
template <class T> inline T *blobw(void *p, size_t off) {
    return reinterpret_cast<T *>(static_cast<char *>(p) + off);
}

// ---------------------------------------------------------------------------------------
// workspace
// ---------------------------------------------------------------------------------------
struct Workspace {
    float *full;   // (B,H,W,C): x_full = cat(We, Wi), later u = relu(upsamp_conv)
    float *x1;     // (B,h,w,C)
    float *z0;     // (B,h,w,2C)
    float *xb;     // (B,h,w,C): ISTA x = x1 - D(z); later Dg output y
    size_t bytes;
};

// every workspace (inference, training forward, backward) starts with this reserved header:
// (reserved: ABI versions <= 2 kept a range flag there), which no carve hands out as scratch
constexpr size_t WS_HEADER = ALIGN;

Workspace carve(void *ws, int B, int H, int W, int C) {
    const size_t hw = (size_t)(H / 2) * (W / 2);
    Workspace w;
    size_t off = WS_HEADER;
    char *base = static_cast<char *>(ws);
    w.full = reinterpret_cast<float *>(base + off); off = align_up(off + (size_t)B * H * W * C * 4);
    w.x1 = reinterpret_cast<float *>(base + off); off = align_up(off + (size_t)B * hw * C * 4);
    w.z0 = reinterpret_cast<float *>(base + off); off = align_up(off + (size_t)B * hw * 2 * C * 4);
    w.xb = reinterpret_cast<float *>(base + off); off = align_up(off + (size_t)B * hw * C * 4);
    w.bytes = off;
    return w;
}

// ---------------------------------------------------------------------------------------
// tile selection
// ---------------------------------------------------------------------------------------
// mseg: 0 = the workgroup's pixels fill its 16-pixel m-tiles in row-major order; > 0 = every
// tile row is cut into mseg row-aligned m-tiles (the last one partly idle), see ConvArgs.mseg
struct Tile { int TH, TW, ty, tx; size_t lds; int mseg; };

size_t lds_bytes(int TH, int TW, int S) {
    const int HP = ((TH - 1) * S + 3) * ((TW - 1) * S + 3);
    return (size_t)((HP + 15) & ~15) * 8 * 16;
}

// One tile candidate: TW columns, row-major m-tiles (mode 0) or row-aligned m-tile segments
// (mode 1), as many rows as the workgroup's pixels, the staging registers (max_items: halo
// items, HP rounded to 8, x4 k-groups, one workgroup may hold; 0 = unlimited) and the LDS
// (nbuf images, occ workgroups per CU) allow.  False if the width admits no tile.
bool tile_candidate(int Hout, int Wout, int block_px, int S, int max_items, int nbuf, int occ, int TW, int mode,
                    Tile &t, int &conf) {
    const int mseg = mode ? (TW + 15) / 16 : 0;
    if (mode && TW % 16 == 0) return false;               // same as row-major
    int TH = mode ? (block_px / 16) / mseg : block_px / TW;
    if (TH > Hout) TH = Hout;
    if (TH < 1) return false;
    auto items = [&](int th) { return ((((th - 1) * S + 3) * ((TW - 1) * S + 3) + 7) & ~7) * 4; };
    while (max_items && TH > 1 && items(TH) > max_items) --TH;
    if (max_items && items(TH) > max_items) return false;
    // the kernel's small_div range (ConvArgs.rcp_pitch, the halo coordinates): halo < 2048
    // pixels, pitch and halo width <= 512 -- a tile outside it is never ranked (launch_conv_cfg
    // would refuse it)
    if (((TH - 1) * S + 3) * ((TW - 1) * S + 3) >= 2048 || (mode ? 16 * mseg : TW) > 512 || (TW - 1) * S + 3 > 512)
        return false;
    const size_t lds = lds_bytes(TH, TW, S) * nbuf;
    if (lds > 160 * 1024 / (size_t)occ) return false;
    t = Tile{TH, TW, (Hout + TH - 1) / TH, (Wout + TW - 1) / TW, lds, mseg};
    // row-major m-tiles that wrap a tile row put two halo rows' slots in one lane group
    conf = (S == 1 && (mode || TW % 16 == 0)) ? 0 : 1;
    return true;
}

// max_items, nbuf, occ: tile_candidate; seg: row-aligned m-tiles allowed (stride-1 stagings).
// Ranking: pixel efficiency (useful / computed pixels) first; at equal efficiency a layout whose
// m-tile A-fragment reads are bank-conflict free (each m-tile's 16 lanes in one halo row:
// ds_read_b128 serves 16 lanes of 16 contiguous slots per cycle), then the smaller LDS image.
// halo_w > 0: rank by cost per useful output pixel instead, tiles x (block_px + halo_w x halo
// pixels) x (1 + 0.05 if the m-tile reads are bank-conflicted): the training dgrads (2-chunk K
// loops at B = 8) otherwise took 48 x 2 tiles (96 px, a 200-pixel halo, conflicted reads) for
// their 96-pixel workgroups
Tile choose_tile(int Hout, int Wout, int block_px, int S, int max_items, int nbuf, int occ = 2, bool seg = false,
                 double halo_w = 0.0) {
    Tile best{1, 1, Hout, Wout, 0, 0};
    double best_eff = -1.0, best_cost = 1e300;
    int best_conf = 1;
    size_t best_lds = ~(size_t)0;
    for (int mode = 0; mode < (seg ? 2 : 1); ++mode)
    for (int TW = 1; TW <= block_px && TW <= Wout; ++TW) {
        Tile t;
        int conf;
        if (!tile_candidate(Hout, Wout, block_px, S, max_items, nbuf, occ, TW, mode, t, conf)) continue;
        const double eff = (double)Hout * Wout / ((double)t.ty * t.tx * block_px);
        bool better;
        double cost = 0.0;
        if (halo_w > 0.0) {
            const double hp = (double)((t.TH - 1) * S + 3) * ((TW - 1) * S + 3);
            cost = (double)t.ty * t.tx * (block_px + halo_w * hp) * (conf ? 1.05 : 1.0) / ((double)Hout * Wout);
            better = cost < best_cost - 1e-9 || (cost < best_cost + 1e-9 && t.lds < best_lds);
        } else {
            better = eff > best_eff + 1e-9 ||
                     (eff > best_eff - 1e-9 && (conf < best_conf || (conf == best_conf && t.lds < best_lds)));
        }
        if (better) {
            best_eff = eff;
            best_cost = cost;
            best_conf = conf;
            best_lds = t.lds;
            best = t;
        }
    }
    return best;
}

// Two-region tiling.  No rectangle of a 192-pixel workgroup tiles 90 x 120 exactly (the best,
// 6 x 32 or 6 x 30 in row segments, computes 0.9375 useful pixels per slot: every row of tiles
// ends in a partly idle tile).  Columns [0, wa) are cut into an exact multiple of one tile width
// (region a) and the strip [wa, Wout) gets its own tile shape (region b); both run in one launch,
// region b's items after region a's: 54 + 3 = 57 tiles per 90 x 120 image instead of 60 (0.987),
// the 96-pixel convs 105 + 8 = 113 instead of 115.  Only where the launch is at least two
// dispatch rounds (B x tiles >= 1024 items on 512 workgroup slots): a one-round launch takes one
// workgroup lifetime whatever its item count.  Memoised per shape in a 64-entry table with
// round-robin replacement (a process serving many resolutions re-plans a shape it evicted,
// ~0.1 ms of host time, instead of re-planning every unseen shape forever); use_cache = false
// (cista_tile_plan introspection) neither reads nor fills it.
struct TilePlan { Tile a, b; int wa; };   // b.tx == 0: one region (a covers every column)

TilePlan plan_tiles(int B, int Hout, int Wout, int block_px, int S, int max_items, int nbuf, int occ, bool seg,
                    double halo_w, bool use_cache = true) {
    TilePlan best{choose_tile(Hout, Wout, block_px, S, max_items, nbuf, occ, seg, halo_w), Tile{}, Wout};
    if (halo_w > 0.0 || (long)B * best.a.ty * best.a.tx < 1024) return best;
    struct Key { int Hout, Wout, block_px, S, max_items, nbuf, occ, seg; };
    struct Ent { Key k; TilePlan p; };
    static std::mutex mu;
    constexpr int NCACHE = 64;
    static Ent cache[NCACHE];
    static int ncache = 0, next = 0;
    const Key key{Hout, Wout, block_px, S, max_items, nbuf, occ, seg ? 1 : 0};
    if (use_cache) {
        std::lock_guard<std::mutex> lock(mu);
        for (int i = 0; i < ncache; ++i)
            if (!memcmp(&cache[i].k, &key, sizeof(Key))) return cache[i].p;
    }
    // ranked by tiles per image, then by tiles whose m-tile reads are bank-conflicted (weighting
    // those 1.05, as the dgrad ranking does, kept the 192-pixel convs at one region: 8410 / 8376
    // frames/s against 8566 / 8541 unweighted, same box)
    long best_tiles = (long)best.a.ty * best.a.tx, best_conf = 0;
    {
        Tile t;
        int conf = 0;
        if (tile_candidate(Hout, Wout, block_px, S, max_items, nbuf, occ, best.a.TW, best.a.mseg ? 1 : 0, t, conf))
            best_conf = conf ? best_tiles : 0;
    }
    for (int mode = 0; mode < (seg ? 2 : 1); ++mode)
        for (int TW = 1; TW <= block_px && TW < Wout; ++TW) {
            const int wa = (Wout / TW) * TW;
            if (wa == Wout) continue;
            Tile ta, tb;
            int ca, cb;
            if (!tile_candidate(Hout, wa, block_px, S, max_items, nbuf, occ, TW, mode, ta, ca)) continue;
            tb = choose_tile(Hout, Wout - wa, block_px, S, max_items, nbuf, occ, seg, 0.0);
            if (!tile_candidate(Hout, Wout - wa, block_px, S, max_items, nbuf, occ, tb.TW, tb.mseg ? 1 : 0, tb, cb))
                continue;
            const long tiles = (long)ta.ty * ta.tx + (long)tb.ty * tb.tx;
            const long conf = (ca ? (long)ta.ty * ta.tx : 0) + (cb ? (long)tb.ty * tb.tx : 0);
            if (tiles < best_tiles || (tiles == best_tiles && conf < best_conf)) {
                best_tiles = tiles;
                best_conf = conf;
                best = TilePlan{ta, tb, wa};
            }
        }
    if (!use_cache) return best;
    std::lock_guard<std::mutex> lock(mu);
    for (int i = 0; i < ncache; ++i)                 // another thread planned it meanwhile
        if (!memcmp(&cache[i].k, &key, sizeof(Key))) return cache[i].p;
    cache[next] = Ent{key, best};
    next = (next + 1) % NCACHE;
    if (ncache < NCACHE) ++ncache;
    return best;
}

// dynamic LDS above 64 KiB must be enabled per kernel (once; not a stream operation).  The
// ABI is reentrant: host threads launching concurrently share this table under a lock.
bool allow_big_lds(const void *kern) {
    static std::mutex mu;
    static const void *done[128];
    static int ndone = 0;
    std::lock_guard<std::mutex> lock(mu);
    for (int i = 0; i < ndone; ++i)
        if (done[i] == kern) return true;
    if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
        return false;
    if (ndone < 128) done[ndone++] = kern;
    return true;
}

// ---------------------------------------------------------------------------------------
// conv launch
// ---------------------------------------------------------------------------------------
// halo weight of the dgrad (STAGE_ZP2) tile ranking; CISTA_ZP2_HALO_W overrides it (A/B runs)
double zp2_halo_weight() {
    static const double w = [] {
        const char *e = getenv("CISTA_ZP2_HALO_W");
        return e ? atof(e) : 0.25;
    }();
    return w;
}

#if CISTA_STAMPS
// diagnostic builds only (scripts/dgrad_stamps.py): every EPI_FOLD launch after
// cista_debug_set_fold_stamps stamps into a region of its own, FOLD_STAMP_WG workgroups x 4
// waves x 24 slots, in launch order, until the ring is full
constexpr size_t FOLD_STAMP_WG = 2048;
std::mutex g_fold_mu;
unsigned long long *g_fold_ring = nullptr;
int g_fold_cap = 0, g_fold_next = 0;
unsigned long long *fold_stamp_region(unsigned nwg) {
    std::lock_guard<std::mutex> lock(g_fold_mu);
    if (!g_fold_ring || g_fold_next >= g_fold_cap || nwg > FOLD_STAMP_WG) return nullptr;
    return g_fold_ring + (size_t)(g_fold_next++) * FOLD_STAMP_WG * 4 * 24;
}
#endif

template <int MT_W, int NW, int WM, int WN, int STAGE, int EPI, int G, bool PF = false, int NI = 0, int OCC = 2>
int launch_conv_cfg(ConvArgs a, hipStream_t st) {
    constexpr int block_px = WM * MT_W * 16;
    constexpr int S = STAGE == STAGE_S2 ? 2 : 1;
    constexpr bool SEG = STAGE == STAGE_S1 || STAGE == STAGE_ZP2 || STAGE == STAGE_CLAMP || STAGE == STAGE_S2D;
    constexpr int NWV = WM * WN, NT = NWV * 64;     // waves, threads per workgroup
    // OCC = waves per SIMD the register budget is sized for (__launch_bounds__): OCC * 4 / NWV
    // workgroups share a CU's LDS
    constexpr bool SPLIT_OK = (STAGE == STAGE_S1 || STAGE == STAGE_S2D || STAGE == STAGE_UP || STAGE == STAGE_CLAMP) &&
                              EPI != EPI_FOLD;
    TilePlan plan{choose_tile(a.Hout, a.Wout, block_px, S, NI ? NI * NT : 0, NI ? 2 : 1, OCC * 4 / NWV, SEG,
                              STAGE == STAGE_ZP2 ? zp2_halo_weight() : 0.0),
                  Tile{}, a.Wout};
    if (SPLIT_OK && a.border == 0)
        plan = plan_tiles(a.B, a.Hout, a.Wout, block_px, S, NI ? NI * NT : 0, NI ? 2 : 1, OCC * 4 / NWV, SEG, 0.0);
    if (a.border == 1)          // rows 0 and Hout-1 in 1-row tiles
        plan.a = Tile{1, block_px, 2, (a.Wout + block_px - 1) / block_px, lds_bytes(1, block_px, S), 0};
    else if (a.border == 2)     // columns 0 and Wout-1 in 1-column tiles
        plan.a = Tile{block_px, 1, (a.Hout + block_px - 1) / block_px, 2, lds_bytes(block_px, 1, S), 0};
    constexpr int nblk_cols = WN * NW * 16;
    if (a.N % nblk_cols) return CISTA_ERR_UNSUPPORTED;
    // the training variant (SV) only for epilogues that save activations, and only when asked
    constexpr bool HAS_SV = EPI == EPI_ISTA_P || EPI == EPI_LSTC_CELL || EPI == EPI_LSTC_OUT || EPI == EPI_LSTM;
    auto kern = conv3x3_split3<MT_W, NW, WM, WN, STAGE, EPI, G, PF, NI, false, OCC>;
    if constexpr (HAS_SV)
        if ((EPI == EPI_LSTM ? a.out2 : a.out1) != nullptr)
            kern = conv3x3_split3<MT_W, NW, WM, WN, STAGE, EPI, G, PF, NI, true, OCC>;
    if (!allow_big_lds((const void *)kern)) return CISTA_ERR_HIP;
    // the epilogue indexes outputs with 32-bit element offsets (pixel * Cout, x4 for out2)
    // and the double-buffered staging reads inputs with 32-bit element offsets
    if ((long long)a.B * a.Hout * a.Wout * a.Cout * (a.out2 || EPI == EPI_PH4 ? 4 : 1) >= (1LL << 31))
        return CISTA_ERR_UNSUPPORTED;
    if ((long long)a.B * a.Hin * a.Win * (a.c0 > a.c1 ? a.c0 : a.c1) >= (1LL << 31)) return CISTA_ERR_UNSUPPORTED;
    // the epilogue's LDS: the pixel table (MT_W x WM x 16 ints), or the final-conv weights of the
    // upsample epilogues (9 x Cout floats)
    const size_t epi_lds = (size_t)MT_W * WM * 16 * 4 > (size_t)9 * a.Cout * 4 ? (size_t)MT_W * WM * 16 * 4
                                                                                 : (size_t)9 * a.Cout * 4;
    // EPI_FOLD: a wave's columns must lie in one FoldSeg
    if (EPI == EPI_FOLD && a.fsplit % (NW * 16)) return CISTA_ERR_UNSUPPORTED;
    // + 3 x NWV words of range-pass scratch (overflow bits, max, min) right after the epilogue's
    // LDS (inside the dead staging images when those are larger)
    a.lds_flag = (int)(epi_lds / 4);
    // one launch; region b's items (plan_tiles: columns [wa, Wout)) follow region a's
    auto geom_ok = [&](const Tile &t) {
        // small_div's range: halo pixels < 2048, pitch and halo width <= 512
        const int pitch = t.mseg ? 16 * t.mseg : t.TW;
        return ((t.TH - 1) * S + 3) * ((t.TW - 1) * S + 3) < 2048 && pitch <= 512 && (t.TW - 1) * S + 3 <= 512;
    };
    if (!geom_ok(plan.a) || (plan.b.tx && !geom_ok(plan.b))) return CISTA_ERR_UNSUPPORTED;
    a.ox_base = 0;
    a.TH = plan.a.TH;
    a.TW = plan.a.TW;
    a.pitch = plan.a.mseg ? 16 * plan.a.mseg : plan.a.TW;
    a.rcp_pitch = 1.0f / (float)a.pitch;
    a.tiles_y = plan.a.ty;
    a.tiles_x = plan.a.tx;
    a.tiles_x_b = plan.b.tx;               // 0: one region
    a.tiles_y_b = plan.b.ty;
    a.TH_b = plan.b.TH;
    a.TW_b = plan.b.TW;
    a.pitch_b = plan.b.mseg ? 16 * plan.b.mseg : plan.b.TW;
    a.rcp_pitch_b = plan.b.tx ? 1.0f / (float)a.pitch_b : 0.0f;
    a.wa = plan.wa;
    const long tiles = (long)plan.a.ty * plan.a.tx + (long)plan.b.ty * plan.b.tx;
#if CISTA_XCD
    dim3 grid((unsigned)((long)a.B * tiles * (a.N / nblk_cols)));   // 1-D, XCD-aware order in the kernel
#else
    dim3 grid((unsigned)((long)a.B * tiles), (unsigned)(a.N / nblk_cols));
#endif
    const size_t tlds = plan.b.lds > plan.a.lds ? plan.b.lds : plan.a.lds;
    const size_t lds = tlds > epi_lds + 12 * NWV ? tlds : epi_lds + 12 * NWV;
#if CISTA_STAMPS
    a.stamps = nullptr;
    if constexpr (EPI == EPI_FOLD) a.stamps = fold_stamp_region(grid.x * grid.y);
#endif
    hipLaunchKernelGGL(kern, grid, dim3(NT), lds, st, a);
    if (hipGetLastError() != hipSuccess) return CISTA_ERR_HIP;
    return CISTA_OK;
}

// pick the wave tiling from the number of packed output columns: the direct stagings (reflect /
// zero / space-to-depth) run the double-buffered K loop (the next halo chunk prefetched into
// registers, B-fragment prefetch); the bilinear staging of C not in {32, 64} a single-buffered one
#ifndef CISTA_SMALL_GRID
#define CISTA_SMALL_GRID 1   // latency tiles for grids that would not fill the chip (small B)
#endif
#ifndef CISTA_W0_PHASE
#define CISTA_W0_PHASE 1         // W0's dgrad as a four-phase MFMA conv (0: the VALU dgrad_s2_kernel)
#endif
// fewer than ~1.5 workgroups per CU with the throughput configuration (px x cols per WG)
inline bool small_grid(const ConvArgs &a, int wg_px, int wg_cols, int limit = 384) {
#if CISTA_SMALL_GRID
    const long px = (long)a.B * a.Hout * a.Wout;
    return ((px + wg_px - 1) / wg_px) * ((a.N + wg_cols - 1) / wg_cols) < limit;
#else
    (void)a; (void)wg_px; (void)wg_cols;
    return false;
#endif
}

template <int STAGE, int EPI, int G>
int launch_conv(const ConvArgs &a, hipStream_t st) {
    if constexpr (STAGE == STAGE_S2) {
        if (a.N % 64 == 0) return launch_conv_cfg<2, 4, 4, 1, STAGE, EPI, G>(a, st);
        if (a.N % 32 == 0) return launch_conv_cfg<2, 2, 4, 1, STAGE, EPI, G>(a, st);
        return CISTA_ERR_UNSUPPORTED;
    } else if constexpr (EPI == EPI_UP4_Q || EPI == EPI_UP4_Q_SAVE) {
        // one wave per phase (NW * 16 == C columns), 96 half-res pixels x 4 phases per workgroup
        if (a.N == 256 && a.Cout == 64) return launch_conv_cfg<6, 4, 1, 4, STAGE, EPI, G, true, 4>(a, st);
        return CISTA_ERR_UNSUPPORTED;
    } else if constexpr (EPI == EPI_UP_Q || EPI == EPI_UP_Q_SAVE) {      // needs WN == 1
        if (a.N == 64) return launch_conv_cfg<8, 4, 4, 1, STAGE, EPI, G>(a, st);
        if (a.N == 32) return launch_conv_cfg<8, 2, 4, 1, STAGE, EPI, G>(a, st);
        return CISTA_ERR_UNSUPPORTED;
    } else if constexpr (STAGE == STAGE_S1 || STAGE == STAGE_ZP2 || STAGE == STAGE_S2D) {
        // double-buffered K loop, 192-pixel workgroups, halo items in 4 x 8 VGPRs per thread
        constexpr bool FWD = STAGE == STAGE_S1 || STAGE == STAGE_S2D;
        if constexpr (FWD) {
            // small batches (B = 1 is the reference harness's case): the throughput tiles below
            // leave most CUs idle, so 64-pixel x 64-column workgroups trade MFMA efficiency
            // for 3-6x more of them (latency per frame)
            const int big_px = a.N % 256 == 0 ? 96 : 192, big_cols = a.N % 256 == 0 ? 256 : a.N % 128 == 0 ? 128 : 64;
            if (a.N % 64 == 0 && small_grid(a, big_px, big_cols)) {
                if constexpr (G == 4) return launch_conv_cfg<1, 4, 4, 1, STAGE, EPI, G, true, 2>(a, st);
                else return launch_conv_cfg<2, 2, 2, 2, STAGE, EPI, G, true, 2>(a, st);
            }
        }
        if constexpr (FWD)      // one workgroup holds all 256 columns, 96 pixels
            if (a.N % 256 == 0) return launch_conv_cfg<6, 4, 1, 4, STAGE, EPI, G, true, 4>(a, st);
        if constexpr (G == 4) {
            if (a.N % 128 == 0) return launch_conv_cfg<6, 4, 2, 2, STAGE, EPI, G, true, 4>(a, st);
        } else {
            if (a.N % 128 == 0) return launch_conv_cfg<12, 2, 1, 4, STAGE, EPI, G, true, 4>(a, st);
            if (a.N % 64 == 0) return launch_conv_cfg<6, 2, 2, 2, STAGE, EPI, G, true, 4>(a, st);
            if (a.N % 32 == 0) return launch_conv_cfg<3, 2, 4, 1, STAGE, EPI, G, true, 4>(a, st);   // N = 32, 96, 160 ...
        }
        return CISTA_ERR_UNSUPPORTED;
    } else if constexpr (G <= 2) {      // STAGE_UP + EPI_RELU (upsample conv of C not in {32, 64})
        if (a.N % 128 == 0) return launch_conv_cfg<12, 2, 1, 4, STAGE, EPI, G, true>(a, st);
        if (a.N % 64 == 0) return launch_conv_cfg<12, 2, 2, 2, STAGE, EPI, G, true>(a, st);
        if (a.N % 32 == 0) return launch_conv_cfg<12, 2, 4, 1, STAGE, EPI, G, true>(a, st);
        return CISTA_ERR_UNSUPPORTED;
    } else {
        return CISTA_ERR_UNSUPPORTED;
    }
}

ConvArgs conv_args(const void *packed, const Layout &L, int id, int C, int B, int Hin, int Win,
                   int Hout, int Wout, const float *in0, int c0, const float *in1, int c1) {
    ConvArgs a;
    memset(&a, 0, sizeof(a));
    const ConvShape s = conv_shape(id, C);
    a.in0 = in0; a.c0 = c0; a.in1 = in1; a.c1 = c1;
    a.B = B; a.Hin = Hin; a.Win = Win; a.Hout = Hout; a.Wout = Wout;
    a.wpack = blob<u32x4>(packed, L.wp[id]);
    a.bias = blob<float>(packed, L.bp[id]);
    a.wscale = blob<float>(packed, L.sc[id]) + 1;
    a.N = s.cout;
    a.Cout = s.cout / s.G;
    return a;
}

#define CHECK(x)                          \
    do {                                  \
        int _s = (x);                     \
        if (_s != CISTA_OK) return _s;    \
    } while (0)
// a gradient-scale pair that could not be produced (pairs used up, or the launch failed) must
// not reach a kernel as a NULL scale pointer
#define CHECK_PTR(p)                                  \
    do {                                              \
        if ((p) == nullptr) return CISTA_ERR_HIP;     \
    } while (0)

bool overlaps(const void *a, size_t na, const void *b, size_t nb) {
    if (!a || !b) return false;
    const char *pa = static_cast<const char *>(a), *pb = static_cast<const char *>(b);
    return pa < pb + nb && pb < pa + na;
}

// ------------------------------------------ frame schedule -----------------------------
// Every buffer one frame touches; the stage entries point some of them at caller memory.
struct Frame {
    const cista_config *cfg;
    const void *packed;
    Layout L;
    int B, H, W, h, w, C;
    const float *events, *prev_image;                  // NCHW inputs
    const float *c_lstc_prev, *z_prev, *h_prev, *c_prev;  // NHWC states (NULL = None)
    float *full;    // x_full = cat(We, Wi) / u = relu(upsamp_conv)   (B,H,W,C)
    float *x1;      // W0 output                                       (B,h,w,C)
    float *z0;      // P0.P0 output                                    (B,h,w,2C)
    float *xb;      // ISTA x = x1 - D(z); later Dg output y           (B,h,w,C)
    float *c_lstc;  // ConvLSTC cell                                   (B,h,w,2C)
    float *z;       // LSTC output, then ISTA iterate (in place)       (B,h,w,2C)
    float *hs, *cs; // ConvLSTM state                                  (B,h,w,C)
    float *rec, *pre;
    // training forward: activations saved for the backward (all NULL at inference)
    float *gi, *gf, *go;   // ConvLSTC gates (sigmoid)                    (B,h,w,2C) each
    float *zl;             // depth x ISTA z_k, z_0 = ConvLSTC output      (B,h,w,2C)
    float *v;              // depth x pre-softshrink ISTA values          (B,h,w,2C)
    float *xs;             // depth x ISTA x_k = x1 - D(z_k)              (B,h,w,C)
    float *y;              // relu(Dg.conv(z))                            (B,h,w,C)
    float *lg;             // ConvLSTM gates (i, r, o, g) post-activation (B,h,w,4C)
    float *u;              // relu(upsamp_conv(...))                      (B,H,W,C)
    bool need_full;        // the input stage must write x_full (the backward's recompute)
    hipStream_t st;
};

// input stage and W0 as one composed linear map (input_w0_kernel) for 1..8 bins
#ifndef CISTA_FUSED_IN
#define CISTA_FUSED_IN 1
#endif
constexpr size_t IN_TILE_LDS = 160 * 1024;   // input-stage transpose tiles (LDS per workgroup)
inline bool fused_input(const cista_config &cfg) { return CISTA_FUSED_IN && cfg.num_bins <= 8; }
#ifndef CISTA_S2D_IN
#define CISTA_S2D_IN 1
#endif
// ... with its interior on MFMA (space-to-depth input, 4 (nb+1) <= 32 channels)
inline bool s2d_input(const cista_config &cfg) { return CISTA_S2D_IN && cfg.num_bins <= 7; }
// ... staged straight from the NCHW planes by the conv (no s2d tensor round trip through HBM)
#ifndef CISTA_S2D_DIRECT
#define CISTA_S2D_DIRECT 1
#endif

// ... and its border pixels by per-sample strip segments (input_border_kernel; 0: the
// class-major input_w0_kernel grid)
#ifndef CISTA_BORDER_STRIPS
#define CISTA_BORDER_STRIPS 1
#endif

// the upsample conv's wave holds all C output channels (WN == 1) for C = 32 and 64
inline bool up_q_path(int C) { return C == 64 || C == 32; }
// ... and for C = 64 it runs phase-decomposed over the half-res input
#ifndef CISTA_UP4
#define CISTA_UP4 1
#endif
inline bool up4_path(int C) { return CISTA_UP4 && C == 64; }

ConvArgs conv_args_f(const Frame &f, int id, int C, int B, int Hin, int Win, int Hout, int Wout,
                     const float *in0, int c0, const float *in1, int c1) {
    ConvArgs a = conv_args(f.packed, f.L, id, C, B, Hin, Win, Hout, Wout, in0, c0, in1, c1);
    return a;
}

#ifndef CISTA_PROBE
#define CISTA_PROBE 0     // diagnostic builds (scripts/l2_probe.py): cista_debug_set_ista_p_probe
#endif
#if CISTA_PROBE
unsigned g_probe_mask = 0;   // != 0: ISTA P's z reads / writes wrapped into [0, mask] elements
#endif

int run_layer(const Frame &f, int layer, int it = 0) {
    const size_t hw = (size_t)f.B * f.h * f.w;
    // training: the ISTA iterates z_0 .. z_{D-1} stay in the saved stack at f.zl (the backward's
    // D wgrad inputs), iteration `it` reading slot it and writing slot it+1 (the last one f.z)
    const bool zstack = f.zl && f.cfg->depth > 0;
    float *z_in = zstack ? f.zl + (size_t)it * hw * 2 * f.C : f.z;
    float *z_out = zstack && it + 1 < f.cfg->depth ? f.zl + (size_t)(it + 1) * hw * 2 * f.C : f.z;
    const int C = f.C, B = f.B, h = f.h, w = f.w;
    ConvArgs a;
    switch (layer) {
        case CISTA_LAYER_INPUT: {                                      // e2v_model.py:62-64
            if (fused_input(*f.cfg) && !f.need_full) {                 // ... and W0, :66
                FusedInArgs fa;
                fa.events = f.events; fa.prev = f.prev_image;
                fa.E = blob<float>(f.packed, f.L.wC); fa.bias = blob<float>(f.packed, f.L.bC);
                fa.out = f.x1; fa.B = B; fa.H = f.H; fa.W = f.W; fa.h = h; fa.w = w; fa.C = C;
                fa.border_only = 0;
                long most = (long)B * (h > 2 ? h - 2 : 1) * (w > 2 ? w - 2 : 1);
                if (s2d_input(*f.cfg) && CISTA_S2D_DIRECT) {
                    // interior on MFMA, the space-to-depth view staged straight from the NCHW
                    // planes (STAGE_S2D); the padded border outputs are then overwritten by the
                    // VALU pass
                    a = conv_args_f(f, CV_IN, C, B, h, w, h, w, f.events, 32, nullptr, 0);
                    a.s2d_img = f.prev_image;
                    a.s2d_nb = f.cfg->num_bins;
                    a.out0 = f.x1;
                    if (const int sc = launch_conv<STAGE_S2D, EPI_BIAS, 1>(a, f.st)) return sc;
                    fa.border_only = 1;
                    most = (long)B * (h > w ? h : w);
                } else if (s2d_input(*f.cfg)) {
                    // interior on MFMA: s2d input (in x_full's space) -> 3x3 split-f16 conv; the
                    // conv's reflect-padded border outputs are then overwritten by the VALU pass
                    const dim3 gs((unsigned)(((long)B * h * w + 255) / 256));
                    switch (f.cfg->num_bins) {
#define NBCASE(n)                                                                                  \
    case n:                                                                                        \
        hipLaunchKernelGGL(s2d_input_kernel<n>, gs, dim3(256), 0, f.st, f.events, f.prev_image,   \
                           f.full, B, f.H, f.W);                                                  \
        break;
                        NBCASE(1) NBCASE(2) NBCASE(3) NBCASE(4) NBCASE(5) NBCASE(6) NBCASE(7)
#undef NBCASE
                    }
                    a = conv_args_f(f, CV_IN, C, B, h, w, h, w, f.full, 32, nullptr, 0);
                    a.out0 = f.x1;
                    if (const int sc = launch_conv<STAGE_S1, EPI_BIAS, 1>(a, f.st)) return sc;
                    fa.border_only = 1;
                    most = (long)B * (h > w ? h : w);
                }
                if (fa.border_only && CISTA_BORDER_STRIPS) {
                    // per-sample strip segments: a sample's border inputs are fetched once; 8
                    // channels per wave at small batch (latency), 32 otherwise
                    const bool small = B < 32;
                    const int ct = small ? 8 : 32;
                    const dim3 gb((unsigned)((long)B * border_segments(h, w)), (unsigned)((C / ct + 1) / 2));
                    switch (f.cfg->num_bins) {
#define NBCASE(n)                                                                          \
    case n:                                                                                \
        if (small) hipLaunchKernelGGL((input_border_kernel<n, 8>), gb, dim3(256), 0, f.st, fa);  \
        else hipLaunchKernelGGL((input_border_kernel<n, 32>), gb, dim3(256), 0, f.st, fa);       \
        break;
                        NBCASE(1) NBCASE(2) NBCASE(3) NBCASE(4) NBCASE(5) NBCASE(6) NBCASE(7)
#undef NBCASE
                    }
                    return hipGetLastError() == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
                }
                // channel split: C / 32 ways for the border pass, else as few as fit the LDS
                int zs = fa.border_only ? C / 32 : 1;
                while (!fa.border_only && ((C / 32) % zs || (size_t)256 * (C / zs + 1) * 4 > IN_TILE_LDS)) ++zs;
                const dim3 g2((unsigned)((most + 255) / 256), fa.border_only ? 8 : 9, (unsigned)zs);
                const size_t lds = (size_t)256 * (C / zs + 1) * 4;
                switch (f.cfg->num_bins) {
#define NBCASE(n)                                                                           \
    case n:                                                                                 \
        if (!allow_big_lds((const void *)input_w0_kernel<n>)) return CISTA_ERR_HIP;        \
        hipLaunchKernelGGL(input_w0_kernel<n>, g2, dim3(256), lds, f.st, fa);              \
        break;
                    NBCASE(1) NBCASE(2) NBCASE(3) NBCASE(4) NBCASE(5) NBCASE(6) NBCASE(7) NBCASE(8)
#undef NBCASE
                }
                return hipGetLastError() == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
            }
            InputArgs ia;
            ia.events = f.events; ia.prev = f.prev_image;
            ia.wE = blob<float>(f.packed, f.L.wE); ia.wI = blob<float>(f.packed, f.L.wI);
            ia.bias = blob<float>(f.packed, f.L.bIn);
            ia.out = f.full; ia.B = B; ia.H = f.H; ia.W = f.W; ia.nb = f.cfg->num_bins; ia.C = C;
            const long npix = (long)B * f.H * f.W;
            // channel split (large C): as few ways as keep the [256][2 CH + 1] tile in the LDS
            int ys = 1;
            while (((C / 32) % ys || (size_t)256 * (C / ys + 1) * 4 > IN_TILE_LDS)) ++ys;
            const dim3 g1((unsigned)((npix + 255) / 256), (unsigned)ys);
            const size_t lds = (size_t)256 * (C / ys + 1) * 4;
            switch (f.cfg->num_bins) {
#define NBCASE(n)                                                                           \
    case n:                                                                                 \
        if (!allow_big_lds((const void *)input_stage_kernel_nb<n>)) return CISTA_ERR_HIP;  \
        hipLaunchKernelGGL(input_stage_kernel_nb<n>, g1, dim3(256), lds, f.st, ia);        \
        break;
                NBCASE(1) NBCASE(2) NBCASE(3) NBCASE(4) NBCASE(5) NBCASE(6) NBCASE(7) NBCASE(8)
#undef NBCASE
                default: {
                    const long total = npix * (C / 16);
                    hipLaunchKernelGGL(input_stage_kernel, dim3((unsigned)((total + 255) / 256)),
                                       dim3(256), 0, f.st, ia);
                }
            }
            return hipGetLastError() == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
        }
        case CISTA_LAYER_W0:                                           // e2v_model.py:66
            if (fused_input(*f.cfg) && !f.need_full) return CISTA_OK;  // done by the input stage
            a = conv_args_f(f, CV_W0, C, B, f.H, f.W, h, w, f.full, C, nullptr, 0);
            a.out0 = f.x1;
            return launch_conv<STAGE_S2, EPI_BIAS, 1>(a, f.st);
        case CISTA_LAYER_P0:                                           // base_layers.py:61
            a = conv_args_f(f, CV_P0, C, B, h, w, h, w, f.x1, C, nullptr, 0);
            a.out0 = f.z0;
            return launch_conv<STAGE_S1, EPI_BIAS, 1>(a, f.st);
        case CISTA_LAYER_GATES:     // c = sig(f) c_prev + sig(i) z0, gates(cat(x1, z_prev)) :57-67
            a = conv_args_f(f, CV_GATES, C, B, h, w, h, w, f.x1, C, f.z_prev, 2 * C);
            a.out0 = f.c_lstc; a.aux0 = f.c_lstc_prev; a.aux1 = f.z0;
            a.out1 = f.gi; a.out2 = f.gf;
            return launch_conv<STAGE_S1, EPI_LSTC_CELL, 2>(a, f.st);
        case CISTA_LAYER_OUT_GATES: // z = sig(out_gates(cat(z0, z_prev))) tanh(c)          :63,69
            a = conv_args_f(f, CV_OUTG, C, B, h, w, h, w, f.z0, 2 * C, f.z_prev, 2 * C);
            a.out0 = (f.zl && f.cfg->depth > 0) ? f.zl : f.z; a.aux0 = f.c_lstc; a.out1 = f.go;
            return launch_conv<STAGE_S1, EPI_LSTC_OUT, 1>(a, f.st);
        case CISTA_LAYER_ISTA_D:    // x = x1 - D(z)                              e2v_model.py:73-74
            a = conv_args_f(f, CV_D, C, B, h, w, h, w, z_in, 2 * C, nullptr, 0);
            a.out0 = f.xs ? f.xs + it * hw * C : f.xb; a.aux0 = f.x1;
            return launch_conv<STAGE_S1, EPI_ISTA_D, 1>(a, f.st);
        case CISTA_LAYER_ISTA_P:    // z = softshrink(P(x) + z, lambda)            :75-77
            a = conv_args_f(f, CV_P, C, B, h, w, h, w, f.xs ? f.xs + it * hw * C : f.xb, C,
                          nullptr, 0);
            a.out0 = z_out; a.aux0 = z_in; a.lambda = blob<float>(f.packed, f.L.lambda);
            a.out1 = f.v ? f.v + it * hw * 2 * C : nullptr;
#if CISTA_PROBE
            if (g_probe_mask && !f.v) {             // diagnostic build: the L2-window ISTA P
                a.probe_mask = g_probe_mask;
                return launch_conv<STAGE_S1, EPI_ISTA_P_L2, 1>(a, f.st);
            }
#endif
            return launch_conv<STAGE_S1, EPI_ISTA_P, 1>(a, f.st);
        case CISTA_LAYER_DG:        // y = relu(Dg.conv(z))                      base_layers.py:222
            a = conv_args_f(f, CV_DG, C, B, h, w, h, w, f.z, 2 * C, nullptr, 0);
            a.out0 = f.y ? f.y : f.xb;
            return launch_conv<STAGE_S1, EPI_RELU, 1>(a, f.st);
        case CISTA_LAYER_LSTM:      // ConvLSTM on cat(y, h_prev)                  :112-128
            a = conv_args_f(f, CV_LSTM, C, B, h, w, h, w, f.y ? f.y : f.xb, C, f.h_prev, C);
            a.out0 = f.hs; a.out1 = f.cs; a.aux0 = f.c_prev; a.out2 = f.lg;
            return launch_conv<STAGE_S1, EPI_LSTM, 4>(a, f.st);
        case CISTA_LAYER_UPSAMPLE:  // relu(conv(ReflectionPad(up2x(h))))          :193-210
            if (up4_path(C)) {
                // phase-decomposed: one 4C-column conv over the half-res h (edge-replicated),
                // then the exact border pass for full-res rows 0, H-1 and columns 0, W-1
                a = conv_args_f(f, CV_UP4, C, B, h, w, h, w, f.hs, C, nullptr, 0);
                a.Cout = C;
                a.out0 = f.full; a.aux0 = blob<float>(f.packed, f.L.wF); a.out1 = f.u;
                const int sc = f.u ? launch_conv<STAGE_CLAMP, EPI_UP4_Q_SAVE, 1>(a, f.st)
                                   : launch_conv<STAGE_CLAMP, EPI_UP4_Q, 1>(a, f.st);
                if (sc) return sc;
                // border strips: the bilinear-staging upsample conv (exact reference arithmetic)
                // on 1-row / 1-column tiles, one fixed configuration for every batch size
                for (int mode = 1; mode <= 2; ++mode) {
                    ConvArgs bo = conv_args_f(f, CV_UP, C, B, h, w, f.H, f.W, f.hs, C, nullptr, 0);
                    bo.out0 = f.full; bo.aux0 = blob<float>(f.packed, f.L.wF); bo.out1 = f.u;
                    bo.border = mode;
                    // 64-pixel strip tiles at every batch size: the 128-pixel configuration gave
                    // border pixels that differ in the last bit from the 64-pixel one (batch
                    // independence, tests/test_gpu_parity.py::test_batch48_persistent_equals_single)
                    const int sb = f.u ? launch_conv_cfg<1, 4, 4, 1, STAGE_UP, EPI_UP_Q_SAVE, 1>(bo, f.st)
                                       : launch_conv_cfg<1, 4, 4, 1, STAGE_UP, EPI_UP_Q, 1>(bo, f.st);
                    if (sb) return sb;
                }
                return CISTA_OK;
            }
            a = conv_args_f(f, CV_UP, C, B, h, w, f.H, f.W, f.hs, C, nullptr, 0);
            a.out0 = f.full;
            if (up_q_path(C)) {     // + final_conv's channel contraction in the epilogue
                a.aux0 = blob<float>(f.packed, f.L.wF);
                a.out1 = f.u;
                if (f.u) return launch_conv<STAGE_UP, EPI_UP_Q_SAVE, 1>(a, f.st);
                return launch_conv<STAGE_UP, EPI_UP_Q, 1>(a, f.st);
            }
            if (f.u) a.out0 = f.u;  // training: u itself is saved (final_stage_kernel reads it there)
            return launch_conv<STAGE_UP, EPI_RELU, 1>(a, f.st);
        case CISTA_LAYER_FINAL: {   // sigmoid(final_conv(u))                  e2v_model.py:87-88
            const long total = (long)B * f.H * f.W;
            const dim3 g1((unsigned)((total + 255) / 256));
            if (up_q_path(C)) {
                FinalQArgs fq;
                fq.q = f.full; fq.bias = blob<float>(f.packed, f.L.bF);
                fq.rec = f.rec; fq.pre = f.pre; fq.B = B; fq.H = f.H; fq.W = f.W;
                hipLaunchKernelGGL(final_q_kernel, g1, dim3(256), 0, f.st, fq);
            } else {
                FinalArgs fa;
                fa.u = f.u ? f.u : f.full; fa.w = blob<float>(f.packed, f.L.wF); fa.bias = blob<float>(f.packed, f.L.bF);
                fa.rec = f.rec; fa.pre = f.pre; fa.B = B; fa.H = f.H; fa.W = f.W; fa.C = C;
                hipLaunchKernelGGL(final_stage_kernel, g1, dim3(256), 0, f.st, fa);
            }
            return hipGetLastError() == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
        }
        default:
            return CISTA_ERR_INVALID;
    }
}

Frame make_frame(const cista_config *cfg, const void *packed, int B, int H, int W, void *ws,
                 void *stream) {
    Frame f;
    memset(&f, 0, sizeof(f));
    f.cfg = cfg; f.packed = packed; f.L = make_layout(*cfg);
    f.B = B; f.H = H; f.W = W; f.h = H / 2; f.w = W / 2; f.C = cfg->base_channels;
    const Workspace wsp = carve(ws, B, H, W, f.C);
    f.full = wsp.full; f.x1 = wsp.x1; f.z0 = wsp.z0; f.xb = wsp.xb;
    f.st = static_cast<hipStream_t>(stream);
    return f;
}

void bind_io(Frame &f, const cista_frame_io *io) {
    f.events = io->events; f.prev_image = io->prev_image;
    f.c_lstc_prev = io->c_lstc_prev; f.z_prev = io->z_prev; f.h_prev = io->h_prev;
    f.c_prev = io->c_prev;
    f.rec = io->rec; f.c_lstc = io->c_lstc; f.z = io->z; f.hs = io->h; f.cs = io->c;
}

int run_layers(const Frame &f, const int *layers, int n) {
    for (int i = 0; i < n; ++i) CHECK(run_layer(f, layers[i]));
    return CISTA_OK;
}

int run_ista(const Frame &f, int iters) {
    for (int i = 0; i < iters; ++i) {                                  // e2v_model.py:72-78
        CHECK(run_layer(f, CISTA_LAYER_ISTA_D, i));
        CHECK(run_layer(f, CISTA_LAYER_ISTA_P, i));
    }
    return CISTA_OK;
}

double layer_macs(const cista_config &cfg, int layer, int B, int H, int W) {
    const double C = cfg.base_channels, hw = (double)(H / 2) * (W / 2), HW = (double)H * W;
    switch (layer) {
        case CISTA_LAYER_INPUT: return B * HW * 9.0 * (C / 2) * (cfg.num_bins + 1);
        case CISTA_LAYER_W0: return B * hw * 9.0 * C * C;
        case CISTA_LAYER_P0: return B * hw * 9.0 * C * 2 * C;
        case CISTA_LAYER_GATES: return B * hw * 9.0 * 3 * C * 4 * C;
        case CISTA_LAYER_OUT_GATES: return B * hw * 9.0 * 4 * C * 2 * C;
        case CISTA_LAYER_ISTA_D: return B * hw * 9.0 * 2 * C * C;
        case CISTA_LAYER_ISTA_P: return B * hw * 9.0 * C * 2 * C;
        case CISTA_LAYER_DG: return B * hw * 9.0 * 2 * C * C;
        case CISTA_LAYER_LSTM: return B * hw * 9.0 * 2 * C * 4 * C;
        case CISTA_LAYER_UPSAMPLE: return B * HW * 9.0 * C * C;
        case CISTA_LAYER_FINAL: return B * HW * 9.0 * C;
        default: return 0.0;
    }
}

int check_common(const cista_config *cfg, const void *packed, int B, int H, int W) {
    if (!cfg_ok(cfg) || !packed || B <= 0 || H <= 0 || W <= 0) return CISTA_ERR_INVALID;
    if (!cfg_supported(cfg)) return CISTA_ERR_UNSUPPORTED;
    return CISTA_OK;
}


// =========================================================================================
// training: saved activations, backward workspace, backward schedule
// =========================================================================================
struct Saved {
    float *x1, *z0, *gi, *gf, *go, *zl, *v, *xs, *y, *lg, *u;
    size_t bytes;
};

Saved carve_saved(void *buf, const cista_config &cfg, int B, int H, int W) {
    const size_t hw = (size_t)B * (H / 2) * (W / 2), HW = (size_t)B * H * W;
    const int C = cfg.base_channels, D = cfg.depth;
    Saved s;
    size_t off = 0;
    char *base = static_cast<char *>(buf);
    auto take = [&](size_t nfloat) {
        float *p = reinterpret_cast<float *>(base + off);
        off = align_up(off + nfloat * 4);
        return p;
    };
    s.x1 = take(hw * C);
    s.z0 = take(hw * 2 * C);
    s.gi = take(hw * 2 * C);
    s.gf = take(hw * 2 * C);
    s.go = take(hw * 2 * C);
    s.zl = take(hw * 2 * C * (D > 0 ? D : 1));   // z_0 = ConvLSTC output, then the ISTA iterates
    s.v = take(hw * 2 * C * (D > 0 ? D : 1));
    s.xs = take(hw * C * (D > 0 ? D : 1));
    s.y = take(hw * C);
    s.lg = take(hw * 4 * C);
    s.u = take(HW * C);
    s.bytes = off;
    return s;
}

#ifndef CISTA_WG_BLOCKS
#define CISTA_WG_BLOCKS 1024
#endif
constexpr int WG_BLOCKS = CISTA_WG_BLOCKS;   // wgrad partial-sum blocks per launch (splits x cout/cin blocks)
constexpr int SCL_PAIRS = 16;                // scale pairs of the non-ISTA gradients of a call (8 used)
constexpr size_t AMAX_WORDS = (size_t)8 * AMAX_SLOTS * AMAX_STRIDE + 8 * 16;   // slot sets + tickets

struct BwdWs {
    float *gpre, *gU, *dxpF, *ghb, *Gl, *dxp, *gy, *gz, *gv, *gxk, *gx1, *Go, *gz0;
    float *fb;          // border lines of an EPI_FOLD dgrad's padded output (fold_border_index)
    float *part, *bpart, *dlp;
    float *part2, *bpart2;   // the side stream's wgrad partials (run_backward, on_side)
    float *wT;          // [9][Cout][Cin] transposed weights for dgrad_vec_kernel
    unsigned *amax;     // [8][AMAX_SLOTS * AMAX_STRIDE] gradient |max| slots (zero between uses),
                        // then [8][16] tickets of ticket_scale (zero between uses)
    float *scl;         // [16] scale pairs
    size_t bytes;
};

BwdWs carve_bwd(void *buf, const cista_config &cfg, int B, int H, int W) {
    const int h = H / 2, w = W / 2, C = cfg.base_channels;
    const size_t hw = (size_t)B * h * w, HW = (size_t)B * H * W;
    BwdWs s;
    size_t off = WS_HEADER;    // the reserved header is never handed out as scratch
    char *base = static_cast<char *>(buf);
    auto take = [&](size_t nfloat) {
        float *p = reinterpret_cast<float *>(base + off);
        off = align_up(off + nfloat * 4);
        return p;
    };
    s.gpre = take(HW);
    s.gU = take(HW * C);
    s.dxpF = take((size_t)B * (H + 2) * (W + 2) * C);
    s.ghb = take(hw * C);
    s.Gl = take(hw * 4 * C);
    s.dxp = take((size_t)B * (h + 2) * (w + 2) * 4 * C);
    s.gy = take(hw * C);
    s.gz = take(hw * 2 * C);
    // the ISTA iterations' gradients and iterates, stacked [iteration][B][h][w][C] so that the
    // tied D / P weight gradients are one wgrad launch each over all iterations
    const size_t nd = cfg.depth > 0 ? (size_t)cfg.depth : 1;
    s.gv = take(nd * hw * 2 * C);
    s.gxk = take(nd * hw * C);
    s.gx1 = take(hw * C);
    s.Go = take(hw * 2 * C);
    s.gz0 = take(hw * 2 * C);
    {
        const size_t lh = (size_t)B * (2 * (w + 2) + 2 * h) * 4 * C, lf = (size_t)B * (2 * (W + 2) + 2 * H) * C;
        s.fb = take(lh > lf ? lh : lf);
    }
    s.part = take((size_t)WG_BLOCKS * 32 * 32 * 9);
    s.bpart = take((size_t)WG_BLOCKS * 4 * C);
    s.dlp = take((size_t)2 * C * 512 * nd);           // lambda partials [iteration][block][2C]
    s.part2 = take((size_t)WG_BLOCKS * 32 * 32 * 9);
    s.bpart2 = take((size_t)WG_BLOCKS * 4 * C);
    s.wT = take((size_t)9 * C * C);
    s.amax = reinterpret_cast<unsigned *>(take(AMAX_WORDS));
    s.scl = take(2 * SCL_PAIRS + 4 * nd + 4);   // the call's pairs, the ISTA P / D pairs per iteration, their minima
    s.bytes = off;
    return s;
}

inline dim3 g1d(long n) { return dim3((unsigned)((n + 255) / 256)); }

// {s, 1/s} from the |max| slots a producing kernel filled (amax_publish), slots re-zeroed
__global__ __launch_bounds__(256) void slots_scale_kernel(unsigned *slots, float *scl) {
    __shared__ float red[4];
    const unsigned u = slots[threadIdx.x * AMAX_STRIDE];
    slots[threadIdx.x * AMAX_STRIDE] = 0u;
    float m = __uint_as_float(u);
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) scale_from_max(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])), scl);
}

struct Bwd {
    const cista_config *cfg;
    const void *packed;
    Layout L;
    int B, H, W, h, w, C;
    hipStream_t st;
    BwdWs ws;
    int slot;   // |max| slot set (rotating over 8)
    int pair;   // next scale pair of the call (never reused within a call)
    hipStream_t side = nullptr;   // weight gradients' stream (NULL: everything on st)
    bool side_busy = false;       // side work not yet joined into st
    int dev = 0, nev = 0;         // device, events used by the call
};

int hip_ok() { return hipGetLastError() == hipSuccess ? CISTA_OK : CISTA_ERR_HIP; }

// Weight gradients on a side stream.  Each wgrad of the backward reads gradients and activations
// that are final when it is issued, so it can run beside the dgrad chain: its workgroups fill the
// matrix pipes while the chain's one-round dgrad launches are in their memory phases
// and while the chain's small elementwise and scale kernels hold a few CUs.  Fork: an event on the
// caller's stream after the wgrad's inputs, waited on by the side stream; the side wgrads use their
// own partial buffers (part2 / bpart2).  Join: before the caller's stream overwrites an input a
// pending side wgrad reads, and at the end of the call (the caller reads the weight gradients on
// its stream).  One side stream per device, created on first use; events from a per-thread pool
// (a wait is bound to the event's record at the time of the call, so reuse is safe).
// CISTA_BWD_SIDE=0 (read per call) keeps everything on the caller's stream: the same kernels in
// the same order, so the gradients are bit-identical either way (tests/test_gpu_train.py).
bool side_enabled() {
    const char *e = getenv("CISTA_BWD_SIDE");
    return !e || atoi(e) != 0;
}
constexpr int MAX_DEV = 64, BWD_EVENTS = 16;
hipStream_t side_stream(int dev) {
    static std::mutex mu;
    static hipStream_t streams[MAX_DEV] = {};
    if (dev < 0 || dev >= MAX_DEV) return nullptr;
    std::lock_guard<std::mutex> lock(mu);
    if (!streams[dev] && hipStreamCreateWithFlags(&streams[dev], hipStreamNonBlocking) != hipSuccess)
        streams[dev] = nullptr;
    return streams[dev];
}
// the calling thread's events on device dev, all created on first use (NULL: could not be;
// cista_backward then keeps everything on the caller's stream)
hipEvent_t *event_pool(int dev) {
    thread_local hipEvent_t pool[MAX_DEV][BWD_EVENTS] = {};
    if (dev < 0 || dev >= MAX_DEV) return nullptr;
    for (int i = 0; i < BWD_EVENTS; ++i)
        if (!pool[dev][i] && hipEventCreateWithFlags(&pool[dev][i], hipEventDisableTiming) != hipSuccess) {
            pool[dev][i] = nullptr;
            return nullptr;
        }
    return pool[dev];
}
// an event recorded on `on` now (NULL on failure)
hipEvent_t mark(Bwd &k, hipStream_t on) {
    hipEvent_t *pool = event_pool(k.dev);
    if (!pool || k.nev >= BWD_EVENTS) return nullptr;
    const hipEvent_t e = pool[k.nev++];
    return hipEventRecord(e, on) == hipSuccess ? e : nullptr;
}
// `waiter` waits for the work issued to `on` so far
int stream_wait(Bwd &k, hipStream_t waiter, hipStream_t on) {
    const hipEvent_t e = mark(k, on);
    return e && hipStreamWaitEvent(waiter, e, 0) == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
}
template <class F>
int on_side(Bwd &k, F &&fn) {
    if (!k.side) return fn();
    const int rw = stream_wait(k, k.side, k.st);
    if (rw != CISTA_OK) return rw;
    const hipStream_t m = k.st;
    float *const p = k.ws.part, *const bp = k.ws.bpart;
    k.st = k.side;
    k.ws.part = k.ws.part2;
    k.ws.bpart = k.ws.bpart2;
    const int r = fn();
    k.st = m;
    k.ws.part = p;
    k.ws.bpart = bp;
    k.side_busy = true;
    return r;
}
int join_side(Bwd &k) {
    if (!k.side || !k.side_busy) return CISTA_OK;
    k.side_busy = false;
    return stream_wait(k, k.st, k.side);
}

// per-tensor power-of-two scale {s, 1/s} of an output gradient for its fp16 splits (split-f16
// dgrad and wgrad), in a rotating slot of the backward workspace: the kernel that produces the
// gradient is launched with scale_slots(k) and publishes its |max| there; scale_of then turns
// the slots into the scale pair (one 256-thread launch)
unsigned *scale_slots(Bwd &k, int ahead = 0) {
    return k.ws.amax + (size_t)((k.slot + ahead) & 7) * AMAX_SLOTS * AMAX_STRIDE;
}
// the smallest of n scale pairs (the largest gradient of a stacked wgrad) -> out
__global__ void min_scale_kernel(const float *pairs, int n, float *out) {
    if (threadIdx.x != 0) return;
    int j = 0;
    for (int i = 1; i < n; ++i) j = pairs[2 * i] < pairs[2 * j] ? i : j;
    out[0] = pairs[2 * j];
    out[1] = pairs[2 * j + 1];
}
// a gradient whose producer does not publish: one grid-stride |max| pass into the slots
__global__ __launch_bounds__(256) void absmax_publish_kernel(const float *x, long n, unsigned *slots) {
    float m = 0.0f;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) m = fmaxf(m, fabsf(x[i]));
    amax_publish(slots, m);
}
const float *scale_of(Bwd &k, float *dst = nullptr);
const float *grad_scale(Bwd &k, const float *G, long n) {
    const long blocks = (n + 255) / 256;
    hipLaunchKernelGGL(absmax_publish_kernel, dim3((unsigned)(blocks < 1 ? 1 : blocks > 1024 ? 1024 : blocks)), dim3(256),
                       0, k.st, G, n, scale_slots(k));
    return scale_of(k);
}
const float *scale_of(Bwd &k, float *dst) {
    unsigned *sl = scale_slots(k);
    // pairs are not reused within a call (a weight gradient on the side stream may read one late)
    float *sc = dst;
    if (!sc) {
        if (k.pair >= SCL_PAIRS) return nullptr;        // more gradients than the workspace has pairs for
        sc = k.ws.scl + 2 * k.pair++;
    }
    ++k.slot;
    hipLaunchKernelGGL(slots_scale_kernel, dim3(1), dim3(AMAX_SLOTS), 0, k.st, sl, sc);
    return hipGetLastError() == hipSuccess ? sc : nullptr;
}

// The pair a producer's last block fills (ticket_scale) in place of scale_of's launch: the same
// pair bookkeeping; the producer publishes into scale_slots(k) and gets ticket_of(k), and the
// caller calls slot_done(k) after its launch (scale_of's ++slot)
float *claim_scale(Bwd &k, float *dst = nullptr) {
    if (dst) return dst;
    if (k.pair >= SCL_PAIRS) return nullptr;
    return k.ws.scl + 2 * k.pair++;
}
unsigned *ticket_of(Bwd &k) { return k.ws.amax + (size_t)8 * AMAX_SLOTS * AMAX_STRIDE + (size_t)(k.slot & 7) * 16; }
void slot_done(Bwd &k) { ++k.slot; }

// dst (+)= sign * the split sum of the wgrad partials, and db from the bias partials, one launch
void reduce_parts_at(Bwd &k, const float *part, const float *bpart, int ns, long n, float *dst, float *db, long nbias,
                     float sign, int accumulate) {
    const long nb = db ? nbias : 0;
    hipLaunchKernelGGL(reduce_partials_kernel, g1d(n + nb), dim3(256), 0, k.st, part, ns, n, dst, sign, accumulate,
                       bpart, nb, db);
}
void reduce_parts(Bwd &k, int ns, long n, float *dst, float *db, long nbias, float sign, int accumulate) {
    reduce_parts_at(k, k.ws.part, k.ws.bpart, ns, n, dst, db, nbias, sign, accumulate);
}

#ifndef CISTA_WIN_NS
#define CISTA_WIN_NS 512        // splits of the fused We / Wi wgrad (wgrad_in_kernel)
#endif
#ifndef CISTA_WGRAD_IN
#define CISTA_WGRAD_IN 1   // We / Wi wgrads in one fp32-MFMA pass over gxfull (0: two wgrad_small_kernel launches)
#endif
// We and Wi weight / bias gradients from gxfull in one launch (wgrad_in_kernel); C in {32, 64},
// num_bins <= 8.  Returns CISTA_ERR_UNSUPPORTED for other shapes (the caller falls back).
int wgrad_inputs(Bwd &k, const float *gx, const float *ev, const float *img, const cista_param_grads &pg) {
    const int C = k.C, nb = k.cfg->num_bins, half = C / 2;
    if (!CISTA_WGRAD_IN || (C != 32 && C != 64) || nb < 1 || nb > 8) return CISTA_ERR_UNSUPPORTED;
    WgradInArgs a;
    a.G = gx; a.ev = ev; a.img = img;
    a.B = k.B; a.H = k.H; a.W = k.W; a.C = C;
    a.tiles_y = (k.H + 7) / 8;
    a.tiles_x = (k.W + 15) / 16;
    const int ntiles = a.B * a.tiles_y * a.tiles_x;
    const int ns = ntiles < CISTA_WIN_NS ? ntiles : CISTA_WIN_NS;
    a.nsplit = ns;
    a.partE = k.ws.part;
    a.partI = k.ws.part + (size_t)ns * half * nb * 9;
    a.bpartE = k.ws.bpart;
    a.bpartI = k.ws.bpart + (size_t)ns * half;
    const size_t lds = ((size_t)WI_TP * (C + 16) + (size_t)(nb + 1) * WI_HPX) * 4;
    switch (nb * 2 + (C == 64 ? 1 : 0)) {
#define WICASE(n)                                                                                      \
    case 2 * n: hipLaunchKernelGGL((wgrad_in_kernel<n, 1>), dim3(ns), dim3(256), lds, k.st, a); break;              \
    case 2 * n + 1: hipLaunchKernelGGL((wgrad_in_kernel<n, 2>), dim3(ns), dim3(256), lds, k.st, a); break;
        WICASE(1) WICASE(2) WICASE(3) WICASE(4) WICASE(5) WICASE(6) WICASE(7) WICASE(8)
#undef WICASE
    }
    reduce_parts_at(k, a.partE, a.bpartE, ns, (long)half * nb * 9, pg.We_w, pg.We_b, half, 1.0f, 0);
    reduce_parts_at(k, a.partI, a.bpartI, ns, (long)half * 9, pg.Wi_w, pg.Wi_b, half, 1.0f, 0);
    return hip_ok();
}

#ifndef CISTA_WGRAD_TR
#define CISTA_WGRAD_TR 1      // split-f16 wgrads on wgrad_tr_kernel (0: wgrad_split_kernel, A/B builds)
#endif
#ifndef CISTA_WSMALL_NS
#define CISTA_WSMALL_NS 512     // splits of the We / Wi wgrads (wgrad_small_kernel)
#endif
#ifndef CISTA_WC1_NS
#define CISTA_WC1_NS 2048       // splits x channel blocks of the final-conv wgrad (wgrad_c1_kernel; 512: 57 us, 2048: 45 us at B = 8)
#endif
#ifndef CISTA_WGRAD_TR_S2
#define CISTA_WGRAD_TR_S2 1   // W0's stride-2 wgrad on wgrad_tr_kernel<XS_S2> (0: exact fp32-MFMA wgrad_kernel)
#endif
constexpr int NCU = 256;      // MI355X compute units (8 XCDs x 32)

// dW (+)= sign * wgrad ; G channels [Goff, Goff+Cout) of a Gc-channel NHWC tensor; and, when
// db != NULL, db (+)= sign * (pixel sum of G) from the same pass over G (bias gradient).
// gsc (the grad_scale of G) selects the split-f16 kernel where the shape allows it.
template <int XS>
int wgrad(Bwd &k, const float *G, int Gc, int Goff, int Cout, const float *X0, int x0c,
          const float *X1, int x1c, int Cin, int Hin, int Win, int Hout, int Wout, float *dst,
          float sign, int accumulate, float *db, const float *gsc = nullptr, int Bn = 0) {
    WgradArgs a;
    memset(&a, 0, sizeof(a));
    a.G = G; a.Gc = Gc; a.Goff = Goff;
    a.X0 = X0; a.x0c = x0c; a.X1 = X1; a.x1c = x1c;
    a.B = Bn > 0 ? Bn : k.B;                 // Bn: samples of a stacked (iterations x batch) G / X
    a.Hin = Hin; a.Win = Win; a.Hout = Hout; a.Wout = Wout;
    a.Cout = Cout; a.Cin = Cin;
    a.partial = k.ws.part;
    a.bpartial = db ? k.ws.bpart : nullptr;
    a.off32 = (long long)a.B * Hout * Wout * Gc < (1LL << 31) &&
              (long long)a.B * Hin * Win * (x0c > x1c ? x0c : x1c) < (1LL << 31);
    constexpr bool TR_S2 = XS == XS_S2 && CISTA_WGRAD_TR_S2;
    if (TR_S2 && a.off32 && gsc && Cout % 64 == 0 && Cin % 32 == 0 && Gc % 4 == 0 && Goff % 4 == 0 && x0c % 32 == 0 &&
        x1c % 32 == 0 && Hin == 2 * Hout && Win == 2 * Wout) {
        // W0 (stride 2): the split-f16 wgrad on 2 x 16-pixel tiles over a parity-split halo
        if constexpr (TR_S2) {
            using GE = WtGeo<XS_S2>;
            a.gscale = gsc;
            a.TH = GE::TH; a.TW = 16;
            a.tiles_y = (Hout + GE::TH - 1) / GE::TH;
            a.tiles_x = (Wout + 15) / 16;
            const int ntiles = a.B * a.tiles_y * a.tiles_x;
            const int nblk = (Cout / 64) * ((Cin + 63) / 64);
            int ns = NCU / nblk;
            const int lim = (int)(((long)WG_BLOCKS * 32 * 32) / ((long)Cout * Cin));
            ns = ns > lim ? lim : ns;
            ns = ns > ntiles ? ntiles : ns;
            ns = ns < 1 ? 1 : ns;
            ns = (ntiles + (ntiles + ns - 1) / ns - 1) / ((ntiles + ns - 1) / ns);   // equal tiles per split
            a.nsplit = ns;
            if (!allow_big_lds((const void *)wgrad_tr_kernel<XS_S2>)) return CISTA_ERR_HIP;
            hipLaunchKernelGGL(wgrad_tr_kernel<XS_S2>, dim3(nblk, ns), dim3(WT_THREADS), GE::LDS, k.st, a);
            reduce_parts(k, ns, (long)Cout * Cin * 9, dst, db, Cout, sign, accumulate);
            return hip_ok();
        }
    }
    if (XS == XS_S1 && gsc && Cout % 64 == 0 && Cin % 32 == 0 && Gc % 4 == 0 &&
        Goff % 4 == 0 && x0c % 32 == 0 && x1c % 32 == 0 && Hin == Hout && Win == Wout) {
        a.gscale = gsc;
        a.TH = WS_TH; a.TW = WS_TW;
        a.tiles_y = (Hout + WS_TH - 1) / WS_TH;
        a.tiles_x = (Wout + WS_TW - 1) / WS_TW;
        const int ntiles = a.B * a.tiles_y * a.tiles_x;
        if (CISTA_WGRAD_TR && a.off32) {
            static_assert(WtGeo<XS_S1>::TH == WS_TH && WS_TW == 16, "wgrad_tr_kernel tiles");
            // 64 x 64 blocks, one 8-wave workgroup per CU: splits fill the CUs once (and fit
            // the partial buffer: ns x Cout x Cin x 9 <= WG_BLOCKS x 32 x 32 x 9)
            const int nblk = (Cout / 64) * ((Cin + 63) / 64);
            int ns = NCU / nblk;
            const int lim = (int)(((long)WG_BLOCKS * 32 * 32) / ((long)Cout * Cin));
            ns = ns > lim ? lim : ns;
            ns = ns > ntiles ? ntiles : ns;
            ns = ns < 1 ? 1 : ns;
            ns = (ntiles + (ntiles + ns - 1) / ns - 1) / ((ntiles + ns - 1) / ns);   // equal tiles per split
            a.nsplit = ns;
            if (!allow_big_lds((const void *)wgrad_tr_kernel<XS_S1>)) return CISTA_ERR_HIP;
            hipLaunchKernelGGL(wgrad_tr_kernel<XS_S1>, dim3(nblk, ns), dim3(WT_THREADS), WtGeo<XS_S1>::LDS, k.st, a);
            reduce_parts(k, ns, (long)Cout * Cin * 9, dst, db, Cout, sign, accumulate);
            return hip_ok();
        }
        const int nblk = (Cout / 64) * (Cin / 32);
        int ns = (WG_BLOCKS / 2) / nblk;   // partials: ns x Cout x Cin x 9 <= WG_BLOCKS x 32 x 32 x 9
        ns = ns > ntiles ? ntiles : ns;
        ns = ns < 1 ? 1 : ns;
        ns = (ntiles + (ntiles + ns - 1) / ns - 1) / ((ntiles + ns - 1) / ns);   // equal tiles per split
        a.nsplit = ns;
        if (!allow_big_lds((const void *)wgrad_split_kernel)) return CISTA_ERR_HIP;
        hipLaunchKernelGGL(wgrad_split_kernel, dim3(nblk, ns), dim3(256), WS_LDS, k.st, a);
        const long n = (long)Cout * Cin * 9;
        reduce_parts(k, ns, n, dst, db, Cout, sign, accumulate);
        return hip_ok();
    }
    if (XS == XS_NCHW && Cout <= 32 && Cin == x0c && Cin >= 1 && Cin <= 8 && !X1 && Hin == Hout && Win == Wout) {
        a.TH = 16; a.TW = 16;                                // We / Wi: VALU over NCHW planes
        a.tiles_y = (Hout + 15) / 16;
        a.tiles_x = (Wout + 15) / 16;
        const int ntiles = a.B * a.tiles_y * a.tiles_x;
        const int ns = ntiles < CISTA_WSMALL_NS ? ntiles : CISTA_WSMALL_NS;
        a.nsplit = ns;
        switch (Cin) {
#define WSCASE(n) \
    case n: hipLaunchKernelGGL(wgrad_small_kernel<n>, dim3(ns), dim3(256), 0, k.st, a); break;
            WSCASE(1) WSCASE(2) WSCASE(3) WSCASE(4) WSCASE(5) WSCASE(6) WSCASE(7) WSCASE(8)
#undef WSCASE
        }
        const long n = (long)Cout * Cin * 9;
        reduce_parts(k, ns, n, dst, db, Cout, sign, accumulate);
        return hip_ok();
    }
    if (XS == XS_S1 && Cout == 1 && Gc == 1 && Goff == 0 && Cin % 32 == 0 && x0c % 4 == 0 && x1c % 4 == 0 &&
        Hin == Hout && Win == Wout) {                        // final_conv: VALU, one output row
        a.TH = 16; a.TW = 16;
        a.tiles_y = (Hout + 15) / 16;
        a.tiles_x = (Wout + 15) / 16;
        const int ncb = Cin / 32;
        const int ntiles = a.B * a.tiles_y * a.tiles_x;
        int ns = CISTA_WC1_NS / ncb;
        ns = ns > ntiles ? ntiles : ns;
        ns = ns < 1 ? 1 : ns;
        a.nsplit = ns;
        hipLaunchKernelGGL(wgrad_c1_kernel, dim3(ncb, ns), dim3(256), 0, k.st, a);
        const long n = (long)Cin * 9;
        reduce_parts(k, ns, n, dst, db, 1, sign, accumulate);
        return hip_ok();
    }
    const int T = XS == XS_S2 ? 8 : 16;
    a.TH = Hout < T ? Hout : T;
    a.TW = Wout < T ? Wout : T;
    a.tiles_y = (Hout + a.TH - 1) / a.TH;
    a.tiles_x = (Wout + a.TW - 1) / a.TW;
    a.Cout = Cout; a.Cin = Cin;
    const int nblk = ((Cout + 31) / 32) * ((Cin + 31) / 32);
    const int ntiles = a.B * a.tiles_y * a.tiles_x;
    int ns = WG_BLOCKS / nblk;
    ns = ns > ntiles ? ntiles : ns;
    ns = ns < 1 ? 1 : ns;
    ns = (ntiles + (ntiles + ns - 1) / ns - 1) / ((ntiles + ns - 1) / ns);   // equal tiles per split
    a.nsplit = ns;
    a.partial = k.ws.part;
    a.bpartial = db ? k.ws.bpart : nullptr;
    a.vec4 = XS != XS_NCHW && Gc % 4 == 0 && Goff % 4 == 0 && x0c % 4 == 0 && x1c % 4 == 0 && Cin % 4 == 0;
    constexpr int S = XS == XS_S2 ? 2 : 1;
    const int HP = ((a.TH - 1) * S + 3) * ((a.TW - 1) * S + 3);
    const size_t lds = ((size_t)((a.TH * a.TW + 3) & ~3) + HP) * 33 * 4;
    auto kern = wgrad_kernel<XS>;
    if (!allow_big_lds((const void *)kern)) return CISTA_ERR_HIP;
    hipLaunchKernelGGL(kern, dim3(nblk, ns), dim3(256), lds, k.st, a);
    const long n = (long)Cout * Cin * 9;
    reduce_parts(k, ns, n, dst, db, Cout, sign, accumulate);
    return hip_ok();
}

// VALU dgrad through a reference-layout weight (W0: stride 2; final conv: Cout 1)
int dgrad_vec(Bwd &k, const DgradSmallArgs &d, const float *Wref) {
    if (d.Cin % 4 || d.Xc % 4 || d.Xoff % 4 || (size_t)d.Cout * d.Cin > (size_t)k.C * k.C) return CISTA_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(transpose_w_kernel, g1d((long)d.Cout * d.Cin * 9), dim3(256), 0, k.st, Wref, d.Cout, d.Cin,
                       k.ws.wT);
    hipLaunchKernelGGL(dgrad_vec_kernel, g1d((long)d.B * d.Hin * d.Win * (d.Cin / 4)), dim3(256), 0, k.st, d,
                       (const float *)k.ws.wT);
    return hip_ok();
}

// dxp (B, h+2, w+2, N) = padded-domain gradient of conv `id`'s input, from G (B,h,w,K)
// sc: grad_scale of G (computed here when NULL)
int dgrad_conv(Bwd &k, int id, const float *G, float *dxp, const float *sc = nullptr) {
    const ConvShape s = conv_shape(id, k.C);
    const int Hin = id == CV_UP ? k.H : k.h, Win = id == CV_UP ? k.W : k.w;
    if (!sc) sc = grad_scale(k, G, (long)k.B * Hin * Win * s.cout);
    if (!sc) return CISTA_ERR_HIP;
    ConvArgs a;
    memset(&a, 0, sizeof(a));
    a.in0 = G; a.c0 = s.cout; a.in1 = nullptr; a.c1 = 0;
    a.B = k.B; a.Hin = Hin; a.Win = Win; a.Hout = Hin + 2; a.Wout = Win + 2;
    a.wpack = blob<u32x4>(k.packed, k.L.dwp[id]);
    a.bias = blob<float>(k.packed, k.L.dbp[id]);
    a.wscale = blob<float>(k.packed, k.L.sc[id]) + 1;
    a.ascale = sc;
    a.N = s.cin; a.Cout = s.cin;
    a.out0 = dxp;
    return launch_conv<STAGE_ZP2, EPI_BIAS, 1>(a, k.st);
}

#ifndef CISTA_FOLD_EPI
#define CISTA_FOLD_EPI 1   // dgrads fold the reflect padding in their epilogue (0: fold_reflect_kernel pass)
#endif
constexpr int FOLD_COL_ALIGN = 32;      // NW * 16 of the STAGE_ZP2 wave tilings

FoldSeg fseg(float *dst, int Cd, int dc0, float scale = 1.0f, int mode = FOLD_SET, float *aux = nullptr,
             unsigned *amax = nullptr) {
    FoldSeg f;
    f.dst = dst; f.aux = aux; f.Cd = Cd; f.dc0 = dc0; f.mode = mode; f.scale = scale; f.amax = amax;
    return f;
}

// input gradient of conv `id` from G (B, Hin, Win, K) with the reflect fold in the conv epilogue:
// packed columns [0, split) -> s0, [split, N) -> s1 (FoldSeg), then fold_fix_kernel for the
// reflected border terms.  sc: grad_scale of G.
int dgrad_fold(Bwd &k, int id, const float *G, const float *sc, const FoldSeg &s0, const FoldSeg &s1, int split,
               float *scl_out = nullptr) {
    const ConvShape s = conv_shape(id, k.C);
    const int Hin = id == CV_UP ? k.H : k.h, Win = id == CV_UP ? k.W : k.w;
    // a wave's NW x 16 columns must lie in one FoldSeg: every STAGE_ZP2 configuration of
    // launch_conv has NW = 2 (checked again by launch_conv_cfg)
    if (Hin < 4 || Win < 4 || split % FOLD_COL_ALIGN) return CISTA_ERR_UNSUPPORTED;
    ConvArgs a;
    memset(&a, 0, sizeof(a));
    a.in0 = G; a.c0 = s.cout; a.in1 = nullptr; a.c1 = 0;
    a.B = k.B; a.Hin = Hin; a.Win = Win; a.Hout = Hin + 2; a.Wout = Win + 2;
    a.wpack = blob<u32x4>(k.packed, k.L.dwp[id]);
    a.bias = blob<float>(k.packed, k.L.dbp[id]);
    a.wscale = blob<float>(k.packed, k.L.sc[id]) + 1;
    a.ascale = sc;
    a.N = s.cin; a.Cout = s.cin;
    a.fseg[0] = s0; a.fseg[1] = s1; a.fsplit = split;
    a.fborder = k.ws.fb;
    CHECK((launch_conv<STAGE_ZP2, EPI_FOLD, 1>(a, k.st)));
    FoldFixArgs f;
    f.fb = k.ws.fb; f.N = s.cin; f.B = k.B; f.n = Hin; f.m = Win;
    f.seg[0] = s0; f.seg[1] = s1; f.fsplit = split;
    // scl_out: fold_fix's last block turns s0's |max| slots (the interior published by the conv
    // epilogue, the border by fold_fix) into the pair (ticket_scale)
    if (scl_out && (!s0.amax || s1.amax)) return CISTA_ERR_INVALID;
    f.scl = scl_out;
    f.ticket = scl_out ? ticket_of(k) : nullptr;
    hipLaunchKernelGGL(fold_fix_kernel, g1d((long)k.B * (2 * Win + 2 * (Hin - 2)) * (s.cin / 4)), dim3(256), 0, k.st, f);
    return hip_ok();
}

// add: dst = add + fold (copy-free identity path; NULL add with accumulate 0 is plain dst = fold);
// dst2: a second destination receiving dst2 += fold from the same pass over src
int fold(Bwd &k, const float *src, int Cs, int sc0, float *dst, int Cd, int dc0, int n, int H, int W,
         float scale, int accumulate, const float *mask, const float *add = nullptr, float *dst2 = nullptr,
         unsigned *amax = nullptr) {
    FoldArgs f;
    f.src = src; f.Cs = Cs; f.sc0 = sc0; f.dst = dst; f.Cd = Cd; f.dc0 = dc0; f.n = n;
    f.B = k.B; f.H = H; f.W = W; f.scale = scale; f.accumulate = accumulate; f.mask = mask;
    f.add = add; f.dst2 = dst2; f.amax = amax;
    hipLaunchKernelGGL(fold_reflect_kernel, g1d((long)k.B * H * W * (n / 4)), dim3(256), 0, k.st, f);
    return hip_ok();
}

int copy_or_zero(float *dst, const float *src, size_t nfloat, hipStream_t st) {
    const hipError_t e = src ? hipMemcpyAsync(dst, src, nfloat * 4, hipMemcpyDeviceToDevice, st)
                             : hipMemsetAsync(dst, 0, nfloat * 4, st);
    return e == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
}

int run_backward(Bwd &k, const cista_params &P, const cista_frame_io &io, const Saved &sv,
                 const cista_grad_io &g, const cista_param_grads &pg) {
    const int B = k.B, H = k.H, W = k.W, h = k.h, w = k.w, C = k.C, D = k.cfg->depth;
    const long hw = (long)B * h * w, HW = (long)B * H * W;
    BwdWs &ws = k.ws;
    hipStream_t st = k.st;
    // the reflect fold in the dgrad epilogue (dgrad_fold) needs input rows 1 and n-2 distinct
    // (n, m >= 4); smaller images take the padded-domain dgrad + fold_reflect_kernel pass
    // (and FoldSeg splits at multiples of a wave's columns: C, 2C with C % 32 == 0 -- cfg_supported)
    const bool fold_ok = CISTA_FOLD_EPI && C % FOLD_COL_ALIGN == 0;
    const bool fold_half = fold_ok && h >= 4 && w >= 4, fold_full = fold_ok && H >= 4 && W >= 4;
    // ---- 1-2. output stage: rec = sigmoid(final_conv(u)), u = relu(upsamp_conv(up(h))) --------
    CHECK(copy_or_zero(ws.ghb, g.g_h, (size_t)hw * C, st));
    if (g.g_rec) {
        hipLaunchKernelGGL(sigmoid_bwd_kernel, g1d(HW), dim3(256), 0, st, g.g_rec, io.rec, ws.gpre, HW);
        CHECK(wgrad<XS_S1>(k, ws.gpre, 1, 0, 1, sv.u, C, nullptr, 0, C, H, W, H, W, pg.final_w, 1.0f, 0, pg.final_b));
        DgradSmallArgs d;
        d.G = ws.gpre; d.Gc = 1; d.Goff = 0; d.W = P.final_w; d.dX = ws.gU; d.Xc = C; d.Xoff = 0;
        d.mask = sv.u; d.B = B; d.Hin = H; d.Win = W; d.Hout = H; d.Wout = W; d.S = 1; d.Cout = 1; d.Cin = C;
        d.accumulate = 0;
        const float *gsu = nullptr;
        if (C % 8 == 0 && C / 8 <= 256) {                                               // g_U (ReLU'd)
            // pixels in a grid-stride loop (weights in registers), <= 8 workgroups per CU; the
            // scale pair of gU from the kernel's last block
            float *sc = claim_scale(k);
            CHECK_PTR(sc);
            const long ppb = 256 / (C / 8), nblk = (HW + ppb - 1) / ppb;
            const dim3 grid((unsigned)(nblk < 8 * NCU ? nblk : 8 * NCU));
            hipLaunchKernelGGL(transpose_w_kernel, g1d((long)C * 9), dim3(256), 0, st, P.final_w, 1, C, ws.wT);
            if (HW + (long)grid.x * ppb < INT32_MAX)
                hipLaunchKernelGGL(dgrad_final_kernel<int>, grid, dim3(256), 0, st, (const float *)ws.gpre, (const float *)ws.wT,
                                   (const float *)sv.u, ws.gU, B, H, W, C, scale_slots(k), ticket_of(k), sc);
            else
                hipLaunchKernelGGL(dgrad_final_kernel<long>, grid, dim3(256), 0, st, (const float *)ws.gpre, (const float *)ws.wT,
                                   (const float *)sv.u, ws.gU, B, H, W, C, scale_slots(k), ticket_of(k), sc);
            CHECK(hip_ok());
            slot_done(k);
            gsu = sc;
        } else {
            CHECK(dgrad_vec(k, d, P.final_w));
            hipLaunchKernelGGL(absmax_publish_kernel, dim3(1024), dim3(256), 0, st, (const float *)ws.gU, (long)HW * C,
                               scale_slots(k));
            gsu = scale_of(k);
            CHECK_PTR(gsu);
        }
        // upsample conv wgrad as a stride-1 wgrad over the materialised up(h) (in dxpF, which
        // the dgrad below overwrites); the gradient scale is shared with that dgrad
        if (HW * (C / 4) < INT32_MAX)
            hipLaunchKernelGGL(upsample2x_kernel<int>, g1d(HW * (C / 4)), dim3(256), 0, st, io.h, ws.dxpF, B, h, w, C);
        else
            hipLaunchKernelGGL(upsample2x_kernel<long>, g1d(HW * (C / 4)), dim3(256), 0, st, io.h, ws.dxpF, B, h, w, C);
        CHECK(wgrad<XS_S1>(k, ws.gU, C, 0, C, ws.dxpF, C, nullptr, 0, C, H, W, H, W, pg.up_w, 1.0f, 0, pg.up_b, gsu));
        float *gup = ws.gU;                              // g wrt up(h)
        if (fold_full) {
            gup = ws.dxpF;                               // (B, H, W, C): the dgrad's input gU is still read
            CHECK(dgrad_fold(k, CV_UP, ws.gU, gsu, fseg(gup, C, 0), fseg(nullptr, 0, 0), C));
        } else {
            CHECK(dgrad_conv(k, CV_UP, ws.gU, ws.dxpF, gsu));
            CHECK(fold(k, ws.dxpF, C, 0, ws.gU, C, 0, C, H, W, 1.0f, 0, nullptr));
        }
        if (hw * C / 4 < INT32_MAX)
            hipLaunchKernelGGL(upsample_bwd_kernel<int>, g1d(hw * C / 4), dim3(256), 0, st, (const float *)gup, ws.ghb,
                               B, h, w, C, 1);
        else
            hipLaunchKernelGGL(upsample_bwd_kernel<long>, g1d(hw * C / 4), dim3(256), 0, st, (const float *)gup, ws.ghb,
                               B, h, w, C, 1);
    } else {
        if (hipMemsetAsync(pg.final_b, 0, 4, st) != hipSuccess ||
            hipMemsetAsync(pg.final_w, 0, (size_t)9 * C * 4, st) != hipSuccess ||
            hipMemsetAsync(pg.up_b, 0, (size_t)C * 4, st) != hipSuccess ||
            hipMemsetAsync(pg.up_w, 0, (size_t)9 * C * C * 4, st) != hipSuccess)
            return CISTA_ERR_HIP;
    }
    // ---- 3. ConvLSTM ---------------------------------------------------------------------
    hipLaunchKernelGGL(lstm_bwd_kernel, g1d(hw * C), dim3(256), 0, st, (const float *)sv.lg, (const float *)io.c,
                       io.c_prev, (const float *)ws.ghb, g.g_c, ws.Gl, io.c_prev ? g.g_c_prev : nullptr, hw, C, scale_slots(k));
    const float *gsc = scale_of(k);
    CHECK_PTR(gsc);
    CHECK(on_side(k, [&] {
        return wgrad<XS_S1>(k, ws.Gl, 4 * C, 0, 4 * C, sv.y, C, io.h_prev, C, 2 * C, h, w, h, w, pg.lstm_w, 1.0f, 0,
                            pg.lstm_b, gsc);
    }));
    // Gl is overwritten by lstc_bwd_kernel (section 6) once this wgrad has read it
    const hipEvent_t lstm_wgrad_done = k.side ? mark(k, k.side) : nullptr;
    if (k.side && !lstm_wgrad_done) return CISTA_ERR_HIP;
    if (fold_half) {                                // relu(Dg) mask; h_prev's part if wanted
        float *sgy = claim_scale(k);                // gy's pair, from fold_fix's last block
        CHECK_PTR(sgy);
        CHECK(dgrad_fold(k, CV_LSTM, ws.Gl, gsc, fseg(ws.gy, C, 0, 1.0f, FOLD_MASK, const_cast<float *>(sv.y), scale_slots(k)),
                         fseg(io.h_prev ? g.g_h_prev : nullptr, C, 0), C, sgy));
        slot_done(k);
        gsc = sgy;
    } else {
        CHECK(dgrad_conv(k, CV_LSTM, ws.Gl, ws.dxp, gsc));
        CHECK(fold(k, ws.dxp, 2 * C, 0, ws.gy, C, 0, C, h, w, 1.0f, 0, sv.y, nullptr, nullptr, scale_slots(k)));
        if (io.h_prev && g.g_h_prev) CHECK(fold(k, ws.dxp, 2 * C, C, g.g_h_prev, C, 0, C, h, w, 1.0f, 0, nullptr));
        gsc = scale_of(k);
        CHECK_PTR(gsc);
    }
    // ---- 4. Dg conv (+ReLU) ----------------------------------------------------------------
    CHECK(on_side(k, [&] {
        return wgrad<XS_S1>(k, ws.gy, C, 0, C, io.z, 2 * C, nullptr, 0, 2 * C, h, w, h, w, pg.Dg_w, 1.0f, 0, pg.Dg_b, gsc);
    }));
    if (fold_half) {                                // g_z + fold
        CHECK(dgrad_fold(k, CV_DG, ws.gy, gsc, fseg(ws.gz, 2 * C, 0, 1.0f, g.g_z ? FOLD_ADD : FOLD_SET, const_cast<float *>(g.g_z)),
                         fseg(nullptr, 0, 0), 2 * C));
    } else {
        CHECK(dgrad_conv(k, CV_DG, ws.gy, ws.dxp, gsc));
        CHECK(fold(k, ws.dxp, 2 * C, 0, ws.gz, 2 * C, 0, 2 * C, h, w, 1.0f, 0, nullptr, g.g_z));
    }
    // ---- 5. ISTA, reversed (tied D, P, lambda accumulate over iterations) -------------------
    const float *lam = blob<float>(k.packed, k.L.lambda);
    if (D == 0) {
        if (hipMemsetAsync(pg.lambda, 0, (size_t)2 * C * 4, st) != hipSuccess ||
            hipMemsetAsync(pg.D_w, 0, (size_t)C * 2 * C * 9 * 4, st) != hipSuccess ||
            hipMemsetAsync(pg.D_b, 0, (size_t)C * 4, st) != hipSuccess ||
            hipMemsetAsync(pg.P_w, 0, (size_t)2 * C * C * 9 * 4, st) != hipSuccess ||
            hipMemsetAsync(pg.P_b, 0, (size_t)2 * C * 4, st) != hipSuccess)
            return CISTA_ERR_HIP;
    }
    if (hipMemsetAsync(ws.gx1, 0, (size_t)hw * C * 4, st) != hipSuccess) return CISTA_ERR_HIP;
    const int nbl = 512;   // softshrink_bwd blocks (lambda partials [nbl][2C])
    float *sclP = ws.scl + 2 * SCL_PAIRS, *sclD = sclP + 2 * D;      // per-iteration scale pairs of gv / gxk
    for (int it = D - 1; it >= 0; --it) {
        const float *v = sv.v + (size_t)it * hw * 2 * C;
        float *gv = ws.gv + (size_t)it * hw * 2 * C, *gxk = ws.gxk + (size_t)it * hw * C;
        // dlambda partials per (channel, block) of this iteration in ws.dlp; all iterations'
        // reduced after the loop (lambda_grad_kernel).  gv's scale pair from the kernel's last block
        if (2 * C <= 1024) {
            hipLaunchKernelGGL(softshrink_bwd4_kernel, dim3(nbl), dim3(256), 0, st, (const float *)ws.gz, v,
                               lam, gv, ws.dlp + (size_t)it * nbl * 2 * C, hw, 2 * C, scale_slots(k), ticket_of(k),
                               sclP + 2 * it);
            slot_done(k);
            gsc = sclP + 2 * it;
        } else {
            hipLaunchKernelGGL(softshrink_bwd_kernel, dim3(nbl), dim3(256), 0, st, (const float *)ws.gz, v,
                               lam, gv, ws.dlp + (size_t)it * nbl * 2 * C, hw, 2 * C, scale_slots(k));
            gsc = scale_of(k, sclP + 2 * it);
            CHECK_PTR(gsc);
        }
        // P: v = z_k + P(x_k) + b_P
        if (fold_half) {                            // gx1 += too; gxk's pair from fold_fix's last block
            CHECK(dgrad_fold(k, CV_P, gv, gsc, fseg(gxk, C, 0, 1.0f, FOLD_DST2, ws.gx1, scale_slots(k)), fseg(nullptr, 0, 0), C,
                             sclD + 2 * it));
            slot_done(k);
            gsc = sclD + 2 * it;
        } else {
            CHECK(dgrad_conv(k, CV_P, gv, ws.dxp, gsc));
            CHECK(fold(k, ws.dxp, C, 0, gxk, C, 0, C, h, w, 1.0f, 0, nullptr, nullptr, ws.gx1, scale_slots(k)));
            gsc = scale_of(k, sclD + 2 * it);
            CHECK_PTR(gsc);
        }
        // D: x_k = x1 - (D(z_k) + b_D)  ->  grad of D's output is -g_xk
        if (fold_half) {                            // identity path + fold
            CHECK(dgrad_fold(k, CV_D, gxk, gsc, fseg(ws.gz, 2 * C, 0, -1.0f, FOLD_ADD, gv), fseg(nullptr, 0, 0), 2 * C));
        } else {
            CHECK(dgrad_conv(k, CV_D, gxk, ws.dxp, gsc));
            CHECK(fold(k, ws.dxp, 2 * C, 0, ws.gz, 2 * C, 0, 2 * C, h, w, -1.0f, 0, nullptr, gv));
        }
    }
    if (D > 0) {
        // tied D / P weights: one wgrad over all iterations each (G and X stacked as D x B samples),
        // the split scale the smallest of the iterations' (their largest gradient)
        float *sP = sclD + 2 * D, *sD = sP + 2;
        CHECK(on_side(k, [&] {
            hipLaunchKernelGGL(min_scale_kernel, dim3(1), dim3(64), 0, k.st, (const float *)sclP, D, sP);
            hipLaunchKernelGGL(min_scale_kernel, dim3(1), dim3(64), 0, k.st, (const float *)sclD, D, sD);
            // lambda is (1, 2C, 1, 1): the per-block partials of every iteration, summed
            hipLaunchKernelGGL(lambda_grad_kernel, dim3(2 * C), dim3(256), 0, k.st, (const float *)ws.dlp, nbl, 2 * C, D,
                               pg.lambda);
            const int r = wgrad<XS_S1>(k, ws.gv, 2 * C, 0, 2 * C, sv.xs, C, nullptr, 0, C, h, w, h, w, pg.P_w, 1.0f, 0,
                                       pg.P_b, sP, D * B);
            if (r != CISTA_OK) return r;
            return wgrad<XS_S1>(k, ws.gxk, C, 0, C, sv.zl, 2 * C, nullptr, 0, 2 * C, h, w, h, w, pg.D_w, -1.0f, 0, pg.D_b,
                                sD, D * B);
        }));
    }
    // ---- 6. ConvLSTC --------------------------------------------------------------------------
    // Gg in Gl (4C: [gi | gf]), Go, gz0 (cell part): Gl held the ConvLSTM gradient that its
    // side-stream wgrad reads (the ISTA wgrads behind it on that stream keep running)
    if (lstm_wgrad_done && hipStreamWaitEvent(st, lstm_wgrad_done, 0) != hipSuccess) return CISTA_ERR_HIP;
    hipLaunchKernelGGL(lstc_bwd_kernel, g1d(hw * 2 * C), dim3(256), 0, st, (const float *)sv.gi,
                       (const float *)sv.gf, (const float *)sv.go, (const float *)sv.z0,
                       (const float *)io.c_lstc, io.c_lstc_prev, (const float *)ws.gz, g.g_c_lstc,
                       ws.Gl, ws.Go, ws.gz0, io.c_lstc_prev ? g.g_c_lstc_prev : nullptr, hw, 2 * C, scale_slots(k, 0), scale_slots(k, 1));
    gsc = scale_of(k);                                   // Go; Gl's scale is the next slot set
    CHECK_PTR(gsc);
    CHECK(on_side(k, [&] {
        return wgrad<XS_S1>(k, ws.Go, 2 * C, 0, 2 * C, sv.z0, 2 * C, io.z_prev, 2 * C, 4 * C, h, w, h, w,
                            pg.out_gates_w, 1.0f, 0, pg.out_gates_b, gsc);
    }));
    const bool want_zp = io.z_prev && g.g_z_prev;
    if (fold_half) {                                // gz0 is final here: its slot set follows Gl's
        CHECK(dgrad_fold(k, CV_OUTG, ws.Go, gsc, fseg(ws.gz0, 2 * C, 0, 1.0f, FOLD_ADD, ws.gz0, scale_slots(k, 1)),
                         fseg(want_zp ? g.g_z_prev : nullptr, 2 * C, 0), 2 * C));
    } else {
        CHECK(dgrad_conv(k, CV_OUTG, ws.Go, ws.dxp, gsc));
        CHECK(fold(k, ws.dxp, 4 * C, 0, ws.gz0, 2 * C, 0, 2 * C, h, w, 1.0f, 1, nullptr, nullptr, nullptr,
                   scale_slots(k, 1)));
        if (want_zp) CHECK(fold(k, ws.dxp, 4 * C, 2 * C, g.g_z_prev, 2 * C, 0, 2 * C, h, w, 1.0f, 0, nullptr));
    }
    gsc = scale_of(k);                                   // Gl (published by lstc_bwd_kernel)
    CHECK_PTR(gsc);
    CHECK(on_side(k, [&] {
        return wgrad<XS_S1>(k, ws.Gl, 4 * C, 0, 4 * C, sv.x1, C, io.z_prev, 2 * C, 3 * C, h, w, h, w,
                            pg.gates_w, 1.0f, 0, pg.gates_b, gsc);
    }));
    if (fold_half) {
        CHECK(dgrad_fold(k, CV_GATES, ws.Gl, gsc, fseg(ws.gx1, C, 0, 1.0f, FOLD_ADD, ws.gx1),
                         fseg(want_zp ? g.g_z_prev : nullptr, 2 * C, 0, 1.0f, FOLD_ADD, want_zp ? g.g_z_prev : nullptr), C));
    } else {
        CHECK(dgrad_conv(k, CV_GATES, ws.Gl, ws.dxp, gsc));
        CHECK(fold(k, ws.dxp, 3 * C, 0, ws.gx1, C, 0, C, h, w, 1.0f, 1, nullptr));
        if (want_zp) CHECK(fold(k, ws.dxp, 3 * C, C, g.g_z_prev, 2 * C, 0, 2 * C, h, w, 1.0f, 1, nullptr));
    }
    gsc = scale_of(k);                                   // gz0 (published by its last fold)
    CHECK_PTR(gsc);
    CHECK(on_side(k, [&] {
        return wgrad<XS_S1>(k, ws.gz0, 2 * C, 0, 2 * C, sv.x1, C, nullptr, 0, C, h, w, h, w, pg.P0_w, 1.0f, 0, pg.P0_b, gsc);
    }));
    const float *gsx = nullptr;                         // gx1 is final: W0's output gradient
    if (fold_half) {                                    // gx1's pair from fold_fix's last block
        float *sx = claim_scale(k);
        CHECK_PTR(sx);
        CHECK(dgrad_fold(k, CV_P0, ws.gz0, gsc, fseg(ws.gx1, C, 0, 1.0f, FOLD_ADD, ws.gx1, scale_slots(k)), fseg(nullptr, 0, 0), C,
                         sx));
        slot_done(k);
        gsx = sx;
    } else {
        CHECK(dgrad_conv(k, CV_P0, ws.gz0, ws.dxp, gsc));
        CHECK(fold(k, ws.dxp, C, 0, ws.gx1, C, 0, C, h, w, 1.0f, 1, nullptr, nullptr, nullptr, scale_slots(k)));
        gsx = scale_of(k);
        CHECK_PTR(gsx);
    }
    // ---- 7. W0 (stride 2) over x_full = cat(We(events), Wi(prev_image)), recomputed ----------
    float *xfull = ws.gU, *gxfull = ws.gU;   // x_full is dead once W0's wgrad has run
    {
        Frame f;
        memset(&f, 0, sizeof(f));
        f.cfg = k.cfg; f.packed = k.packed; f.L = k.L; f.B = B; f.H = H; f.W = W; f.h = h; f.w = w;
        f.C = C; f.events = io.events; f.prev_image = io.prev_image; f.full = xfull; f.st = st;
        f.need_full = true;
        CHECK(run_layer(f, CISTA_LAYER_INPUT));
    }
    CHECK(wgrad<XS_S2>(k, ws.gx1, C, 0, C, xfull, C, nullptr, 0, C, H, W, h, w, pg.W0_w, 1.0f, 0, pg.W0_b, gsx));
    {
        // padded-domain stride-2 dgrad into dxpF (split-f16 MFMA, the four output phases of a
        // G pixel as one 4C-column conv over G, pack_w0phase_kernel), then reflect-fold into gxfull
        int rc = CISTA_ERR_UNSUPPORTED;
        if (CISTA_W0_PHASE) {
            ConvArgs c;
            memset(&c, 0, sizeof(c));
            c.in0 = ws.gx1; c.c0 = C; c.in1 = nullptr; c.c1 = 0;
            c.B = B; c.Hin = h; c.Win = w; c.Hout = h + 1; c.Wout = w + 1;
            c.wpack = blob<u32x4>(k.packed, k.L.w4p);
            c.bias = blob<float>(k.packed, k.L.b4p);
            c.wscale = blob<float>(k.packed, k.L.sc[CV_W0]) + 1;
            c.ascale = gsx;
            c.N = 4 * C; c.Cout = C;
            c.out0 = ws.dxpF;
            rc = launch_conv<STAGE_ZP2, EPI_PH4, 1>(c, st);
        }
        if (rc == CISTA_ERR_UNSUPPORTED) {                 // VALU fallback
            const int Hp = H + 2, Wp = W + 2, ngx = (((Wp + 1) / 2) + S2_NJ - 1) / S2_NJ;
            hipLaunchKernelGGL(transpose_w_kernel, g1d((long)C * C * 9), dim3(256), 0, st, P.W0_w, C, C, ws.wT);
            hipLaunchKernelGGL(dgrad_s2_kernel, g1d((long)B * Hp * 2 * ngx * (C / 8)), dim3(256), 0, st,
                               (const float *)ws.gx1, C, 0, (const float *)ws.wT, C, C, B, h, w, ws.dxpF, Hp, Wp);
            rc = hip_ok();
        }
        CHECK(rc);
        CHECK(fold(k, ws.dxpF, C, 0, gxfull, C, 0, C, H, W, 1.0f, 0, nullptr));
    }
    // ---- 8. We / Wi ----------------------------------------------------------------------------
    const int half = C / 2, nb = k.cfg->num_bins;
    const int rin = wgrad_inputs(k, gxfull, io.events, io.prev_image, pg);
    if (rin != CISTA_ERR_UNSUPPORTED) CHECK(rin);
    else CHECK(wgrad<XS_NCHW>(k, gxfull, C, 0, half, io.events, nb, nullptr, 0, nb, H, W, H, W, pg.We_w, 1.0f, 0, pg.We_b));
    if (rin == CISTA_ERR_UNSUPPORTED) CHECK(wgrad<XS_NCHW>(k, gxfull, C, half, half, io.prev_image, 1, nullptr, 0, 1, H, W, H, W, pg.Wi_w, 1.0f, 0,
                         pg.Wi_b));
    if (g.g_prev_image) {
        DgradSmallArgs d;
        d.G = gxfull; d.Gc = C; d.Goff = half; d.W = P.Wi_w; d.dX = g.g_prev_image; d.Xc = 0; d.Xoff = 0;
        d.mask = nullptr; d.B = B; d.Hin = H; d.Win = W; d.Hout = H; d.Wout = W; d.S = 1; d.Cout = half;
        d.Cin = 1; d.accumulate = 0;
        if (half % 4 == 0 && half <= DC1_MAXC && C % 4 == 0)
            hipLaunchKernelGGL(dgrad_c1_kernel, dim3((unsigned)((long)B * ((H + 15) / 16) * ((W + 15) / 16))),
                               dim3(256), 0, st, (const float *)gxfull, C, half, (const float *)P.Wi_w, half,
                               g.g_prev_image, B, H, W);
        else
            hipLaunchKernelGGL(dgrad_small_kernel, g1d(HW), dim3(256), 0, st, d);
    }
    if (g.g_events) {                            // We dgrad: the events' own gradient
        DgradSmallArgs d;
        d.G = gxfull; d.Gc = C; d.Goff = 0; d.W = P.We_w; d.dX = g.g_events; d.Xc = 0; d.Xoff = 0;
        d.mask = nullptr; d.B = B; d.Hin = H; d.Win = W; d.Hout = H; d.Wout = W; d.S = 1; d.Cout = half;
        d.Cin = nb; d.accumulate = 0;
        hipLaunchKernelGGL(dgrad_small_kernel, g1d(HW * nb), dim3(256), 0, st, d);
    }
    return hip_ok();
}
}  // namespace

// =========================================================================================
extern "C" {

int cista_abi_version(void) { return CISTA_ABI_VERSION; }
#if CISTA_PROBE
// diagnostic builds only: every inference ISTA P launch reads and writes z inside its first
// mask + 1 elements (an L2-resident window of real data; results wrong).  0: off
int cista_debug_set_ista_p_probe(unsigned mask) {
    g_probe_mask = mask;
    return CISTA_OK;
}
#endif
#if CISTA_STAMPS
// diagnostic builds only: the conv kernels' phase timestamps go to buf (NULL: off)
int cista_debug_set_stamps(void *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(cista::g_cista_stamps), &buf, sizeof(buf)) == hipSuccess ? CISTA_OK
                                                                                            : CISTA_ERR_HIP;
}
// ... per EPI_FOLD launch, nlaunch regions of FOLD_STAMP_WG x 96 words (NULL: off); returns
// the number of regions filled since the previous call
int cista_debug_set_fold_stamps(void *buf, int nlaunch) {
    std::lock_guard<std::mutex> lock(g_fold_mu);
    const int used = g_fold_next;
    g_fold_ring = static_cast<unsigned long long *>(buf);
    g_fold_cap = buf ? nlaunch : 0;
    g_fold_next = 0;
    return used;
}
// ... and wgrad_tr_kernel's (scripts/wgrad_stamps.py)
int cista_debug_set_wstamps(void *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(cista::g_cista_wstamps), &buf, sizeof(buf)) == hipSuccess ? CISTA_OK
                                                                                             : CISTA_ERR_HIP;
}
#endif

const char *cista_status_string(int s) {
    switch (s) {
        case CISTA_OK: return "ok";
        case CISTA_ERR_INVALID: return "invalid argument (shape, NULL pointer or inconsistent states)";
        case CISTA_ERR_UNSUPPORTED: return "unsupported configuration (this build needs base_channels % 32 == 0)";
        case CISTA_ERR_HIP: return "HIP runtime error";
        case CISTA_ERR_WORKSPACE: return "workspace too small";
        case CISTA_ERR_ALIAS: return "an output buffer overlaps an input buffer";
        default: return "unknown status";
    }
}

size_t cista_packed_bytes(const cista_config *cfg) {
    if (!cfg_ok(cfg)) return 0;
    return make_layout(*cfg).total;
}

int cista_pack_params(const cista_config *cfg, const cista_params *p, void *packed, void *stream) {
    if (!cfg_ok(cfg) || !p || !packed) return CISTA_ERR_INVALID;
    if (!cfg_supported(cfg)) return CISTA_ERR_UNSUPPORTED;
    const void *req[] = {p->We_w, p->We_b, p->Wi_w, p->Wi_b, p->W0_w, p->W0_b, p->gates_w,
                         p->gates_b, p->out_gates_w, p->out_gates_b, p->P0_w, p->P0_b, p->lambda,
                         p->D_w, p->D_b, p->P_w, p->P_b, p->Dg_w, p->Dg_b, p->lstm_w, p->lstm_b,
                         p->up_w, p->up_b, p->final_w, p->final_b};
    for (const void *q : req)
        if (!q) return CISTA_ERR_INVALID;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int C = cfg->base_channels, nb = cfg->num_bins;
    const Layout L = make_layout(*cfg);
    // alignment gaps included: the packed bytes are a function of the parameters alone (data-
    // parallel replicas compare them bitwise)
    if (hipMemsetAsync(packed, 0, L.total, st) != hipSuccess) return CISTA_ERR_HIP;
    {
        const long ne = 9L * 25 * (nb + 1) * C + C;
        hipLaunchKernelGGL(compose_in_w0_kernel, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st,
                           p->We_w, p->Wi_w, p->We_b, p->Wi_b, p->W0_w, p->W0_b,
                           blobw<float>(packed, L.wC), blobw<float>(packed, L.bC), nb, C);
        const int ns = C * 32 * 9 + C;
        hipLaunchKernelGGL(s2d_weight_kernel, dim3((ns + 255) / 256), dim3(256), 0, st,
                           (const float *)blobw<float>(packed, L.wC), (const float *)blobw<float>(packed, L.bC),
                           blobw<float>(packed, L.wS), blobw<float>(packed, L.bS), nb, C);
    }
    {
        const int nu = 4 * C * C * 9 + 4 * C;
        hipLaunchKernelGGL(compose_up4_kernel, dim3((nu + 255) / 256), dim3(256), 0, st, p->up_w, p->up_b,
                           blobw<float>(packed, L.wU4), blobw<float>(packed, L.bU4), C);
    }
    const float *ws[CV_COUNT] = {p->W0_w, p->P0_w, p->gates_w, p->out_gates_w, p->D_w, p->P_w,
                                 p->Dg_w, p->lstm_w, p->up_w, blobw<float>(packed, L.wS),
                                 blobw<float>(packed, L.wU4)};
    const float *bs[CV_COUNT] = {p->W0_b, p->P0_b, p->gates_b, p->out_gates_b, p->D_b, p->P_b,
                                 p->Dg_b, p->lstm_b, p->up_b, blobw<float>(packed, L.bS),
                                 blobw<float>(packed, L.bU4)};
    {   // every conv's weight scale pair: two launches (WeightScaleJobs)
        static_assert(CV_COUNT <= WS_JOBS, "weight scale jobs");
        WeightScaleJobs j;
        memset(&j, 0, sizeof(j));
        j.jobs = CV_COUNT;
        j.part = blobw<float>(packed, L.wsp);
        for (int i = 0; i < CV_COUNT; ++i) {
            const ConvShape s = conv_shape(i, C);
            j.w[i] = ws[i];
            j.n[i] = (long)s.cout * s.cin * 9;
            j.scale[i] = blobw<float>(packed, L.sc[i]);
        }
        hipLaunchKernelGGL(weight_absmax_kernel, dim3(WS_PARTS, CV_COUNT), dim3(256), 0, st, j);
        hipLaunchKernelGGL(weight_scale_finalize_kernel, dim3(CV_COUNT), dim3(64), 0, st, j);
    }
    for (int i = 0; i < CV_COUNT; ++i) {
        const ConvShape s = conv_shape(i, C);
        PackArgs a;
        a.w = ws[i]; a.b = bs[i];
        a.scale = blobw<float>(packed, L.sc[i]);
        a.wp = blobw<u32x4>(packed, L.wp[i]);
        a.bp = blobw<float>(packed, L.bp[i]);
        a.Cout = s.cout; a.Cin = s.cin; a.G = s.G;
        const long total = (long)(s.cin / 32) * 9 * (s.cout / 16) * 64;
        hipLaunchKernelGGL(pack_conv_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
        // dgrad pack: K = forward Cout, N = forward Cin, same scale
        PackArgs d = a;
        d.wp = blobw<u32x4>(packed, L.dwp[i]);
        d.bp = blobw<float>(packed, L.dbp[i]);
        d.Cout = s.cin; d.Cin = s.cout;
        const long dtotal = (long)(s.cout / 32) * 9 * (s.cin / 16) * 64;
        const long dgrid = dtotal > s.cin ? dtotal : s.cin;
        hipLaunchKernelGGL(pack_dgrad_kernel, dim3((unsigned)((dgrid + 255) / 256)), dim3(256), 0, st, d);
    }
    {   // W0's dgrad as a four-phase conv (training backward), W0's forward scale
        PackArgs q;
        q.w = p->W0_w; q.b = nullptr;
        q.scale = blobw<float>(packed, L.sc[CV_W0]);
        q.wp = blobw<u32x4>(packed, L.w4p);
        q.bp = blobw<float>(packed, L.b4p);
        q.Cin = C; q.Cout = 4 * C; q.G = 1;
        const long total = (long)(C / 32) * 9 * (4 * C / 16) * 64;
        hipLaunchKernelGGL(pack_w0phase_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, q);
    }
    const int half = C / 2;
    hipLaunchKernelGGL(transpose_small_kernel, dim3((half * nb * 9 + 255) / 256), dim3(256), 0, st,
                       p->We_w, blobw<float>(packed, L.wE), half, nb);
    hipLaunchKernelGGL(transpose_small_kernel, dim3((half * 9 + 255) / 256), dim3(256), 0, st,
                       p->Wi_w, blobw<float>(packed, L.wI), half, 1);
    hipLaunchKernelGGL(final_weight_kernel, dim3((C * 9 + 255) / 256), dim3(256), 0, st,
                       p->final_w, blobw<float>(packed, L.wF), C);
    if (hipGetLastError() != hipSuccess) return CISTA_ERR_HIP;
    char *pb = static_cast<char *>(packed);
    if (hipMemcpyAsync(pb + L.bIn, p->We_b, half * 4, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(pb + L.bIn + half * 4, p->Wi_b, half * 4, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(pb + L.bF, p->final_b, 4, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(pb + L.lambda, p->lambda, 2 * C * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return CISTA_ERR_HIP;
    return CISTA_OK;
}

size_t cista_workspace_bytes(const cista_config *cfg, int B, int H, int W) {
    if (!cfg_ok(cfg) || B <= 0 || H <= 0 || W <= 0) return 0;
    return carve(nullptr, B, H, W, cfg->base_channels).bytes;
}

int cista_forward(const cista_config *cfg, const void *packed, int B, int H, int W,
                  const cista_frame_io *io, void *workspace, size_t workspace_bytes, void *stream) {
    CHECK(check_common(cfg, packed, B, H, W));
    if (!io || !io->events || !io->prev_image || !io->rec || !io->c_lstc || !io->z || !io->h ||
        !io->c || !workspace)
        return CISTA_ERR_INVALID;
    if ((H & 1) || (W & 1) || H < 4 || W < 4) return CISTA_ERR_INVALID;
    if ((io->h_prev == nullptr) != (io->c_prev == nullptr)) return CISTA_ERR_INVALID;
    const int C = cfg->base_channels, h = H / 2, w = W / 2;
    const size_t need = carve(nullptr, B, H, W, C).bytes;
    if (workspace_bytes < need) return CISTA_ERR_WORKSPACE;
    // aliasing: outputs must not overlap any input or each other
    const size_t nS2 = (size_t)B * h * w * 2 * C * 4, nS1 = (size_t)B * h * w * C * 4;
    const size_t nF = (size_t)B * H * W * 4, nE = nF * cfg->num_bins;
    const void *outs[] = {io->rec, io->c_lstc, io->z, io->h, io->c};
    const size_t outn[] = {nF, nS2, nS2, nS1, nS1};
    const void *ins[] = {io->events, io->prev_image, io->c_lstc_prev, io->z_prev, io->h_prev,
                         io->c_prev, workspace};
    const size_t inn[] = {nE, nF, nS2, nS2, nS1, nS1, need};
    for (int i = 0; i < 5; ++i) {
        for (int j = 0; j < 7; ++j)
            if (overlaps(outs[i], outn[i], ins[j], inn[j])) return CISTA_ERR_ALIAS;
        for (int j = i + 1; j < 5; ++j)
            if (overlaps(outs[i], outn[i], outs[j], outn[j])) return CISTA_ERR_ALIAS;
    }
    Frame f = make_frame(cfg, packed, B, H, W, workspace, stream);
    bind_io(f, io);
    static const int head[] = {CISTA_LAYER_INPUT, CISTA_LAYER_W0, CISTA_LAYER_P0, CISTA_LAYER_GATES,
                               CISTA_LAYER_OUT_GATES};
    static const int tail[] = {CISTA_LAYER_DG, CISTA_LAYER_LSTM, CISTA_LAYER_UPSAMPLE, CISTA_LAYER_FINAL};
    CHECK(run_layers(f, head, 5));
    CHECK(run_ista(f, cfg->depth));
    return run_layers(f, tail, 4);
}

struct cista_sequence {
    hipGraph_t graph;
    hipGraphExec_t exec;
};

int cista_sequence_capture(const cista_config *cfg, const void *packed, int B, int H, int W,
                           const cista_frame_io *io, int n_frames, void *workspace, size_t workspace_bytes,
                           cista_sequence **out, void *stream) {
    if (!out || !io || n_frames <= 0) return CISTA_ERR_INVALID;
    *out = nullptr;
    hipStream_t cs;
    if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) return CISTA_ERR_HIP;
    // the private stream starts after the work the caller has enqueued on `stream` (inputs,
    // packed parameters, the workspace's previous users)
    int status = CISTA_OK;
    hipEvent_t ready = nullptr;
    if (hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(ready, static_cast<hipStream_t>(stream)) != hipSuccess ||
        hipStreamWaitEvent(cs, ready, 0) != hipSuccess)
        status = CISTA_ERR_HIP;
    // a first eager frame on the private stream: one-time kernel attributes (LDS limits) are set
    // outside the capture, and argument errors surface before any graph exists
    if (status == CISTA_OK) status = cista_forward(cfg, packed, B, H, W, &io[0], workspace, workspace_bytes, cs);
    if (status == CISTA_OK && hipStreamSynchronize(cs) != hipSuccess) status = CISTA_ERR_HIP;
    hipGraph_t g = nullptr;
    if (status == CISTA_OK) {
        if (hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal) != hipSuccess) status = CISTA_ERR_HIP;
        for (int f = 0; status == CISTA_OK && f < n_frames; ++f)
            status = cista_forward(cfg, packed, B, H, W, &io[f], workspace, workspace_bytes, cs);
        const hipError_t e = hipStreamEndCapture(cs, &g);   // always end a begun capture
        if (status == CISTA_OK && e != hipSuccess) status = CISTA_ERR_HIP;
    }
    hipGraphExec_t ex = nullptr;
    if (status == CISTA_OK && hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) != hipSuccess) status = CISTA_ERR_HIP;
    (void)hipStreamDestroy(cs);
    if (ready) (void)hipEventDestroy(ready);
    if (status != CISTA_OK) {
        if (g) (void)hipGraphDestroy(g);
        return status;
    }
    *out = new cista_sequence{g, ex};
    return CISTA_OK;
}

int cista_sequence_launch(cista_sequence *seq, void *stream) {
    if (!seq) return CISTA_ERR_INVALID;
    return hipGraphLaunch(seq->exec, static_cast<hipStream_t>(stream)) == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
}

void cista_sequence_destroy(cista_sequence *seq) {
    if (!seq) return;
    (void)hipGraphExecDestroy(seq->exec);
    (void)hipGraphDestroy(seq->graph);
    delete seq;
}

int cista_stage_input(const cista_config *cfg, const void *packed, int B, int H, int W,
                      const float *events, const float *prev_image, float *x1, void *workspace,
                      size_t workspace_bytes, void *stream) {
    CHECK(check_common(cfg, packed, B, H, W));
    if (!events || !prev_image || !x1 || !workspace || (H & 1) || (W & 1)) return CISTA_ERR_INVALID;
    if (workspace_bytes < carve(nullptr, B, H, W, cfg->base_channels).bytes) return CISTA_ERR_WORKSPACE;
    Frame f = make_frame(cfg, packed, B, H, W, workspace, stream);
    f.events = events; f.prev_image = prev_image; f.x1 = x1;
    static const int l[] = {CISTA_LAYER_INPUT, CISTA_LAYER_W0};
    return run_layers(f, l, 2);
}

int cista_stage_lstc(const cista_config *cfg, const void *packed, int B, int h, int w,
                     const float *x1, const float *z_prev, const float *c_prev, float *z_out,
                     float *c_out, void *workspace, size_t workspace_bytes, void *stream) {
    CHECK(check_common(cfg, packed, B, h, w));
    if (!x1 || !z_out || !c_out || !workspace) return CISTA_ERR_INVALID;
    if (workspace_bytes < carve(nullptr, B, 2 * h, 2 * w, cfg->base_channels).bytes) return CISTA_ERR_WORKSPACE;
    Frame f = make_frame(cfg, packed, B, 2 * h, 2 * w, workspace, stream);
    f.x1 = const_cast<float *>(x1); f.z_prev = z_prev; f.c_lstc_prev = c_prev;
    f.z = z_out; f.c_lstc = c_out;
    static const int l[] = {CISTA_LAYER_P0, CISTA_LAYER_GATES, CISTA_LAYER_OUT_GATES};
    return run_layers(f, l, 3);
}

int cista_stage_ista(const cista_config *cfg, const void *packed, int B, int h, int w,
                     const float *x1, float *z, int iters, void *workspace, size_t workspace_bytes,
                     void *stream) {
    CHECK(check_common(cfg, packed, B, h, w));
    if (!x1 || !z || !workspace || iters < 0) return CISTA_ERR_INVALID;
    if (workspace_bytes < carve(nullptr, B, 2 * h, 2 * w, cfg->base_channels).bytes) return CISTA_ERR_WORKSPACE;
    Frame f = make_frame(cfg, packed, B, 2 * h, 2 * w, workspace, stream);
    f.x1 = const_cast<float *>(x1); f.z = z;
    return run_ista(f, iters);
}

int cista_stage_decoder(const cista_config *cfg, const void *packed, int B, int h, int w,
                        const float *z, const float *h_prev, const float *c_prev, float *h_out,
                        float *c_out, void *workspace, size_t workspace_bytes, void *stream) {
    CHECK(check_common(cfg, packed, B, h, w));
    if (!z || !h_out || !c_out || !workspace || ((h_prev == nullptr) != (c_prev == nullptr)))
        return CISTA_ERR_INVALID;
    if (workspace_bytes < carve(nullptr, B, 2 * h, 2 * w, cfg->base_channels).bytes) return CISTA_ERR_WORKSPACE;
    Frame f = make_frame(cfg, packed, B, 2 * h, 2 * w, workspace, stream);
    f.z = const_cast<float *>(z); f.h_prev = h_prev; f.c_prev = c_prev; f.hs = h_out; f.cs = c_out;
    static const int l[] = {CISTA_LAYER_DG, CISTA_LAYER_LSTM};
    return run_layers(f, l, 2);
}

int cista_stage_output(const cista_config *cfg, const void *packed, int B, int h, int w,
                       const float *hstate, float *rec, float *pre_sigmoid, void *workspace,
                       size_t workspace_bytes, void *stream) {
    CHECK(check_common(cfg, packed, B, h, w));
    if (!hstate || !rec || !workspace) return CISTA_ERR_INVALID;
    if (workspace_bytes < carve(nullptr, B, 2 * h, 2 * w, cfg->base_channels).bytes) return CISTA_ERR_WORKSPACE;
    Frame f = make_frame(cfg, packed, B, 2 * h, 2 * w, workspace, stream);
    f.hs = const_cast<float *>(hstate); f.rec = rec; f.pre = pre_sigmoid;
    static const int l[] = {CISTA_LAYER_UPSAMPLE, CISTA_LAYER_FINAL};
    return run_layers(f, l, 2);
}

double cista_layer_macs(const cista_config *cfg, int layer, int B, int H, int W) {
    if (!cfg_ok(cfg)) return 0.0;
    return layer_macs(*cfg, layer, B, H, W);
}

int cista_tile_plan(int B, int Hout, int Wout, int block_px, int *out) {
    if (!out || B < 1 || Hout < 1 || Wout < 1 || (block_px != 192 && block_px != 96)) return CISTA_ERR_INVALID;
    // the forward double-buffered configurations: NI = 4 halo items per thread x 256 threads,
    // two LDS images, two workgroups per CU, row-aligned m-tiles allowed (launch_conv_cfg)
    const TilePlan p = plan_tiles(B, Hout, Wout, block_px, 1, 4 * 256, 2, 2, true, 0.0, false);
    const Tile *t[2] = {&p.a, &p.b};
    for (int r = 0; r < 2; ++r) {
        out[5 * r + 0] = t[r]->TH; out[5 * r + 1] = t[r]->TW; out[5 * r + 2] = t[r]->ty;
        out[5 * r + 3] = t[r]->tx; out[5 * r + 4] = t[r]->mseg;
    }
    out[10] = p.wa;
    const Tile one = choose_tile(Hout, Wout, block_px, 1, 4 * 256, 2, 2, true, 0.0);
    out[11] = one.ty * one.tx;
    out[12] = one.mseg;
    out[13] = 0;
    return CISTA_OK;
}

int cista_layer_fused(const cista_config *cfg, int layer) {
    if (!cfg_ok(cfg)) return 0;
    return layer == CISTA_LAYER_W0 && fused_input(*cfg) ? 1 : 0;
}

int cista_launch_layer(const cista_config *cfg, const void *packed, int layer, int B, int H, int W,
                       const cista_frame_io *io, void *workspace, size_t workspace_bytes,
                       void *stream) {
    CHECK(check_common(cfg, packed, B, H, W));
    if (!io || !workspace || layer < 0 || layer >= CISTA_LAYER_COUNT) return CISTA_ERR_INVALID;
    if (workspace_bytes < carve(nullptr, B, H, W, cfg->base_channels).bytes) return CISTA_ERR_WORKSPACE;
    Frame f = make_frame(cfg, packed, B, H, W, workspace, stream);
    bind_io(f, io);
    return run_layer(f, layer);
}


size_t cista_saved_bytes(const cista_config *cfg, int B, int H, int W) {
    if (!cfg_ok(cfg) || B <= 0 || H <= 0 || W <= 0) return 0;
    return carve_saved(nullptr, *cfg, B, H, W).bytes;
}

size_t cista_train_workspace_bytes(const cista_config *cfg, int B, int H, int W) {
    if (!cfg_ok(cfg) || B <= 0 || H <= 0 || W <= 0) return 0;
    const size_t a = carve(nullptr, B, H, W, cfg->base_channels).bytes;
    const size_t b = carve_bwd(nullptr, *cfg, B, H, W).bytes;
    return a > b ? a : b;
}

static int train_supported(const cista_config *cfg) {
    return (cfg->base_channels % 32 == 0 && cfg->base_channels <= 256) ? CISTA_OK : CISTA_ERR_UNSUPPORTED;
}

// the backward's dominant launch on its own (timing / PMC hook): the tied ISTA P weight
// gradient over all depth iterations, exactly as run_backward launches it
int cista_wgrad_ista_p(const cista_config *cfg, int B, int H, int W, const float *G, const float *X,
                       const float *gscale, float *dW, float *db, void *workspace, size_t workspace_bytes,
                       void *stream) {
    if (!cfg_ok(cfg) || train_supported(cfg) != CISTA_OK || cfg->depth < 1) return CISTA_ERR_UNSUPPORTED;
    if (!G || !X || !gscale || !dW || !db || !workspace || B <= 0) return CISTA_ERR_INVALID;
    if ((H & 1) || (W & 1) || H < 4 || W < 4) return CISTA_ERR_INVALID;
    Bwd k;
    k.cfg = cfg; k.packed = nullptr; k.L = make_layout(*cfg);
    k.B = B; k.H = H; k.W = W; k.h = H / 2; k.w = W / 2; k.C = cfg->base_channels;
    k.st = static_cast<hipStream_t>(stream);
    k.ws = carve_bwd(workspace, *cfg, B, H, W);
    k.slot = 0;
    k.pair = 0;
    if (workspace_bytes < k.ws.bytes) return CISTA_ERR_WORKSPACE;
    const int C = k.C;
    return wgrad<XS_S1>(k, G, 2 * C, 0, 2 * C, X, C, nullptr, 0, C, k.h, k.w, k.h, k.w, dW, 1.0f, 0, db, gscale,
                        cfg->depth * B);
}

int cista_wgrad_w0(const cista_config *cfg, int B, int H, int W, const float *G, const float *X,
                   const float *gscale, float *dW, float *db, void *workspace, size_t workspace_bytes,
                   void *stream) {
    if (!cfg_ok(cfg) || train_supported(cfg) != CISTA_OK) return CISTA_ERR_UNSUPPORTED;
    if (!G || !X || !gscale || !dW || !db || !workspace || B <= 0) return CISTA_ERR_INVALID;
    if ((H & 1) || (W & 1) || H < 4 || W < 4) return CISTA_ERR_INVALID;
    Bwd k;
    k.cfg = cfg; k.packed = nullptr; k.L = make_layout(*cfg);
    k.B = B; k.H = H; k.W = W; k.h = H / 2; k.w = W / 2; k.C = cfg->base_channels;
    k.st = static_cast<hipStream_t>(stream);
    k.ws = carve_bwd(workspace, *cfg, B, H, W);
    k.slot = 0;
    k.pair = 0;
    if (workspace_bytes < k.ws.bytes) return CISTA_ERR_WORKSPACE;
    const int C = k.C;
    return wgrad<XS_S2>(k, G, C, 0, C, X, C, nullptr, 0, C, H, W, k.h, k.w, dW, 1.0f, 0, db, gscale);
}

int cista_forward_train(const cista_config *cfg, const void *packed, int B, int H, int W,
                        const cista_frame_io *io, void *saved, size_t saved_bytes, void *workspace,
                        size_t workspace_bytes, void *stream) {
    CHECK(check_common(cfg, packed, B, H, W));
    CHECK(train_supported(cfg));
    if (!io || !io->events || !io->prev_image || !io->rec || !io->c_lstc || !io->z || !io->h ||
        !io->c || !workspace || !saved)
        return CISTA_ERR_INVALID;
    if ((H & 1) || (W & 1) || H < 4 || W < 4) return CISTA_ERR_INVALID;
    if ((io->h_prev == nullptr) != (io->c_prev == nullptr)) return CISTA_ERR_INVALID;
    if (workspace_bytes < carve(nullptr, B, H, W, cfg->base_channels).bytes) return CISTA_ERR_WORKSPACE;
    const Saved sv = carve_saved(saved, *cfg, B, H, W);
    if (saved_bytes < sv.bytes) return CISTA_ERR_WORKSPACE;
    Frame f = make_frame(cfg, packed, B, H, W, workspace, stream);
    bind_io(f, io);
    f.x1 = sv.x1; f.z0 = sv.z0; f.gi = sv.gi; f.gf = sv.gf; f.go = sv.go; f.zl = sv.zl;
    f.v = sv.v; f.xs = sv.xs; f.y = sv.y; f.lg = sv.lg; f.u = sv.u;
    static const int head[] = {CISTA_LAYER_INPUT, CISTA_LAYER_W0, CISTA_LAYER_P0, CISTA_LAYER_GATES,
                               CISTA_LAYER_OUT_GATES};
    static const int tail[] = {CISTA_LAYER_DG, CISTA_LAYER_LSTM, CISTA_LAYER_UPSAMPLE, CISTA_LAYER_FINAL};
    CHECK(run_layers(f, head, 5));
    CHECK(run_ista(f, cfg->depth));
    return run_layers(f, tail, 4);
}

int cista_backward(const cista_config *cfg, const void *packed, const cista_params *params, int B,
                   int H, int W, const cista_frame_io *io, const void *saved, size_t saved_bytes,
                   const cista_grad_io *grads, size_t grads_bytes, const cista_param_grads *pg,
                   void *workspace, size_t workspace_bytes, void *stream) {
    CHECK(check_common(cfg, packed, B, H, W));
    CHECK(train_supported(cfg));
    if (!params || !io || !saved || !grads || !pg || !workspace) return CISTA_ERR_INVALID;
    if (!params->W0_w || !params->final_w || !params->Wi_w) return CISTA_ERR_INVALID;
    const void *req[] = {pg->We_w, pg->We_b, pg->Wi_w, pg->Wi_b, pg->W0_w, pg->W0_b, pg->gates_w,
                         pg->gates_b, pg->out_gates_w, pg->out_gates_b, pg->P0_w, pg->P0_b, pg->lambda,
                         pg->D_w, pg->D_b, pg->P_w, pg->P_b, pg->Dg_w, pg->Dg_b, pg->lstm_w, pg->lstm_b,
                         pg->up_w, pg->up_b, pg->final_w, pg->final_b};
    for (const void *q : req)
        if (!q) return CISTA_ERR_INVALID;
    if ((H & 1) || (W & 1) || H < 4 || W < 4) return CISTA_ERR_INVALID;
    const Saved sv = carve_saved(const_cast<void *>(saved), *cfg, B, H, W);
    if (saved_bytes < sv.bytes) return CISTA_ERR_WORKSPACE;
    // the caller's view of cista_grad_io: members it does not have are NULL (never read)
    constexpr size_t GIO_V1 = offsetof(cista_grad_io, g_events);
    if (grads_bytes < GIO_V1) return CISTA_ERR_INVALID;
    cista_grad_io g = {};
    memcpy(&g, grads, grads_bytes < sizeof(g) ? grads_bytes : sizeof(g));
    Bwd k;
    k.cfg = cfg; k.packed = packed; k.L = make_layout(*cfg);
    k.B = B; k.H = H; k.W = W; k.h = H / 2; k.w = W / 2; k.C = cfg->base_channels;
    k.st = static_cast<hipStream_t>(stream);
    k.ws = carve_bwd(workspace, *cfg, B, H, W);
    k.slot = 0;
    k.pair = 0;
    if (workspace_bytes < k.ws.bytes) return CISTA_ERR_WORKSPACE;
    // the gradient |max| slots start at zero (slots_scale_kernel re-zeroes the ones it reads)
    if (hipMemsetAsync(k.ws.amax, 0, AMAX_WORDS * sizeof(unsigned), k.st) != hipSuccess)
        return CISTA_ERR_HIP;
    // the side stream is the current device's: used only when the caller's stream is on it
    hipDevice_t sdev = -1;
    if (side_enabled() && hipGetDevice(&k.dev) == hipSuccess && hipStreamGetDevice(k.st, &sdev) == hipSuccess &&
        sdev == k.dev && event_pool(k.dev))
        k.side = side_stream(k.dev);
    const int r = run_backward(k, *params, *io, sv, g, *pg);
    const int j = join_side(k);               // also after a failed call: nothing left running
    return r != CISTA_OK ? r : j;
}
}  // extern "C"
