// cista_abi.hip -- C ABI (include/cista_lstc.h) of the MI355X CISTA-LSTC hot path:
// parameter packing, workspace carving, per-layer launch configuration and the per-frame
// schedule of CistaLSTCNet.forward (reference e2v/e2v_model.py:41-90).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/cista_lstc.h"
#include "cista_kernels.hpp"

using namespace cista;

namespace {

constexpr size_t ALIGN = 256;
inline size_t align_up(size_t x) { return (x + ALIGN - 1) & ~(ALIGN - 1); }

// ---------------------------------------------------------------------------------------
// packed parameter blob layout
// ---------------------------------------------------------------------------------------
enum ConvId { CV_W0, CV_P0, CV_GATES, CV_OUTG, CV_D, CV_P, CV_DG, CV_LSTM, CV_UP, CV_COUNT };

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
        default: return {C, C, 1};                   // CV_UP
    }
}

struct Layout {
    size_t wp[CV_COUNT], bp[CV_COUNT], sc[CV_COUNT];
    size_t wE, wI, bIn, wF, bF, lambda;
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
    L.wE = off; off = align_up(off + (size_t)nb * 9 * (C / 2) * 4);
    L.wI = off; off = align_up(off + (size_t)9 * (C / 2) * 4);
    L.bIn = off; off = align_up(off + (size_t)C * 4);
    L.wF = off; off = align_up(off + (size_t)9 * C * 4);
    L.bF = off; off = align_up(off + 4);
    L.lambda = off; off = align_up(off + (size_t)2 * C * 4);
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

Workspace carve(void *ws, int B, int H, int W, int C) {
    const size_t hw = (size_t)(H / 2) * (W / 2);
    Workspace w;
    size_t off = 0;
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
struct Tile { int TH, TW, ty, tx; size_t lds; };

size_t lds_bytes(int TH, int TW, int S) {
    const int HP = ((TH - 1) * S + 3) * ((TW - 1) * S + 3);
    return (size_t)((HP + 15) & ~15) * 8 * 16;
}

// max_items: staging items (HP rounded to 8, x4 k-groups) one workgroup may hold in registers
// (0 = unlimited); nbuf: LDS images (2 for the double-buffered loop)
Tile choose_tile(int Hout, int Wout, int block_px, int S, int max_items, int nbuf) {
    Tile best{1, 1, Hout, Wout, 0};
    double best_eff = -1.0;
    size_t best_lds = ~(size_t)0;
    const size_t lds_cap = 80 * 1024;   // two workgroups per CU
    for (int TW = 1; TW <= block_px && TW <= Wout; ++TW) {
#if CISTA_TW16
        // 16-pixel m-tiles that never wrap a tile row read LDS without bank conflicts
        if (Wout >= 16 && (TW % 16) != 0) continue;
#endif
        int TH = block_px / TW;
        if (TH > Hout) TH = Hout;
        if (TH < 1) continue;
        auto items = [&](int th) { return ((((th - 1) * S + 3) * ((TW - 1) * S + 3) + 7) & ~7) * 4; };
        while (max_items && TH > 1 && items(TH) > max_items) --TH;
        if (max_items && items(TH) > max_items) continue;
        const size_t lds = lds_bytes(TH, TW, S) * nbuf;
        if (lds > lds_cap) continue;
        const int ty = (Hout + TH - 1) / TH, tx = (Wout + TW - 1) / TW;
        const double eff = (double)Hout * Wout / ((double)ty * tx * block_px);
        if (eff > best_eff + 1e-9 || (eff > best_eff - 1e-9 && lds < best_lds)) {
            best_eff = eff;
            best_lds = lds;
            best = Tile{TH, TW, ty, tx, lds};
        }
    }
    return best;
}

// dynamic LDS above 64 KiB must be enabled per kernel (once; not a stream operation)
bool allow_big_lds(const void *kern) {
    static const void *done[64];
    static int ndone = 0;
    for (int i = 0; i < ndone; ++i)
        if (done[i] == kern) return true;
    if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
        return false;
    if (ndone < 64) done[ndone++] = kern;
    return true;
}

// ---------------------------------------------------------------------------------------
// conv launch
// ---------------------------------------------------------------------------------------
template <int MT_W, int NW, int WM, int WN, int STAGE, int EPI, int G, bool PF = false, int NI = 0>
int launch_conv_cfg(ConvArgs a, hipStream_t st) {
    constexpr int block_px = WM * MT_W * 16;
    constexpr int S = STAGE == STAGE_S2 ? 2 : 1;
    const Tile t = choose_tile(a.Hout, a.Wout, block_px, S, NI ? NI * 256 : 0, NI ? 2 : 1);
    a.TH = t.TH;
    a.TW = t.TW;
    a.tiles_y = t.ty;
    a.tiles_x = t.tx;
    constexpr int nblk_cols = WN * NW * 16;
    if (a.N % nblk_cols) return CISTA_ERR_UNSUPPORTED;
    auto kern = conv3x3_split3<MT_W, NW, WM, WN, STAGE, EPI, G, PF, NI>;
    if (!allow_big_lds((const void *)kern)) return CISTA_ERR_HIP;
    dim3 grid((unsigned)((long)a.B * t.ty * t.tx), (unsigned)(a.N / nblk_cols));
    // the LDS also holds the epilogue's per-wave transpose tiles (4 waves x 16 x (NW*16+4))
    const size_t epi_lds = (size_t)4 * 16 * (NW * 16 + 4) * 4;
    hipLaunchKernelGGL(kern, grid, dim3(256), t.lds > epi_lds ? t.lds : epi_lds, st, a);
    return hipGetLastError() == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
}

// pick the wave tiling from the number of packed output columns.
// CISTA_VARIANT selects the tiling family (A/B builds for scripts/layer_bench.py):
//   0: MT_W=8 x NW=4 waves, no B prefetch
//   1: MT_W=16 x NW=2 waves with B-fragment prefetch where the epilogue allows NW=2
//   2: double-buffered K loop (next halo chunk prefetched into registers), B prefetch
#ifndef CISTA_VARIANT
#define CISTA_VARIANT 2
#endif
#ifndef CISTA_TW16
#define CISTA_TW16 0
#endif
#ifndef CISTA_PF_MT
#define CISTA_PF_MT 12
#endif
template <int STAGE, int EPI, int G>
int launch_conv(const ConvArgs &a, hipStream_t st) {
    if constexpr (STAGE == STAGE_S2) {
        if (a.N % 64 == 0) return launch_conv_cfg<2, 4, 4, 1, STAGE, EPI, G>(a, st);
        if (a.N % 32 == 0) return launch_conv_cfg<2, 2, 4, 1, STAGE, EPI, G>(a, st);
        return CISTA_ERR_UNSUPPORTED;
    } else if constexpr (EPI == EPI_UP_Q) {      // needs WN == 1
        if (a.N == 64) return launch_conv_cfg<8, 4, 4, 1, STAGE, EPI, G>(a, st);
        if (a.N == 32) return launch_conv_cfg<8, 2, 4, 1, STAGE, EPI, G>(a, st);
        return CISTA_ERR_UNSUPPORTED;
    } else if constexpr (CISTA_VARIANT == 2 && STAGE == STAGE_S1) {
        // double-buffered K loop, 192-pixel workgroups, halo items in 4 x 8 VGPRs per thread
        if constexpr (G == 4) {
            if (a.N % 128 == 0) return launch_conv_cfg<6, 4, 2, 2, STAGE, EPI, G, true, 4>(a, st);
        } else {
            if (a.N % 128 == 0) return launch_conv_cfg<12, 2, 1, 4, STAGE, EPI, G, true, 4>(a, st);
            if (a.N == 64) return launch_conv_cfg<6, 2, 2, 2, STAGE, EPI, G, true, 4>(a, st);
            if (a.N == 32) return launch_conv_cfg<3, 2, 4, 1, STAGE, EPI, G, true, 4>(a, st);
        }
        return CISTA_ERR_UNSUPPORTED;
    } else if constexpr (CISTA_VARIANT >= 1 && G <= 2) {
        constexpr int MT = CISTA_PF_MT;
        if (a.N % 128 == 0) return launch_conv_cfg<MT, 2, 1, 4, STAGE, EPI, G, true>(a, st);
        if (a.N == 64) return launch_conv_cfg<MT, 2, 2, 2, STAGE, EPI, G, true>(a, st);
        if (a.N == 32) return launch_conv_cfg<MT, 2, 4, 1, STAGE, EPI, G, true>(a, st);
        return CISTA_ERR_UNSUPPORTED;
    } else {
        if (a.N >= 256 && a.N % 256 == 0) return launch_conv_cfg<8, 4, 1, 4, STAGE, EPI, G>(a, st);
        if (a.N >= 128 && a.N % 128 == 0) return launch_conv_cfg<8, 4, 2, 2, STAGE, EPI, G>(a, st);
        if constexpr (G <= 2) {
            if (a.N == 64) return launch_conv_cfg<8, 4, 4, 1, STAGE, EPI, G>(a, st);
            if (a.N == 32) return launch_conv_cfg<8, 2, 4, 1, STAGE, EPI, G>(a, st);
        }
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
    hipStream_t st;
};

// the upsample conv's wave holds all C output channels (WN == 1) for C = 32 and 64
inline bool up_q_path(int C) { return C == 64 || C == 32; }

int run_layer(const Frame &f, int layer) {
    const int C = f.C, B = f.B, h = f.h, w = f.w;
    ConvArgs a;
    switch (layer) {
        case CISTA_LAYER_INPUT: {                                      // e2v_model.py:62-64
            InputArgs ia;
            ia.events = f.events; ia.prev = f.prev_image;
            ia.wE = blob<float>(f.packed, f.L.wE); ia.wI = blob<float>(f.packed, f.L.wI);
            ia.bias = blob<float>(f.packed, f.L.bIn);
            ia.out = f.full; ia.B = B; ia.H = f.H; ia.W = f.W; ia.nb = f.cfg->num_bins; ia.C = C;
            const long npix = (long)B * f.H * f.W;
            const dim3 g1((unsigned)((npix + 255) / 256));
            const size_t lds = (size_t)256 * (C + 1) * 4;
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
            a = conv_args(f.packed, f.L, CV_W0, C, B, f.H, f.W, h, w, f.full, C, nullptr, 0);
            a.out0 = f.x1;
            return launch_conv<STAGE_S2, EPI_BIAS, 1>(a, f.st);
        case CISTA_LAYER_P0:                                           // base_layers.py:61
            a = conv_args(f.packed, f.L, CV_P0, C, B, h, w, h, w, f.x1, C, nullptr, 0);
            a.out0 = f.z0;
            return launch_conv<STAGE_S1, EPI_BIAS, 1>(a, f.st);
        case CISTA_LAYER_GATES:     // c = sig(f) c_prev + sig(i) z0, gates(cat(x1, z_prev)) :57-67
            a = conv_args(f.packed, f.L, CV_GATES, C, B, h, w, h, w, f.x1, C, f.z_prev, 2 * C);
            a.out0 = f.c_lstc; a.aux0 = f.c_lstc_prev; a.aux1 = f.z0;
            return launch_conv<STAGE_S1, EPI_LSTC_CELL, 2>(a, f.st);
        case CISTA_LAYER_OUT_GATES: // z = sig(out_gates(cat(z0, z_prev))) tanh(c)          :63,69
            a = conv_args(f.packed, f.L, CV_OUTG, C, B, h, w, h, w, f.z0, 2 * C, f.z_prev, 2 * C);
            a.out0 = f.z; a.aux0 = f.c_lstc;
            return launch_conv<STAGE_S1, EPI_LSTC_OUT, 1>(a, f.st);
        case CISTA_LAYER_ISTA_D:    // x = x1 - D(z)                              e2v_model.py:73-74
            a = conv_args(f.packed, f.L, CV_D, C, B, h, w, h, w, f.z, 2 * C, nullptr, 0);
            a.out0 = f.xb; a.aux0 = f.x1;
            return launch_conv<STAGE_S1, EPI_ISTA_D, 1>(a, f.st);
        case CISTA_LAYER_ISTA_P:    // z = softshrink(P(x) + z, lambda)            :75-77
            a = conv_args(f.packed, f.L, CV_P, C, B, h, w, h, w, f.xb, C, nullptr, 0);
            a.out0 = f.z; a.aux0 = f.z; a.lambda = blob<float>(f.packed, f.L.lambda);
            return launch_conv<STAGE_S1, EPI_ISTA_P, 1>(a, f.st);
        case CISTA_LAYER_DG:        // y = relu(Dg.conv(z))                      base_layers.py:222
            a = conv_args(f.packed, f.L, CV_DG, C, B, h, w, h, w, f.z, 2 * C, nullptr, 0);
            a.out0 = f.xb;
            return launch_conv<STAGE_S1, EPI_RELU, 1>(a, f.st);
        case CISTA_LAYER_LSTM:      // ConvLSTM on cat(y, h_prev)                  :112-128
            a = conv_args(f.packed, f.L, CV_LSTM, C, B, h, w, h, w, f.xb, C, f.h_prev, C);
            a.out0 = f.hs; a.out1 = f.cs; a.aux0 = f.c_prev;
            return launch_conv<STAGE_S1, EPI_LSTM, 4>(a, f.st);
        case CISTA_LAYER_UPSAMPLE:  // relu(conv(ReflectionPad(up2x(h))))          :193-210
            a = conv_args(f.packed, f.L, CV_UP, C, B, h, w, f.H, f.W, f.hs, C, nullptr, 0);
            a.out0 = f.full;
            if (up_q_path(C)) {     // + final_conv's channel contraction in the epilogue
                a.aux0 = blob<float>(f.packed, f.L.wF);
                return launch_conv<STAGE_UP, EPI_UP_Q, 1>(a, f.st);
            }
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
                fa.u = f.full; fa.w = blob<float>(f.packed, f.L.wF); fa.bias = blob<float>(f.packed, f.L.bF);
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
        CHECK(run_layer(f, CISTA_LAYER_ISTA_D));
        CHECK(run_layer(f, CISTA_LAYER_ISTA_P));
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

}  // namespace

// =========================================================================================
extern "C" {

int cista_abi_version(void) { return CISTA_ABI_VERSION; }

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
    const float *ws[CV_COUNT] = {p->W0_w, p->P0_w, p->gates_w, p->out_gates_w, p->D_w, p->P_w,
                                 p->Dg_w, p->lstm_w, p->up_w};
    const float *bs[CV_COUNT] = {p->W0_b, p->P0_b, p->gates_b, p->out_gates_b, p->D_b, p->P_b,
                                 p->Dg_b, p->lstm_b, p->up_b};
    for (int i = 0; i < CV_COUNT; ++i) {
        const ConvShape s = conv_shape(i, C);
        PackArgs a;
        a.w = ws[i]; a.b = bs[i];
        a.scale = blobw<float>(packed, L.sc[i]);
        hipLaunchKernelGGL(weight_scale_kernel, dim3(1), dim3(1024), 0, st, ws[i],
                           (long)s.cout * s.cin * 9, a.scale);
        a.wp = blobw<u32x4>(packed, L.wp[i]);
        a.bp = blobw<float>(packed, L.bp[i]);
        a.Cout = s.cout; a.Cin = s.cin; a.G = s.G;
        const long total = (long)(s.cin / 32) * 9 * (s.cout / 16) * 64;
        hipLaunchKernelGGL(pack_conv_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
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

}  // extern "C"
