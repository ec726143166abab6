// cista_pingpong.hpp -- two-tile ("ping-pong") persistent workgroups for the ISTA convs
// (reference e2v/e2v_model.py:72-78: x = x1 - D(z); z = softshrink(P(x) + z, lambda), D and P
// the tied IstaBlock convs of e2v/base_layers.py:21-35).
//
// Why: in the one-tile kernel (conv_tile) a workgroup's phases run in sequence --
// the halo round trip of its first K-chunk, the MFMA K loop, then an epilogue that reads z / x1
// and writes z / x (98 + 98 KB per ISTA P tile) -- and the two workgroups of a CU drift in lock
// step, so the matrix pipe idles whenever both are in a memory phase: ISTA P's time is the sum of
// its MFMA passes (~0.6 ms at B = 256) and its HBM traffic (~0.6 ms), MFMA busy 53 %.
//
// Here one 512-thread workgroup per CU runs two halves of 4 waves (waves 0-3, 4-7: on every SIMD
// one wave of each half), each half a stream of tiles through the SAME per-tile code as
// conv_tile: the K-chunks ("C" segments: MFMAs on one LDS halo image while the next chunk -- of
// this tile, or chunk 0 of the half's next tile -- is loaded into registers and committed to the
// other image) and the epilogue ("E": aux loads, fused elementwise tail, float4 stores).  The
// halves share the workgroup barrier: every segment ends in one s_barrier, and half 1 runs
// OFF = period / 2 segments behind half 0, so one half's epilogue is always paired with the
// other half's MFMA segment and the matrix pipe of each SIMD is never left without a wave in
// its K loop (two C segments paired share the pipe, which is also fine).  The next tile's first
// chunk is staged inside the previous tile's last C segment, so a tile costs no separate halo
// round trip.  Per-pixel arithmetic, MFMA order and the epilogue's operations are those of
// conv_tile, so the frames are bit-identical to the one-tile kernel (tests/test_gpu_pingpong.py).
//
// Persistent grid: one workgroup per CU (two halves x two 32 KB images = 128 KB of LDS); workgroup
// L runs on XCD L % 8 (round-robin dispatch), the items of XCD x are a contiguous range and its
// 2 x (workgroups on x) half-slots take them round-robin, so tiles processed at the same time on
// one XCD are neighbours (their halos meet in that XCD's L2).
#pragma once
#include "cista_kernels.hpp"

namespace cista {

// Diagnostic build only (CISTA_STAMPS=1, scripts/pp_stamps.py): lane 0 of every wave stamps the
// segment boundaries of its half's third tile into g_cista_stamps[(block * 8 + wave) * 24 + slot]:
// 0 hw id | xcc << 32, 1 tile start, 2 + 2 kc end of K-chunk kc's work, 3 + 2 kc after its barrier,
// 12 epilogue aux loads issued / 13 epilogue math done / 14 epilogue stores issued, 15 after the
// epilogue's barrier, 16 / 17 constant-rate clock at tile start / epilogue end
#if CISTA_STAMPS
#define PP_STAMP(cond, slot, v)                                                                          \
    do {                                                                                                 \
        unsigned long long *_p = g_cista_stamps;                                                         \
        if (_p && (cond) && (threadIdx.x & 63) == 0) _p[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 24 + (slot)] = (v); \
    } while (0)
#else
#define PP_STAMP(cond, slot, v) do { } while (0)
#endif
// timing-only experiment builds (results wrong): 1 = memory segments do nothing, 2 = K segments
// issue no MFMAs
#ifndef PP_EXP
#define PP_EXP 0
#endif


struct PingPongArgs {
    ConvArgs a;          // pointers, region-a geometry (TH, TW, tiles_*, pitch) and region b (*_b, wa)
    int items;           // (tile, column block) items of the launch, region a's first
    int items_a;         // items of region a
    int img_u4;          // u32x4 units of one LDS halo image (>= 8 x HPpad of either region)
    struct PPOverflow *overflow;   // tiles whose staged input overflowed the fp16 hi part
};

// geometry of one tile item (workgroup-uniform per half)
struct PPTile {
    int b, oy0, ox0, nblk;
    int TH, TW, pitch;
    float rcp_pitch;
};

__device__ __forceinline__ PPTile pp_tile(const PingPongArgs &p, int w, int nnb) {
    const ConvArgs &a = p.a;
    PPTile t;
    int tiles_x = a.tiles_x, tiles_y = a.tiles_y;
    t.TH = a.TH; t.TW = a.TW; t.pitch = a.pitch; t.rcp_pitch = a.rcp_pitch;
    int ox_base = 0;
    if (w >= p.items_a) {
        w -= p.items_a;
        tiles_x = a.tiles_x_b; tiles_y = a.tiles_y_b;
        t.TH = a.TH_b; t.TW = a.TW_b; t.pitch = a.pitch_b; t.rcp_pitch = a.rcp_pitch_b;
        ox_base = a.wa;
    }
    t.nblk = w % nnb;
    int r = w / nnb;
    const int tx = r % tiles_x;
    r /= tiles_x;
    const int ty = r % tiles_y;
    t.b = r / tiles_y;
    t.oy0 = ty * t.TH;
    t.ox0 = ox_base + tx * t.TW;
    return t;
}

__device__ __forceinline__ bool pp_pixel(const PPTile &t, int p, int &py, int &px) {
    py = small_div(p, t.rcp_pitch);
    px = p - py * t.pitch;
    const bool ok = py < t.TH && px < t.TW;
    py = py < t.TH ? py : t.TH - 1;
    px = px < t.TW ? px : t.TW - 1;
    return ok;
}

// the conv_tile view of a tile's geometry (stage_pixels / stage_issue_px read Hin, Win, c0, ...)
__device__ __forceinline__ int pp_hwd(const PPTile &t) { return t.TW + 2; }
__device__ __forceinline__ int pp_hppad(const PPTile &t) { return ((t.TH + 2) * (t.TW + 2) + 15) & ~15; }

// One K-chunk of MFMAs for a wave that is ALONE in its K loop on its SIMD (the partner wave of
// the other half is in a memory segment): the same products in the same order as conv_tile's
// mfma_tap loop -- per tap, per m-tile, per n-tile hi*hi, lo*hi, hi*lo -- but with the A (pixel)
// fragments read AH = 2 (tap, m-tile) steps ahead across tap boundaries and B (weight) fragments
// DB taps ahead.  One step ahead (mfma_tap) leaves the read of m-tile m+1 about 2 MFMAs to
// return and stalls on LDS latency every m-tile; in the one-tile kernel the other workgroup's
// wave fills those stalls, a lone wave cannot.
template <int MT_W, int NW, int DB>
__device__ __forceinline__ void pp_chunk(f32x4 (&acc)[MT_W][NW], const u32x4 *smem, const int (&abase)[MT_W], int HWd,
                                         int HPpad, const u32x4 *wp, size_t tapstride) {
    constexpr int AH = 2, NS = 9 * MT_W;
    u32x4 bh[DB + 1][NW], bl[DB + 1][NW];
#pragma unroll
    for (int tt = 0; tt < DB; ++tt)
#pragma unroll
        for (int n = 0; n < NW; ++n) {
            bh[tt][n] = wp[(size_t)tt * tapstride + n * 128];
            bl[tt][n] = wp[(size_t)tt * tapstride + n * 128 + 64];
        }
    auto aaddr = [&](int st) {
        const int tap = st / MT_W, m = st % MT_W;
        return abase[m] + (tap / 3) * HWd + (tap % 3);
    };
    u32x4 ah[AH + 1], al[AH + 1];
#pragma unroll
    for (int st = 0; st < AH; ++st) {
        ah[st] = smem[aaddr(st)];
        al[st] = smem[4 * HPpad + aaddr(st)];
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int m = 0; m < MT_W; ++m) {
        const int st = tap * MT_W + m;
        if (m == 0 && tap + DB <= 8) {
            const u32x4 *wq = wp + (size_t)(tap + DB) * tapstride;
#pragma unroll
            for (int n = 0; n < NW; ++n) {
                bh[(tap + DB) % (DB + 1)][n] = wq[n * 128];
                bl[(tap + DB) % (DB + 1)][n] = wq[n * 128 + 64];
            }
        }
        if (st + AH < NS) {
            ah[(st + AH) % (AH + 1)] = smem[aaddr(st + AH)];
            al[(st + AH) % (AH + 1)] = smem[4 * HPpad + aaddr(st + AH)];
        }
        const f16x8 xh = __builtin_bit_cast(f16x8, ah[st % (AH + 1)]);
        const f16x8 xl = __builtin_bit_cast(f16x8, al[st % (AH + 1)]);
        const int slot = tap % (DB + 1);
#pragma unroll
        for (int n = 0; n < NW; ++n) {
            const f16x8 wh = __builtin_bit_cast(f16x8, bh[slot][n]);
            const f16x8 wl = __builtin_bit_cast(f16x8, bl[slot][n]);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xh, acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, xh, acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xl, acc[m][n], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Epilogue of one tile, math part: conv_tile's generic m-tile loop for EPI_ISTA_D / EPI_ISTA_P
// at G = 1, operation for operation (acc * ws + bias as one fma, then x1 - v or softshrink(v + z,
// lambda)); the results replace the accumulators in place.  Pixel offsets are computed per lane
// (no LDS pixel table, so no barrier inside a segment).  The aux inputs of PD m-tiles are in
// flight at once.  pp_epi_store then writes acc.
template <int MT_W, int NW, int WM>
__device__ __forceinline__ int pp_pix_off(const ConvArgs &a, const PPTile &t, int wm, int m, int pl) {
    int py, px, l = pl;
    asm volatile("" : "+v"(l));          // recomputed per use, not held from the loads to the stores
    const bool in = pp_pixel(t, (wm * MT_W + m) * 16 + l, py, px);
    const int oy = t.oy0 + py, ox = t.ox0 + px;
    return (in && oy < a.Hout && ox < a.Wout) ? ((t.b * a.Hout + oy) * a.Wout + ox) * a.Cout : -1;
}

template <int MT_W, int NW, int WM, int EPI>
__device__ __forceinline__ void pp_epi_math(const ConvArgs &a, const PPTile &t, f32x4 (&acc)[MT_W][NW], int wm, int nt0,
                                            int htid, bool stamp) {
    constexpr bool ISTAP = EPI == EPI_ISTA_P;
    constexpr int NQ = NW;                                   // G == 1
    constexpr int AUXV = NQ * 4;
    constexpr int PD0 = CISTA_AUX_VGPRS / AUXV;
    constexpr int PD = PD0 < 1 ? 1 : (PD0 > MT_W ? MT_W : PD0);
    int etid = htid;
    asm volatile("" : "+v"(etid));
    const int kq = (etid & 63) >> 4, pl = etid & 15;
    const float ws = *a.wscale;
    const int ch0 = nt0 * 16 + 4 * kq;
    float4 bias4[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) bias4[q] = *(const float4 *)(a.bias + (nt0 + q) * 16 + 4 * kq);
    float4 lam4[ISTAP ? NQ : 1];
    bool lam_nonneg = false;
    if constexpr (ISTAP) {
        bool nn = true;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            lam4[q] = *(const float4 *)(a.lambda + ch0 + 16 * q);
            nn = nn && lam4[q].x >= 0.0f && lam4[q].y >= 0.0f && lam4[q].z >= 0.0f && lam4[q].w >= 0.0f;
        }
        lam_nonneg = __builtin_amdgcn_ballot_w64(!nn) == 0;
    }
    auto load_aux = [&](int m, float4 (&A0)[NQ]) {
        const int off = pp_pix_off<MT_W, NW, WM>(a, t, wm, m, pl);
        const unsigned o = (unsigned)(off < 0 ? 0 : off) + (unsigned)ch0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) A0[q] = *(const float4 *)(a.aux0 + o + 16 * q);
    };
    float4 ring[PD][NQ];
#pragma unroll
    for (int d = 0; d < PD; ++d) load_aux(d, ring[d]);
    PP_STAMP(stamp, 12, __builtin_amdgcn_s_memtime());
    auto mloop = [&](auto fast_tag) __attribute__((always_inline)) {
        constexpr bool FAST = decltype(fast_tag)::value;
#pragma unroll
        for (int m = 0; m < MT_W; ++m) {
            float4 (&cur)[NQ] = ring[m % PD];
            asm volatile("" ::: "memory");
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const f32x4 ac = acc[m][q];
                float vv[4];
                vv[0] = fmaf(ac[0], ws, bias4[q].x);
                vv[1] = fmaf(ac[1], ws, bias4[q].y);
                vv[2] = fmaf(ac[2], ws, bias4[q].z);
                vv[3] = fmaf(ac[3], ws, bias4[q].w);
                const float *xa = reinterpret_cast<const float *>(&cur[q]);
                float r[4];
                if constexpr (EPI == EPI_ISTA_D) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) r[e] = xa[e] - vv[e];
                } else {
                    const float *ll = reinterpret_cast<const float *>(&lam4[q]);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float x = vv[e] + xa[e];
                        r[e] = FAST ? x - __builtin_amdgcn_fmed3f(x, -ll[e], ll[e]) : softshrink_(x, ll[e]);
                    }
                }
                acc[m][q] = f32x4{r[0], r[1], r[2], r[3]};
            }
            if (m + PD < MT_W) load_aux(m + PD, cur);
            asm volatile("" ::: "memory");
        }
    };
    if constexpr (ISTAP) {
        if (lam_nonneg) mloop(BoolTag<true>{});
        else mloop(BoolTag<false>{});
    } else {
        (void)lam_nonneg;
        mloop(BoolTag<false>{});
    }
    PP_STAMP(stamp, 13, __builtin_amdgcn_s_memtime());
}

template <int MT_W, int NW, int WM>
__device__ __forceinline__ void pp_epi_store(const ConvArgs &a, const PPTile &t, const f32x4 (&acc)[MT_W][NW], int wm,
                                             int nt0, int htid) {
    int etid = htid;
    asm volatile("" : "+v"(etid));
    const int kq = (etid & 63) >> 4, pl = etid & 15;
    const int ch0 = nt0 * 16 + 4 * kq;
#pragma unroll
    for (int m = 0; m < MT_W; ++m) {
        const int off = pp_pix_off<MT_W, NW, WM>(a, t, wm, m, pl);
        if (off >= 0) {
#pragma unroll
            for (int q = 0; q < NW; ++q)
                *(float4 *)(a.out0 + (unsigned)off + (unsigned)(ch0 + 16 * q)) =
                    make_float4(acc[m][q][0], acc[m][q][1], acc[m][q][2], acc[m][q][3]);
        }
    }
}

// Overflow list (the range pass of the one-tile kernel, deferred): a tile whose staged input does
// not fit the fp16 hi part (|x| >= 65520) writes nothing; its item goes on this list and
// conv3x3_fixup re-runs it with conv_tile (range pass included) right after the launch -- its
// inputs are untouched (ISTA P's in-place z update was skipped too).  The host zeroes count
// before every two-tile launch.
struct PPOverflow {
    unsigned count;
    unsigned pad[63];
    int items[1];        // [capacity]
};

template <int MT_W, int NW, int WM, int WN, int EPI>
__global__ __launch_bounds__(512, 1) void conv3x3_pingpong(const PingPongArgs p) {
    static_assert(WM * WN == 4, "4 waves per half");
    static_assert(EPI == EPI_ISTA_D || EPI == EPI_ISTA_P, "the ISTA epilogues");
    constexpr int NI = 4, NTH = 256;
    extern __shared__ u32x4 smem[];
    const ConvArgs &a = p.a;
    const int half = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);
    u32x4 *const hbuf = smem + (size_t)half * 2 * p.img_u4;                   // this half's two images
    int *const flags = reinterpret_cast<int *>(smem + (size_t)4 * p.img_u4);   // [2 halves][4 waves]

    // items of this workgroup's XCD (contiguous), taken round-robin by its half-slots
    const unsigned nwg = gridDim.x, L = blockIdx.x, xcd = L & 7u;
    const unsigned q8 = (unsigned)p.items >> 3, r8 = (unsigned)p.items & 7u;
    const int xs = (int)(xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8);
    const int xn = (int)(q8 + (xcd < r8 ? 1u : 0u));
    const int slots = 2 * (int)((nwg - xcd + 7u) >> 3);              // half-slots on this XCD
    const int slot0 = 2 * (int)(L >> 3);
    auto ntiles = [&](int slot) { return xn > slot ? (xn - slot + slots - 1) / slots : 0; };
    const int my_slot = slot0 + half;
    const int n_mine = ntiles(my_slot);
    const int nnb = a.N / (WN * NW * 16);
    const int kc0 = a.c0 >> 5;
    const int nch = kc0 + (a.in1 ? (a.c1 >> 5) : 0);
    // per tile: ngrp x [K segment: MFMAs of a group of two chunks | memory segment: staging of the
    // next group, or after the last group the epilogue + staging of the next tile's first group].
    // Half 1 runs one segment behind half 0, so on every SIMD one wave is in a K segment and the
    // other in a memory segment.  Barriers per half: 1 (prologue) + 2 ngrp per tile (+1 for half 1)
    const int ngrp = (nch + 1) >> 1;
    const int own = half + 1 + n_mine * 2 * ngrp;
    const int total = max(1 + ntiles(slot0) * 2 * ngrp, 2 + ntiles(slot0 + 1) * 2 * ngrp);
    const size_t tapstride = (size_t)(a.N >> 4) * 2 * 64;
    auto seg_of = [&](int kc, const float *&seg, int &segC, int &choff) {
        seg = kc < kc0 ? a.in0 : a.in1;
        segC = kc < kc0 ? a.c0 : a.c1;
        choff = (kc < kc0 ? kc : kc - kc0) * 32;
    };
    auto item_of = [&](int k) { return xs + my_slot + slots * k; };
    // a group = chunks 2g, 2g+1 of one tile (the half's two LDS images): the halo loads of both
    // chunks are issued before either is committed.  (A chunk beyond nch -- odd chunk counts --
    // re-loads chunk 2g and is not committed.)
#define PP_GROUP_ISSUE(t, g, htid)                                                                           \
    {                                                                                                        \
        stage_pixels<STAGE_S1, NI, NTH>(a, (t).b, (t).oy0 - 1, (t).ox0 - 1, (t).TH + 2, pp_hwd(t), gspix, gshp, gsg, \
                                        (htid));                                                             \
        const float *seg; int segC, choff;                                                                   \
        seg_of(2 * (g), seg, segC, choff);                                                                   \
        stage_issue_px<STAGE_S1, NI>(a, seg, segC, choff, gspix, gsg, gv0a, gv1a, (t).b);                    \
        seg_of(2 * (g) + 1 < nch ? 2 * (g) + 1 : 2 * (g), seg, segC, choff);                                 \
        stage_issue_px<STAGE_S1, NI>(a, seg, segC, choff, gspix, gsg, gv0b, gv1b, (t).b);                    \
    }
#define PP_GROUP_COMMIT(t, g, amx)                                                                           \
    {                                                                                                        \
        stage_commit<NI>(hbuf, pp_hppad(t), gv0a, gv1a, gshp, gsg, (amx));                                   \
        if (2 * (g) + 1 < nch) stage_commit<NI>(hbuf + p.img_u4, pp_hppad(t), gv0b, gv1b, gshp, gsg, (amx)); \
    }

    f16x2 amax_next = {};                 // |hi| maxima of the next tile's first group (staged early)
    if (half) __syncthreads();            // half 1 starts one segment late
    if (n_mine > 0) {                     // prologue: group 0 of the half's first tile
        const PPTile t = pp_tile(p, item_of(0), nnb);
        float4 gv0a[NI], gv1a[NI], gv0b[NI], gv1b[NI];
        int gspix[NI], gshp[NI], gsg[NI];
        PP_GROUP_ISSUE(t, 0, threadIdx.x & 255);
        PP_GROUP_COMMIT(t, 0, amax_next);
    }
    __syncthreads();

#pragma unroll 1
    for (int k = 0; k < n_mine; ++k) {
        // opaque thread id: nothing derived from it is hoisted out of the tile loop and held
        // across it (that spilled)
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int htid = tid & 255;
        const int lane = tid & 63;
        const int hwave = (tid >> 6) & 3;
        const int wm = hwave % WM, wn = hwave / WM;
        const int item = item_of(k);
        const PPTile t = pp_tile(p, item, nnb);
        const bool stamp = k == 2;
#if CISTA_STAMPS
        if (stamp) {
            unsigned hw, xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            PP_STAMP(true, 0, (unsigned long long)hw | ((unsigned long long)xcc << 32));
            PP_STAMP(true, 16, __builtin_amdgcn_s_memrealtime());
            PP_STAMP(true, 1, __builtin_amdgcn_s_memtime());
        }
#endif
        const int nt0 = (t.nblk * WN + wn) * NW;
        const int HWd = pp_hwd(t), HPpad = pp_hppad(t);
        f32x4 acc[MT_W][NW];
#pragma unroll
        for (int m = 0; m < MT_W; ++m)
#pragma unroll
            for (int n = 0; n < NW; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
        f16x2 amax = amax_next;
        amax_next = f16x2{};
#pragma unroll 1
        for (int g = 0; g < ngrp; ++g) {
            // ------------------------------ K segment: the MFMAs of chunks 2g, 2g+1 (no HBM load
            // in this wave's queue: the B fragments' L2 round trips are the only vmcnt waits)
            if (g == ngrp - 1) {
                // every chunk of this tile is staged: its waves' overflow bits for the epilogue
                const _Float16 hm = amax[0] > amax[1] ? amax[0] : amax[1];
                const bool wany = __ballot(__builtin_isinf((float)hm) ? 1 : 0) != 0;
                if (lane == 0) flags[half * 4 + hwave] = wany ? 1 : 0;
            }
            int abase[MT_W];
            {
                const int kgrp = lane >> 4;
#pragma unroll
                for (int m = 0; m < MT_W; ++m) {
                    int py, px;
                    pp_pixel(t, (wm * MT_W + m) * 16 + (lane & 15), py, px);
                    abase[m] = kgrp * HPpad + py * HWd + px;
                }
            }
#pragma unroll 1
            for (int c = 0; c < 2; ++c) {
                const int kc = 2 * g + c;
                if (kc >= nch) break;
                const u32x4 *cur = hbuf + c * p.img_u4;
#pragma unroll
                for (int m = 0; m < MT_W; ++m) asm volatile("" : "+v"(abase[m]));
                const u32x4 *wp = a.wpack + ((size_t)kc * 9) * tapstride + (size_t)nt0 * 128 + lane;
#if PP_EXP != 2
                pp_chunk<MT_W, NW, 2>(acc, cur, abase, HWd, HPpad, wp, tapstride);
#endif
            }
            PP_STAMP(stamp && g < 2, 2 + 4 * g, __builtin_amdgcn_s_memtime());
            __syncthreads();
            PP_STAMP(stamp && g < 2, 3 + 4 * g, __builtin_amdgcn_s_memtime());
            // ------------------------------ memory segment (the other half is in a K segment)
            float4 gv0a[NI], gv1a[NI], gv0b[NI], gv1b[NI];
            int gspix[NI], gshp[NI], gsg[NI];
#if PP_EXP == 1
            if (false) {
#else
            if (g + 1 < ngrp) {                       // the next group of this tile
#endif
                PP_GROUP_ISSUE(t, g + 1, htid);
                PP_GROUP_COMMIT(t, g + 1, amax);
            } else if (PP_EXP == 1) {
                if (p.items < 0) pp_epi_store<MT_W, NW, WM>(a, t, acc, wm, nt0, htid);   // keeps the MFMAs live
            } else {
                // the epilogue of this tile, then the next tile's first group
                int anyfl = flags[half * 4];
#pragma unroll
                for (int w = 1; w < 4; ++w) anyfl |= flags[half * 4 + w];
                anyfl = __builtin_amdgcn_readfirstlane(anyfl);
                const bool has_next = k + 1 < n_mine;
                if (!anyfl) pp_epi_math<MT_W, NW, WM, EPI>(a, t, acc, wm, nt0, htid, stamp);
                const PPTile tn = pp_tile(p, has_next ? item_of(k + 1) : item, nnb);
                if (has_next) PP_GROUP_ISSUE(tn, 0, htid);          // loads ahead of the stores (vmcnt in order)
                if (anyfl) {                                        // rare: re-run by conv3x3_fixup
                    if (htid == 0) {
                        const unsigned i = atomicAdd(&p.overflow->count, 1u);
                        p.overflow->items[i] = item;
                    }
                } else {
                    pp_epi_store<MT_W, NW, WM>(a, t, acc, wm, nt0, htid);
                }
                PP_STAMP(stamp, 14, __builtin_amdgcn_s_memtime());
                if (has_next) PP_GROUP_COMMIT(tn, 0, amax_next);
                PP_STAMP(stamp, 17, __builtin_amdgcn_s_memrealtime());
            }
            PP_STAMP(stamp && g < 2, 4 + 4 * g, __builtin_amdgcn_s_memtime());
            __syncthreads();
            PP_STAMP(stamp && g < 2, 5 + 4 * g, __builtin_amdgcn_s_memtime());
        }
    }
    for (int i = own; i < total; ++i) __syncthreads();
#undef PP_GROUP_ISSUE
#undef PP_GROUP_COMMIT
}

// The overflowed tiles of a two-tile launch (PPOverflow), each re-run by a 4-wave workgroup
// through conv_tile -- the one-tile kernel's per-item body, whose range pass recomputes the tile
// with pre-scaled inputs.  A fixed grid loops over the list (usually empty: the launch is then a
// few microseconds).
template <int MT_W, int NW, int WM, int WN, int EPI>
__global__ __launch_bounds__(WM * WN * 64, 2) void conv3x3_fixup(const PingPongArgs p) {
    extern __shared__ u32x4 smem[];
    const unsigned n = __atomic_load_n(&p.overflow->count, __ATOMIC_RELAXED);
    for (unsigned i = blockIdx.x; i < n; i += gridDim.x) {
        const unsigned w = (unsigned)p.overflow->items[i];
        ConvArgs ar = p.a;
        unsigned wl = w;
        if (ar.tiles_x_b && w >= (unsigned)p.items_a) {
            ar.TH = ar.TH_b; ar.TW = ar.TW_b; ar.tiles_x = ar.tiles_x_b; ar.tiles_y = ar.tiles_y_b;
            ar.pitch = ar.pitch_b; ar.rcp_pitch = ar.rcp_pitch_b; ar.ox_base = ar.wa;
            wl -= (unsigned)p.items_a;
        }
        conv_tile<MT_W, NW, WM, WN, STAGE_S1, EPI, 1, true, 4, false>(ar, smem, wl);
        __syncthreads();
    }
}

}  // namespace cista
