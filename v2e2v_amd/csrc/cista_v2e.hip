// GPU video-to-events emulator, voxel-grid mode; contract in
// include/cista_v2e.h.  Reference: v2e/v2e_model.py:290-536, v2e/emulator_utils.py:13-207.
//
// Per forward call:
//   v2e_init_kernel   (first call)  base = lp = lin_log(frame 0), thresholds, noise rates, the
//                                   refractory memory                            (_init :158-253)
//   v2e_tmem_kernel   (later calls) refractory memory shifted by one voxel span    (:329-331)
//   per frame n = 1 .. F-1:
//     v2e_diff_kernel  low-pass (:266-289), leak (:361-368), diff / polarity / threshold / event
//                      count (:393-413), image max of the counts per batch element
//     v2e_iters_kernel num_iters, ts_step, max_num_iters, refractory switch    (:414-427,447)
//     v2e_emit_kernel  the per-iteration emission (:436-492) with shot noise (:437-440), the
//                      refractory filter and the voxel accumulation in this pixel's own voxels,
//                      then base += pol * n_events * C                           (:520)
//   event_preprocess_pytorch('std') over the whole tensor                        (:526)
//
// Floating-point contraction is off: every expression rounds like the reference's float32 ops.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "../../include/cista_lstc.h"
#include "../../include/cista_v2e.h"
#include "../../include/cista_voxel.h"

namespace cista_v2e {

// ------------------------------------------------------------------ Philox4x32-10 stream
struct U4 {
    unsigned x, y, z, w;
};

__device__ __forceinline__ U4 philox(U4 c, unsigned k0, unsigned k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const unsigned hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const unsigned hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

__device__ __forceinline__ float u01(unsigned u) { return ((float)(u >> 8) + 0.5f) * (1.0f / 16777216.0f); }

// draw `d` of element `e`: a uniform and a standard normal
__device__ __forceinline__ U4 draw(unsigned long long seed, unsigned long long d, unsigned long long e) {
    return philox(U4{(unsigned)e, (unsigned)(e >> 32), (unsigned)d, (unsigned)(d >> 32)}, (unsigned)seed,
                  (unsigned)(seed >> 32));
}
__device__ __forceinline__ float randn(unsigned long long seed, unsigned long long d, unsigned long long e) {
    const U4 r = draw(seed, d, e);
    return sqrtf(-2.0f * logf(u01(r.x))) * cosf(6.28318530717958647692f * u01(r.y));
}

// ------------------------------------------------------------------ per-call constants
struct Call {
    int B, F, H, W, nb;
    float tf[CISTA_V2E_MAX_FRAMES];            // t_float_frames (:313-317)
    float time_frames[CISTA_V2E_MAX_FRAMES];   // voxel-time of each frame (:319-320)
    float Tr[CISTA_V2E_MAX_BATCH];             // refractory period in voxel time (:322)
    float dt_lp0[CISTA_V2E_MAX_FRAMES];        // delta_time / tau0 per frame (low-pass, ql)
    float dt_lp1[CISTA_V2E_MAX_FRAMES];        // delta_time / tau1 per frame (qs)
    float duration;                            // (nb - 1) / (F - 1) as float32
    double linlog_f;                           // (1 / 20) * log(20)
    unsigned long long seed, draw0;
    cista_v2e_config cfg;
};

struct State {   // device planes, B*H*W each
    float *base, *lp, *pos, *neg, *pos_pre, *neg_pre, *noise_rate, *tmem;
};

constexpr int MAXSLOTS = 64;    // atomic slots per batch element of the image max
constexpr int SLOTW = 32;       // 4-byte words per slot: one 128-byte line each (same-line atomics
                                // serialise in L2: 3600 workgroups on 2 lines took ~20 us)

struct Scratch {
    int *counts;          // B*H*W event counts of the current frame
    float *pol;           // B*H*W polarity (+1 / -1 / 0)
    int *iters_raw;       // [B][MAXSLOTS][SLOTW] image max of counts (partial maxima, word 0 of a slot)
    int *num_iters;       // [B] max(iters_raw, 1)
    float *ts_step;       // [B]
    int *meta;            // [0] max_num_iters, [1] refractory switch
    unsigned long long *nev;   // [MAXSLOTS][SLOTW / 2] partial event totals (workgroup mod MAXSLOTS)
};

__device__ __forceinline__ float lin_log(float v, double f) {
    // emulator_utils.py:13-38 (float64, rounded to 8 decimals, half to even like torch.round)
    const double x = (double)v;
    double y = x <= 20.0 ? x * f : log(x);
    y = rint(y * 1e8) / 1e8;
    return (float)y;
}
__device__ __forceinline__ float rescale(float v) { return (v + 20.0f) / 275.0f; }   // :41-46

__global__ void v2e_init_kernel(Call c, State s, const float *frames) {
    const long long HW = (long long)c.H * c.W;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)c.B * HW) return;
    const int b = (int)(i / HW);
    const long long p = i - b * HW;
    const int y = (int)(p / c.W), x = (int)(p - (long long)y * c.W);
    const float l0 = lin_log(frames[((long long)b * c.F) * HW + p], c.linlog_f);
    s.base[i] = l0;
    s.lp[i] = l0;
    const cista_v2e_config &g = c.cfg;
    float pt = g.pos_thres, nt = g.neg_thres;
    if (g.sigma_thres > 0.0f) {
        const bool half = (y % 2 == 0) && (x % 2 == 0);   // [:, :, 0::2, 0::2] (:213,226)
        const float pm = (half ? g.ps : g.pl) * g.pos_thres, nm = (half ? g.ps : g.pl) * g.neg_thres;
        pt = fmaxf(pm + g.sigma_thres * randn(c.seed, c.draw0 + (half ? 1 : 0), i), 0.01f);
        nt = fmaxf(nm + g.sigma_thres * randn(c.seed, c.draw0 + (half ? 3 : 2), i), 0.01f);
    }
    s.pos[i] = pt;
    s.neg[i] = nt;
    s.pos_pre[i] = pt * (1.0f / g.pos_thres);                 // einsum(1 / nominal, thres) (:232)
    s.neg_pre[i] = nt * (1.0f / g.neg_thres);
    if (g.leak_rate_hz > 0.0f)                                 // log-normal rates (:244-248)
        s.noise_rate[i] = expf((float)(2.302585092994046 * g.noise_rate_cov_decades) * randn(c.seed, c.draw0 + 4, i));
    s.tmem[i] = 0.0f - c.Tr[b];                                // (:252)
}

__global__ void v2e_tmem_kernel(Call c, State s) {
    const long long HW = (long long)c.H * c.W;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)c.B * HW) return;
    float t = s.tmem[i];
    if (t > 0.0f) t -= (float)(c.nb - 1);                      // :330
    if (t < 0.0f) t = -c.Tr[i / HW];                           // :331
    s.tmem[i] = t;
}

__global__ __launch_bounds__(256) void v2e_diff_kernel(Call c, State s, Scratch w, const float *frames, int n,
                                                       float dt_frame) {
    const int HW = c.H * c.W;                  // B * H * W < 2^31 (checked on the host)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const cista_v2e_config &g = c.cfg;
    int cnt = 0;
    int b = 0;
    if (i < c.B * HW) {
        b = i / HW;
        const int p = i - b * HW;
        const int y = p / c.W, x = p - y * c.W;
        // every load is issued before the first store and before the long lin_log: the waves
        // wait for memory once (issued in program order after stores they were 5 round trips)
        const bool lowpass = g.cutoff_hz > 0.0f, leak = g.leak_rate_hz > 0.0f;
        const float fr = frames[((size_t)b * c.F + n) * HW + p];
        const float lp_old = lowpass ? s.lp[i] : 0.0f;
        float base = s.base[i];
        const float nrate = leak ? s.noise_rate[i] : 0.0f;
        const float pos = s.pos[i], neg = s.neg[i];
        float nw = lin_log(fr, c.linlog_f);
        if (lowpass) {                                         // low_pass_filter (:49-101)
            const float inten = rescale(fr);
            const bool half = (y % 2 == 0) && (x % 2 == 0);
            float eps = g.ql > 0.0f ? inten * c.dt_lp0[n] : 1.0f;
            if (half) eps = g.qs > 0.0f ? inten * c.dt_lp1[n] : 1.0f;
            eps = fminf(eps, 1.0f);
            nw = (1.0f - eps) * lp_old + eps * nw;
        }
        if (leak) {                                            // subtract_leak_current (:104-124)
            const float r = randn(c.seed, c.draw0 + 8 + 2 * (unsigned long long)n, i);
            const float rate = g.leak_rate_hz * nrate * (1.0f - g.leak_jitter_fraction * r);
            base = base - dt_frame * rate * pos;
        }
        float diff = nw - base;                                // :386
        if (!(fabsf(diff) > 1e-6f)) diff = 0.0f;               // :405-406
        const float pol = diff > 0.0f ? 1.0f : (diff < 0.0f ? -1.0f : 0.0f);
        const float C = (pol > 0.0f ? pos : 0.0f) + (pol < 0.0f ? neg : 0.0f);   // :412
        cnt = (int)floorf(fabsf(diff) / (C + 1e-9f));          // :413
        if (lowpass) s.lp[i] = nw;
        if (leak) s.base[i] = base;
        w.counts[i] = cnt;
        w.pol[i] = pol;
    }
    // image max of the counts per batch element (exact in any order): wave max, workgroup max
    // in LDS, then one atomic per workgroup into one of MAXSLOTS slots of the element (thousands
    // of workgroups on one address serialise: ~10 ns each, 145 us per 720x1280 frame)
    __shared__ int wmax[4], wb[4];
    int m = cnt;
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o));
    const int b0 = __shfl(b, 0);
    const bool uniform = __all(b == b0);
    const bool live = i - (int)(threadIdx.x & 63) < c.B * HW;            // the wave has pixels
    if (uniform) {
        if ((threadIdx.x & 63) == 0) { wmax[threadIdx.x >> 6] = live ? m : 0; wb[threadIdx.x >> 6] = live ? b0 : -1; }
    } else {
        if (i < c.B * HW && cnt > 0)       // the slots start at 0: a zero maximum changes nothing
            atomicMax(w.iters_raw + ((size_t)b * MAXSLOTS + blockIdx.x % MAXSLOTS) * SLOTW, cnt);
        if ((threadIdx.x & 63) == 0) { wmax[threadIdx.x >> 6] = 0; wb[threadIdx.x >> 6] = -1; }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // waves of one batch element combine; a workgroup spans at most two elements
        for (int k = 0; k < 4; ++k) {
            if (wb[k] < 0) continue;
            int mk = wmax[k];
            for (int l = k + 1; l < 4; ++l)
                if (wb[l] == wb[k]) { mk = max(mk, wmax[l]); wb[l] = -1; }
            if (mk > 0) atomicMax(w.iters_raw + ((size_t)wb[k] * MAXSLOTS + blockIdx.x % MAXSLOTS) * SLOTW, mk);
        }
    }
}

__global__ void v2e_iters_kernel(Call c, Scratch w) {
    if (threadIdx.x != 0) return;
    int mx = 0;
    for (int b = 0; b < c.B; ++b) {
        int r = 0;
        for (int k = 0; k < MAXSLOTS; ++k) {          // read, then cleared for the next frame's diff
            r = max(r, w.iters_raw[((size_t)b * MAXSLOTS + k) * SLOTW]);
            w.iters_raw[((size_t)b * MAXSLOTS + k) * SLOTW] = 0;
        }
        mx = max(mx, r);                                       // max_num_iters (:417)
        const int ni = r == 0 ? 1 : r;                         // :426
        w.num_iters[b] = ni;
        w.ts_step[b] = c.duration / (float)ni;                 // :427
    }
    int refr = 0;                                              // (Tr > ts_step).any(), (B,1) vs (B,)
    for (int b1 = 0; b1 < c.B; ++b1)
        for (int b2 = 0; b2 < c.B; ++b2) refr |= c.Tr[b1] > w.ts_step[b2];
    w.meta[0] = mx;
    w.meta[1] = refr;
}

// One pixel's event iterations of a frame step (v2e_model.py:449-473 with the shot noise of
// emulator_utils.py:159-207): fire(it, ts) says whether iteration `it` emits an event and at
// which voxel time.  Shared by the voxel-grid and the raw-event emission.
struct PixelSteps {
    int cnt, ni, B, b, HW, p, q_have;
    float pol, on_thr, off_thr, step, Tr, t0, tmem;
    bool shot, refr;
    unsigned long long seed, dkey;
    U4 rq;                                             // the 4 uniforms of iterations 4q .. 4q+3

    __device__ __forceinline__ bool fire(int it, float &ts) {
        bool m = cnt >= it + 1;                        // :459
        // num_iter_mask (:196-198); the draw only matters when the count has not already set the
        // mask (mask = count OR shot).  One Philox block serves 4 iterations.
        if (shot && it < ni && !m) {
            const int q = it >> 2;
            if (q != q_have) {
                rq = draw(seed, dkey, ((unsigned long long)q * B + b) * HW + p);
                q_have = q;
            }
            const unsigned u = (it & 3) == 0 ? rq.x : (it & 3) == 1 ? rq.y : (it & 3) == 2 ? rq.z : rq.w;
            const float r = u01(u);
            m = pol > 0.0f ? r > on_thr : r < off_thr;
        }
        ts = it < ni ? t0 + step * (float)(it + 1) : 0.0f;   // :428-432
        if (refr) {                                    // :469-473
            const float since = ts * (m ? 1.0f : 0.0f) - tmem;
            m = since > Tr;
            if (m) tmem = ts;
        }
        return m;
    }
};

__device__ __forceinline__ PixelSteps pixel_steps(const Call &c, const Scratch &w, int n, float dt_frame, int b, int p,
                                                  int cnt, float pol, float fr, float pos_pre, float neg_pre,
                                                  float tmem0) {
    const cista_v2e_config &g = c.cfg;
    PixelSteps q;
    q.cnt = cnt; q.ni = w.num_iters[b]; q.B = c.B; q.b = b; q.HW = c.H * c.W; q.p = p; q.q_have = -1;
    q.pol = pol; q.step = w.ts_step[b]; q.Tr = c.Tr[b]; q.t0 = c.time_frames[n - 1]; q.tmem = tmem0;
    q.shot = g.shot_noise_rate_hz > 0.0f;
    q.refr = w.meta[1] != 0;
    q.seed = c.seed;
    q.dkey = c.draw0 + 9 + 2 * (unsigned long long)n;
    q.rq = U4{0u, 0u, 0u, 0u};
    q.on_thr = 1.0f;
    q.off_thr = 0.0f;
    if (q.shot) {                                      // generate_shot_noise thresholds
        const float inten = rescale(fr);
        const float factor = (g.shot_noise_rate_hz / 2.0f * dt_frame / (float)q.ni) * ((0.25f - 1.0f) * inten + 1.0f);
        q.on_thr = 1.0f - factor * pos_pre;
        q.off_thr = factor * neg_pre;
    }
    return q;
}

// The voxel cells of a pixel are touched by this thread only, so they are loaded once (at the
// pixel's first event) and accumulated in registers, in the reference's order -- bit-identical
// to a read-modify-write per event (a cell never holds -0, so the +0 of the untouched cells'
// selects is exact), without one dependent global round trip per event.
template <int NB>
__global__ __launch_bounds__(256) void v2e_emit_kernel(Call c, State s, Scratch w, const float *frames, float *vox,
                                                       int n, float dt_frame) {
    const int HW = c.H * c.W;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const cista_v2e_config &g = c.cfg;
    unsigned nev = 0;
    if (i < c.B * HW) {
        const int b = i / HW;
        const int p = i - b * HW;
        // the per-pixel operands in one batch of loads (the voxel cells only at the first event)
        const bool shot = g.shot_noise_rate_hz > 0.0f;
        const int cnt = w.counts[i];
        const float pol = w.pol[i];
        const float pos = s.pos[i], neg = s.neg[i], base = s.base[i], tmem0 = s.tmem[i];
        const float fr = shot ? frames[((size_t)b * c.F + n) * HW + p] : 0.0f;
        const float pos_pre = shot ? s.pos_pre[i] : 0.0f, neg_pre = shot ? s.neg_pre[i] : 0.0f;
        const float C = (pol > 0.0f ? pos : 0.0f) + (pol < 0.0f ? neg : 0.0f);
        int final_cnt = 0;
        if (pol != 0.0f) {                 // pol == 0: no count, no shot noise, no event (exact skip)
            const int max_iters = w.meta[0];
            PixelSteps px = pixel_steps(c, w, n, dt_frame, b, p, cnt, pol, fr, pos_pre, neg_pre, tmem0);
            const int nb = c.nb;
            float *vp = vox + (size_t)b * nb * HW + p;
            float cell[NB];
            unsigned touched = 0;
            bool loaded = false;
            for (int it = 0; it < max_iters; ++it) {
                float ts;
                if (!px.fire(it, ts)) continue;
                final_cnt += 1;                                // :476
                const float ti = floorf(ts);                   // :479-484
                const float dts = ts - ti;
                if (ti >= 0.0f) {
                    if (!loaded) {
#pragma unroll
                        for (int j = 0; j < NB; ++j) cell[j] = j < nb ? vp[(size_t)j * HW] : 0.0f;
                        loaded = true;
                    }
                    const int k = (int)ts;
                    nev += 1;
                    const float vl = pol * (1.0f - dts), vr = pol * dts;
                    const bool right = ti + 1.0f < (float)nb;
#pragma unroll
                    for (int j = 0; j < NB; ++j) {             // k >= nb: dropped
                        if (j == k) cell[j] += vl;
                        if (j == k + 1 && right) cell[j] += vr;
                    }
                    if (k < nb) touched |= 1u << k;
                    if (right) touched |= 1u << (k + 1);
                }
            }
#pragma unroll
            for (int j = 0; j < NB; ++j)
                if ((touched >> j) & 1u) vp[(size_t)j * HW] = cell[j];
            if (px.refr) s.tmem[i] = px.tmem;
        }
        s.base[i] = base + pol * (float)final_cnt * C;        // :520
    }
    // events generated: wave sums, then one atomic per workgroup
    __shared__ unsigned red[4];
    unsigned t = nev;
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long tot = (unsigned long long)red[0] + red[1] + red[2] + red[3];
        // slot per workgroup: thousands of same-address atomics serialise in L2 (~10 ns each:
        // 3600 of them were the whole 39 us of this kernel at 720x1280)
        if (tot) atomicAdd(w.nev + (blockIdx.x % MAXSLOTS) * (SLOTW / 2), tot);
    }
}

__global__ void v2e_nev_kernel(Scratch w, unsigned long long *out) {
    unsigned long long t = w.nev[threadIdx.x * (SLOTW / 2)];   // 64 lanes = MAXSLOTS slots
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if (threadIdx.x == 0) *out = t;
}

// ------------------------------------------------------------------ raw-event mode
// output_mode='raw' (v2e_model.py:504-518,527-534): rows [t, x, y, p, b] (float32) of every
// event, sorted by batch element, then timestamp.  Within one element the timestamps grow with
// (frame n, iteration it) -- every event has it < num_iters[b], so t = time_frames[n-1] +
// ts_step * (it + 1) > 0 -- and the rows of one (b, n, it) share t, kept in the reference's
// emission order (y, x): the row order is (b, n, it, y, x), the result of the reference's two
// sorts when ties keep their emission order.  Rows are written in place, no sort: a count pass
// over the whole call gives every element's row range, then the call is replayed from the same
// state and random stream, each iteration block of 32 writing its rows at offsets from an
// exclusive scan of per-wave event counts.
struct RawScratch {
    float *snap;                   // base, lp, tmem planes at the start of the call
    unsigned *bits;                // B*HW: fired iterations of the current 32-iteration block
    unsigned *cnt;                 // [B][32][nchunks] per-wave event counts, then their first rows
    unsigned long long *totb;      // [B][MAXSLOTS][SLOTW/2] partial event totals per element
    unsigned long long *run;       // [B] next output row of each element, [B] the call's total
    int *mis;                      // [CISTA_V2E_MAX_FRAMES] max_num_iters of each frame step
    unsigned *tsum;                // [B][ntiles] tile sums of cnt, then the tiles' first rows
    int nchunks;                   // 64-pixel waves per batch element
    int ntiles;                    // SCAN_TILE-element tiles of one element's cnt
};
constexpr int SCAN_TILE = 4096;    // 256 threads x 16 consecutive counts

// One wave = 64 consecutive pixels of one element (grid (ceil(nchunks / 4), B)).  COUNT: the
// frame step with its state update, adding the events to the element's total.  Otherwise the
// step replayed for iterations [32 blk, 32 blk + 32): fired-iteration bits per pixel and event
// counts per (iteration, wave); `update` (the last block) also writes base / tmem.
template <bool COUNT>
__global__ __launch_bounds__(256) void v2e_raw_emit_kernel(Call c, State s, Scratch w, RawScratch r,
                                                           const float *frames, int n, float dt_frame, int blk,
                                                           int update) {
    const int HW = c.H * c.W;
    const int b = blockIdx.y, chunk = blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int p = chunk * 64 + lane;
    const int i = b * HW + p;
    unsigned bits = 0, nev = 0;
    if (p < HW) {
        const bool shot = c.cfg.shot_noise_rate_hz > 0.0f;
        const int cnt = w.counts[i];
        const float pol = w.pol[i];
        const float pos = s.pos[i], neg = s.neg[i], base = s.base[i], tmem0 = s.tmem[i];
        const float fr = shot ? frames[((size_t)b * c.F + n) * HW + p] : 0.0f;
        const float pos_pre = shot ? s.pos_pre[i] : 0.0f, neg_pre = shot ? s.neg_pre[i] : 0.0f;
        const float C = (pol > 0.0f ? pos : 0.0f) + (pol < 0.0f ? neg : 0.0f);
        int final_cnt = 0;
        if (pol != 0.0f) {
            const int max_iters = w.meta[0];
            const int lo = 32 * blk;
            const int end = update ? max_iters : min(max_iters, lo + 32);
            PixelSteps px = pixel_steps(c, w, n, dt_frame, b, p, cnt, pol, fr, pos_pre, neg_pre, tmem0);
            for (int it = 0; it < end; ++it) {
                float ts;
                if (!px.fire(it, ts)) continue;
                final_cnt += 1;
                if (it >= lo && it < lo + 32) bits |= 1u << (it - lo);
            }
            if (update && px.refr) s.tmem[i] = px.tmem;
        }
        if (update) s.base[i] = base + pol * (float)final_cnt * C;   // :520
        nev = (unsigned)final_cnt;
    }
    if (COUNT) {
        unsigned t = nev;
        for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
        if (lane == 0 && t != 0u)
            atomicAdd(r.totb + ((size_t)b * MAXSLOTS + chunk % MAXSLOTS) * (SLOTW / 2), (unsigned long long)t);
    } else {
        if (p < HW) r.bits[i] = bits;
        unsigned mine = 0;
        for (int j = 0; j < 32; ++j) {
            const unsigned cj = (unsigned)__popcll(__ballot((bits >> j) & 1u));
            if (lane == j) mine = cj;
        }
        if (lane < 32 && chunk < r.nchunks) r.cnt[((size_t)b * 32 + lane) * r.nchunks + chunk] = mine;
    }
}

// Row ranges of the elements from the count pass: run[b] = rows of elements < b, run[B] = total.
__global__ void v2e_raw_offsets_kernel(RawScratch r, int B) {
    if (threadIdx.x != 0) return;
    unsigned long long acc = 0;
    for (int b = 0; b < B; ++b) {
        unsigned long long t = 0;
        for (int k = 0; k < MAXSLOTS; ++k) t += r.totb[((size_t)b * MAXSLOTS + k) * (SLOTW / 2)];
        r.run[b] = acc;
        acc += t;
    }
    r.run[B] = acc;
}

// The counts [32][nchunks] of an element (iteration-major, then pixel order) become exclusive
// row offsets continuing from run[b], in three launches over SCAN_TILE-count tiles: tile sums,
// one workgroup per element scanning its tile sums (and moving run[b] past this block's rows),
// then each tile rescanned from its offset.
__device__ __forceinline__ unsigned block_excl_scan256(unsigned v, unsigned *wsum, unsigned &total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    unsigned before = 0;
    for (int k = 0; k < wv; ++k) before += wsum[k];
    total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    return before + incl - v;
}

__global__ __launch_bounds__(256) void v2e_raw_tile_sum_kernel(RawScratch r) {
    __shared__ unsigned wsum[4];
    const int b = blockIdx.y, n = 32 * r.nchunks;
    const unsigned *a = r.cnt + (size_t)b * n;
    const int base = blockIdx.x * SCAN_TILE + threadIdx.x * 16;
    unsigned v = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (base + k < n) v += a[base + k];
    unsigned total;
    block_excl_scan256(v, wsum, total);
    if (threadIdx.x == 0) r.tsum[(size_t)b * r.ntiles + blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void v2e_raw_tile_scan_kernel(RawScratch r) {
    __shared__ unsigned wsum[16];
    const int b = blockIdx.x;
    const int n = r.ntiles;
    unsigned *a = r.tsum + (size_t)b * n;
    const int per = (n + 1023) / 1024;
    const int lo = min(n, (int)threadIdx.x * per), hi = min(n, lo + per);
    const unsigned long long start = r.run[b];       // read before the barrier, written after
    unsigned sum = 0;
    for (int k = lo; k < hi; ++k) sum += a[k];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned v = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    if (lane == 63) wsum[wv] = v;
    __syncthreads();
    unsigned before = 0;
    for (int k = 0; k < wv; ++k) before += wsum[k];
    unsigned pos = (unsigned)start + before + v - sum;
    for (int k = lo; k < hi; ++k) {
        const unsigned x = a[k];
        a[k] = pos;
        pos += x;
    }
    if (threadIdx.x == 1023) r.run[b] = start + before + v;
}

__global__ __launch_bounds__(256) void v2e_raw_tile_apply_kernel(RawScratch r) {
    __shared__ unsigned wsum[4];
    const int b = blockIdx.y, n = 32 * r.nchunks;
    unsigned *a = r.cnt + (size_t)b * n;
    const int base = blockIdx.x * SCAN_TILE + threadIdx.x * 16;
    unsigned c[16], v = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        c[k] = base + k < n ? a[base + k] : 0u;
        v += c[k];
    }
    unsigned total;
    unsigned pos = r.tsum[(size_t)b * r.ntiles + blockIdx.x] + block_excl_scan256(v, wsum, total);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (base + k < n) a[base + k] = pos;
        pos += c[k];
    }
}

// The rows of iteration block `blk`: an event's row is its (iteration, wave) offset plus its rank
// among the wave's lanes firing at that iteration (pixel order).
__global__ __launch_bounds__(256) void v2e_raw_fill_kernel(Call c, Scratch w, RawScratch r, int n, int blk,
                                                           float *events, unsigned long long capacity) {
    const int HW = c.H * c.W;
    const int b = blockIdx.y, chunk = blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (chunk >= r.nchunks) return;                   // whole waves
    const int p = chunk * 64 + lane;
    const unsigned bits = p < HW ? r.bits[b * HW + p] : 0u;
    if (__ballot(bits != 0u) == 0ull) return;
    const float step = w.ts_step[b], t0 = c.time_frames[n - 1];
    const float pol = p < HW ? w.pol[b * HW + p] : 0.0f;
    const int y = p / c.W, x = p - y * c.W;
    const unsigned *off = r.cnt + (size_t)b * 32 * r.nchunks + chunk;
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int j = 0; j < 32; ++j) {
        const bool m = (bits >> j) & 1u;
        const unsigned long long bal = __ballot(m);
        if (bal == 0ull) continue;
        if (m) {
            const unsigned long long row = (unsigned long long)off[(size_t)j * r.nchunks] + __popcll(bal & below);
            if (row < capacity) {
                float *e = events + row * 5;
                e[0] = t0 + step * (float)(32 * blk + j + 1);   // the PixelSteps::fire timestamp
                e[1] = (float)x;
                e[2] = (float)y;
                e[3] = pol;
                e[4] = (float)b;
            }
        }
    }
}

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

State carve_state(void *base, int B, int H, int W) {
    State s;
    size_t off = 0;
    const size_t n = (size_t)B * H * W;
    char *p = static_cast<char *>(base);
    auto take = [&]() {
        float *r = p ? reinterpret_cast<float *>(p + off) : nullptr;
        off = align_up(off + n * 4);
        return r;
    };
    s.base = take(); s.lp = take(); s.pos = take(); s.neg = take();
    s.pos_pre = take(); s.neg_pre = take(); s.noise_rate = take(); s.tmem = take();
    (void)off;
    return s;
}

size_t state_bytes(int B, int H, int W) { return 8 * align_up((size_t)B * H * W * 4); }

struct WsLayout {
    Scratch sc;
    void *vox_ws;       // voxel preprocess workspace
    size_t vox_ws_bytes, bytes;
};

WsLayout carve_ws(void *base, int B, int H, int W, int nb) {
    WsLayout L;
    size_t off = 0;
    const size_t n = (size_t)B * H * W;
    char *p = static_cast<char *>(base);
    auto take = [&](size_t bytes) {
        void *r = p ? p + off : nullptr;
        off = align_up(off + bytes);
        return r;
    };
    L.sc.counts = static_cast<int *>(take(n * 4));
    L.sc.pol = static_cast<float *>(take(n * 4));
    L.sc.iters_raw = static_cast<int *>(take((size_t)CISTA_V2E_MAX_BATCH * MAXSLOTS * SLOTW * 4));
    L.sc.num_iters = static_cast<int *>(take(CISTA_V2E_MAX_BATCH * 4));
    L.sc.ts_step = static_cast<float *>(take(CISTA_V2E_MAX_BATCH * 4));
    L.sc.meta = static_cast<int *>(take(16));
    L.sc.nev = static_cast<unsigned long long *>(take(MAXSLOTS * SLOTW * 4));
    L.vox_ws_bytes = cista_voxel_workspace_bytes(1, 0, B * nb, H, W);
    L.vox_ws = take(L.vox_ws_bytes);
    L.bytes = off;
    return L;
}

inline dim3 g1d(long long n) { return dim3((unsigned)((n + 255) / 256)); }

// torch.linspace(start, end, steps) in float32 (symmetric formula of ATen's linspace kernel)
void linspace_f32(float start, float end, int steps, float *out) {
    if (steps == 1) {
        out[0] = start;
        return;
    }
    const float step = (end - start) / (float)(steps - 1);
    const int halfway = steps / 2;
    for (int k = 0; k < steps; ++k)
        out[k] = k < halfway ? start + step * (float)k : end - step * (float)(steps - k - 1);
}

RawScratch carve_raw(void *base, int B, int H, int W, size_t *bytes) {
    RawScratch r;
    size_t off = 0;
    const size_t n = (size_t)B * H * W;
    char *p = static_cast<char *>(base);
    auto take = [&](size_t nbytes) {
        void *q = p ? p + off : nullptr;
        off = align_up(off + nbytes);
        return q;
    };
    r.nchunks = (H * W + 63) / 64;
    r.snap = static_cast<float *>(take(3 * n * 4));
    r.bits = static_cast<unsigned *>(take(n * 4));
    r.cnt = static_cast<unsigned *>(take((size_t)B * 32 * r.nchunks * 4));
    r.totb = static_cast<unsigned long long *>(take((size_t)B * MAXSLOTS * (SLOTW / 2) * 8));
    r.run = static_cast<unsigned long long *>(take(((size_t)B + 1) * 8));
    r.mis = static_cast<int *>(take(CISTA_V2E_MAX_FRAMES * 4));
    r.ntiles = (32 * r.nchunks + SCAN_TILE - 1) / SCAN_TILE;
    r.tsum = static_cast<unsigned *>(take((size_t)B * r.ntiles * 4));
    *bytes = off;
    return r;
}

// The per-call constants (v2e_model.py:303-322 and the low-pass time constants :266-289).
int make_call(const cista_v2e_config *cfg, const double *t_frames, int t_cols, int B, int F, int H, int W, Call &c) {
    if (B <= 0 || B > CISTA_V2E_MAX_BATCH || F < 2 || F > CISTA_V2E_MAX_FRAMES || H <= 0 || W <= 0)
        return B > CISTA_V2E_MAX_BATCH || F > CISTA_V2E_MAX_FRAMES ? CISTA_ERR_UNSUPPORTED : CISTA_ERR_INVALID;
    if (cfg->num_bins < 2 || cfg->num_bins > 16 || (t_cols != 2 && t_cols != F)) return CISTA_ERR_INVALID;
    if ((long long)B * H * W >= (1LL << 31)) return CISTA_ERR_UNSUPPORTED;        // 32-bit pixel index
    const int nb = cfg->num_bins;
    memset(&c, 0, sizeof(c));
    c.B = B; c.F = F; c.H = H; c.W = W; c.nb = nb;
    c.cfg = *cfg;
    c.seed = cfg->seed;
    // frame times (:313-317): linspace over the first sample's first/last time, or its row
    if (t_cols == 2) linspace_f32((float)t_frames[0], (float)t_frames[1], F, c.tf);
    else
        for (int k = 0; k < F; ++k) c.tf[k] = (float)t_frames[k];
    const double duration = (double)(nb - 1) / (double)(F - 1);                    // :319
    c.duration = (float)duration;
    linspace_f32(0.0f, (float)(duration * (F - 1)), F, c.time_frames);            // :320
    for (int b = 0; b < B; ++b) {                                                  // :322
        const float span = (float)(t_frames[(size_t)b * t_cols + t_cols - 1] - t_frames[(size_t)b * t_cols]);
        c.Tr[b] = (float)(nb - 1) * cfg->refractory_period_s * (1.0f / span);
    }
    const double pi2 = 3.14159265358979323846 * 2.0;
    for (int k = 1; k < F; ++k) {
        const float dt = c.tf[k] - c.tf[k - 1];                                    // :275
        if (cfg->cutoff_hz > 0.0f) {
            c.dt_lp0[k] = cfg->ql > 0.0f ? dt / (float)(1.0 / (pi2 * cfg->cutoff_hz * cfg->ql)) : 1.0f;
            c.dt_lp1[k] = cfg->qs > 0.0f ? dt / (float)(1.0 / (pi2 * cfg->cutoff_hz * cfg->qs)) : 1.0f;
        }
    }
    c.linlog_f = (1.0 / 20.0) * log(20.0);
    return CISTA_OK;
}

// Start of a forward call: _init on the first call, else the refractory-memory shift (:324-331);
// the frame-time check (:339-342); cleared event / image-max slots; this call's random stream.
int begin_call(Call &c, const State &s, const Scratch &sc, cista_v2e_host_state *hs, const float *frames,
               const double *t_frames, hipStream_t st) {
    const long long npx = (long long)c.B * c.H * c.W;
    if (!hs->initialized) {
        c.draw0 = hs->draw;
        hipLaunchKernelGGL(v2e_init_kernel, g1d(npx), dim3(256), 0, st, c, s, frames);
        hs->draw += 8;
        hs->t_previous = (float)t_frames[0];
        hs->initialized = 1;
    } else if (c.cfg.refractory_period_s > 0.0f) {
        hipLaunchKernelGGL(v2e_tmem_kernel, g1d(npx), dim3(256), 0, st, c, s);
    }
    if (!(c.tf[1] > hs->t_previous)) return CISTA_ERR_INVALID;                     // :339-342
    if (hipMemsetAsync(sc.nev, 0, MAXSLOTS * SLOTW * 4, st) != hipSuccess) return CISTA_ERR_HIP;
    c.draw0 = hs->draw;
    hs->draw += 2 * (unsigned long long)c.F + 16;
    // the image-max slots start cleared; each frame's v2e_iters_kernel clears them after reading
    if (hipMemsetAsync(sc.iters_raw, 0, (size_t)c.B * MAXSLOTS * SLOTW * 4, st) != hipSuccess) return CISTA_ERR_HIP;
    return CISTA_OK;
}

}  // namespace cista_v2e

using namespace cista_v2e;

extern "C" {

size_t cista_v2e_state_bytes(int B, int H, int W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    return state_bytes(B, H, W);
}

size_t cista_v2e_workspace_bytes(int B, int H, int W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    return carve_ws(nullptr, B, H, W, 16).bytes;   // sized for up to 16 bins
}

size_t cista_v2e_raw_workspace_bytes(int B, int H, int W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    size_t raw = 0;
    carve_raw(nullptr, B, H, W, &raw);
    return carve_ws(nullptr, B, H, W, 16).bytes + raw;
}

int cista_v2e_forward(const cista_v2e_config *cfg, cista_v2e_host_state *hs, void *state, const float *frames,
                      const double *t_frames, int t_cols, int B, int F, int H, int W, float *voxels,
                      unsigned long long *num_events, void *workspace, size_t workspace_bytes, void *stream) {
    if (!cfg || !hs || !state || !frames || !t_frames || !voxels || !workspace) return CISTA_ERR_INVALID;
    Call c;
    const int rc = make_call(cfg, t_frames, t_cols, B, F, H, W, c);
    if (rc != CISTA_OK) return rc;
    const WsLayout L = carve_ws(workspace, B, H, W, cfg->num_bins);
    if (workspace_bytes < L.bytes) return CISTA_ERR_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const State s = carve_state(state, B, H, W);
    const int nb = cfg->num_bins;
    const long long npx = (long long)B * H * W;
    const int rb = begin_call(c, s, L.sc, hs, frames, t_frames, st);
    if (rb != CISTA_OK) return rb;
    if (hipMemsetAsync(voxels, 0, (size_t)B * nb * H * W * 4, st) != hipSuccess) return CISTA_ERR_HIP;
    for (int n = 1; n < F; ++n) {
        const float dt = c.tf[n] - hs->t_previous;                                 // :352
        hipLaunchKernelGGL(v2e_diff_kernel, g1d(npx), dim3(256), 0, st, c, s, L.sc, frames, n, dt);
        hipLaunchKernelGGL(v2e_iters_kernel, dim3(1), dim3(64), 0, st, c, L.sc);
        if (nb <= 5)
            hipLaunchKernelGGL(v2e_emit_kernel<5>, g1d(npx), dim3(256), 0, st, c, s, L.sc, frames, voxels, n, dt);
        else
            hipLaunchKernelGGL(v2e_emit_kernel<16>, g1d(npx), dim3(256), 0, st, c, s, L.sc, frames, voxels, n, dt);
        hs->t_previous = c.tf[n];                                                  // :518
    }
    if (num_events) hipLaunchKernelGGL(v2e_nev_kernel, dim3(1), dim3(MAXSLOTS), 0, st, L.sc, num_events);
    if (hipGetLastError() != hipSuccess) return CISTA_ERR_HIP;
    // event_preprocess_pytorch(mode='std', filter_hot_pixel=False) over the whole tensor (:526)
    return cista_voxel_preprocess(voxels, 1, B * nb, H, W, CISTA_VOXEL_STD_F32, 0.0f, L.vox_ws, L.vox_ws_bytes,
                                  stream);
}

int cista_v2e_forward_raw(const cista_v2e_config *cfg, cista_v2e_host_state *hs, void *state, const float *frames,
                          const double *t_frames, int t_cols, int B, int F, int H, int W, float *events,
                          unsigned long long capacity, unsigned long long *num_events, int *loop_iterations,
                          void *workspace, size_t workspace_bytes, void *stream) {
    if (!cfg || !hs || !state || !frames || !t_frames || !num_events || !workspace || (capacity && !events))
        return CISTA_ERR_INVALID;
    Call c;
    const int rc = make_call(cfg, t_frames, t_cols, B, F, H, W, c);
    if (rc != CISTA_OK) return rc;
    const WsLayout L = carve_ws(workspace, B, H, W, cfg->num_bins);
    size_t raw_bytes = 0;
    const RawScratch r = carve_raw(static_cast<char *>(workspace) + L.bytes, B, H, W, &raw_bytes);
    if (workspace_bytes < L.bytes + raw_bytes) return CISTA_ERR_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const State s = carve_state(state, B, H, W);
    const long long npx = (long long)B * H * W;
    const size_t plane = (size_t)npx * 4;
    const dim3 wgrid((unsigned)((r.nchunks + 3) / 4), (unsigned)B);
    const cista_v2e_host_state hs0 = *hs;
    // base / lp / tmem are the state a call changes once initialised (thresholds and noise rates
    // are fixed at _init, which replays identically from the same random-stream counter)
    if (hs0.initialized) {
        if (hipMemcpyAsync(r.snap, s.base, plane, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipMemcpyAsync(r.snap + npx, s.lp, plane, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipMemcpyAsync(r.snap + 2 * npx, s.tmem, plane, hipMemcpyDeviceToDevice, st) != hipSuccess)
            return CISTA_ERR_HIP;
    }
    auto restore = [&]() -> int {
        *hs = hs0;
        if (!hs0.initialized) return CISTA_OK;
        if (hipMemcpyAsync(s.base, r.snap, plane, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipMemcpyAsync(s.lp, r.snap + npx, plane, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipMemcpyAsync(s.tmem, r.snap + 2 * npx, plane, hipMemcpyDeviceToDevice, st) != hipSuccess)
            return CISTA_ERR_HIP;
        return CISTA_OK;
    };

    // pass 1: the call's frame steps, counting each element's events
    int rb = begin_call(c, s, L.sc, hs, frames, t_frames, st);
    if (rb != CISTA_OK) return rb;
    if (hipMemsetAsync(r.totb, 0, (size_t)B * MAXSLOTS * (SLOTW / 2) * 8, st) != hipSuccess) return CISTA_ERR_HIP;
    for (int n = 1; n < F; ++n) {
        const float dt = c.tf[n] - hs->t_previous;
        hipLaunchKernelGGL(v2e_diff_kernel, g1d(npx), dim3(256), 0, st, c, s, L.sc, frames, n, dt);
        hipLaunchKernelGGL(v2e_iters_kernel, dim3(1), dim3(64), 0, st, c, L.sc);
        if (hipMemcpyAsync(r.mis + n, L.sc.meta, 4, hipMemcpyDeviceToDevice, st) != hipSuccess) return CISTA_ERR_HIP;
        hipLaunchKernelGGL(v2e_raw_emit_kernel<true>, wgrid, dim3(256), 0, st, c, s, L.sc, r, frames, n, dt, 0, 1);
        hs->t_previous = c.tf[n];
    }
    hipLaunchKernelGGL(v2e_raw_offsets_kernel, dim3(1), dim3(64), 0, st, r, B);
    if (hipGetLastError() != hipSuccess) return CISTA_ERR_HIP;
    unsigned long long total = 0;
    int mis[CISTA_V2E_MAX_FRAMES] = {0};
    if (hipMemcpyAsync(&total, r.run + B, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(mis + 1, r.mis + 1, (size_t)(F - 1) * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return CISTA_ERR_HIP;
    *num_events = total;
    if (loop_iterations) {
        int sum = 0;
        for (int n = 1; n < F; ++n) sum += mis[n];
        *loop_iterations = sum;
    }
    if (total > capacity || total >= (1ull << 32)) {   // the caller sizes `events` and calls again
        const int rr = restore();
        if (rr != CISTA_OK) return rr;
        return total >= (1ull << 32) ? CISTA_ERR_UNSUPPORTED : CISTA_ERR_WORKSPACE;
    }

    // pass 2: the same steps from the same state and random stream, writing the rows
    rb = restore();
    if (rb != CISTA_OK) return rb;
    rb = begin_call(c, s, L.sc, hs, frames, t_frames, st);
    if (rb != CISTA_OK) return rb;
    for (int n = 1; n < F; ++n) {
        const float dt = c.tf[n] - hs->t_previous;
        hipLaunchKernelGGL(v2e_diff_kernel, g1d(npx), dim3(256), 0, st, c, s, L.sc, frames, n, dt);
        hipLaunchKernelGGL(v2e_iters_kernel, dim3(1), dim3(64), 0, st, c, L.sc);
        const int nblk = mis[n] > 0 ? (mis[n] + 31) / 32 : 1;
        for (int blk = 0; blk < nblk; ++blk) {
            hipLaunchKernelGGL(v2e_raw_emit_kernel<false>, wgrid, dim3(256), 0, st, c, s, L.sc, r, frames, n, dt, blk,
                               blk == nblk - 1 ? 1 : 0);
            if (mis[n] == 0) continue;
            const dim3 tgrid((unsigned)r.ntiles, (unsigned)B);
            hipLaunchKernelGGL(v2e_raw_tile_sum_kernel, tgrid, dim3(256), 0, st, r);
            hipLaunchKernelGGL(v2e_raw_tile_scan_kernel, dim3((unsigned)B), dim3(1024), 0, st, r);
            hipLaunchKernelGGL(v2e_raw_tile_apply_kernel, tgrid, dim3(256), 0, st, r);
            hipLaunchKernelGGL(v2e_raw_fill_kernel, wgrid, dim3(256), 0, st, c, L.sc, r, n, blk, events, capacity);
        }
        hs->t_previous = c.tf[n];
    }
    return hipGetLastError() == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
}

}  // extern "C"
