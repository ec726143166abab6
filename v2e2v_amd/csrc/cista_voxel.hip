// GPU event voxelizer + event_preprocess for the CISTA-LSTC input.
//
// Reference: utils/event_process.py:15-63 (events_to_voxel_grid, numpy), :132-154
// (event_preprocess), :157-176 (event_preprocess_pytorch).  The results are bit-identical to the
// numpy path; see include/cista_voxel.h for the argument contract.
//
// Pipeline (one stream, no host sync):
//   1. vox_keys_kernel   : event i -> key (window, pixel), value i; out-of-grid -> sentinel
//   2. stable radix sort : groups each (window, pixel)'s events, keeping event order
//   3. vox_accum_kernel  : one thread per group walks its events in order, left contributions
//                          first, then right ones, acc = float(double(acc) + val)  (np.add.at)
//   4. vox_chunk_kernel  : per (window, 8192-element chunk): hot-pixel filter, numpy-pairwise
//                          float32 sums of v and v*v, non-zero count, min, max
//   5. vox_stats_kernel  : per window: chunk sums in order -> mean/std (float64) or min/max
//   6. vox_apply_kernel  : filter + normalise in place
//
// Floating-point contraction is OFF for this file: every add/mul must round exactly like numpy.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <mutex>

#include "../../include/cista_lstc.h"
#include "../../include/cista_voxel.h"

namespace cista_vox {

constexpr int CHUNK = 8192;    // numpy ufunc buffer size: the float32 reduction runs per chunk
constexpr int LEAF = 128;      // numpy pairwise-sum block (PW_BLOCKSIZE)
constexpr int MAX_LEAVES = 128;

struct ChunkPart {
    float sum, sq, mn, mx;
    int nnz;
};
struct WinStats {
    double mean, std;
    float mn, mx;
    long long nnz;
};

__device__ __forceinline__ int window_of(const long long *off, int B, long long i) {
    int lo = 0, hi = B;   // off[lo] <= i < off[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

// Events outside the H x W frame (x >= W, y >= H, or negative).  Reference :53-58: np.add.at on
// the flat index x + y W + bin H W raises IndexError when an index leaves the grid, and otherwise
// adds the event to another cell: x >= W moves it down a row, y >= H to a later bin, a negative x
// back a row.  x, y as np.uint are truncated toward zero and wrapped modulo 2^64 (float -3.0 ->
// 2^64 - 3), and np.add.at reads the uint64 index as intp, so the sum is a signed index: in
// [-size, size) it is valid (a negative one counts from the end of the grid, Python-style),
// outside it raises.  The torch twin (:113-124, int64 index_add_) raises on negative indices too.
// flat_cell: the grid index (normalised into [0, size)) of contribution `bin` of such an event, or
// -1 where the reference raises.
__device__ __forceinline__ long long flat_cell(double x, double y, long long bin, int nb, int H, int W, bool torch_idx) {
    const long long HW = (long long)H * W, size = (long long)nb * HW;
    if (!(fabs(x) < 1.0e15) || !(fabs(y) < 1.0e15)) return -1;             // NaN / inf included
    const long long i = (long long)x + (long long)y * W + bin * HW;        // trunc, signed
    if (i >= size || i < (torch_idx ? 0 : -size)) return -1;
    return i < 0 ? i + size : i;
}

// Classifies one out-of-frame event (rare path): ORs CISTA_VOXEL_OUT_OF_RANGE (the reference
// raises) or CISTA_VOXEL_SPILL (it adds the event elsewhere) into *status, and returns the pixel
// (in [0, HW)) its contributions land on -- both share it: the right one is the left one plus
// H W, modulo the grid -- or -1 when it hits no bin or the reference raises.  Such an event is
// then sorted and accumulated with that pixel's own events, in event order, its bins taken from
// flat_cell (spill_bins), so the grid is bit-identical to np.add.at's.
__device__ __noinline__ long long grid_status(const double *e, double x, double y, double first, double dT, int nb,
                                              int H, int W, bool torch_floor, int *status) {
    const double ts = (double)(nb - 1) * (e[0] - first) / dT;
    const double tf = torch_floor ? floor(ts) : ts;
    if (!(tf > -1.0) || !(tf < 9.0e18) || (torch_floor && tf < 0.0)) return -1;   // hits no bin
    const long long ti = (long long)tf;
    const long long HW = (long long)H * W;
    int f = 0;
    long long cl = -1, cr = -1;
    if (ti < nb) {
        cl = flat_cell(x, y, ti, nb, H, W, torch_floor);
        f |= cl < 0 ? CISTA_VOXEL_OUT_OF_RANGE : CISTA_VOXEL_SPILL;
    }
    if (ti + 1 < nb) {
        cr = flat_cell(x, y, ti + 1, nb, H, W, torch_floor);
        f |= cr < 0 ? CISTA_VOXEL_OUT_OF_RANGE : CISTA_VOXEL_SPILL;
    }
    if (f && status) atomicOr(status, f);
    if (f == 0 || (f & CISTA_VOXEL_OUT_OF_RANGE)) return -1;
    return cl % HW;                                  // ti + 1 < nb implies ti < nb: cl is set
}

// bins of the left / right contribution of an event with time bin ti: (ti, ti + 1) inside the
// frame; for an out-of-frame event the bins of its flat cells (its pixel is its sort key)
__device__ __forceinline__ void spill_bins(double x, double y, unsigned long long ti, int nb, int H, int W,
                                           bool torch_idx, unsigned long long &bl, unsigned long long &br) {
    bl = ti;
    br = ti + 1;
    if (x > -1.0 && x < (double)W && y > -1.0 && y < (double)H) return;
    const long long HW = (long long)H * W;
    const long long cl = ti < (unsigned long long)nb ? flat_cell(x, y, (long long)ti, nb, H, W, torch_idx) : -1;
    const long long cr = ti + 1 < (unsigned long long)nb ? flat_cell(x, y, (long long)ti + 1, nb, H, W, torch_idx) : -1;
    // an invalid cell (the reference raised: reported by grid_status) gets bin nb, i.e. none
    bl = cl < 0 ? (unsigned long long)nb : (unsigned long long)(cl / HW);
    br = cr < 0 ? (unsigned long long)nb : (unsigned long long)(cr / HW);
}

__global__ void vox_keys_kernel(const double *ev, const long long *off, int B, long long N, int H, int W,
                                unsigned long long *keys, int *vals, int nb, int torch_acc, int *status) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int b = window_of(off, B, i);
    const double x = ev[4 * i + 1], y = ev[4 * i + 2];
    const unsigned long long HW = (unsigned long long)H * W;
    unsigned long long key = (unsigned long long)B * HW;   // sentinel: sorts last, ignored
    // reference :42-43: astype(np.uint) truncates toward zero, so (-1, W) maps into [0, W)
    if (x > -1.0 && x < (double)W && y > -1.0 && y < (double)H) {
        key = (unsigned long long)b * HW + (unsigned long long)y * W + (unsigned long long)x;
    } else {                                  // rare: the pixel the reference's flat index hits
        const long long e0 = off[b], e1 = off[b + 1] - 1;
        double dT = ev[4 * e1] - ev[4 * e0];
        if (dT == 0.0) dT = 1.0;
        const long long p = grid_status(ev + 4 * i, x, y, ev[4 * e0], dT, nb, H, W, torch_acc != 0, status);
        if (p >= 0) key = (unsigned long long)b * HW + (unsigned long long)p;
    }
    keys[i] = key;
    vals[i] = (int)i;
}

// time normalisation of one event (reference :36-50); false if the event hits no bin
struct EvVal {
    unsigned long long ti;
    double vl, vr;
};
__device__ __forceinline__ bool event_value(const double *e, double first, double dT, int nb, EvVal &o) {
    const double ts = (double)(nb - 1) * (e[0] - first) / dT;        // :40
    if (!(ts > -1.0) || !(ts < 9.0e18)) return false;                  // uint cast defined only here
    o.ti = (unsigned long long)ts;                                     // :48
    const double dts = ts - (double)o.ti;                              // :49
    double pol = e[3];
    if (pol == 0.0) pol = -1.0;                                        // :45
    o.vl = pol * (1.0 - dts);                                          // :50
    o.vr = pol * dts;                                                  // :51
    return true;
}

// events_to_voxel_grid_pytorch (:66-129) on a float64 events tensor: tis = floor(ts) must be
// >= 0, the contributions are float32 (pols.float() * (1 - dts.float())), and index_add_ adds
// them to the float32 grid in float32
struct EvValT {
    unsigned long long ti;
    float vl, vr;
};
__device__ __forceinline__ bool event_value_torch(const double *e, double first, double dT, int nb, EvValT &o) {
    const double ts = (double)(nb - 1) * (e[0] - first) / dT;        // :99
    const double tis = floor(ts);                                      // :106
    if (!(tis >= 0.0) || !(tis < 9.0e18)) return false;                // valid_indices &= tis >= 0
    o.ti = (unsigned long long)tis;
    const float dts = (float)(ts - tis);                               // :108, .float()
    float pol = (float)e[3];
    if (pol == 0.0f) pol = -1.0f;                                      // :104
    o.vl = pol * (1.0f - dts);                                         // :109
    o.vr = pol * dts;                                                  // :110
    return true;
}

__global__ void vox_accum_kernel(const unsigned long long *keys, const int *vals, long long N, const double *ev,
                                 const long long *off, int B, int nb, int H, int W, float *vox, int torch_acc) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= N) return;
    const unsigned long long HW = (unsigned long long)H * W;
    const unsigned long long key = keys[j];
    if (key >= (unsigned long long)B * HW) return;
    if (j > 0 && keys[j - 1] == key) return;                           // not the group head
    const int b = (int)(key / HW);
    const unsigned long long p = key - (unsigned long long)b * HW;
    const double first = ev[4 * off[b]], last = ev[4 * (off[b + 1] - 1)];
    double dT = last - first;                                          // :37-38
    if (dT == 0.0) dT = 1.0;                                           // :40-41
    float *out = vox + (size_t)b * nb * HW + p;
    long long end = j;
    while (end < N && keys[end] == key) ++end;
    // an out-of-frame event grouped here (its flat index hits pixel p) adds to the bins of its
    // flat cells (spill_bins); in-frame events to (ti, ti + 1)
    if (torch_acc) {                    // index_add_ #1 / #2 (:112-127), float32 adds
        for (int ph = 0; ph < 2; ++ph)
            for (long long k = j; k < end; ++k) {
                const double *e = ev + 4 * (long long)vals[k];
                EvValT v;
                if (!event_value_torch(e, first, dT, nb, v)) continue;
                unsigned long long bl, br;
                spill_bins(e[1], e[2], v.ti, nb, H, W, true, bl, br);
                const unsigned long long bin = ph ? br : bl;
                if (bin < (unsigned long long)nb) out[bin * HW] += ph ? v.vr : v.vl;
            }
        return;
    }
    // np.add.at #1 (:53-54): left contributions of the whole window, in event order; then
    // np.add.at #2 (:56-58): right contributions
    for (int ph = 0; ph < 2; ++ph)
        for (long long k = j; k < end; ++k) {
            const double *e = ev + 4 * (long long)vals[k];
            EvVal v;
            if (!event_value(e, first, dT, nb, v)) continue;
            unsigned long long bl, br;
            spill_bins(e[1], e[2], v.ti, nb, H, W, false, bl, br);
            const unsigned long long bin = ph ? br : bl;
            if (bin < (unsigned long long)nb) {
                float *d = out + bin * HW;
                *d = (float)((double)*d + (ph ? v.vr : v.vl));
            }
        }
}

// ------------------------------------------------------------------------------------------
// Per-window sort + tiled accumulation (replaces keys + global radix sort + memset + accum when
// the grid has < 2^18 pixels and num_bins <= WNB):
//   vox_sort_kernel (one 512-thread workgroup per window): the window's events in segments of
//     WSEG, key = pixel << 14 | event-in-segment (unique: the sort needs no stability; events
//     outside the grid get a sentinel that sorts last), block radix sort in LDS, sorted keys to
//     the workspace; for single-segment windows also the first sorted position of every tile;
//   vox_tile_kernel (one workgroup per (tile of TP pixels x num_bins bins, window)): zero the
//     tile in LDS, walk the pixel groups of the tile (contiguous in the sorted keys) -- one
//     thread per group, left contributions first, then right ones, in event order: the
//     reference's per-voxel order -- and write the tile out densely (zeros included: no memset).
// Windows of more than one segment walk every segment's range of the tile, left passes of all
// segments first, then right passes, barriers in between.
// ------------------------------------------------------------------------------------------
constexpr int WT = 512;                    // threads of the sort kernel
constexpr int WITEMS = 32;                 // sort items per thread
constexpr int WSEG = WT * WITEMS;          // events per sorted segment (14-bit local index)
constexpr int WNB = 8;                     // bins held in registers by a group walk
constexpr int TT = 256;                    // threads of the tile kernel
constexpr int WTILE = 12288;               // floats of a tile (TP = WTILE / num_bins pixels)
constexpr int TBMAX = 256;                 // tiles per window (TP >= 1536 and HW < 2^18: <= 171)
typedef hipcub::BlockRadixSort<unsigned, WT, WITEMS> WinSort;
typedef hipcub::BlockExchange<unsigned, WT, WITEMS> WinExch;
struct WinLds {
    union {
        typename WinSort::TempStorage sort;
        typename WinExch::TempStorage exch;
        unsigned keys[WSEG];               // the sorted segment
    } u;
};

__host__ __device__ inline int tile_pixels(int nb) { return (WTILE / nb) & ~3; }

// first sorted position in [0, n) whose pixel (key >> 14) is >= p
__device__ __forceinline__ int key_lower(const unsigned *k, int n, unsigned p) {
    int lo = 0, hi = n;
    const unsigned kk = p << 14;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (k[mid] < kk) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// grid (B), block WT, dynamic LDS sizeof(WinLds).  scratch: n_events sorted keys (window b's
// segments at its event offsets); tb: TBMAX + 1 tile starts per window (single-segment windows)
__global__ __launch_bounds__(WT) void vox_sort_kernel(const double *ev, const long long *off, int nb, int H, int W,
                                                      int end_bit, unsigned *scratch, double2 *tp_sorted, int *tb,
                                                      int *spw, int torch_acc, int *status) {
    extern __shared__ __align__(16) char wsm[];
    WinLds &L = *reinterpret_cast<WinLds *>(wsm);
    const int b = blockIdx.x, tid = threadIdx.x;
    int spill = 0;                      // this thread keyed an out-of-frame event to a pixel
    const long long e0 = off[b];
    const int n = (int)(off[b + 1] - e0);
    const int nseg = (n + WSEG - 1) / WSEG;
    for (int sg = 0; sg < nseg; ++sg) {
        const long long base = e0 + (long long)sg * WSEG;
        const int cnt = min(WSEG, n - sg * WSEG);
        unsigned key[WITEMS];
        // striped (coalesced) rows, loads issued branch-free in batches (a load under a branch is
        // waited for before the branch joins: 32 serial HBM round trips per thread)
        constexpr int LB = 8;
#pragma unroll
        for (int i0 = 0; i0 < WITEMS; i0 += LB) {
            double x[LB], y[LB];
#pragma unroll
            for (int i = 0; i < LB; ++i) {
                const int l = min((i0 + i) * WT + tid, cnt - 1);
                const double2 r = *reinterpret_cast<const double2 *>(ev + 4 * (base + l) + 1);
                x[i] = r.x;
                y[i] = r.y;
            }
#pragma unroll
            for (int i = 0; i < LB; ++i) {
                const int l = (i0 + i) * WT + tid;
                // reference :42-43: astype(np.uint) truncates toward zero
                const bool in = l < cnt && x[i] > -1.0 && x[i] < (double)W && y[i] > -1.0 && y[i] < (double)H;
                key[i0 + i] = in ? ((((unsigned)y[i] * (unsigned)W + (unsigned)x[i]) << 14) | (unsigned)l) : 0xFFFFFFFFu;
                if (__builtin_expect(l < cnt && !in, 0)) {      // rare: keyed to the pixel it spills to
                    double dT = ev[4 * (e0 + n - 1)] - ev[4 * e0];
                    if (dT == 0.0) dT = 1.0;
                    const long long p = grid_status(ev + 4 * (base + l), x[i], y[i], ev[4 * e0], dT, nb, H, W,
                                                    torch_acc != 0, status);
                    if (p >= 0) {
                        key[i0 + i] = ((unsigned)p << 14) | (unsigned)l;
                        spill = 1;
                    }
                }
            }
        }
        __syncthreads();                                                // LDS union reuse
        WinExch(L.u.exch).StripedToBlocked(key, key);
        __syncthreads();
        WinSort(L.u.sort).SortBlockedToStriped(key, 0, end_bit);
        __syncthreads();
        // (t, polarity) of every event in sorted order, for the tile kernel to stream: the rows
        // are re-read in event order (coalesced, L2 / Infinity-Cache hot) in rounds of WPR
        // events, staged in LDS (the sort storage) and picked up by the sorted positions
        constexpr int WPR = 4096;
        double2 *pay = reinterpret_cast<double2 *>(&L.u);
        static_assert(WPR * sizeof(double2) <= sizeof(L.u), "payload round fits the sort storage");
        for (int r0 = 0; r0 < cnt; r0 += WPR) {
            __syncthreads();
            for (int l = r0 + tid; l < min(cnt, r0 + WPR); l += WT) {
                const double *e = ev + 4 * (base + l);
                pay[l - r0] = make_double2(e[0], e[3]);
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < WITEMS; ++i) {
                const int l = i * WT + tid;
                const int idx = (int)(key[i] & 0x3FFF);
                if (l < cnt && key[i] != 0xFFFFFFFFu && idx >= r0 && idx < r0 + WPR) tp_sorted[base + l] = pay[idx - r0];
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < WITEMS; ++i) {
            const int l = i * WT + tid;
            if (nseg == 1) L.u.keys[l] = key[i];
            if (l < cnt) scratch[base + l] = key[i];
        }
    }
    spill = __syncthreads_or(spill);
    if (tid == 0) spw[b] = spill;
    if (nseg == 1) {
        __syncthreads();
        const unsigned HW = (unsigned)H * (unsigned)W;
        const int TP = tile_pixels(nb);
        const int ntiles = (int)((HW + TP - 1) / TP);
        for (int t = tid; t <= ntiles; t += WT) tb[(size_t)b * (TBMAX + 1) + t] = key_lower(L.u.keys, n, min((unsigned)t * TP, HW));
    }
}

// ---- group walks of the tile kernel; cell (bin, pixel p) = tile[bin * TP + p - pa] ----
// General walk (RMW on the LDS cells): sorted positions [s, e) of one segment; pass 1 = left
// contributions, 2 = right, 3 = both (in that order: single-segment windows)
// evs: the segment's event rows (window with spilled events: evs != nullptr, every event's bins
// through spill_bins from its own x, y; the key's low 14 bits index the row)
template <bool TORCH>
__device__ void walk_groups(const unsigned *k, int s, int e, const double2 *tps, double first, double dT, int nb,
                            float *tile, int TP, unsigned pa, int pass, const double *evs = nullptr, int H = 0,
                            int W = 0) {
    for (int j = s + (int)threadIdx.x; j < e; j += TT) {
        const unsigned p = k[j] >> 14;
        if (j > s && (k[j - 1] >> 14) == p) continue;                   // not the group head
        int g = j;
        while (g < e && (k[g] >> 14) == p) ++g;                         // group [j, g)
        float *cell = tile + (p - pa);
        for (int ph = 1; ph <= 2; ++ph) {
            if (!(pass & ph)) continue;
            for (int q = j; q < g; ++q) {
                const double2 r = tps[q];
                const double ev[4] = {r.x, 0.0, 0.0, r.y};
                double ex = 0.0, ey = 0.0;
                if (evs) {
                    const double *row = evs + 4 * (long long)(k[q] & 0x3FFFu);
                    ex = row[1];
                    ey = row[2];
                }
                if (TORCH) {
                    EvValT v;
                    if (!event_value_torch(ev, first, dT, nb, v)) continue;
                    unsigned long long bin = v.ti + (ph == 2 ? 1 : 0);
                    if (evs) {
                        unsigned long long bl, br;
                        spill_bins(ex, ey, v.ti, nb, H, W, true, bl, br);
                        bin = ph == 2 ? br : bl;
                    }
                    if (bin < (unsigned long long)nb) cell[bin * TP] += ph == 1 ? v.vl : v.vr;
                } else {
                    EvVal v;
                    if (!event_value(ev, first, dT, nb, v)) continue;
                    unsigned long long bin = v.ti + (ph == 2 ? 1 : 0);
                    if (evs) {
                        unsigned long long bl, br;
                        spill_bins(ex, ey, v.ti, nb, H, W, false, bl, br);
                        bin = ph == 2 ? br : bl;
                    }
                    if (bin < (unsigned long long)nb) {
                        float *d = cell + bin * TP;
                        *d = (float)((double)*d + (ph == 1 ? v.vl : v.vr));
                    }
                }
            }
        }
    }
}

// Fast walk (single-segment windows, nb <= WNB): a group's nb cells start at zero and only its
// thread touches them, so they are accumulated in registers -- the same adds in the same order
// -- and only the touched cells are stored; a lone event (most pixels) is evaluated once.  The
// thread's positions are taken WB at a time and their event rows gathered up front.
constexpr int WB = 4;
template <bool TORCH>
__device__ void walk_fast(const unsigned *k, int e, const double2 *tps, double first, double dT, int nb,
                          float *tile, int TP, unsigned pa) {
    // positions [0, e) of the tile: k[j] its sorted keys, tps[j] their (t, polarity)
    for (int j0 = (int)threadIdx.x; j0 < e; j0 += WB * TT) {
        unsigned kp[WB];
        double t[WB], pl[WB];
#pragma unroll
        for (int u = 0; u < WB; ++u) {                                  // branch-free gathers
            const int j = min(j0 + u * TT, e - 1);
            kp[u] = k[j];
            const double2 r = tps[j];
            t[u] = r.x;
            pl[u] = r.y;
        }
#pragma unroll
        for (int u = 0; u < WB; ++u) {
            const int j = j0 + u * TT;
            if (j >= e) break;
            const unsigned p = kp[u] >> 14;
            if (j > 0 && (k[j - 1] >> 14) == p) continue;               // not the group head
            float *cell = tile + (p - pa);
            const bool lone = j + 1 == e || (k[j + 1] >> 14) != p;
            if (lone) {             // the only left and the only right contribution of two cells
                double e4[4];
                e4[0] = t[u];
                e4[3] = pl[u];
                if (TORCH) {
                    EvValT v;
                    if (!event_value_torch(e4, first, dT, nb, v)) continue;
                    if (v.ti < (unsigned long long)nb) cell[v.ti * TP] = 0.0f + v.vl;
                    if (v.ti + 1 < (unsigned long long)nb) cell[(v.ti + 1) * TP] = 0.0f + v.vr;
                } else {
                    EvVal v;
                    if (!event_value(e4, first, dT, nb, v)) continue;
                    if (v.ti < (unsigned long long)nb) cell[v.ti * TP] = (float)(0.0 + v.vl);
                    if (v.ti + 1 < (unsigned long long)nb) cell[(v.ti + 1) * TP] = (float)(0.0 + v.vr);
                }
                continue;
            }
            int g = j + 1;
            while (g < e && (k[g] >> 14) == p) ++g;                     // group [j, g)
            float acc[WNB];
#pragma unroll
            for (int bb = 0; bb < WNB; ++bb) acc[bb] = 0.0f;
            unsigned touched = 0;
            for (int ph = 1; ph <= 2; ++ph)                             // left, then right
                for (int q = j; q < g; ++q) {
                    const double2 rr = tps[q];
                    const double r[4] = {rr.x, 0.0, 0.0, rr.y};
                    unsigned long long bin;
                    double vd = 0.0;
                    float vf = 0.0f;
                    if (TORCH) {
                        EvValT v;
                        if (!event_value_torch(r, first, dT, nb, v)) continue;
                        bin = v.ti + (ph == 2 ? 1 : 0);
                        vf = ph == 1 ? v.vl : v.vr;
                    } else {
                        EvVal v;
                        if (!event_value(r, first, dT, nb, v)) continue;
                        bin = v.ti + (ph == 2 ? 1 : 0);
                        vd = ph == 1 ? v.vl : v.vr;
                    }
                    if (bin >= (unsigned long long)nb) continue;
#pragma unroll
                    for (int bb = 0; bb < WNB; ++bb)
                        if ((unsigned long long)bb == bin) acc[bb] = TORCH ? acc[bb] + vf : (float)((double)acc[bb] + vd);
                    touched |= 1u << bin;
                }
#pragma unroll
            for (int bb = 0; bb < WNB; ++bb)
                if (touched & (1u << bb)) cell[bb * TP] = acc[bb];
        }
    }
}

// grid (ntiles, B), block TT
template <bool TORCH>
__global__ __launch_bounds__(TT) void vox_tile_kernel(const double *ev, const long long *off, int nb, int H, int W,
                                                      const unsigned *scratch, const double2 *tps, const int *tb,
                                                      const int *spw, float *vox) {
    __shared__ __align__(16) float tile[WTILE];
    __shared__ int rng[2];
    const int t = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const long long e0 = off[b];
    const int n = (int)(off[b + 1] - e0);
    const int nseg = (n + WSEG - 1) / WSEG;
    const unsigned HW = (unsigned)H * (unsigned)W;
    const int TP = tile_pixels(nb);
    const unsigned pa = (unsigned)t * TP;
    const int np = (int)min((unsigned)TP, HW - pa);
    double first = 0.0, dT = 1.0;
    if (n > 0) {
        first = ev[4 * e0];
        dT = ev[4 * (e0 + n - 1)] - first;                              // :37-38
        if (dT == 0.0) dT = 1.0;                                        // :40-41
    }
    for (int i = tid; i < nb * TP; i += TT) tile[i] = 0.0f;
    __syncthreads();
    if (nseg == 1) {
        const int *tbw = tb + (size_t)b * (TBMAX + 1);
        const int s = tbw[t], e = tbw[t + 1];
        if (spw[b]) {                      // rare: events spilled into this window's grid
            walk_groups<TORCH>(scratch + e0, s, e, tps + e0, first, dT, nb, tile, TP, pa, 3, ev + 4 * e0, H, W);
        } else if (nb <= WNB) {
            walk_fast<TORCH>(scratch + e0 + s, e - s, tps + e0 + s, first, dT, nb, tile, TP, pa);
        } else {
            walk_groups<TORCH>(scratch + e0, s, e, tps + e0, first, dT, nb, tile, TP, pa, 3);
        }
    } else if (nseg > 1) {
        for (int pass = 1; pass <= 2; ++pass)                            // np.add.at #1, then #2
            for (int sg = 0; sg < nseg; ++sg) {
                const long long base = e0 + (long long)sg * WSEG;
                const int cnt = min(WSEG, n - sg * WSEG);
                if (tid == 0) {
                    rng[0] = key_lower(scratch + base, cnt, pa);
                    rng[1] = key_lower(scratch + base, cnt, pa + np);
                }
                __syncthreads();
                walk_groups<TORCH>(scratch + base, rng[0], rng[1], tps + base, first, dT, nb, tile, TP, pa, pass,
                                   spw[b] ? ev + 4 * base : nullptr, H, W);
                __syncthreads();
            }
    }
    __syncthreads();
    float *out = vox + (size_t)b * nb * HW + pa;
    const bool vec = (((size_t)out) & 15) == 0 && (HW & 3) == 0;
    for (int kb = 0; kb < nb; ++kb) {                                    // dense rows, zeros included
        float *row = out + (size_t)kb * HW;
        const float *src = tile + kb * TP;
        if (vec) {
            for (int i = tid; i < np / 4; i += TT)
                reinterpret_cast<float4 *>(row)[i] = reinterpret_cast<const float4 *>(src)[i];
            for (int i = (np & ~3) + tid; i < np; i += TT) row[i] = src[i];
        } else {
            for (int i = tid; i < np; i += TT) row[i] = src[i];
        }
    }
}

__device__ __forceinline__ float hot(float v, float thr) { return (thr > 0.0f && fabsf(v) > thr) ? 0.0f : v; }

__device__ __forceinline__ int pw_split(int n) {
    int n2 = n / 2;
    return n2 - n2 % 8;
}

// The chunk is first staged into LDS with coalesced loads (one element per thread per step,
// hot-pixel filter applied), then every leaf is summed by its own thread from LDS.  Leaf l of
// the LDS image starts at l * LSTRIDE: a stride of 129 floats puts the 128-element leaves of
// consecutive threads on consecutive banks (conflict-free), and element i lives at
// (i >> 7) * LSTRIDE + (i & 127) for any leaf boundary of a partial chunk.
constexpr int LSTRIDE = LEAF + 1;

__device__ __forceinline__ float lds_at(const float *buf, int i) { return buf[(i >> 7) * LSTRIDE + (i & 127)]; }

// numpy pairwise_sum leaf (n <= 128) of v and v^2 over LDS elements [s, s + n) (already filtered)
__device__ void leaf_sums_lds(const float *buf, int s0, int n, float &s, float &q) {
    if (n < 8) {
        s = -0.0f;
        q = -0.0f;
        for (int i = 0; i < n; ++i) {
            const float v = lds_at(buf, s0 + i);
            s += v;
            q += v * v;
        }
        return;
    }
    float r[8], rq[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        r[k] = lds_at(buf, s0 + k);
        rq[k] = r[k] * r[k];
    }
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float v = lds_at(buf, s0 + i + k);
            r[k] += v;
            rq[k] += v * v;
        }
    }
    s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    q = ((rq[0] + rq[1]) + (rq[2] + rq[3])) + ((rq[4] + rq[5]) + (rq[6] + rq[7]));
    for (; i < n; ++i) {
        const float v = lds_at(buf, s0 + i);
        s += v;
        q += v * v;
    }
}

// grid (nchunks, B), block MAX_LEAVES
__global__ __launch_bounds__(MAX_LEAVES) void vox_chunk_kernel(const float *vox, long long n, int nchunks,
                                                               float thr, ChunkPart *parts) {
    __shared__ float buf[(CHUNK / LEAF) * LSTRIDE];
    __shared__ int lstart[MAX_LEAVES], llen[MAX_LEAVES];
    __shared__ float ls[MAX_LEAVES], lq[MAX_LEAVES];
    __shared__ int rcnt[MAX_LEAVES];
    __shared__ float rmn[MAX_LEAVES], rmx[MAX_LEAVES];
    __shared__ int nleaves;
    // thread 0's recursion stacks live in LDS: as private arrays with dynamic indices they were
    // scratch memory, and the serial walks dominated the kernel (4 ms for 960 windows)
    __shared__ int st_s[32], st_n[32], st_state[32];
    __shared__ float st_ls[32], st_lq[32];
    const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const long long start = (long long)c * CHUNK;
    const int m = (int)((n - start) < CHUNK ? (n - start) : CHUNK);
    const float *a = vox + (size_t)b * n + start;
    // a full chunk's recursion is the balanced tree over 64 leaves of 128 (8192 = 64 * 128 and
    // every split halves a multiple of 8): leaves and combination are static, done in parallel
    const bool full = m == CHUNK;
    static_assert(CHUNK % LEAF == 0 && (CHUNK / LEAF & (CHUNK / LEAF - 1)) == 0, "balanced full chunk");
    if (full) {
        if (tid < CHUNK / LEAF) { lstart[tid] = tid * LEAF; llen[tid] = LEAF; }
        if (tid == 0) nleaves = CHUNK / LEAF;
    } else if (tid == 0) {      // leaves of numpy's pairwise recursion, left to right
        int top = 0, nl = 0;
        st_s[top] = 0; st_n[top] = m; ++top;
        while (top > 0) {
            --top;
            const int s = st_s[top], len = st_n[top];
            if (len <= LEAF) {
                lstart[nl] = s; llen[nl] = len; ++nl;
            } else {
                const int n2 = pw_split(len);
                st_s[top] = s + n2; st_n[top] = len - n2; ++top;   // right, popped second
                st_s[top] = s; st_n[top] = n2; ++top;              // left, popped first
            }
        }
        nleaves = nl;
    }
    // coalesced staging + count / min / max (order-independent)
    int cnt = 0;
    float mn = INFINITY, mx = -INFINITY;
    if (full && (((size_t)a) & 15) == 0) {
        // float4 loads: 4 consecutive elements always lie in one leaf row of the LDS image
        constexpr int U4 = CHUNK / 4 / MAX_LEAVES;                   // 16 float4 per thread
        float4 v[U4];
#pragma unroll
        for (int u = 0; u < U4; ++u) v[u] = reinterpret_cast<const float4 *>(a)[tid + u * MAX_LEAVES];
#pragma unroll
        for (int u = 0; u < U4; ++u) {
            const int i = (tid + u * MAX_LEAVES) * 4;
            const float e[4] = {hot(v[u].x, thr), hot(v[u].y, thr), hot(v[u].z, thr), hot(v[u].w, thr)};
            float *dst = buf + (i >> 7) * LSTRIDE + (i & 127);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                dst[k] = e[k];
                cnt += e[k] != 0.0f;
                mn = fminf(mn, e[k]);
                mx = fmaxf(mx, e[k]);
            }
        }
    } else {
        constexpr int U = 8;
        for (int i0 = tid; i0 < m; i0 += U * MAX_LEAVES) {
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + u * MAX_LEAVES;
                v[u] = i < m ? hot(a[i], thr) : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + u * MAX_LEAVES;
                if (i < m) {
                    buf[(i >> 7) * LSTRIDE + (i & 127)] = v[u];
                    cnt += v[u] != 0.0f;
                    mn = fminf(mn, v[u]);
                    mx = fmaxf(mx, v[u]);
                }
            }
        }
    }
    rcnt[tid] = cnt; rmn[tid] = mn; rmx[tid] = mx;
    __syncthreads();
    if (full) {
        // the 64 full leaves' 8 accumulator chains (numpy's unrolled leaf: r[c] = v[c], then
        // r[c] += v[c + 8i]) spread over all 128 threads: thread (o, l) runs chains 4o..4o+3 of
        // leaf l and forms ((r[4o] + r[4o+1]) + (r[4o+2] + r[4o+3])); the leaf sum is the o = 0
        // half + the o = 1 half, exactly numpy's association
        const int l = tid & 63, o = tid >> 6;
        const float *row = buf + l * LSTRIDE + 4 * o;
        float r[4], rq[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            r[k] = row[k];
            rq[k] = r[k] * r[k];
        }
#pragma unroll
        for (int i = 1; i < LEAF / 8; ++i)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float v = row[8 * i + k];
                r[k] += v;
                rq[k] += v * v;
            }
        const float hs = (r[0] + r[1]) + (r[2] + r[3]), hq = (rq[0] + rq[1]) + (rq[2] + rq[3]);
        if (o == 1) { ls[l] = hs; lq[l] = hq; }
        __syncthreads();
        if (o == 0) { ls[l] = hs + ls[l]; lq[l] = hq + lq[l]; }
    } else if (tid < nleaves) {
        leaf_sums_lds(buf, lstart[tid], llen[tid], ls[tid], lq[tid]);
    }
    for (int k = MAX_LEAVES / 2; k > 0; k >>= 1) {
        if (tid < k) {
            rcnt[tid] += rcnt[tid + k];
            rmn[tid] = fminf(rmn[tid], rmn[tid + k]);
            rmx[tid] = fmaxf(rmx[tid], rmx[tid + k]);
        }
        __syncthreads();
    }
    if (full) {
        // node = left + right, level by level (the same additions as the recursion)
        for (int k = CHUNK / LEAF / 2; k >= 1; k >>= 1) {
            __syncthreads();
            float s2 = 0.0f, q2 = 0.0f;
            if (tid < k) { s2 = ls[2 * tid] + ls[2 * tid + 1]; q2 = lq[2 * tid] + lq[2 * tid + 1]; }
            __syncthreads();
            if (tid < k) { ls[tid] = s2; lq[tid] = q2; }
        }
        __syncthreads();
        if (tid == 0) {
            ChunkPart p;
            p.sum = ls[0]; p.sq = lq[0]; p.nnz = rcnt[0]; p.mn = rmn[0]; p.mx = rmx[0];
            parts[(size_t)b * nchunks + c] = p;
        }
        return;
    }
    if (tid == 0) {
        // post-order evaluation of the same recursion: node = left + right
        int top = 0, leaf = 0;
        st_n[0] = m; st_state[0] = 0; top = 1;
        float vs = 0.0f, vq = 0.0f;
        bool have = false;   // (vs, vq) holds a finished child value to deliver
        while (top > 0) {
            if (have) {
                const int t = top - 1;
                if (st_state[t] == 1) {            // left child finished: descend right
                    st_ls[t] = vs; st_lq[t] = vq; st_state[t] = 2; have = false;
                    const int len = st_n[t], n2 = pw_split(len);
                    st_n[top] = len - n2; st_state[top] = 0; ++top;
                } else {                           // right child finished: combine, pop
                    vs = st_ls[t] + vs; vq = st_lq[t] + vq;
                    --top;
                }
                continue;
            }
            const int t = top - 1;
            const int len = st_n[t];
            if (len <= LEAF) {
                vs = ls[leaf]; vq = lq[leaf]; ++leaf;
                --top;
                have = true;
            } else {
                st_state[t] = 1;
                st_n[top] = pw_split(len); st_state[top] = 0; ++top;
            }
        }
        ChunkPart p;
        p.sum = vs; p.sq = vq; p.nnz = rcnt[0]; p.mn = rmn[0]; p.mx = rmx[0];
        parts[(size_t)b * nchunks + c] = p;
    }
}

// one thread per window: numpy's chunk-sequential float32 accumulation, then float64 stats
// one workgroup per window: the chunk partials are staged in LDS (coalesced; read one by one
// from memory the dependent loads of the sequential sum took ~0.2 us each), then one thread
// does numpy's chunk-sequential float32 accumulation; float64 stats
constexpr int SBATCH = 1024;
__global__ __launch_bounds__(256) void vox_stats_kernel(const ChunkPart *parts, int nchunks, int mode, WinStats *st) {
    __shared__ ChunkPart sp[SBATCH];
    const int b = blockIdx.x;
    float s = 0.0f, q = 0.0f, mn = INFINITY, mx = -INFINITY;
    long long nnz = 0;
    for (int c0 = 0; c0 < nchunks; c0 += SBATCH) {
        const int nc = min(SBATCH, nchunks - c0);
        __syncthreads();
        for (int c = threadIdx.x; c < nc; c += blockDim.x) sp[c] = parts[(size_t)b * nchunks + c0 + c];
        __syncthreads();
        if (threadIdx.x == 0)
            for (int c = 0; c < nc; ++c) {
                const ChunkPart p = sp[c];
                s += p.sum;
                q += p.sq;
                nnz += p.nnz;
                mn = fminf(mn, p.mn);
                mx = fmaxf(mx, p.mx);
            }
    }
    if (threadIdx.x != 0) return;
    WinStats w;
    w.nnz = nnz; w.mn = mn; w.mx = mx;
    w.mean = 0.0; w.std = 0.0;
    if (nnz > 0 && mode == CISTA_VOXEL_STD) {
        const double dn = (double)nnz;
        const double mean = (double)s / dn;                  // :148
        w.mean = mean;
        w.std = sqrt((double)q / dn - mean * mean);          // :150
    }
    st[b] = w;
}

__device__ __forceinline__ float apply1(float v0, int mode, float thr, const WinStats &w) {
    const float v = hot(v0, thr);                            // :137-138
    float r = v;
    if (mode == CISTA_VOXEL_STD) {
        if (w.nnz > 0) {                                     // :146
            const double mask = v != 0.0f ? 1.0 : 0.0;
            r = (float)(mask * ((double)v - w.mean) / (w.std + 1e-8));   // :152
        }
    } else if (mode == CISTA_VOXEL_STD_F32) {
        if (w.nnz > 0) {                                     // :170, float32: mask * (v - mean) / (std + 1e-8)
            const float mask = v != 0.0f ? 1.0f : 0.0f;
            r = mask * (v - (float)w.mean) / ((float)w.std + 1e-8f);
        }
    } else if (mode == CISTA_VOXEL_MAXMIN) {
        r = (v - w.mn) / (w.mx - w.mn + 1e-8f);              // :140
    }
    return r;
}

// grid (ceil(n / 1024), B), block 256: 4 consecutive elements of window blockIdx.y per thread,
// as one float4 when the window's grid is 16-byte aligned
__global__ void vox_apply_kernel(float *vox, long long n, int mode, float thr, const WinStats *st) {
    const int b = blockIdx.y;
    const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i >= n) return;
    WinStats w;
    if (mode != CISTA_VOXEL_RAW) w = st[b];
    float *g = vox + (size_t)b * n + i;
    if (i + 4 <= n && (((size_t)g) & 15) == 0) {
        float4 v = *reinterpret_cast<float4 *>(g);
        v.x = apply1(v.x, mode, thr, w);
        v.y = apply1(v.y, mode, thr, w);
        v.z = apply1(v.z, mode, thr, w);
        v.w = apply1(v.w, mode, thr, w);
        *reinterpret_cast<float4 *>(g) = v;
    } else {
        for (long long k = 0; k < 4 && i + k < n; ++k) g[k] = apply1(g[k], mode, thr, w);
    }
}

// ---- CISTA_VOXEL_STD_F32 statistics: every element's v and float32(v * v) summed in float64 in a
// fixed order (a workgroup per (block, window), then one per window), rounded once to float32
// as the mode states.  Unlike the numpy modes there is no float32 pairwise order to reproduce,
// so the whole grid streams at HBM rate instead of 8192-element chunks with serial tree walks.
struct Part64 {
    double s, q;
    long long nnz;
};

inline int nblk64(long long n) {
    const long long b = (n + 4095) / 4096;               // >= 16 elements per thread
    return (int)(b < 1 ? 1 : b > 512 ? 512 : b);
}

__device__ __forceinline__ void acc64(float v0, float thr, double &s, double &q, int &nz) {
    const float v = hot(v0, thr);
    s += (double)v;
    q += (double)(v * v);                                 // (v ** 2) in float32, then summed
    nz += v != 0.0f;
}

// grid (nblk, B), block 256; thread t of block k takes float4 groups t + 256 (k + nblk j)
__global__ __launch_bounds__(256) void vox_sum64_kernel(const float *vox, long long n, float thr, Part64 *parts) {
    const int b = blockIdx.y, nblk = gridDim.x;
    const float *a = vox + (size_t)b * n;
    double s = 0.0, q = 0.0;
    int nz = 0;
    const bool al = (((size_t)a) & 15) == 0;
    const long long n4 = al ? n / 4 : 0;
    for (long long k = (long long)blockIdx.x * 256 + threadIdx.x; k < n4; k += (long long)nblk * 256) {
        const float4 v = reinterpret_cast<const float4 *>(a)[k];
        acc64(v.x, thr, s, q, nz); acc64(v.y, thr, s, q, nz);
        acc64(v.z, thr, s, q, nz); acc64(v.w, thr, s, q, nz);
    }
    for (long long k = 4 * n4 + (long long)blockIdx.x * 256 + threadIdx.x; k < n; k += (long long)nblk * 256)
        acc64(a[k], thr, s, q, nz);
    __shared__ double ss[256], sq[256];
    __shared__ long long sn[256];
    ss[threadIdx.x] = s; sq[threadIdx.x] = q; sn[threadIdx.x] = nz;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) {
            ss[threadIdx.x] += ss[threadIdx.x + k];
            sq[threadIdx.x] += sq[threadIdx.x + k];
            sn[threadIdx.x] += sn[threadIdx.x + k];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) parts[(size_t)b * nblk + blockIdx.x] = Part64{ss[0], sq[0], sn[0]};
}

// grid B, block 256: the window's block partials in a fixed tree, then the float32 statistics
__global__ __launch_bounds__(256) void vox_stats64_kernel(const Part64 *parts, int nblk, WinStats *st) {
    const int b = blockIdx.x;
    double s = 0.0, q = 0.0;
    long long nz = 0;
    for (int k = threadIdx.x; k < nblk; k += 256) {
        const Part64 p = parts[(size_t)b * nblk + k];
        s += p.s; q += p.q; nz += p.nnz;
    }
    __shared__ double ss[256], sq[256];
    __shared__ long long sn[256];
    ss[threadIdx.x] = s; sq[threadIdx.x] = q; sn[threadIdx.x] = nz;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) {
            ss[threadIdx.x] += ss[threadIdx.x + k];
            sq[threadIdx.x] += sq[threadIdx.x + k];
            sn[threadIdx.x] += sn[threadIdx.x + k];
        }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    WinStats w;
    w.nnz = sn[0]; w.mn = 0.0f; w.mx = 0.0f;
    w.mean = 0.0; w.std = 0.0;
    if (w.nnz > 0) {                                     // event_preprocess_pytorch (:168-175)
        const float nf = (float)w.nnz;
        const float mean = (float)ss[0] / nf;                // sum() / num_nonzeros
        const float var = (float)sq[0] / nf - mean * mean;   // (v ** 2).sum() / n - mean ** 2
        w.mean = mean;
        w.std = sqrtf(var);
    }
    st[b] = w;
}

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

struct VoxWs {
    unsigned long long *k0, *k1;
    int *v0, *v1;
    int *tb;                 // per-window tile starts of the sort + tile path
    int *spw;                // per-window flag of the same path: out-of-frame events spill into the grid
    void *tps;               // (t, polarity) of every event in sorted order (same path)
    ChunkPart *parts;
    Part64 *parts64;         // CISTA_VOXEL_STD_F32 block partials
    WinStats *stats;
    void *cub;
    size_t cub_bytes, bytes;
};

int end_bits(unsigned long long maxkey) {
    int bits = 1;
    while (bits < 64 && (maxkey >> bits) != 0) ++bits;
    return bits;
}

VoxWs carve(void *base, int B, long long N, int nb, int H, int W) {
    VoxWs w;
    size_t off = 0;
    char *p = static_cast<char *>(base);
    auto take = [&](size_t bytes) {
        void *r = p ? p + off : nullptr;
        off = align_up(off + bytes);
        return r;
    };
    const long long n = (long long)nb * H * W;
    const int nchunks = (int)((n + CHUNK - 1) / CHUNK);
    const size_t NN = (size_t)(N > 0 ? N : 1);
    w.k0 = static_cast<unsigned long long *>(take(NN * 8));
    w.k1 = static_cast<unsigned long long *>(take(NN * 8));
    w.v0 = static_cast<int *>(take(NN * 4));
    w.v1 = static_cast<int *>(take(NN * 4));
    w.tb = static_cast<int *>(take((size_t)(B > 0 ? B : 1) * (TBMAX + 1) * 4));
    w.tps = take(NN * 16);
    w.spw = static_cast<int *>(take((size_t)(B > 0 ? B : 1) * 4));
    w.parts = static_cast<ChunkPart *>(take((size_t)(B > 0 ? B : 1) * nchunks * sizeof(ChunkPart)));
    w.stats = static_cast<WinStats *>(take((size_t)(B > 0 ? B : 1) * sizeof(WinStats)));
    w.parts64 = static_cast<Part64 *>(take((size_t)(B > 0 ? B : 1) * nblk64(n) * sizeof(Part64)));
    w.cub_bytes = 0;
    if (N > 0) {
        const hipError_t e = hipcub::DeviceRadixSort::SortPairs(
            nullptr, w.cub_bytes, (const unsigned long long *)nullptr, (unsigned long long *)nullptr,
            (const int *)nullptr, (int *)nullptr, (int)NN, 0, 64);
        if (e != hipSuccess) w.cub_bytes = ~(size_t)0 >> 8;   // unusable: forces CISTA_ERR_WORKSPACE
    }
    w.cub = take(w.cub_bytes);
    w.bytes = off;
    return w;
}

inline dim3 g1d(long long n, int bs = 256) { return dim3((unsigned)((n + bs - 1) / bs)); }

// dynamic LDS above 64 KiB is enabled per kernel, once (thread-safe)
bool big_lds(const void *kern) {
    static std::mutex mu;
    static const void *done[4];
    static int ndone = 0;
    std::lock_guard<std::mutex> lock(mu);
    for (int i = 0; i < ndone; ++i)
        if (done[i] == kern) return true;
    if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(WinLds)) != hipSuccess)
        return false;
    if (ndone < 4) done[ndone++] = kern;
    return true;
}

// hot-pixel filter + normalisation of B grids of n floats, in place
int preprocess(float *voxels, int B, long long n, int mode, float thr, const VoxWs &w, hipStream_t st) {
    const int nchunks = (int)((n + CHUNK - 1) / CHUNK);
    if (mode == CISTA_VOXEL_STD_F32) {
        const int nb64 = nblk64(n);
        hipLaunchKernelGGL(vox_sum64_kernel, dim3(nb64, B), dim3(256), 0, st, (const float *)voxels, n, thr,
                           w.parts64);
        hipLaunchKernelGGL(vox_stats64_kernel, dim3(B), dim3(256), 0, st, (const Part64 *)w.parts64, nb64, w.stats);
    } else if (mode != CISTA_VOXEL_RAW) {
        hipLaunchKernelGGL(vox_chunk_kernel, dim3(nchunks, B), dim3(MAX_LEAVES), 0, st, (const float *)voxels, n,
                           nchunks, thr, w.parts);
        hipLaunchKernelGGL(vox_stats_kernel, dim3(B), dim3(256), 0, st, (const ChunkPart *)w.parts, nchunks, mode,
                           w.stats);
    }
    if (mode != CISTA_VOXEL_RAW || thr > 0.0f)
        for (int b0 = 0; b0 < B; b0 += 65535)                 // grid.y <= 65535 windows per launch
            hipLaunchKernelGGL(vox_apply_kernel, dim3((unsigned)((n + 1023) / 1024), min(B - b0, 65535)), dim3(256),
                               0, st, voxels + (size_t)b0 * n, n, mode, thr, (const WinStats *)w.stats + b0);
    return hipGetLastError() == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
}

}  // namespace cista_vox

using namespace cista_vox;

extern "C" {

size_t cista_voxel_workspace_bytes(int B, long long n_events, int num_bins, int height, int width) {
    if (B < 0 || n_events < 0 || num_bins <= 0 || height <= 0 || width <= 0) return 0;
    return carve(nullptr, B, n_events, num_bins, height, width).bytes;
}

int cista_voxelize(const double *events, const long long *offsets, int B, long long n_events, int num_bins,
                   int height, int width, int mode, float hot_threshold, float *voxels, void *workspace,
                   size_t workspace_bytes, void *stream) {
    return cista_voxelize_checked(events, offsets, B, n_events, num_bins, height, width, mode, hot_threshold, voxels,
                                  workspace, workspace_bytes, nullptr, stream);
}

int cista_voxelize_checked(const double *events, const long long *offsets, int B, long long n_events, int num_bins,
                           int height, int width, int mode, float hot_threshold, float *voxels, void *workspace,
                           size_t workspace_bytes, int *grid_status, void *stream) {
    if (B < 0 || n_events < 0 || n_events > 0x7fffffffLL || num_bins <= 0 || height <= 0 || width <= 0)
        return CISTA_ERR_INVALID;
    const int torch_acc = (mode & CISTA_VOXEL_TORCH_ACCUM) != 0;
    mode &= ~CISTA_VOXEL_TORCH_ACCUM;
    if (mode < CISTA_VOXEL_RAW || mode > CISTA_VOXEL_STD_F32) return CISTA_ERR_INVALID;
    if (B == 0) return CISTA_OK;
    if (!offsets || !voxels || !workspace || (n_events > 0 && !events)) return CISTA_ERR_INVALID;
    const VoxWs w = carve(workspace, B, n_events, num_bins, height, width);
    if (workspace_bytes < w.bytes) return CISTA_ERR_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const long long n = (long long)num_bins * height * width;
    const unsigned long long HW = (unsigned long long)height * width;
    const long long tp = num_bins * 4 <= WTILE ? tile_pixels(num_bins) : 0;
    if (HW < (1ull << 18) - 1 && tp > 0 && ((long long)HW + tp - 1) / tp <= TBMAX) {
        // per-window sort + tiled accumulation (no memset, no global sort)
        if (!big_lds(reinterpret_cast<const void *>(vox_sort_kernel))) return CISTA_ERR_HIP;
        const int ntiles = (int)(((long long)HW + tp - 1) / tp);
        unsigned *scr = reinterpret_cast<unsigned *>(w.k0);
        int *tb = reinterpret_cast<int *>(w.tb);
        double2 *tps = reinterpret_cast<double2 *>(w.tps);
        hipLaunchKernelGGL(vox_sort_kernel, dim3(B), dim3(WT), sizeof(WinLds), st, events, offsets, num_bins, height,
                           width, 14 + end_bits(HW), scr, tps, tb, w.spw, torch_acc, grid_status);
        hipLaunchKernelGGL(torch_acc ? vox_tile_kernel<true> : vox_tile_kernel<false>, dim3(ntiles, B), dim3(TT), 0,
                           st, events, offsets, num_bins, height, width, (const unsigned *)scr, (const double2 *)tps,
                           (const int *)tb, (const int *)w.spw, voxels);
        if (hipGetLastError() != hipSuccess) return CISTA_ERR_HIP;
        return preprocess(voxels, B, n, mode, hot_threshold, w, st);
    }
    if (hipMemsetAsync(voxels, 0, (size_t)B * n * sizeof(float), st) != hipSuccess) return CISTA_ERR_HIP;
    if (n_events > 0) {
        hipLaunchKernelGGL(vox_keys_kernel, g1d(n_events), dim3(256), 0, st, events, offsets, B, n_events, height,
                           width, w.k0, w.v0, num_bins, torch_acc, grid_status);
        size_t cb = w.cub_bytes;
        const int bits = end_bits((unsigned long long)B * height * width);
        if (hipcub::DeviceRadixSort::SortPairs(w.cub, cb, (const unsigned long long *)w.k0, w.k1,
                                               (const int *)w.v0, w.v1, (int)n_events, 0, bits, st) != hipSuccess)
            return CISTA_ERR_HIP;
        hipLaunchKernelGGL(vox_accum_kernel, g1d(n_events), dim3(256), 0, st, (const unsigned long long *)w.k1,
                           (const int *)w.v1, n_events, events, offsets, B, num_bins, height, width, voxels,
                           torch_acc);
    }
    return preprocess(voxels, B, n, mode, hot_threshold, w, st);
}

int cista_voxel_preprocess(float *voxels, int B, int num_bins, int height, int width, int mode,
                           float hot_threshold, void *workspace, size_t workspace_bytes, void *stream) {
    if (B < 0 || num_bins <= 0 || height <= 0 || width <= 0) return CISTA_ERR_INVALID;
    if (mode < CISTA_VOXEL_RAW || mode > CISTA_VOXEL_STD_F32) return CISTA_ERR_INVALID;
    if (B == 0) return CISTA_OK;
    if (!voxels || !workspace) return CISTA_ERR_INVALID;
    const VoxWs w = carve(workspace, B, 0, num_bins, height, width);
    if (workspace_bytes < w.bytes) return CISTA_ERR_WORKSPACE;
    return preprocess(voxels, B, (long long)num_bins * height * width, mode, hot_threshold, w,
                      static_cast<hipStream_t>(stream));
}

}  // extern "C"
