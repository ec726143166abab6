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

__global__ void vox_keys_kernel(const double *ev, const long long *off, int B, long long N, int H, int W,
                                unsigned long long *keys, int *vals) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int b = window_of(off, B, i);
    const double x = ev[4 * i + 1], y = ev[4 * i + 2];
    const unsigned long long HW = (unsigned long long)H * W;
    unsigned long long key = (unsigned long long)B * HW;   // sentinel: sorts last, ignored
    // reference :42-43: astype(np.uint) truncates toward zero, so (-1, W) maps into [0, W)
    if (x > -1.0 && x < (double)W && y > -1.0 && y < (double)H)
        key = (unsigned long long)b * HW + (unsigned long long)y * W + (unsigned long long)x;
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
    if (torch_acc) {                    // index_add_ #1 / #2 (:112-127), float32 adds
        for (long long k = j; k < end; ++k) {
            EvValT v;
            if (event_value_torch(ev + 4 * (long long)vals[k], first, dT, nb, v) && v.ti < (unsigned long long)nb)
                out[v.ti * HW] += v.vl;
        }
        for (long long k = j; k < end; ++k) {
            EvValT v;
            if (event_value_torch(ev + 4 * (long long)vals[k], first, dT, nb, v) && v.ti + 1 < (unsigned long long)nb)
                out[(v.ti + 1) * HW] += v.vr;
        }
        return;
    }
    // np.add.at #1 (:53-54): left contributions of the whole window, in event order
    for (long long k = j; k < end; ++k) {
        EvVal v;
        if (!event_value(ev + 4 * (long long)vals[k], first, dT, nb, v)) continue;
        if (v.ti < (unsigned long long)nb) {
            float *d = out + v.ti * HW;
            *d = (float)((double)*d + v.vl);
        }
    }
    // np.add.at #2 (:56-58): right contributions
    for (long long k = j; k < end; ++k) {
        EvVal v;
        if (!event_value(ev + 4 * (long long)vals[k], first, dT, nb, v)) continue;
        if (v.ti + 1 < (unsigned long long)nb) {
            float *d = out + (v.ti + 1) * HW;
            *d = (float)((double)*d + v.vr);
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
    rcnt[tid] = cnt; rmn[tid] = mn; rmx[tid] = mx;
    __syncthreads();
    if (tid < nleaves) leaf_sums_lds(buf, lstart[tid], llen[tid], ls[tid], lq[tid]);
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
__global__ void vox_stats_kernel(const ChunkPart *parts, int nchunks, int B, int mode, WinStats *st) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    float s = 0.0f, q = 0.0f, mn = INFINITY, mx = -INFINITY;
    long long nnz = 0;
    for (int c = 0; c < nchunks; ++c) {
        const ChunkPart p = parts[(size_t)b * nchunks + c];
        s += p.sum;
        q += p.sq;
        nnz += p.nnz;
        mn = fminf(mn, p.mn);
        mx = fmaxf(mx, p.mx);
    }
    WinStats w;
    w.nnz = nnz; w.mn = mn; w.mx = mx;
    w.mean = 0.0; w.std = 0.0;
    if (nnz > 0 && mode == CISTA_VOXEL_STD_F32) {
        // event_preprocess_pytorch (:168-175): float32 scalars throughout.  The sums are taken
        // in float64 over the chunk partials and rounded once (ATen's float32 reduction order is
        // not restated; the difference is the last bit of sum())
        double sd = 0.0, qd = 0.0;
        for (int c = 0; c < nchunks; ++c) {
            sd += (double)parts[(size_t)b * nchunks + c].sum;
            qd += (double)parts[(size_t)b * nchunks + c].sq;
        }
        const float nf = (float)nnz;
        const float mean = (float)sd / nf;                   // sum() / num_nonzeros
        const float var = (float)qd / nf - mean * mean;      // (v ** 2).sum() / n - mean ** 2
        w.mean = mean;
        w.std = sqrtf(var);
    } else if (nnz > 0) {
        const double dn = (double)nnz;
        const double mean = (double)s / dn;                  // :148
        w.mean = mean;
        w.std = sqrt((double)q / dn - mean * mean);          // :150
    }
    st[b] = w;
}

__global__ void vox_apply_kernel(float *vox, long long n, int B, int mode, float thr, const WinStats *st) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * B) return;
    const int b = (int)(i / n);
    const float v = hot(vox[i], thr);                        // :137-138
    float r = v;
    if (mode == CISTA_VOXEL_STD) {
        const WinStats w = st[b];
        if (w.nnz > 0) {                                     // :146
            const double mask = v != 0.0f ? 1.0 : 0.0;
            r = (float)(mask * ((double)v - w.mean) / (w.std + 1e-8));   // :152
        }
    } else if (mode == CISTA_VOXEL_STD_F32) {
        const WinStats w = st[b];
        if (w.nnz > 0) {                                     // :170, float32: mask * (v - mean) / (std + 1e-8)
            const float mask = v != 0.0f ? 1.0f : 0.0f;
            r = mask * (v - (float)w.mean) / ((float)w.std + 1e-8f);
        }
    } else if (mode == CISTA_VOXEL_MAXMIN) {
        const WinStats w = st[b];
        r = (v - w.mn) / (w.mx - w.mn + 1e-8f);              // :140
    }
    vox[i] = r;
}

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

struct VoxWs {
    unsigned long long *k0, *k1;
    int *v0, *v1;
    ChunkPart *parts;
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
    w.parts = static_cast<ChunkPart *>(take((size_t)(B > 0 ? B : 1) * nchunks * sizeof(ChunkPart)));
    w.stats = static_cast<WinStats *>(take((size_t)(B > 0 ? B : 1) * sizeof(WinStats)));
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

// hot-pixel filter + normalisation of B grids of n floats, in place
int preprocess(float *voxels, int B, long long n, int mode, float thr, const VoxWs &w, hipStream_t st) {
    const int nchunks = (int)((n + CHUNK - 1) / CHUNK);
    if (mode != CISTA_VOXEL_RAW) {
        hipLaunchKernelGGL(vox_chunk_kernel, dim3(nchunks, B), dim3(MAX_LEAVES), 0, st, (const float *)voxels, n,
                           nchunks, thr, w.parts);
        hipLaunchKernelGGL(vox_stats_kernel, g1d(B, 64), dim3(64), 0, st, (const ChunkPart *)w.parts, nchunks, B,
                           mode, w.stats);
    }
    if (mode != CISTA_VOXEL_RAW || thr > 0.0f)
        hipLaunchKernelGGL(vox_apply_kernel, g1d(n * B), dim3(256), 0, st, voxels, n, B, mode, thr,
                           (const WinStats *)w.stats);
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
    if (hipMemsetAsync(voxels, 0, (size_t)B * n * sizeof(float), st) != hipSuccess) return CISTA_ERR_HIP;
    if (n_events > 0) {
        hipLaunchKernelGGL(vox_keys_kernel, g1d(n_events), dim3(256), 0, st, events, offsets, B, n_events, height,
                           width, w.k0, w.v0);
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
