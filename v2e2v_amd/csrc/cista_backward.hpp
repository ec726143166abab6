// cista_backward.hpp -- BPTT backward kernels of the CISTA-LSTC frame (SURVEY section 8 row a11;
// reference train_e2v.py:108-130 drives autograd through e2v/e2v_model.py:41-90).
//
//  * dgrad of the MFMA-sized reflect-padded convs reuses conv3x3_split3 with STAGE_ZP2: a
//    correlation of the zero-padded output gradient with the flipped, transposed weights
//    (packed by pack_dgrad_kernel) produces the gradient on the PADDED input domain, which
//    fold_reflect_kernel folds back (padded index -1 -> 1, H -> H-2) and accumulates;
//  * wgrad is a pixel-reduction GEMM on exact fp32 MFMA (v_mfma_f32_16x16x4f32): per pixel tile
//    the output gradient and the reflect-padded input halo are staged in LDS, every wave owns
//    one 16x16 (cout x cin) block for all 9 taps; per-split partial sums are reduced by
//    reduce_partials_kernel (deterministic, no atomics);
//  * the elementwise tails (sigmoid/tanh gate algebra, softshrink, ReLU masks, bilinear x2,
//    the final 64->1 conv) have dedicated fp32 kernels.
#pragma once
#include "cista_kernels.hpp"

namespace cista {

// --------------------------------------------------------------------------------------------
// fold the padded-domain gradient of a reflect-padded (pad 1) conv back onto its input:
// dst[b,y,x,dc0+c] (+)= scale * sum of src[b, Y, X, sc0+c] over padded (Y, X) whose reflected
// index is (y, x).  src is (B, H+2, W+2, Cs); dst (B, H, W, Cd).  Optional ReLU-style mask:
// multiply by (mask[b,y,x,c] > 0) after accumulation (mask NHWC with Cd channels).
// --------------------------------------------------------------------------------------------
struct FoldArgs {
    const float *src; int Cs, sc0;
    float *dst; int Cd, dc0;
    int n;                 // channels folded
    int B, H, W;
    float scale;
    int accumulate;        // 0: dst = fold, 1: dst += fold
    const float *mask;     // optional, applied to the result (NHWC, Cd channels)
    const float *add;      // optional (accumulate == 0): dst = add + fold (add laid out as dst)
    float *dst2;           // optional second destination (laid out as dst): dst2 += fold
    unsigned *amax;        // optional: publish max |dst| (after the mask) to these slots
};

__device__ __forceinline__ int refl_sources(int i, int n, int (&out)[3]) {
    // padded indices P in [0, n+2) with reflect(P - 1) == i, i.e. the padded positions that
    // read input index i: P = i + 1, plus P = 0 when i == 1 and P = n + 1 when i == n - 2
    int k = 0;
    out[k++] = i + 1;
    if (i == 1) out[k++] = 0;
    if (i == n - 2) out[k++] = n + 1;
    return k;
}

// Per-tensor |x| maximum for the power-of-two gradient scales of the split-f16 dgrad / wgrad,
// accumulated by the kernel that PRODUCES the gradient: a workgroup maximum (every thread of the
// 256-thread block calls this, with 0 for no element), then one atomicMax of its bits (non-
// negative floats order as unsigned; fmaxf drops NaN, inf stays inf) into one of 256 slots on
// separate 64-B lines, so no address sees more than ~1/256 of the workgroups.  slots_scale_kernel
// turns the slots into {s, 1/s} and re-zeroes them.  (Replaces a separate absmax pass per
// gradient tensor, 16 us each at B = 8.)
// (AMAX_SLOTS / AMAX_STRIDE / amax4f: cista_kernels.hpp)
__device__ __forceinline__ void amax_publish(unsigned *slots, float m) {
    __shared__ float amax_red[4];
    __syncthreads();                            // a previous call's reads of amax_red are done
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) amax_red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float b = fmaxf(fmaxf(amax_red[0], amax_red[1]), fmaxf(amax_red[2], amax_red[3]));
        if (b > 0.0f) atomicMax(slots + (blockIdx.x & (AMAX_SLOTS - 1)) * AMAX_STRIDE, __float_as_uint(b));
    }
}
// per-tensor power-of-two scale for an fp16-split dgrad / wgrad input: {s, 1/s} -> scl
__device__ __forceinline__ void scale_from_max(float mx, float *scl) {
    int e = 0;
    if (mx > 0.0f && isfinite(mx)) {
        e = (int)floorf(log2f(16384.0f / mx));
        e = e < -60 ? -60 : (e > 60 ? 60 : e);
    }
    scl[0] = ldexpf(1.0f, e);
    scl[1] = ldexpf(1.0f, -e);
}
// The last block of a publishing kernel turns the |max| slots into the scale pair, in place of a
// slots_scale_kernel launch of its own.  The only data that crosses blocks are the slots' atomics,
// which execute at the memory side, so no fence is needed (a release fence here writes back the
// XCD's L2 in every block): each block's thread 0 publishes its maximum with a returning atomic
// and consumes the result (the wave waits until the memory side has performed it), then takes a
// ticket with a relaxed device-scope atomic; the block that takes the last ticket reads and
// re-zeroes the slots with atomic exchanges, writes {s, 1/s} (read by the next launch) and re-arms
// the ticket.  A maximum does not depend on the order of the blocks, so the pair is the one the
// separate launch computes.  Every block of the grid must call it (no early exits).
__device__ __forceinline__ void ticket_scale(const float *red4, unsigned *slots, unsigned *ticket, float *scl) {
    __shared__ int last;
    __shared__ float red[4];
    if (threadIdx.x == 0) {
        const float b = fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3]));
        unsigned old = 0u;
        if (b > 0.0f)
            old = __hip_atomic_fetch_max(slots + (blockIdx.x & (AMAX_SLOTS - 1)) * AMAX_STRIDE, __float_as_uint(b),
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(old) : "memory");   // performed before the ticket below
        last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1 ? 1 : 0;
    }
    __syncthreads();
    if (!last) return;
    float m = 0.0f;
    for (int i = threadIdx.x; i < AMAX_SLOTS; i += blockDim.x)
        m = fmaxf(m, __uint_as_float(__hip_atomic_exchange(slots + i * AMAX_STRIDE, 0u, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT)));
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = red[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) b = fmaxf(b, red[w]);
        scale_from_max(b, scl);
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// amax_publish's block reduction without the atomic (ticket_scale publishes it): red4 <- the
// block's four wave maxima
__device__ __forceinline__ void amax_block(float *red4, float m) {
    __syncthreads();                            // a previous call's reads of red4 are done
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = m;
    __syncthreads();
}

__global__ __launch_bounds__(256) void fold_reflect_kernel(const FoldArgs a) {
    const int g4 = a.n / 4;
    const long total = (long)a.B * a.H * a.W * g4;
    const long idx0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = idx0 < total;
    if (!a.amax && !live) return;               // (a block that publishes keeps every thread)
    const long idx = live ? idx0 : total - 1;   // dead threads recompute the last item, store nothing
    const int c = (int)(idx % g4) * 4;
    const long pix = idx / g4;
    const int x = (int)(pix % a.W);
    const int y = (int)((pix / a.W) % a.H);
    const int b = (int)(pix / ((long)a.W * a.H));
    int ys[3], xs[3];
    const int ny = refl_sources(y, a.H, ys), nx = refl_sources(x, a.W, xs);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = 0; i < ny; ++i)
        for (int j = 0; j < nx; ++j) {
            const float4 v = *(const float4 *)(a.src + (((size_t)b * (a.H + 2) + ys[i]) * (a.W + 2) + xs[j]) * a.Cs + a.sc0 + c);
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    const size_t od = (size_t)pix * a.Cd + a.dc0 + c;
    float4 *d = (float4 *)(a.dst + od);
    const float4 f = make_float4(s.x * a.scale, s.y * a.scale, s.z * a.scale, s.w * a.scale);
    float4 r = f;
    if (a.accumulate || a.add) {
        const float4 o = a.accumulate ? *d : *(const float4 *)(a.add + od);
        r.x = o.x + f.x; r.y = o.y + f.y; r.z = o.z + f.z; r.w = o.w + f.w;
    }
    if (a.dst2 && live) {
        float4 *d2 = (float4 *)(a.dst2 + od);
        const float4 o = *d2;
        *d2 = make_float4(o.x + f.x, o.y + f.y, o.z + f.z, o.w + f.w);
    }
    if (a.mask) {
        const float4 m = *(const float4 *)(a.mask + (size_t)pix * a.Cd + a.dc0 + c);
        r.x = m.x > 0.f ? r.x : 0.f; r.y = m.y > 0.f ? r.y : 0.f;
        r.z = m.z > 0.f ? r.z : 0.f; r.w = m.w > 0.f ? r.w : 0.f;
    }
    if (live) *d = r;
    if (a.amax) amax_publish(a.amax, live ? amax4f(0.0f, r) : 0.0f);
}

// --------------------------------------------------------------------------------------------
// The reflected terms of an EPI_FOLD dgrad (the conv epilogue wrote each input pixel's own term,
// padded pixel (i+1, j+1), with its segment's mode): input rows 1 and n-2 and columns 1 and m-2
// also read the padded border lines (P = 0 / n+1, Q = 0 / m+1; refl_sources), which the epilogue
// left in fb.  Thread = (sample, border input pixel, 4 channels); the modes are linear in the
// folded value, so the terms are added to what the epilogue stored (a masked pixel stays 0).
// Needs n, m >= 4 (rows 1 and n-2 distinct).
// --------------------------------------------------------------------------------------------
struct FoldFixArgs {
    const float *fb;        // (B, 2 (m+2) + 2 n, N)
    int N, B, n, m;
    FoldSeg seg[2];
    int fsplit;
    float *scl;             // non-NULL: the last block turns seg[0].amax into this pair (ticket_scale)
    unsigned *ticket;
};

__global__ __launch_bounds__(256) void fold_fix_kernel(const FoldFixArgs a) {
    const int g4 = a.N / 4, n = a.n, m = a.m;
    const int nb = 2 * m + 2 * (n - 2);                     // border input pixels per sample
    const long total = (long)a.B * nb * g4;
    const long idx0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = idx0 < total;
    const bool pub = a.seg[0].amax || a.seg[1].amax;
    if (!pub && !live) return;                               // (a block that publishes keeps every thread)
    const long idx = live ? idx0 : total - 1;
    const int c = (int)(idx % g4) * 4;
    const long r = idx / g4;
    const int k = (int)(r % nb), b = (int)(r / nb);
    int i, j;
    if (k < 2 * m) {                                         // rows 1 and n-2, every column
        i = k < m ? 1 : n - 2;
        j = k < m ? k : k - m;
    } else {                                                 // columns 1 and m-2 of the other rows
        const int k2 = k - 2 * m, rr = k2 >> 1;              // rows 0, 2 .. n-3, n-1
        i = rr == 0 ? 0 : (rr <= n - 4 ? rr + 1 : n - 1);
        j = (k2 & 1) ? m - 2 : 1;
    }
    int ys[3], xs[3];
    const int ny = refl_sources(i, n, ys), nx = refl_sources(j, m, xs);
    const int L = 2 * (m + 2) + 2 * n;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int u = 0; u < ny; ++u)
        for (int v = 0; v < nx; ++v) {
            if (u == 0 && v == 0) continue;                  // (i+1, j+1): the epilogue's own term
            const float4 t = *(const float4 *)(a.fb + ((size_t)b * L + fold_border_index(ys[u], xs[v], n, m)) * a.N + c);
            s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
        }
    const bool s1 = c >= a.fsplit;
    const FoldSeg &S = s1 ? a.seg[1] : a.seg[0];
    float mx = 0.0f;
    if (live && S.dst) {
        const size_t o = (((size_t)b * n + i) * m + j) * S.Cd + S.dc0 + c - (s1 ? a.fsplit : 0);
        float4 f = make_float4(s.x * S.scale, s.y * S.scale, s.z * S.scale, s.w * S.scale);
        if (S.mode == FOLD_MASK) {
            const float4 mk = *(const float4 *)(S.aux + o);
            f.x = mk.x > 0.f ? f.x : 0.f; f.y = mk.y > 0.f ? f.y : 0.f;
            f.z = mk.z > 0.f ? f.z : 0.f; f.w = mk.w > 0.f ? f.w : 0.f;
        }
        float4 *d = (float4 *)(S.dst + o);
        float4 v = *d;
        v.x += f.x; v.y += f.y; v.z += f.z; v.w += f.w;
        *d = v;
        mx = amax4f(0.0f, v);
        if (S.mode == FOLD_DST2 && S.aux) {
            float4 *d2 = (float4 *)(S.aux + o);
            float4 w = *d2;
            w.x += f.x; w.y += f.y; w.z += f.z; w.w += f.w;
            *d2 = w;
        }
    }
    if (a.scl) {                          // the host passes a pair only with seg[0].amax alone
        __shared__ float red4[4];
        amax_block(red4, s1 ? 0.0f : mx);
        ticket_scale(red4, a.seg[0].amax, a.ticket, a.scl);
        return;
    }
    if (a.seg[0].amax) amax_publish(a.seg[0].amax, s1 ? 0.0f : mx);
    if (a.seg[1].amax) amax_publish(a.seg[1].amax, s1 ? mx : 0.0f);
}

// dgrad weight packing: B fragment of the dgrad conv = W[k=cout][col=cin] at the flipped tap
// (t' = 8 - t), same [kc][tap][ntile][part][lane] layout and per-layer scale as the forward.
__global__ void pack_dgrad_kernel(const PackArgs a) {
    // here a.Cin = forward Cout (the dgrad K), a.Cout = forward Cin (the dgrad N)
    const int NT = a.Cout / 16;
    const int KC = a.Cin / 32;
    const long total = (long)KC * 9 * NT * 64;
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < a.Cout) a.bp[idx] = 0.0f;
    if (idx >= total) return;
    const int lane = (int)(idx % 64);
    long r = idx / 64;
    const int nt = (int)(r % NT);
    r /= NT;
    const int tap = (int)(r % 9);
    const int kc = (int)(r / 9);
    const int ci_fwd = nt * 16 + (lane & 15);        // dgrad output channel = forward input channel
    const float s = a.scale[0];
    f16x8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int co_fwd = kc * 32 + 8 * (lane >> 4) + j;
        // forward weight layout [co][ci][ky][kx], a.Cin (= fwd Cout) rows of a.Cout (= fwd Cin)
        const float v = a.w[((size_t)co_fwd * a.Cout + ci_fwd) * 9 + (8 - tap)] * s;
        const _Float16 hb = (_Float16)v;
        h[j] = hb;
        l[j] = (_Float16)(v - (float)hb);
    }
    const size_t base = ((((size_t)kc * 9 + tap) * NT + nt) * 2) * 64 + lane;
    a.wp[base] = __builtin_bit_cast(u32x4, h);
    a.wp[base + 64] = __builtin_bit_cast(u32x4, l);
}

// W0 (stride 2) dgrad as a four-phase stride-1 conv over G (conv3x3_split3<STAGE_ZP2, EPI_PH4>):
// the padded-domain input gradient at (2i + a, 2j + b) = sum over the forward taps (dy, dx) with
// 2y + dy = 2i + a of G(y, x) W[co][ci][dy][dx]: even rows take dy = 0 from G row i and dy = 2
// from row i - 1, odd rows dy = 1 from row i (columns alike).  As a ZP2 correlation (output i reads
// G rows i - 2 + ty) that is ty = 2 -> dy 0 | 1 and ty = 1 -> dy 2; the other taps are zero and
// the kernel skips them.  B fragment: K = forward cout, column = phase (a*2+b) x forward cin; same
// [kc][tap][ntile][part][lane] layout and per-layer scale as the forward pack (a.Cin = forward
// Cout, a.Cout = 4 x forward Cin).
__device__ __forceinline__ int w0_phase_tap(int parity, int t) {
    return parity ? (t == 2 ? 1 : -1) : (t == 2 ? 0 : (t == 1 ? 2 : -1));
}
__global__ void pack_w0phase_kernel(const PackArgs a) {
    const int Cf = a.Cout / 4;
    const int NT = a.Cout / 16;
    const int KC = a.Cin / 32;
    const long total = (long)KC * 9 * NT * 64;
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < a.Cout) a.bp[idx] = 0.0f;
    if (idx >= total) return;
    const int lane = (int)(idx % 64);
    long r = idx / 64;
    const int nt = (int)(r % NT);
    r /= NT;
    const int tap = (int)(r % 9);
    const int kc = (int)(r / 9);
    const int col = nt * 16 + (lane & 15), ph = col / Cf, ci = col - ph * Cf;
    const int dy = w0_phase_tap(ph >> 1, tap / 3), dx = w0_phase_tap(ph & 1, tap % 3);
    const float s = a.scale[0];
    f16x8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int co = kc * 32 + 8 * (lane >> 4) + j;
        const float v = (dy < 0 || dx < 0) ? 0.0f : a.w[((size_t)co * Cf + ci) * 9 + dy * 3 + dx] * s;
        const _Float16 hb = (_Float16)v;
        h[j] = hb;
        l[j] = (_Float16)(v - (float)hb);
    }
    const size_t base = ((((size_t)kc * 9 + tap) * NT + nt) * 2) * 64 + lane;
    a.wp[base] = __builtin_bit_cast(u32x4, h);
    a.wp[base + 64] = __builtin_bit_cast(u32x4, l);
}

// --------------------------------------------------------------------------------------------
// wgrad: dW[co][ci][t] (+)= sign * sum_P G(P, co) * Xpad(S*P + t, ci) on exact fp32 MFMA.
// --------------------------------------------------------------------------------------------
enum XStage { XS_S1 = 0, XS_S2 = 1, XS_UP = 2, XS_NCHW = 3 };

struct WgradArgs {
    const float *G; int Gc, Goff;       // output gradient NHWC (B, Hout, Wout, Gc); cout j at Goff + j
    const float *X0; int x0c;           // input segment 0 (NHWC, or NCHW planes for XS_NCHW)
    const float *X1; int x1c;           // input segment 1 (may be NULL: zeros)
    int B, Hin, Win, Hout, Wout;        // XS_UP: Hin/Win = half-res source, Hout = 2 Hin
    int TH, TW, tiles_x, tiles_y;
    int Cout, Cin;                      // forward conv shape
    int nsplit;
    float *partial;                     // [nsplit][Cout][Cin][9]
    float *bpartial;                    // optional [nsplit][Cout]: bias grads (pixel sums of G),
                                        // produced by the ci-block-0 workgroups
    int vec4;                           // float4 staging: Gc, Goff, x0c, x1c, Cin % 4 == 0, NHWC
                                        // input, tile <= 16x16 (S1/UP) or 8x8 (S2)
    const float *gscale;                // wgrad_split_kernel: {s, 1/s} power-of-two scale of G
    int off32;                          // G and X element offsets fit 31 bits (wgrad_tr fast path)
};

typedef float f32x4w __attribute__((ext_vector_type(4)));

template <int XS>
__device__ __forceinline__ float wg_load_x(const WgradArgs &a, int b, int iy, int ix, int ci) {
    // one input value of the (virtual) reflect-padded conv input; 0 beyond Cin
    if (ci >= a.Cin) return 0.0f;
    const float *seg = ci < a.x0c ? a.X0 : a.X1;
    const int segC = ci < a.x0c ? a.x0c : a.x1c;
    const int cc = ci < a.x0c ? ci : ci - a.x0c;
    if (!seg) return 0.0f;
    if constexpr (XS == XS_UP) {
        const int Hu = 2 * a.Hin, Wu = 2 * a.Win;
        const int Y = reflect_clamp(iy, Hu), X = reflect_clamp(ix, Wu);
        float sy = fmaxf(((float)Y + 0.5f) * 0.5f - 0.5f, 0.0f);
        float sx = fmaxf(((float)X + 0.5f) * 0.5f - 0.5f, 0.0f);
        const int y0 = (int)sy, x0 = (int)sx;
        const int y1 = y0 + (y0 < a.Hin - 1 ? 1 : 0), x1 = x0 + (x0 < a.Win - 1 ? 1 : 0);
        const float ly1 = sy - (float)y0, ly0 = 1.0f - ly1, lx1 = sx - (float)x0, lx0 = 1.0f - lx1;
        const float *base = seg + (size_t)b * a.Hin * a.Win * segC + cc;
        const float v00 = base[((size_t)y0 * a.Win + x0) * segC], v01 = base[((size_t)y0 * a.Win + x1) * segC];
        const float v10 = base[((size_t)y1 * a.Win + x0) * segC], v11 = base[((size_t)y1 * a.Win + x1) * segC];
        return bilerp(ly0, ly1, lx0, lx1, v00, v01, v10, v11);
    } else if constexpr (XS == XS_NCHW) {
        const int y = reflect_clamp(iy, a.Hin), x = reflect_clamp(ix, a.Win);
        return seg[(((size_t)b * segC + cc) * a.Hin + y) * a.Win + x];
    } else {
        const int y = reflect_clamp(iy, a.Hin), x = reflect_clamp(ix, a.Win);
        return seg[(((size_t)b * a.Hin + y) * a.Win + x) * segC + cc];
    }
}

// four consecutive input channels ci..ci+3 (ci % 4 == 0, segment bounds % 4 == 0; NHWC only)
template <int XS>
__device__ __forceinline__ float4 wg_load_x4(const WgradArgs &a, int b, int iy, int ix, int ci) {
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ci >= a.Cin) return z;
    const bool s0 = ci < a.x0c;
    const float *seg = s0 ? a.X0 : a.X1;
    const int segC = s0 ? a.x0c : a.x1c;
    const int cc = s0 ? ci : ci - a.x0c;
    if (!seg) return z;
    if constexpr (XS == XS_UP) {
        const int Hu = 2 * a.Hin, Wu = 2 * a.Win;
        const int Y = reflect_clamp(iy, Hu), X = reflect_clamp(ix, Wu);
        float sy = fmaxf(((float)Y + 0.5f) * 0.5f - 0.5f, 0.0f);
        float sx = fmaxf(((float)X + 0.5f) * 0.5f - 0.5f, 0.0f);
        const int y0 = (int)sy, x0 = (int)sx;
        const int y1 = y0 + (y0 < a.Hin - 1 ? 1 : 0), x1 = x0 + (x0 < a.Win - 1 ? 1 : 0);
        const float ly1 = sy - (float)y0, ly0 = 1.0f - ly1, lx1 = sx - (float)x0, lx0 = 1.0f - lx1;
        const float *base = seg + (size_t)b * a.Hin * a.Win * segC + cc;
        const float4 v00 = *reinterpret_cast<const float4 *>(base + ((size_t)y0 * a.Win + x0) * segC);
        const float4 v01 = *reinterpret_cast<const float4 *>(base + ((size_t)y0 * a.Win + x1) * segC);
        const float4 v10 = *reinterpret_cast<const float4 *>(base + ((size_t)y1 * a.Win + x0) * segC);
        const float4 v11 = *reinterpret_cast<const float4 *>(base + ((size_t)y1 * a.Win + x1) * segC);
        float4 r;
        r.x = bilerp(ly0, ly1, lx0, lx1, v00.x, v01.x, v10.x, v11.x);
        r.y = bilerp(ly0, ly1, lx0, lx1, v00.y, v01.y, v10.y, v11.y);
        r.z = bilerp(ly0, ly1, lx0, lx1, v00.z, v01.z, v10.z, v11.z);
        r.w = bilerp(ly0, ly1, lx0, lx1, v00.w, v01.w, v10.w, v11.w);
        return r;
    } else {
        if constexpr (XS == XS_NCHW)   // never selected on the host (vec4 = 0); plain loads
            return make_float4(wg_load_x<XS>(a, b, iy, ix, ci), wg_load_x<XS>(a, b, iy, ix, ci + 1),
                               wg_load_x<XS>(a, b, iy, ix, ci + 2), wg_load_x<XS>(a, b, iy, ix, ci + 3));
        const int y = reflect_clamp(iy, a.Hin), x = reflect_clamp(ix, a.Win);
        return *reinterpret_cast<const float4 *>(seg + (((size_t)b * a.Hin + y) * a.Win + x) * segC + cc);
    }
}

// workgroup: 4 waves = 2 (cout 16-blocks) x 2 (cin 16-blocks); blockIdx.x = (co32, ci32) block,
// blockIdx.y = split; the split loops over pixel tiles t = split, split + nsplit, ...
template <int XS>
__global__ __launch_bounds__(256) void wgrad_kernel(const WgradArgs a) {
    extern __shared__ float wsm[];
    constexpr int S = XS == XS_S2 ? 2 : 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nci = (a.Cin + 31) / 32;
    const int co0 = (blockIdx.x / nci) * 32, ci0 = (blockIdx.x % nci) * 32;
    const int wco = (wave >> 1) * 16, wci = (wave & 1) * 16;
    const int TH = a.TH, TW = a.TW;
    const int HWd = (TW - 1) * S + 3, HH = (TH - 1) * S + 3;
    const int HP = HH * HWd;
    const int NPX = TH * TW;
    const int NPX4 = (NPX + 3) & ~3;
    float *Gs = wsm;                       // [NPX4][33]
    float *Xs = wsm + NPX4 * 33;           // [HP][33]
    f32x4w acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = f32x4w{0.f, 0.f, 0.f, 0.f};
    const bool do_bias = a.bpartial && (blockIdx.x % nci) == 0;
    float bsum = 0.0f;                       // thread: channel tid & 31, pixel phase tid >> 5
    const int ntiles = a.B * a.tiles_y * a.tiles_x;
    for (int tile = blockIdx.y; tile < ntiles; tile += a.nsplit) {
        int tt = tile;
        const int tx = tt % a.tiles_x;
        tt /= a.tiles_x;
        const int ty = tt % a.tiles_y;
        const int b = tt / a.tiles_y;
        const int oy0 = ty * TH, ox0 = tx * TW;
        __syncthreads();
        // stage G tile (zero outside the image / beyond Cout) and the input halo: all of a
        // thread's global loads are issued before the first LDS store (latency overlap)
        const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
        if (a.vec4) {
            constexpr int UG = 8, UX = 11;   // 256 px x 8 quads; (17*2+1)^2 or 18^2 halo x 8 quads
            float4 gv[UG], xv[UX];
#pragma unroll
            for (int u = 0; u < UG; ++u) {
                const int i = threadIdx.x + u * 256;
                const int p = i >> 3, c = (i & 7) * 4;
                const int py = p / TW, px = p - py * TW;
                const int oy = oy0 + py, ox = ox0 + px;
                gv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (p < NPX && oy < a.Hout && ox < a.Wout && co0 + c < a.Cout)
                    gv[u] = *reinterpret_cast<const float4 *>(
                        a.G + (((size_t)b * a.Hout + oy) * a.Wout + ox) * a.Gc + a.Goff + co0 + c);
            }
#pragma unroll
            for (int u = 0; u < UX; ++u) {
                const int i = threadIdx.x + u * 256;
                const int hp = i >> 3, c = (i & 7) * 4;
                const int hy = hp / HWd, hx = hp - hy * HWd;
                xv[u] = hp < HP ? wg_load_x4<XS>(a, b, iy0 + hy, ix0 + hx, ci0 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < UG; ++u) {
                const int i = threadIdx.x + u * 256;
                const int p = i >> 3, c = (i & 7) * 4;
                if (p < NPX4) {
                    float *d = Gs + p * 33 + c;
                    d[0] = gv[u].x; d[1] = gv[u].y; d[2] = gv[u].z; d[3] = gv[u].w;
                }
            }
#pragma unroll
            for (int u = 0; u < UX; ++u) {
                const int i = threadIdx.x + u * 256;
                const int hp = i >> 3, c = (i & 7) * 4;
                if (hp < HP) {
                    float *d = Xs + hp * 33 + c;
                    d[0] = xv[u].x; d[1] = xv[u].y; d[2] = xv[u].z; d[3] = xv[u].w;
                }
            }
        } else {
            for (int i0 = threadIdx.x; i0 < NPX4 * 32; i0 += 256 * 8) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int i = i0 + u * 256;
                    const int p = i >> 5, c = i & 31;
                    const int py = p / TW, px = p - py * TW;
                    const int oy = oy0 + py, ox = ox0 + px;
                    v[u] = 0.0f;
                    if (p < NPX && oy < a.Hout && ox < a.Wout && co0 + c < a.Cout)
                        v[u] = a.G[(((size_t)b * a.Hout + oy) * a.Wout + ox) * a.Gc + a.Goff + co0 + c];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int i = i0 + u * 256;
                    if (i < NPX4 * 32) Gs[(i >> 5) * 33 + (i & 31)] = v[u];
                }
            }
            for (int i0 = threadIdx.x; i0 < HP * 32; i0 += 256 * 8) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int i = i0 + u * 256;
                    const int hp = i >> 5, c = i & 31;
                    const int hy = hp / HWd, hx = hp - hy * HWd;
                    v[u] = i < HP * 32 ? wg_load_x<XS>(a, b, iy0 + hy, ix0 + hx, ci0 + c) : 0.0f;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int i = i0 + u * 256;
                    if (i < HP * 32) Xs[(i >> 5) * 33 + (i & 31)] = v[u];
                }
            }
        }
        __syncthreads();
        if (do_bias)
            for (int p = threadIdx.x >> 5; p < NPX4; p += 8) bsum += Gs[p * 33 + (threadIdx.x & 31)];
        for (int p4 = 0; p4 < NPX4; p4 += 4) {
            const int p = p4 + (lane >> 4);
            const float av = Gs[p * 33 + wco + (lane & 15)];
            const int pp = p < NPX ? p : NPX - 1;
            const int py = pp / TW, px = pp - py * TW;
            const int hb = (py * S) * HWd + px * S;
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const float bv = Xs[(hb + (t / 3) * HWd + (t % 3)) * 33 + wci + (lane & 15)];
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[t], 0, 0, 0);
            }
        }
    }
    if (do_bias) {
        __syncthreads();
        Gs[threadIdx.x] = bsum;
        __syncthreads();
        if (threadIdx.x < 32) {
            float t = 0.0f;
            for (int k = 0; k < 8; ++k) t += Gs[k * 32 + threadIdx.x];
            if (co0 + (int)threadIdx.x < a.Cout)
                a.bpartial[(size_t)blockIdx.y * a.Cout + co0 + threadIdx.x] = t;
        }
    }
    // acc[t][j]: row (cout) 4*(lane>>4) + j, col (cin) lane & 15
    float *part = a.partial + (size_t)blockIdx.y * a.Cout * a.Cin * 9;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int co = co0 + wco + 4 * (lane >> 4) + j;
        const int ci = ci0 + wci + (lane & 15);
        if (co < a.Cout && ci < a.Cin)
#pragma unroll
            for (int t = 0; t < 9; ++t) part[((size_t)co * a.Cin + ci) * 9 + t] = acc[t][j];
    }
}

// --------------------------------------------------------------------------------------------
// wgrad on split-f16 MFMA (v_mfma_f32_16x16x32_f16, 3 passes hi*hi + hi*lo + lo*hi, fp32
// accumulate) for the stride-1 NHWC convs (XS_S1, 64-aligned Cout, 32-aligned Cin):
//   dW[co][ci][t] = sum_P G(P, co) * Xpad(P + t, ci)  =  per tap a (co x ci) GEMM, K = pixels.
// Workgroup = 64 co x 32 ci block; 4 waves = 2 (32 co) x 2 (16 ci), 2 x 9 accumulators each.
// Pixel tile 6 x 16 = 96 = 3 K-steps of 32; a lane's 8 K values are 8 consecutive pixels of
// one row.  LDS (fp16, hi and lo planes):
//   Gs[part][co][GST]           output gradient, pre-scaled by the per-tensor power of two
//                               gscale[0] so its fp16 split keeps fp32 accuracy;
//   Xs[part][dx][ci][XST]       the reflect-padded input halo (8 rows x 18 cols) as three
//                               column-shifted 8 x 16 copies (dx = 0, 1, 2), so that every
//                               tap's B fragment is one aligned ds_read_b128.
// Row strides GST = 104 and XST = 136 halves (odd in 16-byte units) with the pair swizzle of
// ws_swz put the 16 lanes of each ds_read_b128 lane group on 16 distinct 16-byte bank groups.  The staging stores
// (ds_write_b128: 8-lane groups, 32 banks) are conflict-free by the item order: G item
// i = 12 cq + pg (pixel group pg fastest) -- 8 consecutive items write 128 contiguous bytes of
// one co row, or the tail of one row and the head of the row 4 below it, which is 832 B = 64
// mod 128 further on; X item = (column half xcg fastest, halo row xr, channel quad xq), so the
// 8 lanes of a group write one plane's 128 contiguous bytes.  G is staged by threads 0..191, X
// by threads 128..255 (float4 loads).  (Channel-pair X items on all 256 threads, float2 loads,
// were tried: twice the load instructions and their address math cost more than the balance.)
// Range: X is a forward activation with no per-tensor scale.  Every tile's X maximum is reduced
// across the workgroup (on the barrier that is there anyway); once it reaches 16384 the
// workgroup switches to a power-of-two pre-scale sx of X (the accumulators, in units of sx,
// are rescaled exactly) -- gradients stay fp32-faithful for activations beyond the fp16 range.
// Per-split partials as wgrad_kernel (same reduce).
// --------------------------------------------------------------------------------------------
constexpr int WS_TH = 6, WS_TW = 16, WS_NPX = 96, WS_HH = 8, WS_HW = 18;
constexpr int WS_GST = WS_NPX + 8;                  // halves per co row
constexpr int WS_XST = WS_HH * WS_TW + 8;           // halves per (dx, ci) plane
constexpr size_t WS_LDS = (size_t)2 * 64 * WS_GST * 2 + (size_t)2 * 3 * 32 * WS_XST * 2 + 16;   // + X maxima

__device__ __forceinline__ void split_pack8(const float (&v)[8], u32x4 &hi, u32x4 &lo) {
    f16x8 h, l;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const _Float16 hb = (_Float16)v[i];
        h[i] = hb;
        l[i] = (_Float16)(v[i] - (float)hb);
    }
    hi = __builtin_bit_cast(u32x4, h);
    lo = __builtin_bit_cast(u32x4, l);
}

// fragment-read swizzle: rows (co) / planes (ci) r with bit 2 != bit 3 keep their 8-pixel groups
// pairwise swapped (group j stored in slot j ^ 1), so the lane groups of ds_read_b128 ({0-3,12-15,
// 20-27}, ...: rows r = 0-3,12-15 at K slot kg beside rows 4-11 at kg + 1) hit 16 distinct bank
// groups for any odd row stride (16-byte units) -- without it every read was 2-way (8 cycles, not 4)
__device__ __forceinline__ int ws_swz(int r) { return ((r >> 2) ^ (r >> 3)) & 1; }

__global__ __launch_bounds__(256, 2) void wgrad_split_kernel(const WgradArgs a) {
    extern __shared__ u32x4 wsm4[];
    _Float16 *Gs = reinterpret_cast<_Float16 *>(wsm4);           // [2][64][GST]
    _Float16 *Xs = Gs + 2 * 64 * WS_GST;                          // [2][3][32][XST]
    float *xmx = reinterpret_cast<float *>(Xs + 2 * 3 * 32 * WS_XST);   // [4] per-wave X maxima
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nci = a.Cin / 32;
    const int co0 = (blockIdx.x / nci) * 64, ci0 = (blockIdx.x % nci) * 32;
    const int wco = (wave >> 1) * 32, wci = (wave & 1) * 16;
    const float gsc = a.gscale[0];
    f32x4 acc[2][9];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool do_bias = a.bpartial && (blockIdx.x % nci) == 0;
    float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);
    const int ntiles = a.B * a.tiles_y * a.tiles_x;
    // staging items: G (tid < 192): co quad cq, pixel group pg (8 px), i = 12 cq + pg;
    //                X (tid >= 128): x = tid - 128, column half xcg = x & 1 (halo columns
    //                8 xcg .. 8 xcg + 9), halo row xr = (x >> 1) & 7, channel quad xq = x >> 4
    const int cq = tid / 12, pg = tid - cq * 12;
    const bool xt = tid >= 128;
    const int xi = tid & 127, xcg = xi & 1, xr = (xi >> 1) & 7, xq = xi >> 4;
    // the global loads of BOTH operands of the next pixel tile are issued right after this
    // tile's LDS image is written, so they land under its MFMAs (register double buffer);
    // the split + LDS stores of a tile wait only for loads issued a whole tile earlier
    float4 gv[8], xv[10];
    auto load_tile = [&](int tile) {
        int tt = tile;
        const int tx = tt % a.tiles_x;
        tt /= a.tiles_x;
        const int ty = tt % a.tiles_y;
        const int b = tt / a.tiles_y;
        const int oy0 = ty * WS_TH, ox0 = tx * WS_TW;
        if (tid < 192) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int p = pg * 8 + j;
                const int oy = oy0 + (p >> 4), ox = ox0 + (p & 15);
                gv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (oy < a.Hout && ox < a.Wout)
                    gv[j] = *reinterpret_cast<const float4 *>(
                        a.G + (((size_t)b * a.Hout + oy) * a.Wout + ox) * a.Gc + a.Goff + co0 + 4 * cq);
            }
        }
        if (xt) {
#pragma unroll
            for (int j = 0; j < 10; ++j)
                xv[j] = wg_load_x4<XS_S1>(a, b, oy0 - 1 + xr, ox0 - 1 + 8 * xcg + j, ci0 + 4 * xq);
        }
    };
    float sx = 1.0f;                            // X pre-scale in force (power of two, <= 1)
    if ((int)blockIdx.y < ntiles) load_tile(blockIdx.y);
    for (int tile = blockIdx.y; tile < ntiles; tile += a.nsplit) {
        {   // this tile's X maximum, reduced on the barrier that retires the previous tile's reads
            float m = 0.0f;
            if (xt)
#pragma unroll
                for (int j = 0; j < 10; ++j)
                    m = fmaxf(m, fmaxf(fmaxf(fabsf(xv[j].x), fabsf(xv[j].y)), fmaxf(fabsf(xv[j].z), fabsf(xv[j].w))));
            for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
            if (lane == 0) xmx[wave] = m;
        }
        __syncthreads();                       // the previous tile's fragment reads are done
        {
            const float m = fmaxf(fmaxf(xmx[0], xmx[1]), fmaxf(xmx[2], xmx[3]));
            if (__builtin_expect(m >= 16384.0f && m < 3.0e38f, 0)) {
                int e = (int)floorf(log2f(16384.0f / m));
                e = e < -126 ? -126 : e;
                const float st = ldexpf(1.0f, e);
                if (st < sx) {                 // rescale what is accumulated (exact)
                    const float r = st / sx;
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int t = 0; t < 9; ++t) acc[u][t] *= r;
                    sx = st;
                }
            }
        }
        if (tid < 192) {
            if (do_bias) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    bsum.x += gv[j].x; bsum.y += gv[j].y; bsum.z += gv[j].z; bsum.w += gv[j].w;
                }
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (&gv[j].x)[c] * gsc;    // exact: power of two
                u32x4 hi, lo;
                split_pack8(v, hi, lo);
                const int row = 4 * cq + c, slot = (pg ^ ws_swz(row)) * 8;
                *reinterpret_cast<u32x4 *>(Gs + row * WS_GST + slot) = hi;
                *reinterpret_cast<u32x4 *>(Gs + (64 + row) * WS_GST + slot) = lo;
            }
        }
        if (xt)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float hs[10], ls[10];
#pragma unroll
            for (int j = 0; j < 10; ++j) {
                float x = (&xv[j].x)[c];
                if (__builtin_expect(sx != 1.0f, 0)) x *= sx;             // exact: power of two
                const _Float16 hb = (_Float16)x;
                hs[j] = (float)hb;
                ls[j] = x - hs[j];
            }
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                f16x8 h, l;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    h[j] = (_Float16)hs[j + dx];
                    l[j] = (_Float16)ls[j + dx];
                }
                const int plane = dx * 32 + 4 * xq + c;
                _Float16 *d = Xs + plane * WS_XST + xr * WS_TW + 8 * (xcg ^ ws_swz(4 * xq + c));
                *reinterpret_cast<u32x4 *>(d) = __builtin_bit_cast(u32x4, h);
                *reinterpret_cast<u32x4 *>(d + 3 * 32 * WS_XST) = __builtin_bit_cast(u32x4, l);
            }
        }
        __syncthreads();
        if (tile + a.nsplit < ntiles) load_tile(tile + a.nsplit);
        const int kg = lane >> 4, r16 = lane & 15, ks = kg ^ ws_swz(r16);
#pragma unroll
        for (int s = 0; s < WS_NPX / 32; ++s) {
            const int p0 = 32 * s + 8 * ks;                         // stored slot of pixel group 4 s + kg
            const int py = 2 * s + (kg >> 1), px0 = 8 * (ks & 1);
            u32x4 ah[2], al[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int row = wco + 16 * u + r16;
                ah[u] = *reinterpret_cast<const u32x4 *>(Gs + row * WS_GST + p0);
                al[u] = *reinterpret_cast<const u32x4 *>(Gs + (64 + row) * WS_GST + p0);
            }
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int dy = t / 3, dx = t % 3;
                const _Float16 *src = Xs + (dx * 32 + wci + r16) * WS_XST + (py + dy) * WS_TW + px0;
                const f16x8 bh = __builtin_bit_cast(f16x8, *reinterpret_cast<const u32x4 *>(src));
                const f16x8 bl = __builtin_bit_cast(f16x8, *reinterpret_cast<const u32x4 *>(src + 3 * 32 * WS_XST));
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const f16x8 xh = __builtin_bit_cast(f16x8, ah[u]);
                    const f16x8 xl = __builtin_bit_cast(f16x8, al[u]);
                    acc[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, bh, acc[u][t], 0, 0, 0);
                    acc[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, bl, acc[u][t], 0, 0, 0);
                    acc[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xl, bh, acc[u][t], 0, 0, 0);
                }
            }
        }
    }
    if (do_bias) {
        // per-thread partial sums of 4 co over its pixel groups -> co sums in a fixed order
        __syncthreads();
        float4 *red = reinterpret_cast<float4 *>(wsm4);
        if (tid < 192) red[tid] = bsum;
        __syncthreads();
        if (tid < 64) {                        // co = tid: quad cq = tid / 4, its 12 pixel groups
            float t = 0.0f;
            for (int k = 0; k < 12; ++k) t += (&red[(tid >> 2) * 12 + k].x)[tid & 3];
            a.bpartial[(size_t)blockIdx.y * a.Cout + co0 + tid] = t;
        }
    }
    // acc[u][t][j]: row (cout) wco + 16u + 4*(lane>>4) + j, col (cin) wci + (lane & 15)
    const float inv = a.gscale[1] * (1.0f / sx);
    float *part = a.partial + (size_t)blockIdx.y * a.Cout * a.Cin * 9;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = co0 + wco + 16 * u + 4 * (lane >> 4) + j;
            const int ci = ci0 + wci + (lane & 15);
#pragma unroll
            for (int t = 0; t < 9; ++t) part[((size_t)co * a.Cin + ci) * 9 + t] = acc[u][t][j] * inv;
        }
}

// --------------------------------------------------------------------------------------------
// wgrad on split-f16 MFMA with transposed LDS reads (the default for the stride-1 NHWC convs with
// 64-aligned Cout): dW[co][ci][t] = sum_P G(P, co) * Xpad(P + t, ci), per tap a (co x ci) GEMM
// with K = pixels.  Workgroup = 64 co x 64 ci, 8 waves = 2 (32 co) x 4 (16 ci), 2 x 9
// accumulators each; one workgroup per CU (two LDS buffers).
//  * Both operands keep the natural channel-contiguous layout in LDS, as fp16 hi / lo planes of
//    16 channels: plane[pixel][16 halves], 32 B per pixel.  The K (pixel) values of an MFMA
//    fragment are gathered with gfx950's ds_read_b64_tr_b16 (lane 4q+p of a 16-lane group
//    addresses pixel q, channels 4p..4p+3; lane i receives channel i of the 4 pixels), so a tap's
//    shift is just another pixel address: the input halo is stored ONCE, not as the three
//    column-shifted copies of wgrad_split_kernel (a third of its conversions and LDS stores).
//  * K order of a 32-pixel K-step (tile rows 2s, 2s+1): lane group kg, read r covers pixels
//    4kg..4kg+3 of row 2s+r, so a 32-lane half reads 8 consecutive pixels = 256 contiguous bytes
//    of one plane (all 64 banks, conflict-free) for every tap shift.
//  * Staging item (pixel, 4 channels): lanes 16k..16k+15 hold 4 pixels x 4 quads of plane k, so
//    one pixel's 64 channels are one 256-B load run, and each ds_write_b64 lane group stores 128
//    contiguous bytes (conflict-free).  The next tile's loads are issued before this tile's MFMAs
//    and stored to the other buffer after them: one barrier per 96-pixel tile.
//  * G is pre-scaled by the per-tensor power of two gscale[0] (exact).  X carries no per-tensor
//    scale: every tile's X maximum rides on the tile's barrier; a tile whose |X| would overflow
//    the fp16 hi part (>= 32768 after the scale in force) is re-staged with a smaller power-of-two
//    pre-scale sx and the accumulators are rescaled exactly (rare path, uniform per workgroup).
// --------------------------------------------------------------------------------------------
// Tile geometry per input stage.  Stride 1: 6 x 16 output pixels (3 K-steps), reflect-padded
// 8 x 18 input halo.  Stride 2 (W0): 2 x 16 output pixels (1 K-step) over a 5 x 33 input halo
// whose columns are stored parity-split (the 17 even columns, then the 16 odd ones), so the
// input columns 2x + dx - 1 of four consecutive output pixels are four consecutive LDS pixels.
// 4 MFMA waves (32 co x 32 ci each) + 4 staging waves (8 MFMA waves and two-step-ahead fragment
// reads measured slower; commit c9c3ef1 has both)
constexpr int WT_NMW = 4, WT_THREADS = (WT_NMW + 4) * 64;
#ifndef CISTA_WT_PRIO
#define CISTA_WT_PRIO 1   // staging waves at s_setprio CISTA_WT_PRIO (1: training 1727-1743 -> 1744-1745 frames/s same-box)
#endif
template <int XS> struct WtGeo {
    static constexpr int S = XS == XS_S2 ? 2 : 1;
    static constexpr int TH = S == 2 ? 2 : 6;           // output rows per tile (x 16 columns)
    static constexpr int NPX = TH * 16;                 // output pixels per tile
    static constexpr int KS = NPX / 32;                 // 32-pixel K-steps per tile
    static constexpr int HR = (TH - 1) * S + 3;         // halo rows
    static constexpr int HW = 15 * S + 3;               // halo columns (= LDS row pitch in pixels)
    static constexpr int HP = HR * HW;                  // halo pixels
    static constexpr int UG = NPX / 16, UX = (HP + 15) / 16;   // staging items per loader lane
    static constexpr int GPL = NPX * 16;                // halves per G plane (part, 16-co block)
    static constexpr int XPL = HP * 16;                 // halves per X plane (part, 16-ci block)
    static constexpr int BUF = 8 * GPL + 8 * XPL;       // halves per buffer: G planes [2][4], X [2][4]
    static constexpr size_t LDS = (size_t)2 * BUF * 2 + 16 * 4;   // + maxima, flags, scale
    // LDS pixel of halo pixel (hy, hx)
    static __device__ __forceinline__ int xpos(int hy, int hx) {
        return hy * HW + (S == 1 ? hx : (hx & 1) * 17 + (hx >> 1));
    }
    // LDS pixel read by K row r (0, 1) of K-step s, tap (dy, dx), column offset c (0..15)
    static __device__ __forceinline__ int kpos(int s, int r, int dy, int dx, int c) {
        return S == 1 ? (2 * s + r + dy) * HW + c + dx : (4 * s + 2 * r + dy) * HW + (dx & 1) * 17 + (dx >> 1) + c;
    }
};
static_assert(WtGeo<XS_S1>::HP == 144 && WtGeo<XS_S2>::HP == 165, "wgrad_tr halo geometry");

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// transposed read of 4 pixels x 16 channels of one plane (see above); off in halves, 8-B aligned
__device__ __forceinline__ s16x4 tr_read(const _Float16 *sm, int off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4 *)((__attribute__((address_space(3))) _Float16 *)sm + off));
}

__device__ __forceinline__ f16x8 cat_frag(const s16x4 &x0, const s16x4 &x1) {
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(f16x8, v);
}

// 4 fp32 -> fp16 hi and lo (x ~= hi + lo), packed as 2 dwords each
__device__ __forceinline__ void split4(const float4 &v, uint2 &hi, uint2 &lo) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const f2 v01 = {v.x, v.y}, v23 = {v.z, v.w};
    const h2 h01 = __builtin_convertvector(v01, h2), h23 = __builtin_convertvector(v23, h2);
    const f2 r01 = v01 - __builtin_convertvector(h01, f2), r23 = v23 - __builtin_convertvector(h23, f2);
    hi = make_uint2(__builtin_bit_cast(unsigned, h01), __builtin_bit_cast(unsigned, h23));
    lo = make_uint2(__builtin_bit_cast(unsigned, __builtin_convertvector(r01, h2)),
                    __builtin_bit_cast(unsigned, __builtin_convertvector(r23, h2)));
}

// Diagnostic build only (CISTA_STAMPS=1, scripts/wgrad_stamps.py): lane 0 of wave 0 (MFMA) and
// wave 4 (staging) records shader-clock timestamps into g_cista_wstamps[workgroup * 512 + role * 256
// + slot].  MFMA wave: 0 start, 1 past the first barrier, 2 + 2 it MFMAs of tile it done, 3 + 2 it
// past its barrier (it < 120), 250 MFMA loop done, 251 partials stored, 252 / 253 constant-rate
// clock at start / end.  Staging wave: 0 start, 1 first tile committed, 2 past the first barrier,
// 3 + 3 it next tile committed, 4 + 3 it its successor's loads issued, 5 + 3 it past the barrier.
#if CISTA_STAMPS
__device__ unsigned long long *g_cista_wstamps;
#define WT_STAMP(slot, v)                                                                           \
    do {                                                                                            \
        unsigned long long *_p = g_cista_wstamps;                                                   \
        if (_p && lane == 0 && (wave == 0 || wave == WT_NMW) && (slot) < 256)                       \
            _p[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 512 + (wave >= WT_NMW) * 256 + (slot)] = (v); \
    } while (0)
#else
#define WT_STAMP(slot, v) do { } while (0)
#endif

// (channel block, split) of this workgroup.  Workgroups are dispatched to the 8 XCDs round-robin
// by linear id, so in blockIdx order the channel blocks of one split -- which stage the same X
// tiles at the same time -- sit on different XCDs and each fetches X from HBM.  Renumbering the
// workgroups so that every XCD holds a contiguous run of (split, block) puts them, and the
// neighbouring splits whose halos overlap, behind one L2 (stacked ISTA P wgrad: 551 -> 428 MB per
// launch, time unchanged; the blockIdx-order arm is in commit 8ce774e).  Each split computes the
// same tiles either way (results unchanged).
__device__ __forceinline__ void wt_block_split(int &blk, int &split) {
    const int n = gridDim.x * gridDim.y, l = blockIdx.y * gridDim.x + blockIdx.x;
    const int xcd = l & 7, per = n >> 3, rem = n & 7;
    const int q = xcd * per + (xcd < rem ? xcd : rem) + (l >> 3);
    blk = q % gridDim.x;
    split = q / gridDim.x;
}

template <int XS>
__global__ __launch_bounds__(WT_THREADS, 1) void wgrad_tr_kernel(const WgradArgs a) {
    using GE = WtGeo<XS>;
    constexpr int WT_GPL = GE::GPL, WT_XPL = GE::XPL, WT_BUF = GE::BUF;
    extern __shared__ u32x4 wsm4[];
    _Float16 *sm = reinterpret_cast<_Float16 *>(wsm4);
    float *xmx = reinterpret_cast<float *>(sm + 2 * WT_BUF);     // [4] loader X maxima (rare path)
    int *xfl = reinterpret_cast<int *>(xmx + 4);                 // [2][4] per-buffer overflow flags
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ncb = (a.Cin + 63) / 64;
    int blk, split;
    wt_block_split(blk, split);
    const int co0 = (blk / ncb) * 64, ci0 = (blk % ncb) * 64;
    const bool loader = wave >= WT_NMW;        // waves 0 .. NMW-1: MFMAs; the last 4: staging
    const int ntiles = a.B * a.tiles_y * a.tiles_x;
    const float gsc = a.gscale[0];
    // X pre-scale, per tile: 1, or for a tile whose |X| would overflow the fp16 hi part a power of
    // two <= 1 from that tile's own maximum (so one outlier tile does not push the O(1) values of
    // every later tile towards the fp16 subnormals).  sx: the re-staged tile's scale (loaders) /
    // the scale the accumulators are in (MFMA waves)
    float sx = 1.0f;

    // ---- staging (loader waves): item (pixel 4 set + sp, channel quad sq of plane sb) ----
    const int lw = wave - WT_NMW;
    const int sb = lane >> 4, sp = (lane >> 2) & 3, sq = lane & 3;
    const bool do_bias = a.bpartial && (blk % ncb) == 0;
    float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 gv[GE::UG], xv[GE::UX];
    auto tile_origin = [&](int tile, int &b, int &oy0, int &ox0) __attribute__((always_inline)) {
        int tt = tile;
        const int tx = tt % a.tiles_x;
        tt /= a.tiles_x;
        const int ty = tt % a.tiles_y;
        b = tt / a.tiles_y;
        oy0 = ty * GE::TH;
        ox0 = tx * 16;
    };
    // the lane's X channel quad: segment, its channel count and offset (the host launches this
    // kernel only when every G and X element offset fits 31 bits: 32-bit index math throughout)
    const int cix = ci0 + 16 * sb + 4 * sq;
    const bool xs0 = cix < a.x0c;
    const float *xseg = xs0 ? a.X0 : a.X1;
    const int xsegC = xs0 ? a.x0c : a.x1c, xcc = xs0 ? cix : cix - a.x0c;
    const bool xlane = cix < a.Cin && xseg != nullptr;
    auto load_x = [&](int b, int oy0, int ox0, int u) __attribute__((always_inline)) {
        const int hp = 4 * (lw + 4 * u) + sp;                            // 0..HP-1 (+ masked)
        const int hy = hp / GE::HW, hx = hp - hy * GE::HW;
        if (GE::HP % 16 && hp >= GE::HP) return make_float4(0.f, 0.f, 0.f, 0.f);
        const int y = reflect_clamp(GE::S * oy0 - 1 + hy, a.Hin), x = reflect_clamp(GE::S * ox0 - 1 + hx, a.Win);
        return xlane ? *reinterpret_cast<const float4 *>(xseg + (unsigned)(((b * a.Hin + y) * a.Win + x) * xsegC + xcc))
                     : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    auto load_g = [&](int b, int oy0, int ox0, int u) __attribute__((always_inline)) {
        const int p = 4 * (lw + 4 * u) + sp;                             // 0..NPX-1
        const int oy = oy0 + (p >> 4), ox = ox0 + (p & 15);
        return (oy < a.Hout && ox < a.Wout)
                   ? *reinterpret_cast<const float4 *>(a.G + (unsigned)(((b * a.Hout + oy) * a.Wout + ox) * a.Gc + a.Goff +
                                                                        co0 + 16 * sb + 4 * sq))
                   : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    auto load_tile = [&](int tile) __attribute__((always_inline)) {
        int b, oy0, ox0;
        tile_origin(tile, b, oy0, ox0);
#pragma unroll
        for (int u = 0; u < GE::UG; ++u) gv[u] = load_g(b, oy0, ox0, u);
#pragma unroll
        for (int u = 0; u < GE::UX; ++u) xv[u] = load_x(b, oy0, ox0, u);
    };
    auto put_x = [&](_Float16 *Xp, int u, float4 v, float scale) __attribute__((always_inline)) {
        const int hp = 4 * (lw + 4 * u) + sp;
        if (GE::HP % 16 && hp >= GE::HP) return;
        const int hy = hp / GE::HW, pos = GE::xpos(hy, hp - hy * GE::HW);
        if (__builtin_expect(scale != 1.0f, 0)) { v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale; }
        uint2 hi, lo;
        split4(v, hi, lo);
        *reinterpret_cast<uint2 *>(Xp + sb * WT_XPL + pos * 16 + 4 * sq) = hi;
        *reinterpret_cast<uint2 *>(Xp + (4 + sb) * WT_XPL + pos * 16 + 4 * sq) = lo;
    };
    // registers -> LDS buffer (hi / lo planes); publishes whether this wave's X overflowed
    auto commit = [&](_Float16 *buf, int *flag) __attribute__((always_inline)) {
        _Float16 *Gp = buf, *Xp = buf + 8 * WT_GPL;
#pragma unroll
        for (int u = 0; u < GE::UG; ++u) {
            const int p = 4 * (lw + 4 * u) + sp;
            if (do_bias) { bsum.x += gv[u].x; bsum.y += gv[u].y; bsum.z += gv[u].z; bsum.w += gv[u].w; }
            const float4 v = make_float4(gv[u].x * gsc, gv[u].y * gsc, gv[u].z * gsc, gv[u].w * gsc);
            uint2 hi, lo;
            split4(v, hi, lo);
            *reinterpret_cast<uint2 *>(Gp + sb * WT_GPL + p * 16 + 4 * sq) = hi;
            *reinterpret_cast<uint2 *>(Gp + (4 + sb) * WT_GPL + p * 16 + 4 * sq) = lo;
        }
        float m = 0.0f;
#pragma unroll
        for (int u = 0; u < GE::UX; ++u) {
            m = fmaxf(m, fmaxf(fmaxf(fabsf(xv[u].x), fabsf(xv[u].y)), fmaxf(fabsf(xv[u].z), fabsf(xv[u].w))));
            put_x(Xp, u, xv[u], 1.0f);
        }
        const bool ovf = m >= 32768.0f && m < 3.0e38f;                    // hi part would overflow
        const bool any = __ballot(ovf ? 1 : 0) != 0;
        if (lane == 0) flag[lw] = any ? 1 : 0;
    };
    // rare path (uniform: every wave read the same flags): the tile in buf is re-staged with a
    // pre-scale from its own maximum, the MFMA waves rescale their accumulators exactly (and back
    // at the next unflagged tile).  The loaders re-read the tile's X one item at a time (their
    // registers hold the next tile's loads in flight).  Both roles pass the same three barriers
    // and derive the same scale from the same maxima.
    auto tile_scale = [&]() __attribute__((always_inline)) {
        const float m = fmaxf(fmaxf(xmx[0], xmx[1]), fmaxf(xmx[2], xmx[3]));
        int e = (int)floorf(log2f(16384.0f / m));
        e = e < -126 ? -126 : (e > 0 ? 0 : e);
        return ldexpf(1.0f, e);
    };
    auto acc_zero = [](auto &acc) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int v = 0; v < (int)(sizeof(acc[0]) / sizeof(acc[0][0])); ++v)
#pragma unroll
                for (int t = 0; t < 9; ++t) acc[u][v][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    auto flagged = [&](int bi) __attribute__((always_inline)) {
        return (xfl[4 * bi] | xfl[4 * bi + 1] | xfl[4 * bi + 2] | xfl[4 * bi + 3]) != 0;
    };

    if (loader) {
        // the roles run separate loops with the same barrier sequence, so the loaders' staging
        // registers and the MFMA waves' accumulators are never live at the same time
#if CISTA_WT_PRIO
        // the staging waves (the younger half) win VALU issue arbitration against the MFMA waves
        if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 64 * WT_NMW) __builtin_amdgcn_s_setprio(CISTA_WT_PRIO);
#endif
        WT_STAMP(0, __builtin_amdgcn_s_memtime());
        if (split < ntiles) {
            load_tile(split);
            commit(sm, xfl);
            WT_STAMP(1, __builtin_amdgcn_s_memtime());
            if (split + a.nsplit < ntiles) load_tile(split + a.nsplit);
        }
        __syncthreads();
        WT_STAMP(2, __builtin_amdgcn_s_memtime());
        int it = 0;
        for (int tile = split; tile < ntiles; tile += a.nsplit, ++it) {
            const int bi = it & 1;
            if (__builtin_expect(flagged(bi), 0)) {
                __syncthreads();
                int b, oy0, ox0;
                tile_origin(tile, b, oy0, ox0);
                float m = 0.0f;
#pragma unroll 1
                for (int u = 0; u < GE::UX; ++u) {
                    const float4 v = load_x(b, oy0, ox0, u);
                    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
                }
                for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
                if (lane == 0) xmx[lw] = m;
                __syncthreads();
                sx = tile_scale();
#pragma unroll 1
                for (int u = 0; u < GE::UX; ++u) put_x(sm + bi * WT_BUF + 8 * WT_GPL, u, load_x(b, oy0, ox0, u), sx);
                __syncthreads();
            }
            if (tile + a.nsplit < ntiles) {
                // the other buffer was last read before the barrier that opened this iteration
                commit(sm + (bi ^ 1) * WT_BUF, xfl + 4 * (bi ^ 1));
                WT_STAMP(3 + 3 * it, __builtin_amdgcn_s_memtime());
                if (tile + 2 * a.nsplit < ntiles) load_tile(tile + 2 * a.nsplit);
                WT_STAMP(4 + 3 * it, __builtin_amdgcn_s_memtime());
            }
            __syncthreads();
            WT_STAMP(5 + 3 * it, __builtin_amdgcn_s_memtime());
        }
        if (do_bias) {
            reinterpret_cast<float4 *>(wsm4)[tid - 64 * WT_NMW] = bsum;
            __syncthreads();
        }
        return;
    }

    // ---- MFMA waves: 32 co (planes pco, pco + 1) x NV x 16 ci (planes pci .. pci + NV - 1) ----
    constexpr int NV = 2, WPC = 4 / NV;                            // ci planes per wave, waves per co pair
    const int pco = 2 * (wave / WPC), pci = NV * (wave % WPC);
    const int kg = lane >> 4, rq = (lane >> 2) & 3, rp = lane & 3;   // transposed-read roles
    f32x4 acc[2][NV][9];
    acc_zero(acc);
    WT_STAMP(0, __builtin_amdgcn_s_memtime());
    WT_STAMP(252, __builtin_amdgcn_s_memrealtime());
    __syncthreads();
    WT_STAMP(1, __builtin_amdgcn_s_memtime());
    int it = 0;
    for (int tile = split; tile < ntiles; tile += a.nsplit, ++it) {
        const int bi = it & 1;
        // the tile's X scale: from its own maximum when flagged, else 1 (powers of two, so the
        // accumulator rescale by r is exact)
        const bool fl = flagged(bi);
        if (__builtin_expect(fl || sx != 1.0f, 0)) {    // uniform rare path
            float st = 1.0f;
            if (fl) {
                __syncthreads();
                __syncthreads();
                st = tile_scale();
            }
            const float r = st / sx;
            sx = st;
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int v = 0; v < NV; ++v)
#pragma unroll
                    for (int t = 0; t < 9; ++t) acc[u][v][t] *= r;
            if (fl) __syncthreads();
        }
        const _Float16 *Gp = sm + bi * WT_BUF, *Xp = Gp + 8 * WT_GPL;
        // 27 (K-step, tap) steps, software-pipelined: the fragments of step n + 1 are read before
        // step n's 12 MFMAs are issued, so their LDS latency hides under those MFMAs
        auto read_g = [&](int s, f16x8 (&gh)[2], f16x8 (&gl)[2]) __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int off = (pco + u) * WT_GPL + ((2 * s) * 16 + 4 * kg + rq) * 16 + 4 * rp;
                gh[u] = cat_frag(tr_read(Gp, off), tr_read(Gp, off + 256));
                gl[u] = cat_frag(tr_read(Gp, off + 4 * WT_GPL), tr_read(Gp, off + 4 * WT_GPL + 256));
            }
        };
        auto read_x = [&](int s, int t, f16x8 (&xh)[NV], f16x8 (&xl)[NV]) __attribute__((always_inline)) {
            const int dy = t / 3, dx = t % 3;
            constexpr int R1 = GE::S * GE::HW * 16;     // K row 1 (the next output row) in halves
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const int off = (pci + v) * WT_XPL + GE::kpos(s, 0, dy, dx, 4 * kg + rq) * 16 + 4 * rp;
                xh[v] = cat_frag(tr_read(Xp, off), tr_read(Xp, off + R1));
                xl[v] = cat_frag(tr_read(Xp, off + 4 * WT_XPL), tr_read(Xp, off + 4 * WT_XPL + R1));
            }
        };
        // fragments read one step ahead (double buffer)
        constexpr int XD = 1, NXB = XD + 1, NSTEP = 9 * GE::KS;
        f16x8 gh[2][2], gl[2][2], xh[NXB][NV], xl[NXB][NV];
        read_g(0, gh[0], gl[0]);
#pragma unroll
        for (int d = 0; d < XD; ++d) read_x(d / 9, d % 9, xh[d], xl[d]);
#pragma unroll
        for (int n = 0; n < NSTEP; ++n) {
            const int s = n / 9, t = n % 9, xb = n % NXB, gb = s & 1;
            if (n + XD < NSTEP) read_x((n + XD) / 9, (n + XD) % 9, xh[(n + XD) % NXB], xl[(n + XD) % NXB]);
            if (s + 1 < GE::KS && t == 9 - XD) read_g(s + 1, gh[gb ^ 1], gl[gb ^ 1]);
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    acc[u][v][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gh[gb][u], xh[xb][v], acc[u][v][t], 0, 0, 0);
                    acc[u][v][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gh[gb][u], xl[xb][v], acc[u][v][t], 0, 0, 0);
                    acc[u][v][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gl[gb][u], xh[xb][v], acc[u][v][t], 0, 0, 0);
                }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (it < 120) WT_STAMP(2 + 2 * it, __builtin_amdgcn_s_memtime());
        __syncthreads();
        if (it < 120) WT_STAMP(3 + 2 * it, __builtin_amdgcn_s_memtime());
    }
    WT_STAMP(250, __builtin_amdgcn_s_memtime());
    if (do_bias) {
        // loader sums of co quad 16 sb + 4 sq -> per-co sums in a fixed order (waves, then sp)
        __syncthreads();
        if (tid < 64) {
            const float4 *red = reinterpret_cast<const float4 *>(wsm4);
            const int b16 = tid >> 4, q4 = (tid >> 2) & 3, e = tid & 3;
            float t = 0.0f;
            for (int w = 0; w < 4; ++w)
                for (int p = 0; p < 4; ++p) t += (&red[64 * w + 16 * b16 + 4 * p + q4].x)[e];
            a.bpartial[(size_t)split * a.Cout + co0 + tid] = t;
        }
    }
    // acc[u][v][t][j]: row (cout) 16 (pco + u) + 4 (lane >> 4) + j, col (cin) 16 (pci + v) + (lane & 15)
    const float inv = a.gscale[1] * (1.0f / sx);
    float *part = a.partial + (size_t)split * a.Cout * a.Cin * 9;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int ci = ci0 + 16 * (pci + v) + (lane & 15);
        if (ci >= a.Cin) continue;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int co = co0 + 16 * (pco + u) + 4 * (lane >> 4) + j;
#pragma unroll
                for (int t = 0; t < 9; ++t) part[((size_t)co * a.Cin + ci) * 9 + t] = acc[u][v][t][j] * inv;
            }
    }
    WT_STAMP(251, __builtin_amdgcn_s_memtime());
    WT_STAMP(253, __builtin_amdgcn_s_memrealtime());
}

// --------------------------------------------------------------------------------------------
// wgrad of a one-output-channel stride-1 conv (final_conv, 64 -> 1): dW[ci][t] = sum_P g(P) *
// Xpad(P + t, ci) on VALU (an MFMA block would waste 31 of 32 rows).  blockIdx.x = 32-channel
// block, blockIdx.y = split over 16 x 16 pixel tiles.  The reflect-padded 18 x 18 x 32 input
// halo sits in LDS (row stride 33: conflict-free); thread = (channel tid & 31, pixel phase
// tid >> 5) accumulates 9 taps over its phase's pixels; phases are summed in a fixed order.
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void wgrad_c1_kernel(const WgradArgs a) {
    __shared__ float Xs[18 * 18 * 33];
    __shared__ float gs[256];
    __shared__ float red[8][32 * 9 + 1];
    const int tid = threadIdx.x, ci = tid & 31, ph = tid >> 5;
    const int ci0 = blockIdx.x * 32;
    float acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = 0.0f;
    float bsum = 0.0f;
    const int ntiles = a.B * a.tiles_y * a.tiles_x;
    for (int tile = blockIdx.y; tile < ntiles; tile += a.nsplit) {
        int tt = tile;
        const int tx = tt % a.tiles_x;
        tt /= a.tiles_x;
        const int ty = tt % a.tiles_y;
        const int b = tt / a.tiles_y;
        const int oy0 = ty * 16, ox0 = tx * 16;
        __syncthreads();
        {
            const int oy = oy0 + (tid >> 4), ox = ox0 + (tid & 15);
            gs[tid] = (oy < a.Hout && ox < a.Wout)
                          ? a.G[((size_t)b * a.Hout + oy) * a.Wout + ox] : 0.0f;
        }
        for (int i = tid; i < 18 * 18 * 8; i += 256) {          // 8 channel quads per pixel
            const int hp = i >> 3, q = i & 7;
            const int hy = hp / 18, hx = hp - hy * 18;
            const float4 v = wg_load_x4<XS_S1>(a, b, oy0 - 1 + hy, ox0 - 1 + hx, ci0 + 4 * q);
            float *d = Xs + hp * 33 + 4 * q;
            d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
        __syncthreads();
        // phase ph walks tile rows 2ph, 2ph+1 left to right with the 3 x 3 input window of its
        // channel in registers: 3 LDS reads per pixel instead of 9
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const int py = 2 * ph + rr;
            float w[3][3];
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                w[dy][1] = Xs[((py + dy) * 18 + 0) * 33 + ci];
                w[dy][2] = Xs[((py + dy) * 18 + 1) * 33 + ci];
            }
#pragma unroll 4
            for (int px = 0; px < 16; ++px) {
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    w[dy][0] = w[dy][1];
                    w[dy][1] = w[dy][2];
                    w[dy][2] = Xs[((py + dy) * 18 + px + 2) * 33 + ci];
                }
                const float g = gs[py * 16 + px];
                if (blockIdx.x == 0 && ci == 0) bsum += g;
#pragma unroll
                for (int t = 0; t < 9; ++t) acc[t] = fmaf(g, w[t / 3][t % 3], acc[t]);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 9; ++t) red[ph][ci * 9 + t] = acc[t];
    if (ci == 0) red[ph][32 * 9] = bsum;
    __syncthreads();
    float *part = a.partial + (size_t)blockIdx.y * a.Cin * 9;
    for (int i = tid; i < 32 * 9; i += 256) {
        float s = 0.0f;
        for (int k = 0; k < 8; ++k) s += red[k][i];
        if (ci0 + i / 9 < a.Cin) part[ci0 * 9 + i] = s;
    }
    if (blockIdx.x == 0 && tid == 0 && a.bpartial) {
        float s = 0.0f;
        for (int k = 0; k < 8; ++k) s += red[k][32 * 9];
        a.bpartial[blockIdx.y] = s;
    }
}

// --------------------------------------------------------------------------------------------
// wgrad of the input-stage convs We (num_bins -> C/2) and Wi (1 -> C/2): CI <= 8 NCHW input
// planes, Cout <= 32 output channels of G (channels [Goff, Goff + Cout) of a Gc-channel NHWC
// tensor).  VALU: thread = (output channel tid & 31, pixel phase tid >> 5) accumulates CI x 9
// taps; G tile (256 px x 32, stride 33) and the reflect-padded CI x 18 x 18 input halo in
// LDS; blockIdx.x = split over 16 x 16 tiles; phases summed in a fixed order.
// --------------------------------------------------------------------------------------------
template <int CI>
__global__ __launch_bounds__(256) void wgrad_small_kernel(const WgradArgs a) {
    __shared__ float Gt[256 * 33];
    __shared__ float Xh[CI * 18 * 18];
    const int tid = threadIdx.x, co = tid & 31, ph = tid >> 5;
    float acc[CI][9];
#pragma unroll
    for (int c = 0; c < CI; ++c)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[c][t] = 0.0f;
    float bsum = 0.0f;
    const int ntiles = a.B * a.tiles_y * a.tiles_x;
    for (int tile = blockIdx.x; tile < ntiles; tile += a.nsplit) {
        int tt = tile;
        const int tx = tt % a.tiles_x;
        tt /= a.tiles_x;
        const int ty = tt % a.tiles_y;
        const int b = tt / a.tiles_y;
        const int oy0 = ty * 16, ox0 = tx * 16;
        __syncthreads();
        for (int i = tid; i < 256 * 32; i += 256) {
            const int p = i >> 5, c = i & 31;
            const int oy = oy0 + (p >> 4), ox = ox0 + (p & 15);
            Gt[p * 33 + c] = (c < a.Cout && oy < a.Hout && ox < a.Wout)
                                 ? a.G[(((size_t)b * a.Hout + oy) * a.Wout + ox) * a.Gc + a.Goff + c] : 0.0f;
        }
        for (int i = tid; i < CI * 324; i += 256) {
            const int c = i / 324, hp = i - c * 324;
            const int hy = hp / 18, hx = hp - hy * 18;
            const int y = reflect_clamp(oy0 - 1 + hy, a.Hin), x = reflect_clamp(ox0 - 1 + hx, a.Win);
            Xh[i] = a.X0[(((size_t)b * a.x0c + c) * a.Hin + y) * a.Win + x];
        }
        __syncthreads();
        // phase ph walks tile rows 2ph, 2ph+1 left to right with the CI x 3 x 3 input window in
        // registers (wave-uniform: LDS broadcasts): 3 CI reads per pixel instead of 9 CI
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const int py = 2 * ph + rr;
            float w[CI][3][3];
#pragma unroll
            for (int c = 0; c < CI; ++c)
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    w[c][dy][1] = Xh[c * 324 + (py + dy) * 18 + 0];
                    w[c][dy][2] = Xh[c * 324 + (py + dy) * 18 + 1];
                }
#pragma unroll 2
            for (int px = 0; px < 16; ++px) {
#pragma unroll
                for (int c = 0; c < CI; ++c)
#pragma unroll
                    for (int dy = 0; dy < 3; ++dy) {
                        w[c][dy][0] = w[c][dy][1];
                        w[c][dy][1] = w[c][dy][2];
                        w[c][dy][2] = Xh[c * 324 + (py + dy) * 18 + px + 2];
                    }
                const float g = Gt[(py * 16 + px) * 33 + co];
                bsum += g;
#pragma unroll
                for (int c = 0; c < CI; ++c)
#pragma unroll
                    for (int t = 0; t < 9; ++t) acc[c][t] = fmaf(g, w[c][t / 3][t % 3], acc[c][t]);
            }
        }
    }
    // sum the 8 phases in order 0..7 (phase 0 accumulates the others through LDS)
    float *red = Gt;                                   // 32 x (CI*9 + 1) floats per round
    constexpr int RS = CI * 9 + 1;
    for (int src = 1; src < 8; ++src) {
        __syncthreads();
        if (ph == src) {
#pragma unroll
            for (int c = 0; c < CI; ++c)
#pragma unroll
                for (int t = 0; t < 9; ++t) red[co * RS + c * 9 + t] = acc[c][t];
            red[co * RS + CI * 9] = bsum;
        }
        __syncthreads();
        if (ph == 0) {
#pragma unroll
            for (int c = 0; c < CI; ++c)
#pragma unroll
                for (int t = 0; t < 9; ++t) acc[c][t] += red[co * RS + c * 9 + t];
            bsum += red[co * RS + CI * 9];
        }
    }
    if (ph == 0 && co < a.Cout) {
        float *part = a.partial + (size_t)blockIdx.x * a.Cout * CI * 9;
#pragma unroll
        for (int c = 0; c < CI; ++c)
#pragma unroll
            for (int t = 0; t < 9; ++t) part[((size_t)co * CI + c) * 9 + t] = acc[c][t];
        if (a.bpartial) a.bpartial[(size_t)blockIdx.x * a.Cout + co] = bsum;
    }
}

// --------------------------------------------------------------------------------------------
// We and Wi weight (and bias) gradients in ONE pass over gxfull (B, H, W, C NHWC; was one
// wgrad_small_kernel launch per half, each fetching the whole 256-B pixel rows for its 128 B):
//   dWe[co][ci][t] = sum_P G(P, co) ev_pad(P + t, ci)        co < C/2, ci < NB
//   dWi[co][t]     = sum_P G(P, C/2 + co) img_pad(P + t)
// as pixel-reduction GEMMs on exact fp32 MFMA (v_mfma_f32_16x16x4f32): K = pixels of an 8 x 16
// tile, M = output channel 16-blocks (MB = C/32 per half), N = im2col columns (plane, tap) read
// straight from the reflect-padded (NB+1) x 10 x 18 input halo in LDS, plus a ones column whose
// result is the bias gradient.  4 waves split each tile's 32 K-steps; the next tile's G / halo
// loads are issued before this tile's MFMAs (registers); the waves' sums are added in a fixed
// order at the end (deterministic), one partial per split ([split][co][n], reduce_partials_kernel).
// --------------------------------------------------------------------------------------------
struct WgradInArgs {
    const float *G;            // gxfull (B, H, W, C)
    const float *ev, *img;     // events (B, NB, H, W), previous image (B, 1, H, W)
    float *partE, *partI;      // [nsplit][C/2][NB*9], [nsplit][C/2][9]
    float *bpartE, *bpartI;    // [nsplit][C/2]
    int B, H, W, C, tiles_x, tiles_y, nsplit;
};
constexpr int WI_TP = 128, WI_HR = 10, WI_HW = 18, WI_HPX = WI_HR * WI_HW;

template <int NB, int MB>
__global__ __launch_bounds__(256) void wgrad_in_kernel(const WgradInArgs a) {
    constexpr int C = 32 * MB, HALF = 16 * MB, LDG = C + 16;   // LDG: lanes 0-15 / 16-31 on other banks
    constexpr int NE = NB * 9 + 1, NBE = (NE + 15) / 16;        // E columns incl. the ones column
    constexpr int GI = WI_TP * C / 4 / 256;                     // G float4 items per thread
    constexpr int XI = ((NB + 1) * WI_HPX + 255) / 256;         // halo items per thread
    extern __shared__ float wism[];
    float *Gs = wism, *Xs = wism + WI_TP * LDG;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ntiles = a.B * a.tiles_y * a.tiles_x;
    // per-lane im2col offset of column n = 16 nb + (lane & 15): halo offset, -1 ones, -2 zero
    int offE[NBE], offI;
#pragma unroll
    for (int nb = 0; nb < NBE; ++nb) {
        const int n = nb * 16 + (lane & 15);
        offE[nb] = n < NB * 9 ? (n / 9) * WI_HPX + ((n % 9) / 3) * WI_HW + (n % 3) : (n == NB * 9 ? -1 : -2);
    }
    {
        const int n = lane & 15;
        offI = n < 9 ? NB * WI_HPX + (n / 3) * WI_HW + (n % 3) : (n == 9 ? -1 : -2);
    }
    f32x4 accE[MB][NBE], accI[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
        accI[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int nb = 0; nb < NBE; ++nb) accE[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float4 gv[GI];
    float xv[XI];
    auto load = [&](int tile) __attribute__((always_inline)) {
        int tt = tile;
        const int tx = tt % a.tiles_x;
        tt /= a.tiles_x;
        const int ty = tt % a.tiles_y;
        const int b = tt / a.tiles_y;
        const int oy0 = ty * 8, ox0 = tx * 16;
#pragma unroll
        for (int u = 0; u < GI; ++u) {
            const int i = tid + u * 256;
            const int p = i / (C / 4), c4 = i - p * (C / 4);
            const int oy = oy0 + (p >> 4), ox = ox0 + (p & 15);
            gv[u] = (oy < a.H && ox < a.W)
                        ? *reinterpret_cast<const float4 *>(a.G + (((size_t)b * a.H + oy) * a.W + ox) * C + 4 * c4)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < XI; ++u) {
            const int i = tid + u * 256;
            const int c = i / WI_HPX, hp = i - c * WI_HPX;
            const int hy = hp / WI_HW, hx = hp - hy * WI_HW;
            const int y = reflect_clamp(oy0 - 1 + hy, a.H), x = reflect_clamp(ox0 - 1 + hx, a.W);
            xv[u] = i >= (NB + 1) * WI_HPX ? 0.0f
                    : c < NB ? a.ev[(((size_t)b * NB + c) * a.H + y) * a.W + x]
                             : a.img[((size_t)b * a.H + y) * a.W + x];
        }
    };
    if ((int)blockIdx.x < ntiles) load(blockIdx.x);
    for (int tile = blockIdx.x; tile < ntiles; tile += a.nsplit) {
        __syncthreads();                                    // the previous tile's reads are done
#pragma unroll
        for (int u = 0; u < GI; ++u) {
            const int i = tid + u * 256;
            const int p = i / (C / 4), c4 = i - p * (C / 4);
            *reinterpret_cast<float4 *>(Gs + p * LDG + 4 * c4) = gv[u];
        }
#pragma unroll
        for (int u = 0; u < XI; ++u) {
            const int i = tid + u * 256;
            if (i < (NB + 1) * WI_HPX) Xs[i] = xv[u];
        }
        __syncthreads();
        if (tile + a.nsplit < ntiles) load(tile + a.nsplit);
#pragma unroll 2
        for (int j = 0; j < WI_TP / 16; ++j) {
            const int P = 4 * (wave + 4 * j) + (lane >> 4), base = (P >> 4) * WI_HW + (P & 15);
            const float *gp = Gs + P * LDG + (lane & 15);
            float bE[NBE];
#pragma unroll
            for (int nb = 0; nb < NBE; ++nb)
                bE[nb] = offE[nb] >= 0 ? Xs[offE[nb] + base] : (offE[nb] == -1 ? 1.0f : 0.0f);
            const float bI = offI >= 0 ? Xs[offI + base] : (offI == -1 ? 1.0f : 0.0f);
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) {
                const float aE = gp[mb * 16], aI = gp[HALF + mb * 16];
#pragma unroll
                for (int nb = 0; nb < NBE; ++nb)
                    accE[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(aE, bE[nb], accE[mb][nb], 0, 0, 0);
                accI[mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(aI, bI, accI[mb], 0, 0, 0);
            }
        }
    }
    // waves 1..3 hand their sums to wave 0 through LDS, added in wave order
    constexpr int NACC = MB * (NBE + 1) * 4;               // floats per lane
    __syncthreads();
    float *red = wism;                                      // [3][NACC][64]
    if (wave > 0) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
#pragma unroll
            for (int nb = 0; nb < NBE; ++nb)
#pragma unroll
                for (int r = 0; r < 4; ++r) red[((wave - 1) * NACC + (mb * (NBE + 1) + nb) * 4 + r) * 64 + lane] = accE[mb][nb][r];
#pragma unroll
            for (int r = 0; r < 4; ++r) red[((wave - 1) * NACC + (mb * (NBE + 1) + NBE) * 4 + r) * 64 + lane] = accI[mb][r];
        }
    }
    __syncthreads();
    if (wave == 0) {
        const int sp = blockIdx.x;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = mb * 16 + 4 * (lane >> 4) + r;
#pragma unroll
                for (int nb = 0; nb <= NBE; ++nb) {
                    float v = nb < NBE ? accE[mb][nb][r] : accI[mb][r];
#pragma unroll
                    for (int w = 0; w < 3; ++w) v += red[(w * NACC + (mb * (NBE + 1) + nb) * 4 + r) * 64 + lane];
                    const int n = (nb < NBE ? nb * 16 : 0) + (lane & 15);
                    if (nb < NBE) {
                        if (n < NB * 9) a.partE[((size_t)sp * HALF + co) * (NB * 9) + n] = v;
                        else if (n == NB * 9) a.bpartE[(size_t)sp * HALF + co] = v;
                    } else {
                        if (n < 9) a.partI[((size_t)sp * HALF + co) * 9 + n] = v;
                        else if (n == 9) a.bpartI[(size_t)sp * HALF + co] = v;
                    }
                }
            }
    }
}

// up = interpolate(x, 2x, bilinear, align_corners=False) materialised, NHWC (B,h,w,C) ->
// (B,2h,2w,C), the operation order of the forward's STAGE_UP gather (base_layers.py:198), so
// the upsample conv's wgrad can run as a stride-1 wgrad on it
template <typename I>     // the element index type (int when the count fits 31 bits)
__global__ __launch_bounds__(256) void upsample2x_kernel(const float *x, float *up, int B, int h, int w, int C) {
    const int c4 = C / 4, H = 2 * h, W = 2 * w;
    const I total = (I)B * H * W * c4;
    const I idx = (I)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int q = (int)(idx % c4);
    const I pix = idx / c4;
    const I row = pix / W;
    const int X = (int)(pix - row * W), Y = (int)(row % H), b = (int)(row / H);
    const float sy = fmaxf(((float)Y + 0.5f) * 0.5f - 0.5f, 0.0f);
    const float sx = fmaxf(((float)X + 0.5f) * 0.5f - 0.5f, 0.0f);
    const int y0 = (int)sy, x0 = (int)sx;
    const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
    const float ly1 = sy - (float)y0, ly0 = 1.0f - ly1, lx1 = sx - (float)x0, lx0 = 1.0f - lx1;
    const float *base = x + (size_t)b * h * w * C + 4 * q;
    const float4 v00 = *(const float4 *)(base + ((size_t)y0 * w + x0) * C);
    const float4 v01 = *(const float4 *)(base + ((size_t)y0 * w + x1) * C);
    const float4 v10 = *(const float4 *)(base + ((size_t)y1 * w + x0) * C);
    const float4 v11 = *(const float4 *)(base + ((size_t)y1 * w + x1) * C);
    float4 r;
    r.x = bilerp(ly0, ly1, lx0, lx1, v00.x, v01.x, v10.x, v11.x);
    r.y = bilerp(ly0, ly1, lx0, lx1, v00.y, v01.y, v10.y, v11.y);
    r.z = bilerp(ly0, ly1, lx0, lx1, v00.z, v01.z, v10.z, v11.z);
    r.w = bilerp(ly0, ly1, lx0, lx1, v00.w, v01.w, v10.w, v11.w);
    *(float4 *)(up + (size_t)pix * C + 4 * q) = r;
}

// dW (+)= sign * sum over splits of partial  (n = Cout*Cin*9); threads n .. n + nb - 1 do the
// bias gradient db from bpartial in the same launch.  The split sum is latency-bound (each
// thread walks nsplit rows): 16 rows are loaded per round, then added in the order of four
// interleaved accumulators (row k into s[k % 4]), so the result does not depend on the batching.
__device__ __forceinline__ float sum_splits(const float *partial, int nsplit, long n, long i) {
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
    int k = 0;
    for (; k + 16 <= nsplit; k += 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = partial[(size_t)(k + u) * n + i];
#pragma unroll
        for (int u = 0; u < 16; u += 4) {
            s0 += v[u];
            s1 += v[u + 1];
            s2 += v[u + 2];
            s3 += v[u + 3];
        }
    }
    for (; k + 4 <= nsplit; k += 4) {
        s0 += partial[(size_t)k * n + i];
        s1 += partial[(size_t)(k + 1) * n + i];
        s2 += partial[(size_t)(k + 2) * n + i];
        s3 += partial[(size_t)(k + 3) * n + i];
    }
    for (; k < nsplit; ++k) s0 += partial[(size_t)k * n + i];
    return (s0 + s1) + (s2 + s3);
}

__global__ __launch_bounds__(256) void reduce_partials_kernel(const float *partial, int nsplit, long n,
                                                              float *dst, float sign, int accumulate,
                                                              const float *bpartial = nullptr, long nb = 0,
                                                              float *bdst = nullptr) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) {
        i -= n;
        if (i >= nb) return;
        partial = bpartial;
        n = nb;
        dst = bdst;
    }
    dst[i] = (accumulate ? dst[i] : 0.0f) + sign * sum_splits(partial, nsplit, n, i);
}

// --------------------------------------------------------------------------------------------
// generic VALU dgrad of a small reflect-padded 3x3 conv with stride S (W0, final_conv, Wi):
// dX[b,Q,ci] (+)= sum over (P, t) with reflect(S*P + t - 1) == Q of G[b,P,co] W[co][ci][t]
// G NHWC (B, Hout, Wout, Gc) channels [Goff, Goff+Cout); dX layout NHWC (Xc, Xoff) or, for
// Xc == 0, NCHW planes (prev_image: Cin == 1; events: Cin == num_bins).
// --------------------------------------------------------------------------------------------
struct DgradSmallArgs {
    const float *G; int Gc, Goff;
    const float *W;       // [Cout][Cin][3][3]
    float *dX; int Xc, Xoff;
    const float *mask;    // optional: dX *= (mask > 0), mask laid out like dX
    int B, Hin, Win, Hout, Wout, S, Cout, Cin;
    int accumulate;
};

__device__ __forceinline__ int refl_taps(int q, int n_in, int n_out, int S, int (&P)[6], int (&T)[6]) {
    // all (P, t) with reflect(S*P + t - 1) == q, 0 <= P < n_out, t in 0..2
    int k = 0;
    const int lo = (q - 2) / S - 2, hi = (q + 1) / S + 2;
    for (int p = lo; p <= hi; ++p) {
        if (p < 0 || p >= n_out) continue;
        for (int t = 0; t < 3; ++t) {
            int i = S * p + t - 1;
            i = i < 0 ? -i : i;
            i = i >= n_in ? 2 * n_in - 2 - i : i;
            if (i == q && k < 6) {
                P[k] = p;
                T[k] = t;
                ++k;
            }
        }
    }
    return k;
}

__global__ __launch_bounds__(256) void dgrad_small_kernel(const DgradSmallArgs a) {
    const long total = (long)a.B * a.Hin * a.Win * a.Cin;
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int ci = (int)(idx % a.Cin);
    const long pix = idx / a.Cin;
    const int x = (int)(pix % a.Win);
    const int y = (int)((pix / a.Win) % a.Hin);
    const int b = (int)(pix / ((long)a.Win * a.Hin));
    int Py[6], Ty[6], Px[6], Tx[6];
    const int ny = refl_taps(y, a.Hin, a.Hout, a.S, Py, Ty);
    const int nx = refl_taps(x, a.Win, a.Wout, a.S, Px, Tx);
    float s = 0.0f;
    for (int i = 0; i < ny; ++i)
        for (int j = 0; j < nx; ++j) {
            const float *g = a.G + (((size_t)b * a.Hout + Py[i]) * a.Wout + Px[j]) * a.Gc + a.Goff;
            const int t = Ty[i] * 3 + Tx[j];
            if (((a.Cout | a.Gc | a.Goff) & 3) == 0) {      // float4 along Cout
                for (int co = 0; co < a.Cout; co += 4) {
                    const float4 gv = *reinterpret_cast<const float4 *>(g + co);
                    const float *wp = a.W + ((size_t)co * a.Cin + ci) * 9 + t;
                    const size_t ws = (size_t)a.Cin * 9;
                    s = fmaf(gv.x, wp[0], fmaf(gv.y, wp[ws], fmaf(gv.z, wp[2 * ws], fmaf(gv.w, wp[3 * ws], s))));
                }
            } else {
                for (int co = 0; co < a.Cout; ++co) s = fmaf(g[co], a.W[((size_t)co * a.Cin + ci) * 9 + t], s);
            }
        }
    const size_t o = a.Xc ? (size_t)pix * a.Xc + a.Xoff + ci
                          : ((size_t)b * a.Cin + ci) * a.Hin * a.Win + (size_t)y * a.Win + x;
    if (a.accumulate) s += a.dX[o];
    if (a.mask && !(a.mask[o] > 0.0f)) s = 0.0f;
    a.dX[o] = s;
}

// dgrad_small_kernel for one input channel (Wi: the previous image's gradient), stride 1, with
// the output gradient staged in LDS: workgroup = 16 x 16 pixel tile, thread = pixel.  The G
// channels [Goff, Goff + Cout) of the tile's 18 x 18 neighbourhood (every (P, t) of a pixel lies
// in it, the reflected P = 0 / n - 1 included) are loaded once, coalesced (the per-lane 9-tap
// gathers of the generic kernel re-fetched G ~15x from HBM: 675 MB per launch at B = 8); pixel
// stride Cout + 4 floats makes the 16-lane ds_read_b128 groups conflict-free.  Same arithmetic
// and order as dgrad_small_kernel (bit-identical).  Cout % 4 == 0, Cout <= 32, Gc, Goff % 4 == 0.
constexpr int DC1_MAXC = 32;
__global__ __launch_bounds__(256) void dgrad_c1_kernel(const float *G, int Gc, int Goff, const float *W, int Cout,
                                                       float *dX, int B, int H, int Wd) {
    __shared__ float4 gs[18 * 18 * (DC1_MAXC + 4) / 4];
    const int tilesx = (Wd + 15) / 16, tilesy = (H + 15) / 16;
    const int b = blockIdx.x / (tilesx * tilesy), t2 = blockIdx.x - b * tilesx * tilesy;
    const int y0 = (t2 / tilesx) * 16, x0 = (t2 % tilesx) * 16;
    const int ps = (Cout + 4) / 4;                              // pixel stride in float4
    const int cq = Cout / 4;
    for (int i = threadIdx.x; i < 18 * 18 * cq; i += 256) {
        const int q = i % cq, px = i / cq, ly = px / 18, lx = px - ly * 18;
        const int gy = min(max(y0 - 1 + ly, 0), H - 1), gx = min(max(x0 - 1 + lx, 0), Wd - 1);
        gs[px * ps + q] = *reinterpret_cast<const float4 *>(G + (((size_t)b * H + gy) * Wd + gx) * Gc + Goff + 4 * q);
    }
    __syncthreads();
    const int y = y0 + (threadIdx.x >> 4), x = x0 + (threadIdx.x & 15);
    if (y >= H || x >= Wd) return;
    int Py[6], Ty[6], Px[6], Tx[6];
    const int ny = refl_taps(y, H, H, 1, Py, Ty), nx = refl_taps(x, Wd, Wd, 1, Px, Tx);
    float s = 0.0f;
    for (int i = 0; i < ny; ++i)
        for (int j = 0; j < nx; ++j) {
            const float4 *g = gs + ((Py[i] - y0 + 1) * 18 + (Px[j] - x0 + 1)) * ps;
            const int t = Ty[i] * 3 + Tx[j];
            for (int co = 0; co < Cout; co += 4) {
                const float4 gv = g[co >> 2];
                const float *wp = W + (size_t)co * 9 + t;
                s = fmaf(gv.x, wp[0], fmaf(gv.y, wp[9], fmaf(gv.z, wp[18], fmaf(gv.w, wp[27], s))));
            }
        }
    dX[((size_t)b * H + y) * Wd + x] = s;
}

// W [Cout][Cin][9] -> WT [9][Cout][Cin] (the layout dgrad_vec_kernel reads as float4 along Cin)
__global__ void transpose_w_kernel(const float *W, int Cout, int Cin, float *WT) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Cout * Cin * 9) return;
    const int t = i % 9, ci = (i / 9) % Cin, co = i / (9 * Cin);
    WT[((size_t)t * Cout + co) * Cin + ci] = W[i];
}

// dgrad_small_kernel with 4 input channels per thread (Cin % 4 == 0, Xc % 4 == 0): one
// float4 weight load feeds 4 FMAs, the G value is a wave-uniform-per-pixel broadcast.
// Used for W0 (stride 2, 64 -> 64) and the final conv (1 -> C, ReLU mask).
__global__ __launch_bounds__(256) void dgrad_vec_kernel(const DgradSmallArgs a, const float *WT) {
    const int cq = a.Cin >> 2;
    const long total = (long)a.B * a.Hin * a.Win * cq;
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int ci = (int)(idx % cq) * 4;
    const long pix = idx / cq;
    const int x = (int)(pix % a.Win);
    const int y = (int)((pix / a.Win) % a.Hin);
    const int b = (int)(pix / ((long)a.Win * a.Hin));
    int Py[6], Ty[6], Px[6], Tx[6];
    const int ny = refl_taps(y, a.Hin, a.Hout, a.S, Py, Ty);
    const int nx = refl_taps(x, a.Win, a.Wout, a.S, Px, Tx);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = 0; i < ny; ++i)
        for (int j = 0; j < nx; ++j) {
            const float *g = a.G + (((size_t)b * a.Hout + Py[i]) * a.Wout + Px[j]) * a.Gc + a.Goff;
            const float *w = WT + (size_t)(Ty[i] * 3 + Tx[j]) * a.Cout * a.Cin + ci;
#pragma unroll 4
            for (int co = 0; co < a.Cout; ++co) {
                const float gv = g[co];
                const float4 wv = *reinterpret_cast<const float4 *>(w + (size_t)co * a.Cin);
                s.x = fmaf(gv, wv.x, s.x);
                s.y = fmaf(gv, wv.y, s.y);
                s.z = fmaf(gv, wv.z, s.z);
                s.w = fmaf(gv, wv.w, s.w);
            }
        }
    const size_t o = (size_t)pix * a.Xc + a.Xoff + ci;
    float4 *dst = reinterpret_cast<float4 *>(a.dX + o);
    if (a.accumulate) {
        const float4 d = *dst;
        s.x += d.x; s.y += d.y; s.z += d.z; s.w += d.w;
    }
    if (a.mask) {
        const float4 m = *reinterpret_cast<const float4 *>(a.mask + o);
        s.x = m.x > 0.0f ? s.x : 0.0f;
        s.y = m.y > 0.0f ? s.y : 0.0f;
        s.z = m.z > 0.0f ? s.z : 0.0f;
        s.w = m.w > 0.0f ? s.w : 0.0f;
    }
    *dst = s;
}

// final_conv dgrad (Cout 1, stride 1, reflect padding) with the upsample ReLU mask: dX (B,H,W,C)
// = [u > 0] * sum over (P, t) with reflect(P + t - 1) == Q of G[P] W[t][c].  Thread = (pixel, 8
// channels): two float4 weight loads ([9][C] layout, L1-resident) per tap feed 8 FMAs; the
// general dgrad_vec_kernel spent 4 threads and 64-bit index math per such group (211 us at B=8).
// Pixels in a grid-stride loop, a thread = 8 channels of one pixel per step, so that the 9 x 8
// weights of the thread's channels are loaded once, into registers.  Interior pixels (2 <= y <=
// H-3, 2 <= x <= W-3) take refl_taps' three taps per axis in its order -- (y-1, tap 2), (y, 1),
// (y+1, 0) -- with those registers; the border pixels walk refl_taps and read the weights from
// memory.  Same products in the same order either way.  I: the pixel index type (int when B x H
// x W fits 31 bits, chosen by the host; memory offsets are size_t).
template <typename I>
__global__ __launch_bounds__(256) void dgrad_final_kernel(const float *G, const float *WT, const float *mask,
                                                          float *dX, int B, int H, int W, int C,
                                                          unsigned *amax, unsigned *ticket = nullptr,
                                                          float *scl = nullptr) {
    const int c8 = C >> 3, ppb = 256 / c8;                     // threads per pixel, pixels per block-step
    const bool lane_on = (int)threadIdx.x < ppb * c8;
    const int c = ((int)threadIdx.x % c8) * 8;
    float4 wr0[9], wr1[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        wr0[t] = *reinterpret_cast<const float4 *>(WT + t * C + c);
        wr1[t] = *reinterpret_cast<const float4 *>(WT + t * C + c + 4);
    }
    const I plane = (I)H * W, npix = (I)B * plane;
    float mx = 0.0f;
    for (I pix = (I)blockIdx.x * ppb + (I)threadIdx.x / c8; lane_on && pix < npix; pix += (I)gridDim.x * ppb) {
        const I b = pix / plane, r = pix - b * plane;
        const int y = (int)(r / W), x = (int)(r - (I)y * W);
        const float *g = G + (size_t)b * plane;
        float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
        auto tap = [&](float gv, const float4 &w0, const float4 &w1) __attribute__((always_inline)) {
            s0.x = fmaf(gv, w0.x, s0.x); s0.y = fmaf(gv, w0.y, s0.y); s0.z = fmaf(gv, w0.z, s0.z); s0.w = fmaf(gv, w0.w, s0.w);
            s1.x = fmaf(gv, w1.x, s1.x); s1.y = fmaf(gv, w1.y, s1.y); s1.z = fmaf(gv, w1.z, s1.z); s1.w = fmaf(gv, w1.w, s1.w);
        };
        if (y >= 2 && y <= H - 3 && x >= 2 && x <= W - 3) {
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int t = (2 - i) * 3 + (2 - j);
                    tap(g[(size_t)(y - 1 + i) * W + (x - 1 + j)], wr0[t], wr1[t]);
                }
        } else {
            int Py[6], Ty[6], Px[6], Tx[6];
            const int ny = refl_taps(y, H, H, 1, Py, Ty), nx = refl_taps(x, W, W, 1, Px, Tx);
            for (int i = 0; i < ny; ++i)
                for (int j = 0; j < nx; ++j) {
                    const float *w = WT + (Ty[i] * 3 + Tx[j]) * C + c;
                    tap(g[(size_t)Py[i] * W + Px[j]], *reinterpret_cast<const float4 *>(w),
                        *reinterpret_cast<const float4 *>(w + 4));
                }
        }
        const size_t o = (size_t)pix * C + c;
        const float4 m0 = *reinterpret_cast<const float4 *>(mask + o), m1 = *reinterpret_cast<const float4 *>(mask + o + 4);
        s0.x = m0.x > 0.0f ? s0.x : 0.0f; s0.y = m0.y > 0.0f ? s0.y : 0.0f;
        s0.z = m0.z > 0.0f ? s0.z : 0.0f; s0.w = m0.w > 0.0f ? s0.w : 0.0f;
        s1.x = m1.x > 0.0f ? s1.x : 0.0f; s1.y = m1.y > 0.0f ? s1.y : 0.0f;
        s1.z = m1.z > 0.0f ? s1.z : 0.0f; s1.w = m1.w > 0.0f ? s1.w : 0.0f;
        *reinterpret_cast<float4 *>(dX + o) = s0;
        *reinterpret_cast<float4 *>(dX + o + 4) = s1;
        mx = amax4f(amax4f(mx, s0), s1);
    }
    if (amax && scl) {                        // the scale pair from the last block (ticket_scale)
        __shared__ float red4[4];
        amax_block(red4, mx);
        ticket_scale(red4, amax, ticket, scl);
    } else if (amax) {
        amax_publish(amax, mx);
    }
}

// W0 (stride 2) dgrad on the zero-padded input domain: dxp (B, H+2, W+2, Cin) gets
//   dxp[qy][qx] = sum over taps (ty, tx) with qy = 2 Py + ty, qx = 2 Px + tx of G[Py][Px] . W[t]
// (reflect folding follows in fold_reflect_kernel).  A thread owns 8 input channels of NJ = 8
// same-parity columns qx = px + 2 (NJ xg + j), which share the tap set: per 4 output channels a
// tap costs 8 weight float4 + NJ gradient float4 loads for 256 FMAs (the 4 x 4 version was bound
// by the CU's vector-memory address rate: 8 loads per 64 FMAs, 250 us at B = 8).
// G (B, h, w, Gc) NHWC, WT [9][Cout][Cin]; Cin % 8, Cout, Gc, Goff % 4 == 0.
constexpr int S2_NJ = 8;
__global__ __launch_bounds__(256) void dgrad_s2_kernel(const float *G, int Gc, int Goff, const float *WT, int Cout,
                                                       int Cin, int B, int h, int w, float *dxp, int Hp, int Wp) {
    const int cq = Cin >> 3;
    const int ngx = (((Wp + 1) >> 1) + S2_NJ - 1) / S2_NJ;
    const long total = (long)B * Hp * 2 * ngx * cq;
    long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int ci = (int)(idx % cq) * 8;
    idx /= cq;
    const int xg = (int)(idx % ngx);
    idx /= ngx;
    const int px = (int)(idx & 1);
    idx >>= 1;
    const int qy = (int)(idx % Hp);
    const int b = (int)(idx / Hp);
    const int cnt = (Wp - px + 1) >> 1;
    if (S2_NJ * xg >= cnt) return;
    float4 acc[S2_NJ][2];
#pragma unroll
    for (int j = 0; j < S2_NJ; ++j) acc[j][0] = acc[j][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int ty = 0; ty < 3; ++ty) {
        if ((qy - ty) & 1) continue;
        const int Py = (qy - ty) >> 1;
        if (Py < 0 || Py >= h) continue;
        const float *grow = G + ((size_t)b * h + Py) * w * Gc + Goff;
        for (int tx = px; tx < 3; tx += 2) {
            const int pofs = S2_NJ * xg + ((px - tx) >> 1);     // Px of column j = pofs + j
            bool ok[S2_NJ];
            const float *gp[S2_NJ];
#pragma unroll
            for (int j = 0; j < S2_NJ; ++j) {
                const int Px = pofs + j;
                ok[j] = Px >= 0 && Px < w && S2_NJ * xg + j < cnt;
                gp[j] = grow + (size_t)(ok[j] ? Px : 0) * Gc;
            }
            const float *wt = WT + (size_t)(ty * 3 + tx) * Cout * Cin + ci;
            for (int co = 0; co < Cout; co += 4) {
                float4 wv[4][2];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    wv[k][0] = *reinterpret_cast<const float4 *>(wt + (size_t)(co + k) * Cin);
                    wv[k][1] = *reinterpret_cast<const float4 *>(wt + (size_t)(co + k) * Cin + 4);
                }
#pragma unroll
                for (int j = 0; j < S2_NJ; ++j) {
                    float4 g = *reinterpret_cast<const float4 *>(gp[j] + co);
                    if (!ok[j]) g = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh) {
                        float4 &A = acc[j][hh];
                        A.x = fmaf(g.x, wv[0][hh].x, fmaf(g.y, wv[1][hh].x, fmaf(g.z, wv[2][hh].x, fmaf(g.w, wv[3][hh].x, A.x))));
                        A.y = fmaf(g.x, wv[0][hh].y, fmaf(g.y, wv[1][hh].y, fmaf(g.z, wv[2][hh].y, fmaf(g.w, wv[3][hh].y, A.y))));
                        A.z = fmaf(g.x, wv[0][hh].z, fmaf(g.y, wv[1][hh].z, fmaf(g.z, wv[2][hh].z, fmaf(g.w, wv[3][hh].z, A.z))));
                        A.w = fmaf(g.x, wv[0][hh].w, fmaf(g.y, wv[1][hh].w, fmaf(g.z, wv[2][hh].w, fmaf(g.w, wv[3][hh].w, A.w))));
                    }
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < S2_NJ; ++j) {
        const int qx = px + 2 * (S2_NJ * xg + j);
        if (qx < Wp) {
            float *o = dxp + (((size_t)b * Hp + qy) * Wp + qx) * Cin + ci;
            *reinterpret_cast<float4 *>(o) = acc[j][0];
            *reinterpret_cast<float4 *>(o + 4) = acc[j][1];
        }
    }
}

// --------------------------------------------------------------------------------------------
// elementwise backward tails
// --------------------------------------------------------------------------------------------
// rec = sigmoid(pre): g_pre = g_rec * rec * (1 - rec)
__global__ void sigmoid_bwd_kernel(const float *g, const float *y, float *out, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = g[i] * y[i] * (1.0f - y[i]);
}

// ConvLSTM cell backward (reference base_layers.py:112-128), per (pixel, channel):
// gates saved post-activation [i | r | o | g] (4C, original order); gh, gc: grads of h, c
// (gc may be NULL); c_prev may be NULL (zeros).  Writes G (4C, pre-activation grads, original
// order) and g_c_prev (C; skipped when NULL).
__global__ void lstm_bwd_kernel(const float *gates, const float *c, const float *c_prev,
                                const float *gh, const float *gc, float *G, float *gcp, long npix,
                                int C, unsigned *amax) {
    const long idx0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = idx0 < npix * C;
    if (!amax && !live) return;
    const long idx = live ? idx0 : npix * C - 1;
    const long p = idx / C;
    const int ch = (int)(idx % C);
    const float *gt = gates + p * 4 * C;
    const float i = gt[ch], r = gt[C + ch], o = gt[2 * C + ch], g = gt[3 * C + ch];
    const float cc = c[idx];
    const float cp = c_prev ? c_prev[idx] : 0.0f;
    const float th = gate_tanh(cc);
    const float dh = gh ? gh[idx] : 0.0f;
    const float dc = (gc ? gc[idx] : 0.0f) + dh * o * (1.0f - th * th);
    float *Gp = G + p * 4 * C;
    const float v0 = dc * g * i * (1.0f - i), v1 = dc * cp * r * (1.0f - r);
    const float v2 = dh * th * o * (1.0f - o), v3 = dc * i * (1.0f - g * g);
    if (live) {
        Gp[ch] = v0;
        Gp[C + ch] = v1;
        Gp[2 * C + ch] = v2;
        Gp[3 * C + ch] = v3;
        if (gcp) gcp[idx] = dc * r;
    }
    if (amax) amax_publish(amax, live ? amax4f(0.0f, make_float4(v0, v1, v2, v3)) : 0.0f);
}

// softshrink backward (reference base_layers.py:11-12): z = relu(v-l) - relu(-v-l)
// gv = gz * ([v > l] + [v < -l]);  dl_partial[block][c] = sum gz * (-[v > l] + [v < -l]).
// Thread -> (pixel, channel) with a grid stride that is a multiple of C (fixed channel per
// thread: the first (256 / C) * C threads of a workgroup work; C <= 256), coalesced over channels.
__global__ __launch_bounds__(256) void softshrink_bwd_kernel(const float *gz, const float *v,
                                                             const float *lam, float *gv,
                                                             float *dl_partial, long npix, int C,
                                                             unsigned *amax) {
    __shared__ float red[256];
    float mx = 0.0f;
    const int c = threadIdx.x % C, nl = (256 / C) * C;
    const float l = lam[c];
    const long total = npix * C;
    float acc = 0.0f;
    for (long i = (long)blockIdx.x * nl + threadIdx.x; (int)threadIdx.x < nl && i < total; i += (long)gridDim.x * nl) {
        const float vv = v[i], g = gz[i];
        const bool up = vv > l, dn = vv < -l;
        gv[i] = g * ((up ? 1.0f : 0.0f) + (dn ? 1.0f : 0.0f));
        mx = fmaxf(mx, fabsf(gv[i]));
        acc += g * ((dn ? 1.0f : 0.0f) - (up ? 1.0f : 0.0f));
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if ((int)threadIdx.x < C) {
        float s = 0.0f;
        for (int k = threadIdx.x; k < nl; k += C) s += red[k];
        dl_partial[(size_t)blockIdx.x * C + threadIdx.x] = s;
    }
    if (amax) amax_publish(amax, mx);
}

// softshrink_bwd_kernel over float4 channel groups (C % 4 == 0, C <= 1024): the same gv and, per
// workgroup, the same dlambda partials up to the order of the per-channel sums.  The first
// (256 / (C/4)) * (C/4) threads work (all 256 when 1024 % C == 0).
__global__ __launch_bounds__(256) void softshrink_bwd4_kernel(const float *gz, const float *v,
                                                              const float *lam, float *gv,
                                                              float *dl_partial, long npix, int C,
                                                              unsigned *amax, unsigned *ticket = nullptr,
                                                              float *scl = nullptr) {
    __shared__ float4 red[256];
    float mx = 0.0f;
    const int cq = C >> 2, c = (threadIdx.x % cq) * 4, nl = (256 / cq) * cq;
    const float4 l = *reinterpret_cast<const float4 *>(lam + c);
    const long total = npix * cq;
    const float4 *v4 = reinterpret_cast<const float4 *>(v), *g4 = reinterpret_cast<const float4 *>(gz);
    float4 *o4 = reinterpret_cast<float4 *>(gv);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    auto one = [](float vv, float g, float lv, float &a) {
        const bool up = vv > lv, dn = vv < -lv;
        a += g * ((dn ? 1.0f : 0.0f) - (up ? 1.0f : 0.0f));
        return g * ((up ? 1.0f : 0.0f) + (dn ? 1.0f : 0.0f));
    };
    for (long i = (long)blockIdx.x * nl + threadIdx.x; (int)threadIdx.x < nl && i < total; i += (long)gridDim.x * nl) {
        const float4 vv = v4[i], g = g4[i];
        float4 r;
        r.x = one(vv.x, g.x, l.x, acc.x);
        r.y = one(vv.y, g.y, l.y, acc.y);
        r.z = one(vv.z, g.z, l.z, acc.z);
        r.w = one(vv.w, g.w, l.w, acc.w);
        o4[i] = r;
        mx = amax4f(mx, r);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if ((int)threadIdx.x < cq) {
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int k = threadIdx.x; k < nl; k += cq) {
            s.x += red[k].x; s.y += red[k].y; s.z += red[k].z; s.w += red[k].w;
        }
        *reinterpret_cast<float4 *>(dl_partial + (size_t)blockIdx.x * C + 4 * threadIdx.x) = s;
    }
    if (amax && scl) {
        __shared__ float red4[4];
        amax_block(red4, mx);
        ticket_scale(red4, amax, ticket, scl);
    } else if (amax) {
        amax_publish(amax, mx);
    }
}

// dlambda[c] (+)= sum over the nbl per-block partials ([block][c]) of softshrink_bwd_kernel;
// one workgroup per channel, tree reduction
// dst[c] = sum over the ISTA iterations, the last one first (the backward's order), of the
// per-block partials dlp[it][b][c] -- the fixed-order block sum of each iteration, then the
// running sum over iterations (one launch for all of them, after the ISTA loop)
__global__ __launch_bounds__(256) void lambda_grad_kernel(const float *dlp, int nbl, int C, int niter, float *dst) {
    __shared__ float red[256];
    const int c = blockIdx.x;
    float acc = 0.0f;
    for (int it = niter - 1; it >= 0; --it) {
        const float *p = dlp + (size_t)it * nbl * C;
        float s = 0.0f;
        for (int b = threadIdx.x; b < nbl; b += 256) s += p[(size_t)b * C + c];
        __syncthreads();                       // the previous iteration's red[0] has been read
        red[threadIdx.x] = s;
        __syncthreads();
        for (int k = 128; k > 0; k >>= 1) {
            if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
            __syncthreads();
        }
        acc = acc + red[0];                    // the first: 0 + s, as a fresh accumulation
    }
    if (threadIdx.x == 0) dst[c] = acc;
}

// ConvLSTC cell backward (reference base_layers.py:52-71), per (pixel, channel), Cz = 2C:
// saved i, f (post-sigmoid, Cz each), o (Cz), z0, c (cell), c_prev (nullable);
// gz: grad of the LSTC output z (= ISTA z_0); gcl: grad of c (from the next frame, nullable).
// Writes Gg (2*Cz: [gi | gf] pre-activation), Go (Cz), gz0 (Cz, cell part: = dc * i),
// gcp (Cz, nullable).
__global__ void lstc_bwd_kernel(const float *gi_, const float *gf_, const float *go_, const float *z0,
                                const float *c, const float *c_prev, const float *gz, const float *gcl,
                                float *Gg, float *Go, float *gz0, float *gcp, long npix, int Cz,
                                unsigned *amax_go, unsigned *amax_gg) {
    const long idx0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = idx0 < npix * Cz;
    if (!amax_go && !live) return;
    const long idx = live ? idx0 : npix * Cz - 1;
    const long p = idx / Cz;
    const int ch = (int)(idx % Cz);
    const float i = gi_[idx], f = gf_[idx], o = go_[idx];
    const float cc = c[idx], th = gate_tanh(cc);
    const float cp = c_prev ? c_prev[idx] : 0.0f;
    const float dz = gz[idx];
    const float dc = (gcl ? gcl[idx] : 0.0f) + dz * o * (1.0f - th * th);
    const float vo = dz * th * o * (1.0f - o);
    const float vi = dc * z0[idx] * i * (1.0f - i), vf = dc * cp * f * (1.0f - f);
    if (live) {
        Go[idx] = vo;
        Gg[p * 2 * Cz + ch] = vi;
        Gg[p * 2 * Cz + Cz + ch] = vf;
        gz0[idx] = dc * i;
        if (gcp) gcp[idx] = dc * f;
    }
    if (amax_go) {                              // both or neither (the host passes both)
        amax_publish(amax_go, live ? fabsf(vo) : 0.0f);
        amax_publish(amax_gg, live ? fmaxf(fabsf(vi), fabsf(vf)) : 0.0f);
    }
}

// bilinear x2 (align_corners=False) backward: gh[b,y,x,c] (+)= sum over up-pixels (Y, X) of
// gup[b,Y,X,c] * wy(Y->y) * wx(X->x), with the forward's weights (reference base_layers.py:198)
__device__ __forceinline__ int up_weights(int y, int n, float (&w)[6], int (&Y)[6]) {
    int k = 0;
    for (int yy = 2 * y - 2; yy <= 2 * y + 3; ++yy) {
        if (yy < 0 || yy >= 2 * n) continue;
        const float sy = fmaxf(((float)yy + 0.5f) * 0.5f - 0.5f, 0.0f);
        const int y0 = (int)sy;
        const int y1 = y0 + (y0 < n - 1 ? 1 : 0);
        const float l1 = sy - (float)y0, l0 = 1.0f - l1;
        float wt = 0.0f;
        if (y0 == y) wt += l0;
        if (y1 == y) wt += l1;
        if (wt != 0.0f && k < 6) {
            w[k] = wt;
            Y[k] = yy;
            ++k;
        }
    }
    return k;
}

// thread = (half-res pixel, 4 channels): the tap weights once per 4 channels, float4 loads; the
// per-channel sums keep the scalar kernel's order (rows i, then columns j)
template <typename I>     // the element index type (int when the count fits 31 bits)
__global__ void upsample_bwd_kernel(const float *gup, float *gh, int B, int h, int w, int C,
                                    int accumulate) {
    const int cq = C >> 2;
    const I total = (I)B * h * w * cq;
    const I idx = (I)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int c = (int)(idx % cq) * 4;
    const I pix = idx / cq;
    const int plane = h * w;
    const int b = (int)(pix / plane), r = (int)(pix - (I)b * plane);
    const int y = r / w, x = r - y * w;
    float wy[6], wx[6];
    int Ys[6], Xs[6];
    const int ny = up_weights(y, h, wy, Ys), nx = up_weights(x, w, wx, Xs);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = 0; i < ny; ++i) {
        const float *row = gup + (((size_t)b * 2 * h + Ys[i]) * 2 * w) * C + c;
        float4 sr = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int j = 0; j < nx; ++j) {
            const float4 v = *reinterpret_cast<const float4 *>(row + (size_t)Xs[j] * C);
            sr.x += v.x * wx[j]; sr.y += v.y * wx[j]; sr.z += v.z * wx[j]; sr.w += v.w * wx[j];
        }
        s.x += sr.x * wy[i]; s.y += sr.y * wy[i]; s.z += sr.z * wy[i]; s.w += sr.w * wy[i];
    }
    float4 *o = reinterpret_cast<float4 *>(gh + (size_t)pix * C + c);
    if (accumulate) {
        const float4 d = *o;
        s.x = d.x + s.x; s.y = d.y + s.y; s.z = d.z + s.z; s.w = d.w + s.w;
    }
    *o = s;
}

// a = a * (b > 0)   (ReLU mask, elementwise, n floats)
__global__ void relu_mask_kernel(float *a, const float *b, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && !(b[i] > 0.0f)) a[i] = 0.0f;
}

}  // namespace cista
