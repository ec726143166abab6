// SSIM loss forward/backward for the training loop; contract and the restated
// pytorch_msssim 0.2.1 algorithm in include/cista_loss.h.
//
// The valid separable Gaussian filter is two passes through HBM-resident planes (the frames are
// 0.17 MB each, so every plane stays in L2): a vertical pass over the 5 moments
// (X, Y, X^2, Y^2, XY), a horizontal pass that forms the SSIM map -- or, in the backward, the
// three per-position derivatives dS/dmu1, dS/dE[X^2], dS/dE[XY] -- and, in the backward, the
// transposed (full) horizontal and vertical passes that scatter them back onto X.
// Per-image means are deterministic tree reductions (one workgroup per image).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "../../include/cista_lstc.h"
#include "../../include/cista_loss.h"

namespace cista_ssim {

struct Win {
    float w[CISTA_SSIM_MAX_WIN];
    int n;
};

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

struct Ws {
    float *V;    // [5][NC][Ho][W]   vertical moments
    float *M;    // [2][NC][Ho][Wo]  ssim map, cs map   | backward: [3][NC][Ho][Wo] derivative maps
    float *T;    // [3][NC][Ho][W]   backward: transposed horizontal pass
    size_t bytes;
};

Ws carve(void *base, int NC, int H, int W, int ws) {
    const size_t Ho = H - ws + 1, Wo = W - ws + 1;
    Ws s;
    size_t off = 0;
    char *p = static_cast<char *>(base);
    auto take = [&](size_t nf) {
        float *r = p ? reinterpret_cast<float *>(p + off) : nullptr;
        off = align_up(off + nf * 4);
        return r;
    };
    s.V = take(5 * (size_t)NC * Ho * W);
    s.M = take(3 * (size_t)NC * Ho * Wo);
    s.T = take(3 * (size_t)NC * Ho * W);
    s.bytes = off;
    return s;
}

inline dim3 g1d(long long n) { return dim3((unsigned)((n + 255) / 256)); }

// V[q][nc][y][x] = sum_k w[k] * m_q(y + k, x),  m = (X, Y, X*X, Y*Y, X*Y)
__global__ void ssim_vpass_kernel(const float *X, const float *Y, int NC, int H, int W, Win win, float *V) {
    const int Ho = H - win.n + 1;
    const long long plane = (long long)NC * Ho * W;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= plane) return;
    const int x = (int)(i % W);
    const int y = (int)((i / W) % Ho);
    const long long nc = i / ((long long)W * Ho);
    const float *xp = X + (size_t)nc * H * W + (size_t)y * W + x;
    const float *yp = Y + (size_t)nc * H * W + (size_t)y * W + x;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
    for (int k = 0; k < win.n; ++k) {
        const float a = xp[(size_t)k * W], b = yp[(size_t)k * W], w = win.w[k];
        s0 += w * a;
        s1 += w * b;
        s2 += w * (a * a);
        s3 += w * (b * b);
        s4 += w * (a * b);
    }
    V[i] = s0;
    V[plane + i] = s1;
    V[2 * plane + i] = s2;
    V[3 * plane + i] = s3;
    V[4 * plane + i] = s4;
}

struct Moments {
    float m1, m2, e11, e22, e12;
};

__device__ __forceinline__ Moments hsum(const float *V, long long plane, long long row, int x, const Win &win) {
    Moments m{0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < win.n; ++k) {
        const long long o = row + x + k;
        const float w = win.w[k];
        m.m1 += w * V[o];
        m.m2 += w * V[plane + o];
        m.e11 += w * V[2 * plane + o];
        m.e22 += w * V[3 * plane + o];
        m.e12 += w * V[4 * plane + o];
    }
    return m;
}

// forward: ssim_map and cs_map (pytorch_msssim _ssim, same operation order)
__global__ void ssim_hpass_kernel(const float *V, int NC, int H, int W, Win win, float C1, float C2, float *S,
                                  float *CS) {
    const int Ho = H - win.n + 1, Wo = W - win.n + 1;
    const long long n = (long long)NC * Ho * Wo;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int x = (int)(i % Wo);
    const long long r = i / Wo;                      // nc * Ho + y
    const Moments m = hsum(V, (long long)NC * Ho * W, r * W, x, win);
    const float mu1_sq = m.m1 * m.m1, mu2_sq = m.m2 * m.m2, mu1_mu2 = m.m1 * m.m2;
    const float s11 = 1.0f * (m.e11 - mu1_sq), s22 = 1.0f * (m.e22 - mu2_sq), s12 = 1.0f * (m.e12 - mu1_mu2);
    const float cs = (2.0f * s12 + C2) / (s11 + s22 + C2);
    S[i] = ((2.0f * mu1_mu2 + C1) / (mu1_sq + mu2_sq + C1)) * cs;
    CS[i] = cs;
}

// one workgroup per image: out[nc] = mean of map[nc] (fixed-order tree reduction)
__global__ __launch_bounds__(256) void ssim_mean_kernel(const float *map, long long per, float *out) {
    __shared__ float red[256];
    const long long nc = blockIdx.x;
    const float *m = map + nc * per;
    float s = 0.0f;
    for (long long i = threadIdx.x; i < per; i += 256) s += m[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[nc] = red[0] / (float)per;
}

// backward: G_q = g[nc] / P * dS/dq at every valid position, q = (mu1, E[X^2], E[XY])
__global__ void ssim_hpass_bwd_kernel(const float *V, int NC, int H, int W, Win win, float C1, float C2,
                                      const float *g, float *G) {
    const int Ho = H - win.n + 1, Wo = W - win.n + 1;
    const long long n = (long long)NC * Ho * Wo;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int x = (int)(i % Wo);
    const long long r = i / Wo;
    const long long nc = r / Ho;
    const Moments m = hsum(V, (long long)NC * Ho * W, r * W, x, win);
    const float mu1_sq = m.m1 * m.m1, mu2_sq = m.m2 * m.m2, mu1_mu2 = m.m1 * m.m2;
    const float s11 = m.e11 - mu1_sq, s22 = m.e22 - mu2_sq, s12 = m.e12 - mu1_mu2;
    const float na = 2.0f * mu1_mu2 + C1, da = mu1_sq + mu2_sq + C1;
    const float nc_ = 2.0f * s12 + C2, dc = s11 + s22 + C2;
    const float A = na / da, CS = nc_ / dc;
    const float dA_dm1 = (2.0f * m.m2 * da - na * 2.0f * m.m1) / (da * da);
    const float dCS_dm1 = (-2.0f * m.m2 * dc + nc_ * 2.0f * m.m1) / (dc * dc);
    const float scale = g[nc] / (float)((long long)Ho * Wo);
    G[i] = scale * (dA_dm1 * CS + A * dCS_dm1);
    G[n + i] = scale * (A * (-nc_ / (dc * dc)));
    G[2 * n + i] = scale * (A * 2.0f / dc);
}

// T_q(y, x) = sum_k w[k] G_q(y, x - k), x in [0, W)
__global__ void ssim_thpass_kernel(const float *G, int NC, int H, int W, Win win, float *T) {
    const int Ho = H - win.n + 1, Wo = W - win.n + 1;
    const long long n = (long long)NC * Ho * W, ng = (long long)NC * Ho * Wo;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int x = (int)(i % W);
    const long long r = i / W;
    float t0 = 0.f, t1 = 0.f, t2 = 0.f;
    for (int k = 0; k < win.n; ++k) {
        const int xs = x - k;
        if (xs < 0 || xs >= Wo) continue;
        const long long o = r * Wo + xs;
        const float w = win.w[k];
        t0 += w * G[o];
        t1 += w * G[ng + o];
        t2 += w * G[2 * ng + o];
    }
    T[i] = t0;
    T[n + i] = t1;
    T[2 * n + i] = t2;
}

// F_q(y, x) = sum_k w[k] T_q(y - k, x);  dX = F_mu1 + 2 X F_e11 + Y F_e12
__global__ void ssim_tvpass_kernel(const float *T, const float *X, const float *Y, int NC, int H, int W, Win win,
                                   float *gX) {
    const int Ho = H - win.n + 1;
    const long long n = (long long)NC * H * W, nt = (long long)NC * Ho * W;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int x = (int)(i % W);
    const int y = (int)((i / W) % H);
    const long long nc = i / ((long long)W * H);
    float f0 = 0.f, f1 = 0.f, f2 = 0.f;
    for (int k = 0; k < win.n; ++k) {
        const int ys = y - k;
        if (ys < 0 || ys >= Ho) continue;
        const long long o = (nc * Ho + ys) * W + x;
        const float w = win.w[k];
        f0 += w * T[o];
        f1 += w * T[nt + o];
        f2 += w * T[2 * nt + o];
    }
    gX[i] = f0 + 2.0f * X[i] * f1 + Y[i] * f2;
}

int check(const cista_ssim_config *cfg, const void *X, const void *Y, int N, int C, int H, int W, Win &win,
          float &C1, float &C2) {
    if (!cfg || !X || !Y || N <= 0 || C <= 0) return CISTA_ERR_INVALID;
    if (cfg->win_size <= 0 || cfg->win_size > CISTA_SSIM_MAX_WIN || (cfg->win_size & 1) == 0) return CISTA_ERR_INVALID;
    if (H < cfg->win_size || W < cfg->win_size) return CISTA_ERR_INVALID;
    win.n = cfg->win_size;
    for (int k = 0; k < CISTA_SSIM_MAX_WIN; ++k) win.w[k] = k < win.n ? cfg->win[k] : 0.0f;
    const double c1 = cfg->K1 * cfg->data_range, c2 = cfg->K2 * cfg->data_range;
    C1 = (float)(c1 * c1);
    C2 = (float)(c2 * c2);
    return CISTA_OK;
}

}  // namespace cista_ssim

using namespace cista_ssim;

extern "C" {

size_t cista_ssim_workspace_bytes(int N, int C, int H, int W, int win_size) {
    if (N <= 0 || C <= 0 || win_size <= 0 || H < win_size || W < win_size) return 0;
    return carve(nullptr, N * C, H, W, win_size).bytes;
}

int cista_ssim_forward(const cista_ssim_config *cfg, const float *X, const float *Y, int N, int C, int H, int W,
                       float *ssim_out, float *cs_out, void *workspace, size_t workspace_bytes, void *stream) {
    Win win;
    float C1, C2;
    int st = check(cfg, X, Y, N, C, H, W, win, C1, C2);
    if (st != CISTA_OK) return st;
    if (!ssim_out || !workspace) return CISTA_ERR_INVALID;
    const int NC = N * C, Ho = H - win.n + 1, Wo = W - win.n + 1;
    const Ws w = carve(workspace, NC, H, W, win.n);
    if (workspace_bytes < w.bytes) return CISTA_ERR_WORKSPACE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const long long per = (long long)Ho * Wo;
    hipLaunchKernelGGL(ssim_vpass_kernel, g1d((long long)NC * Ho * W), dim3(256), 0, s, X, Y, NC, H, W, win, w.V);
    float *S = w.M, *CSm = w.M + (size_t)NC * per;
    hipLaunchKernelGGL(ssim_hpass_kernel, g1d(NC * per), dim3(256), 0, s, (const float *)w.V, NC, H, W, win, C1, C2,
                       S, CSm);
    hipLaunchKernelGGL(ssim_mean_kernel, dim3(NC), dim3(256), 0, s, (const float *)S, per, ssim_out);
    if (cs_out) hipLaunchKernelGGL(ssim_mean_kernel, dim3(NC), dim3(256), 0, s, (const float *)CSm, per, cs_out);
    return hipGetLastError() == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
}

int cista_ssim_backward(const cista_ssim_config *cfg, const float *X, const float *Y, int N, int C, int H, int W,
                        const float *g_ssim, float *grad_X, void *workspace, size_t workspace_bytes, void *stream) {
    Win win;
    float C1, C2;
    int st = check(cfg, X, Y, N, C, H, W, win, C1, C2);
    if (st != CISTA_OK) return st;
    if (!g_ssim || !grad_X || !workspace) return CISTA_ERR_INVALID;
    const int NC = N * C, Ho = H - win.n + 1, Wo = W - win.n + 1;
    const Ws w = carve(workspace, NC, H, W, win.n);
    if (workspace_bytes < w.bytes) return CISTA_ERR_WORKSPACE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(ssim_vpass_kernel, g1d((long long)NC * Ho * W), dim3(256), 0, s, X, Y, NC, H, W, win, w.V);
    hipLaunchKernelGGL(ssim_hpass_bwd_kernel, g1d((long long)NC * Ho * Wo), dim3(256), 0, s, (const float *)w.V, NC, H,
                       W, win, C1, C2, g_ssim, w.M);
    hipLaunchKernelGGL(ssim_thpass_kernel, g1d((long long)NC * Ho * W), dim3(256), 0, s, (const float *)w.M, NC, H,
                       W, win, w.T);
    hipLaunchKernelGGL(ssim_tvpass_kernel, g1d((long long)NC * H * W), dim3(256), 0, s, (const float *)w.T, X, Y, NC,
                       H, W, win, grad_X);
    return hipGetLastError() == hipSuccess ? CISTA_OK : CISTA_ERR_HIP;
}

}  // extern "C"
