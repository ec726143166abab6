/*
 * cista_loss.h -- C ABI of the training-loss kernels (part of
 * libcista_hip.so, gfx950).
 *
 * SSIM as used by the reference's training loops: `pytorch_msssim.SSIM(data_range=1,
 * size_average=True, channel=1, nonnegative_ssim=False)` and `loss_ssim = 1 - ssim(output, gt)`
 * (reference train_e2v.py:27,70,119; train.py:23,76,131).  pytorch_msssim is a third-party
 * dependency pinned at 0.2.1 (reference requirements.txt:10) and is NOT vendored in the
 * reference; this restates its published algorithm:
 *
 *   win      = 1-D Gaussian, size win_size (11), sigma 1.5, normalised to sum 1 (float32)
 *   filter   = valid (no padding) separable correlation with win: along H, then along W
 *   mu1 = f(X), mu2 = f(Y), s11 = f(X*X) - mu1^2, s22 = f(Y*Y) - mu2^2, s12 = f(X*Y) - mu1*mu2
 *   cs_map   = (2 s12 + C2) / (s11 + s22 + C2),  C1 = (K1 R)^2, C2 = (K2 R)^2, R = data_range
 *   ssim_map = (2 mu1 mu2 + C1) / (mu1^2 + mu2^2 + C1) * cs_map
 *   ssim[n, c] = mean of ssim_map over the (H - win + 1) x (W - win + 1) valid positions
 *
 * The backward gives d loss / dX for an upstream gradient per (n, c); the target Y takes no
 * gradient (it is the ground-truth frame in the reference).  size_average and nonnegative_ssim
 * (a relu on ssim[n, c]) are host-side reductions of ssim_out (v2e2v_amd/losses.py).
 *
 * Conventions as in cista_lstc.h: device pointers (fp32, NCHW), `stream` = hipStream_t as void*,
 * no allocation, no host sync; CISTA_* status codes.
 */
#ifndef CISTA_LOSS_H
#define CISTA_LOSS_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CISTA_SSIM_MAX_WIN 31

typedef struct {
    int win_size;                      /* odd, <= CISTA_SSIM_MAX_WIN, <= H and <= W            */
    float win[CISTA_SSIM_MAX_WIN];     /* the 1-D window (host values, passed by value)         */
    double data_range;                 /* R; C1 = float((K1 R)^2), C2 = float((K2 R)^2) as the   */
    double K1, K2;                     /* reference's Python-float constants (0.01, 0.03)       */
} cista_ssim_config;

size_t cista_ssim_workspace_bytes(int N, int C, int H, int W, int win_size);

/* ssim_out[n*C + c] = SSIM of image (n, c); cs_out (optional, may be NULL) = mean of cs_map */
int cista_ssim_forward(const cista_ssim_config *cfg, const float *X, const float *Y, int N, int C, int H, int W,
                       float *ssim_out, float *cs_out, void *workspace, size_t workspace_bytes, void *stream);

/* grad_X = sum over (n, c) of g_ssim[n*C + c] * d ssim[n, c] / d X  (written, not accumulated) */
int cista_ssim_backward(const cista_ssim_config *cfg, const float *X, const float *Y, int N, int C, int H, int W,
                        const float *g_ssim, float *grad_X, void *workspace, size_t workspace_bytes, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CISTA_LOSS_H */
