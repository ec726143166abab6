/*
 * cista_lstc.h -- C ABI of the MI355X-native CISTA-LSTC event-to-video hot path
 * (libcista_hip.so, built for gfx950).
 *
 * The reference exposes this path only as a Python nn.Module (lsying009/V2E2V has no native
 * code and no FFI), so each entry point below replaces one reference Python call site; a
 * ctypes binding (v2e2v_amd/_lib.py) sits between them and the unchanged
 * `CistaLSTCNet` surface:
 *
 *   cista_pack_params      <- nn.Conv2d parameter storage of CistaLSTCNet.__init__
 *                             (reference e2v/e2v_model.py:6-38); re-run after every
 *                             load_state_dict / optimizer step (weights -> split-fp16 MFMA fragments)
 *   cista_forward          <- CistaLSTCNet.forward(events, prev_image, prev_states)
 *                             (reference e2v/e2v_model.py:41-90)
 *   cista_stage_input      <- We / Wi / cat / W0                 (e2v_model.py:62-66)
 *   cista_stage_lstc       <- ConvLSTC.forward                   (e2v/base_layers.py:52-71)
 *   cista_stage_ista       <- tied IstaBlock loop + softshrink   (e2v_model.py:72-78,
 *                                                                  base_layers.py:11-12)
 *   cista_stage_decoder    <- RecurrentConvLayer + ConvLSTM      (base_layers.py:214-225,90-130)
 *   cista_stage_output     <- UpsampleConvLayer + final_conv + sigmoid
 *                                                                 (base_layers.py:193-210,
 *                                                                  e2v_model.py:85-88)
 *
 * Conventions (all functions):
 *   - plain C types only; `stream` is a hipStream_t passed as void* (NULL = legacy default);
 *   - every tensor argument is a DEVICE pointer to fp32 data;
 *   - events (B, num_bins, H, W) and frames (B, 1, H, W) are NCHW (== the module surface);
 *     recurrent states are NHWC ("channels_last"), half resolution h = H/2, w = W/2:
 *       c_lstc, z : (B, h, w, 2*C)        h, c : (B, h, w, C)
 *   - a NULL previous-state pointer means "None" in the reference (zeros), per state;
 *   - outputs never alias inputs (checked: CISTA_ERR_ALIAS); inputs are never written;
 *   - work is only enqueued on `stream` (no host sync, no allocation) -> graph-capturable;
 *   - return value: CISTA_OK or an error code; cista_status_string() describes it.  The Python
 *     shim turns every non-zero status into a RuntimeError, like the reference's torch errors.
 */
#ifndef CISTA_LSTC_H
#define CISTA_LSTC_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CISTA_ABI_VERSION 3

enum {
    CISTA_OK = 0,
    CISTA_ERR_INVALID = 1,      /* bad shape / NULL pointer / inconsistent arguments        */
    CISTA_ERR_UNSUPPORTED = 2,  /* valid in the reference but not built here (e.g. C % 32)  */
    CISTA_ERR_HIP = 3,          /* a HIP runtime call failed                                */
    CISTA_ERR_WORKSPACE = 4,    /* workspace smaller than cista_workspace_bytes()           */
    CISTA_ERR_ALIAS = 5         /* an output buffer overlaps an input buffer                */
};

/* CistaLSTCNet(image_dim, base_channels, depth, num_bins) -- image_dim is unused by the
 * reference forward (e2v_model.py:13), so it is not part of the config. */
typedef struct {
    int base_channels;   /* C; this build requires C % 32 == 0 (reference default 64) */
    int depth;           /* ISTA iterations (tied weights), >= 0                        */
    int num_bins;        /* voxel bins, >= 1                                            */
} cista_config;

/* The 25 UNIQUE parameter tensors, device fp32, reference layouts
 * (conv weight [Cout][Cin][3][3], bias [Cout], Lambda [1][2C][1][1]).
 * Gate orders follow the reference: P0.gates = (in, forget) (base_layers.py:58),
 * Dg.recurrent_block.Gates = (in, remember, out, cell) (base_layers.py:116). */
typedef struct {
    const float *We_w, *We_b;                 /* We.conv2d            [C/2][nb][3][3]   */
    const float *Wi_w, *Wi_b;                 /* Wi.conv2d            [C/2][1][3][3]    */
    const float *W0_w, *W0_b;                 /* W0.conv2d            [C][C][3][3], s2  */
    const float *gates_w, *gates_b;           /* P0.gates             [4C][3C][3][3]    */
    const float *out_gates_w, *out_gates_b;   /* P0.out_gates         [2C][4C][3][3]    */
    const float *P0_w, *P0_b;                 /* P0.P0                [2C][C][3][3]     */
    const float *lambda;                      /* lista_blocks.*.Lambda [1][2C][1][1]    */
    const float *D_w, *D_b;                   /* lista_blocks.*.D     [C][2C][3][3]     */
    const float *P_w, *P_b;                   /* lista_blocks.*.P     [2C][C][3][3]     */
    const float *Dg_w, *Dg_b;                 /* Dg.conv.conv2d       [C][2C][3][3]     */
    const float *lstm_w, *lstm_b;             /* Dg.recurrent_block.Gates [4C][2C][3][3]*/
    const float *up_w, *up_b;                 /* upsamp_conv.conv2d   [C][C][3][3]      */
    const float *final_w, *final_b;           /* final_conv.conv2d    [1][C][3][3]      */
} cista_params;

typedef struct {
    const float *events;       /* (B, nb, H, W) NCHW                                 */
    const float *prev_image;   /* (B, 1, H, W)                                       */
    const float *c_lstc_prev;  /* prev_states[0]    NHWC (B,h,w,2C) or NULL          */
    const float *z_prev;       /* prev_states[1]    NHWC (B,h,w,2C) or NULL          */
    const float *h_prev;       /* prev_states[2][0] NHWC (B,h,w,C)  or NULL          */
    const float *c_prev;       /* prev_states[2][1] NHWC (B,h,w,C)  (NULL iff h_prev)*/
    float *rec;                /* out (B, 1, H, W) in (0, 1)                          */
    float *c_lstc;             /* out states[0] NHWC (B,h,w,2C)                       */
    float *z;                  /* out states[1] NHWC (B,h,w,2C)                       */
    float *h;                  /* out states[2][0] NHWC (B,h,w,C)                     */
    float *c;                  /* out states[2][1] NHWC (B,h,w,C)                     */
} cista_frame_io;

int         cista_abi_version(void);
const char *cista_status_string(int status);

/* packed (MFMA-fragment, split-fp16) parameter blob */
size_t cista_packed_bytes(const cista_config *cfg);
int    cista_pack_params(const cista_config *cfg, const cista_params *params, void *packed,
                         void *stream);

/* scratch needed by cista_forward / the stage entries for one (B, H, W) */
size_t cista_workspace_bytes(const cista_config *cfg, int B, int H, int W);

/* Range.  The split-fp16 MFMA path has no range limit a caller must respect: a conv tile whose
 * input holds a value the fp16 hi part cannot (|x| >= 65520) is recomputed in the same launch
 * with its inputs pre-scaled by a power of two.  Workspace bytes [0, 256)
 * stay reserved (ABI versions <= 2 kept a range flag there); nothing is written to them. */
#define CISTA_WORKSPACE_RESERVED_BYTES 256

/* one recurrent frame for B independent sequences */
int cista_forward(const cista_config *cfg, const void *packed, int B, int H, int W,
                  const cista_frame_io *io, void *workspace, size_t workspace_bytes,
                  void *stream);

/* ---- HIP graphs (no reference counterpart: a launch-overhead optimisation) ----
 * cista_sequence_capture records `n_frames` consecutive cista_forward frames -- ~21 kernel
 * launches each -- into ONE hipGraph (captured on a private stream, so any caller stream can
 * replay it).  Frame f reads io[f] and must have the buffers cista_forward would; the recurrent
 * chaining is the caller's choice of pointers (io[f+1]'s prev pointers = io[f]'s outputs).
 * Every pointer is baked into the graph: replays recompute on whatever those buffers hold.
 * The parameters must be packed (and stay packed) before capture.  Capture runs frame 0 once,
 * eagerly, on its private stream before recording (one-time kernel attributes, argument errors):
 * that stream first waits for the work already enqueued on `stream` (an event), so inputs and
 * parameters produced there are ready; the call returns after that frame has finished.
 * cista_sequence_launch enqueues one replay on `stream`; cista_sequence_destroy frees the graph. */
typedef struct cista_sequence cista_sequence;
int  cista_sequence_capture(const cista_config *cfg, const void *packed, int B, int H, int W,
                            const cista_frame_io *io, int n_frames, void *workspace,
                            size_t workspace_bytes, cista_sequence **out, void *stream);
int  cista_sequence_launch(cista_sequence *seq, void *stream);
void cista_sequence_destroy(cista_sequence *seq);

/* ---- stage entries (the reference module boundaries; used by parity tests) ---- */
/* x1 (B,h,w,C) NHWC = W0(cat(We(events), Wi(prev_image)))                              */
int cista_stage_input(const cista_config *cfg, const void *packed, int B, int H, int W,
                      const float *events, const float *prev_image, float *x1,
                      void *workspace, size_t workspace_bytes, void *stream);
/* ConvLSTC: (z_out, c_out) = P0(x1, z_prev, c_prev); z0 scratch inside workspace        */
int cista_stage_lstc(const cista_config *cfg, const void *packed, int B, int h, int w,
                     const float *x1, const float *z_prev, const float *c_prev,
                     float *z_out, float *c_out, void *workspace, size_t workspace_bytes,
                     void *stream);
/* z <- S_lambda(z + P(x1 - D(z))) applied `iters` times IN PLACE on z (B,h,w,2C)        */
int cista_stage_ista(const cista_config *cfg, const void *packed, int B, int h, int w,
                     const float *x1, float *z, int iters, void *workspace,
                     size_t workspace_bytes, void *stream);
/* (h_out, c_out) = ConvLSTM(relu(Dg.conv(z)), (h_prev, c_prev))                          */
int cista_stage_decoder(const cista_config *cfg, const void *packed, int B, int h, int w,
                        const float *z, const float *h_prev, const float *c_prev,
                        float *h_out, float *c_out, void *workspace, size_t workspace_bytes,
                        void *stream);
/* rec (B,1,2h,2w) = sigmoid(final_conv(relu(upsamp_conv(h)))); pre_sigmoid may be NULL   */
int cista_stage_output(const cista_config *cfg, const void *packed, int B, int h, int w,
                       const float *hstate, float *rec, float *pre_sigmoid, void *workspace,
                       size_t workspace_bytes, void *stream);

/* ---- measurement hook (bench.py): launch ONE step of the frame schedule on the
 * buffers of a previous cista_forward with the same io/workspace (CISTA_LAYER_INPUT: its 1-3
 * kernels), so its duration can be
 * timed with events on `stream`.  Not a reference interface.  layer ids: */
enum {
    CISTA_LAYER_INPUT = 0,      /* We/Wi and W0 as one composed map (num_bins <= 8; x1 out) */
    CISTA_LAYER_W0 = 1,         /* stride-2 conv; launches nothing when INPUT composed it */
    CISTA_LAYER_P0 = 2,
    CISTA_LAYER_GATES = 3,      /* ConvLSTC gates + cell update     */
    CISTA_LAYER_OUT_GATES = 4,
    CISTA_LAYER_ISTA_D = 5,
    CISTA_LAYER_ISTA_P = 6,
    CISTA_LAYER_DG = 7,
    CISTA_LAYER_LSTM = 8,
    CISTA_LAYER_UPSAMPLE = 9,
    CISTA_LAYER_FINAL = 10,
    CISTA_LAYER_COUNT = 11
};
/* multiply-accumulates of one launch of `layer` (per frame x B) -- the algorithmic work */
double cista_layer_macs(const cista_config *cfg, int layer, int B, int H, int W);
/* 1 when this build computes `layer` inside another layer's launch at inference (then
 * cista_launch_layer(layer) launches nothing): W0 inside the composed input stage for 1..8 bins */
int cista_layer_fused(const cista_config *cfg, int layer);
int cista_launch_layer(const cista_config *cfg, const void *packed, int layer, int B, int H,
                       int W, const cista_frame_io *io, void *workspace, size_t workspace_bytes,
                       void *stream);
/* the tiling of a forward conv's throughput launch over a Hout x Wout output (stride 1,
 * block_px = 192 or 96 pixels per workgroup, B samples): region a = ty x tx tiles of TH x TW
 * pixels over columns [0, wa), region b (tx == 0: none) over columns [wa, Wout) -- the two-region
 * tiling of cista_abi.hip plan_tiles, both regions in one launch.  out[14] = {TH, TW, ty, tx,
 * mseg} of region a, the same of region b, wa, the tile count and mseg of the best one-region
 * tiling, 0; mseg > 0: each tile row is mseg 16-pixel m-tiles (row-aligned, conflict-free LDS
 * reads), 0: row-major m-tiles.  Host-only (no device call); introspection for tests, not a
 * reference interface. */
int cista_tile_plan(int B, int Hout, int Wout, int block_px, int *out);

/* ---- training: BPTT backward (reference train_e2v.py:108-130
 * differentiates through the whole recurrent sequence with autograd) ----
 * A training frame runs cista_forward_train, which also fills a `saved` buffer with the
 * activations the backward needs; cista_backward then takes the gradients of the frame's five
 * outputs and returns the gradients of its inputs (previous image and states: BPTT) and of
 * all 25 parameters.  Both require base_channels % 32 == 0 and base_channels <= 256 (the
 * wgrad partial-sum buffer holds the gates conv's 4C x 3C x 9 block). */
size_t cista_saved_bytes(const cista_config *cfg, int B, int H, int W);
size_t cista_train_workspace_bytes(const cista_config *cfg, int B, int H, int W);
int cista_forward_train(const cista_config *cfg, const void *packed, int B, int H, int W,
                        const cista_frame_io *io, void *saved, size_t saved_bytes,
                        void *workspace, size_t workspace_bytes, void *stream);

typedef struct {
    const float *g_rec;        /* dL/d rec      (B,1,H,W)       NULL = 0            */
    const float *g_c_lstc;     /* dL/d states[0] NHWC (B,h,w,2C) NULL = 0           */
    const float *g_z;          /* dL/d states[1] NHWC (B,h,w,2C) NULL = 0           */
    const float *g_h;          /* dL/d states[2][0] (B,h,w,C)    NULL = 0           */
    const float *g_c;          /* dL/d states[2][1] (B,h,w,C)    NULL = 0           */
    float *g_prev_image;       /* out (B,1,H,W); NULL = not needed                  */
    float *g_c_lstc_prev;      /* out (B,h,w,2C); NULL = not needed / prev was None */
    float *g_z_prev;           /* out (B,h,w,2C)                                    */
    float *g_h_prev;           /* out (B,h,w,C)                                     */
    float *g_c_prev;           /* out (B,h,w,C)                                     */
    float *g_events;           /* out (B,nb,H,W) NCHW; NULL = not needed (appended in */
                               /* ABI version 2: read only when grads_bytes covers it) */
} cista_grad_io;

/* parameter gradients, same fields / layouts as cista_params; written (not accumulated) */
typedef struct {
    float *We_w, *We_b, *Wi_w, *Wi_b, *W0_w, *W0_b;
    float *gates_w, *gates_b, *out_gates_w, *out_gates_b, *P0_w, *P0_b;
    float *lambda, *D_w, *D_b, *P_w, *P_b;
    float *Dg_w, *Dg_b, *lstm_w, *lstm_b, *up_w, *up_b, *final_w, *final_b;
} cista_param_grads;

/* grads_bytes = sizeof(cista_grad_io) as the caller compiled it: members beyond it (fields
 * appended by later ABI versions) are treated as NULL, never read.  All results are ordered on
 * `stream`; the weight gradients run on a library-owned per-device stream forked from and joined
 * back into `stream` within the call (CISTA_BWD_SIDE=0 in the environment: all on `stream`,
 * bit-identical results). */
int cista_backward(const cista_config *cfg, const void *packed, const cista_params *params,
                   int B, int H, int W, const cista_frame_io *io, const void *saved,
                   size_t saved_bytes, const cista_grad_io *grads, size_t grads_bytes,
                   const cista_param_grads *pgrads, void *workspace, size_t workspace_bytes,
                   void *stream);

/* Timing / PMC hook (bench.py --mode train): the backward's dominant launch on its own -- the
 * tied ISTA P weight gradient over all `depth` iterations (split-f16 wgrad + partial reduction),
 * as cista_backward runs it.  G (depth*B, h, w, 2C) and X (depth*B, h, w, C) NHWC fp32, gscale
 * {s, 1/s} the power-of-two fp16 split scale of G (device), dW (2C, C, 3, 3) and db (2C) written.
 * workspace: cista_train_workspace_bytes. */
int cista_wgrad_ista_p(const cista_config *cfg, int B, int H, int W, const float *G, const float *X,
                       const float *gscale, float *dW, float *db, void *workspace,
                       size_t workspace_bytes, void *stream);

/* Test / timing hook: W0's stride-2 weight gradient as cista_backward runs it (split-f16 wgrad
 * over a parity-split halo + partial reduction).  G (B, H/2, W/2, C) and X (B, H, W, C) NHWC
 * fp32, gscale {s, 1/s} of G, dW (C, C, 3, 3) and db (C) written.  workspace:
 * cista_train_workspace_bytes. */
int cista_wgrad_w0(const cista_config *cfg, int B, int H, int W, const float *G, const float *X,
                   const float *gscale, float *dW, float *db, void *workspace, size_t workspace_bytes,
                   void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CISTA_LSTC_H */
