/*
 * cista_voxel.h -- C ABI of the GPU event voxelizer that feeds the CISTA-LSTC path
 * (part of libcista_hip.so, built for gfx950).
 *
 * Replaces, for a whole batch of event windows in one call:
 *
 *   events_to_voxel_grid(events, num_bins, width, height)   reference utils/event_process.py:15-63
 *   event_preprocess(voxel, mode, filter_hot_pixel)         reference utils/event_process.py:132-154
 *   event_preprocess_pytorch(...)                           reference utils/event_process.py:157-176
 *
 * as called by the data readers (data_readers/train_data_loaders.py:187-193,
 * data_readers/video_readers.py:161-178) and the V2E emulator (v2e/v2e_model.py:526).
 *
 * Results are BIT-IDENTICAL to the reference's numpy path:
 *   - every voxel is accumulated in the reference's order (all left contributions of a voxel in
 *     event order, then all right contributions), each add as float32(float64(acc) + val),
 *     which is what np.add.at does on a float32 grid with float64 values: events are grouped per
 *     (window, pixel) by a stable radix sort, one thread walks each group in event order;
 *   - the 'std' statistics reproduce numpy's float32 reduction exactly: chunks of 8192 elements
 *     (the ufunc buffer), each summed by numpy's pairwise scheme (8-accumulator leaves of <= 128
 *     elements), chunk sums accumulated in order; mean/std and the normalisation in float64.
 *
 * Conventions: device pointers; `stream` is a hipStream_t passed as void*; no host sync, no
 * allocation.  Status codes are the CISTA_* codes of cista_lstc.h.
 */
#ifndef CISTA_VOXEL_H
#define CISTA_VOXEL_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* event_preprocess modes (reference utils/event_process.py:139-152) */
enum {
    CISTA_VOXEL_RAW = 0,     /* no normalisation (events_to_voxel_grid output)                 */
    CISTA_VOXEL_STD = 1,     /* mode='std': mean/std of the non-zero voxels -> (0, 1)          */
    CISTA_VOXEL_MAXMIN = 2,  /* mode='maxmin': (v - min) / (max - min + 1e-8)                  */
    CISTA_VOXEL_STD_F32 = 3, /* mode='std' of event_preprocess_pytorch (:157-176): float32
                                scalars and elementwise math, as torch computes them (the sums
                                rounded once to float32; ATen's reduction order may differ in
                                the last bit of sum())                                          */
    CISTA_VOXEL_TORCH_ACCUM = 0x10  /* cista_voxelize flag: accumulate like
                                events_to_voxel_grid_pytorch (:66-129): float32 contributions
                                and float32 index_add_ (bit-identical to the reference on a
                                float64 events tensor) instead of numpy's np.add.at           */
};

/* grid_status bits of cista_voxelize_checked: what the reference does with an event outside the
 * H x W frame (its np.add.at on the flat index x + y W + bin H W, utils/event_process.py:53-58) */
enum {
    CISTA_VOXEL_OUT_OF_RANGE = 1,  /* a flat index (np.uint: truncated, wrapped modulo 2^64, read
                                      back as intp) outside [-size, size) -- for the torch twin
                                      outside [0, size): the reference raises IndexError; the
                                      event is dropped here                                     */
    CISTA_VOXEL_SPILL = 2          /* a flat index inside the grid: the reference adds the event
                                      to another pixel / bin (a negative numpy index counts from
                                      the end of the grid), and so does this build, in event
                                      order with that cell's own events (bit-identical)         */
};

/* Workspace for cista_voxelize: n_events = total events of the batch (offsets[B]). */
size_t cista_voxel_workspace_bytes(int B, long long n_events, int num_bins, int height, int width);

/*
 * events   : (n_events, 4) float64 rows (t, x, y, p) -- the reference's [N x 4] array; the windows
 *            are concatenated, window b = rows [offsets[b], offsets[b+1]).  Each window must be
 *            time-sorted (first/last rows define the time normalisation, as in the reference);
 *            p == 0 means negative polarity (-1), any other value is used as is.
 * offsets  : DEVICE array of B+1 int64, offsets[0] = 0, offsets[B] = n_events.
 * voxels   : (B, num_bins, height, width) float32 output.
 * mode     : CISTA_VOXEL_*; hot_threshold > 0 zeroes |v| > hot_threshold before normalising
 *            (reference: 25/num_bins for event_preprocess(filter_hot_pixel=True),
 *            20/num_bins for event_preprocess_pytorch); <= 0 disables the filter.
 * Events whose x, y fall outside the H x W frame are added where the reference's flat index puts
 * them, or dropped where the reference raises; cista_voxelize_checked reports which (grid_status).
 * The input is never modified (the reference rewrites events[:, 0] and the polarity column).
 */
int cista_voxelize(const double *events, const long long *offsets, int B, long long n_events, int num_bins,
                   int height, int width, int mode, float hot_threshold, float *voxels, void *workspace,
                   size_t workspace_bytes, void *stream);

/* cista_voxelize that also ORs CISTA_VOXEL_OUT_OF_RANGE / CISTA_VOXEL_SPILL into *grid_status (a
 * DEVICE int the caller zeroes; NULL = no report) for the events outside the frame, so that a
 * caller can raise where the reference raises (read it after the stream has run the call). */
int cista_voxelize_checked(const double *events, const long long *offsets, int B, long long n_events, int num_bins,
                           int height, int width, int mode, float hot_threshold, float *voxels, void *workspace,
                           size_t workspace_bytes, int *grid_status, void *stream);

/* event_preprocess alone, in place, on B existing (num_bins, height, width) float32 voxel grids
 * (reference utils/event_process.py:132-154 / :157-176); workspace from
 * cista_voxel_workspace_bytes(B, 0, num_bins, height, width). */
int cista_voxel_preprocess(float *voxels, int B, int num_bins, int height, int width, int mode,
                           float hot_threshold, void *workspace, size_t workspace_bytes, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CISTA_VOXEL_H */
