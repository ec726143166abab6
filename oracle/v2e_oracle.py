"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the V2E event emulator in voxel-grid mode
(SURVEY section 8 row f2): reference v2e/v2e_model.py:290-536 (EventEmulator.forward, _init
:158-253, IIR_temporal_filtering :266-289) and v2e/emulator_utils.py:13-207 (lin_log,
rescale_intensity_frame, low_pass_filter, subtract_leak_current, generate_shot_noise).

Parity: the emulator's forward (v2e_model.py:290-536) cannot be imported here (the module
imports cv2 and matplotlib, both absent), so the composition below is restated, not
executed from the reference.  Its BUILDING BLOCKS are pinned: lin_log, rescale_intensity_frame,
low_pass_filter, subtract_leak_current, compute_event_map (v2e/emulator_utils.py) and the torch
voxel twins events_to_voxel_grid_pytorch / event_preprocess_pytorch (utils/event_process.py)
are checked against vectors the real reference functions produced
(tests/golden/make_golden_v2e.py -> v2e_blocks.npz; tests/test_oracle_v2e_golden.py).  The
random draws (torch.normal / randn / rand) make whole-forward parity statistical anyway; this
restatement takes the random arrays from a pluggable source so the deterministic configuration
(sigma_thres = 0, leak_rate_hz = 0, shot_noise_rate_hz = 0) can be compared value for value.
Only tests/ import this module.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32


def lin_log(x, threshold=20):
    """emulator_utils.py:13-38: linear below `threshold`, log above, in float64, rounded to 1e-8."""
    x = x.astype(np.float64)
    f = (1.0 / threshold) * math.log(threshold)
    with np.errstate(divide="ignore"):
        y = np.where(x <= threshold, x * f, np.log(x))
    y = np.round(y * 1e8) / 1e8
    return y.astype(f32)


def torch_linspace_f32(start, end, steps):
    """torch.linspace(..., dtype=float32): ATen's symmetric float32 formula (start + step*k for
    the first half, end - step*(steps-1-k) for the second)."""
    start, end = f32(start), f32(end)
    if steps == 1:
        return np.array([start], f32)
    step = f32((end - start) / f32(steps - 1))
    half = steps // 2
    return np.array([start + step * f32(k) if k < half else end - step * f32(steps - k - 1) for k in range(steps)],
                    f32)


def rescale_intensity_frame(x):
    """emulator_utils.py:41-46."""
    return ((x + f32(20)) / f32(275)).astype(f32)


def low_pass_filter(log_new, lp0, inten01, dt, cutoff_hz, ql=1.0, qs=1.0):
    """emulator_utils.py:49-101: first-order intensity-dependent IIR; the (0::2, 0::2) pixels
    use the qs time constant.  float32 like the reference's tensors (dt a float32 scalar)."""
    if cutoff_hz <= 0:
        return log_new
    inten01 = inten01.astype(f32)
    if ql > 0:
        tau0 = 1 / (math.pi * 2 * cutoff_hz * ql)
        eps = (inten01 * (f32(dt) / f32(tau0))).astype(f32)
    else:
        eps = np.ones_like(inten01)
    if qs > 0:
        tau1 = 1 / (math.pi * 2 * cutoff_hz * qs)
        eps1 = (inten01 * (f32(dt) / f32(tau1))).astype(f32)
        eps[:, :, 0::2, 0::2] = eps1[:, :, 0::2, 0::2]
    else:
        eps[:, :, 0::2, 0::2] = 1
    eps = np.minimum(eps, f32(1))
    return ((f32(1) - eps) * lp0 + eps * log_new).astype(f32)


def subtract_leak_current(base, leak_rate_hz, dt, pos_thres, leak_jitter_fraction, noise_rate, rand):
    """emulator_utils.py:104-126; `rand` is the standard-normal draw (torch.randn there)."""
    cur = (f32(leak_rate_hz) * noise_rate * (f32(1) - f32(leak_jitter_fraction) * rand)).astype(f32)
    return (base - (f32(dt) * cur).astype(f32) * pos_thres).astype(f32)


def _div_floor(a, b):
    """ATen's float floor division (torch.div(..., rounding_mode='floor')): Python semantics via
    fmod, not floor(a / b)."""
    a, b = a.astype(f32), b.astype(f32)
    mod = np.fmod(a, b)
    div = ((a - mod) / b).astype(f32)
    div = np.where((mod != 0) & ((b < 0) != (mod < 0)), div - f32(1), div).astype(f32)
    fl = np.floor(div)
    fl = np.where(div - fl > f32(0.5), fl + f32(1), fl)
    return np.where(div != 0, fl, np.copysign(f32(0), a / b)).astype(f32)


def compute_event_map(diff, pos_thres, neg_thres):
    """emulator_utils.py:129-162: ON / OFF event counts of a log-intensity difference."""
    pos = np.maximum(diff, f32(0)).astype(f32)
    neg = np.maximum(-diff, f32(0)).astype(f32)
    return _div_floor(pos, pos_thres).astype(np.int32), _div_floor(neg, neg_thres).astype(np.int32)


def events_to_voxel_grid_pytorch(events, num_bins, width, height):
    """utils/event_process.py:66-129 with a float64 events tensor: timestamps normalised in
    float64, the contributions rounded to float32 (`dts.float()`, float32 polarities), and
    index_add_ on the float32 grid adding them in event order, left contributions first."""
    vox = np.zeros(num_bins * height * width, f32)
    if len(events) == 0:
        return vox.reshape(num_bins, height, width)
    t = events[:, 0].astype(np.float64)
    dT = t[-1] - t[0]
    if dT == 0:
        dT = 1.0
    ts = (num_bins - 1) * (t - t[0]) / dT
    xs = events[:, 1].astype(np.int64)
    ys = events[:, 2].astype(np.int64)
    pol = events[:, 3].astype(f32).copy()
    pol[pol == 0] = -1
    tis = np.floor(ts)
    dts = (ts - tis).astype(f32)
    vl = (pol * (f32(1) - dts)).astype(f32)
    vr = (pol * dts).astype(f32)
    ti = tis.astype(np.int64)
    ok = (tis < num_bins) & (tis >= 0)
    np.add.at(vox, xs[ok] + ys[ok] * width + ti[ok] * width * height, vl[ok])
    ok = ((tis + 1) < num_bins) & (tis >= 0)
    np.add.at(vox, xs[ok] + ys[ok] * width + (ti[ok] + 1) * width * height, vr[ok])
    return vox.reshape(num_bins, height, width)


def event_preprocess_pytorch(vox, mode="std", filter_hot_pixel=True):
    """utils/event_process.py:157-176 in float32 torch semantics: sum() is a float32 scalar
    (here the exact sum rounded once to float32; ATen's own reduction order may differ in the
    last bits), `/ num_nonzeros` in float32, sqrt of a float32 expression, and the elementwise
    normalisation in float32.  Statistics over the whole array, whatever its rank."""
    v = np.asarray(vox, f32).copy()
    nb = v.shape[0]
    if filter_hot_pixel:
        v[np.abs(v) > f32(20.0 / nb)] = 0
    if mode == "maxmin":
        return ((v - v.min()) / (v.max() - v.min() + f32(1e-8))).astype(f32)
    if mode != "std":
        return v
    nz = v != 0
    n = int(nz.sum())
    if n == 0:
        return v
    nf = f32(n)
    mean = f32(f32(v.astype(np.float64).sum()) / nf)
    sq = f32(f32((v.astype(np.float64) ** 2).sum()) / nf)
    std = np.sqrt(f32(sq - f32(mean * mean)), dtype=f32)
    return (nz.astype(f32) * (v - mean) / f32(std + f32(1e-8))).astype(f32)


class NoRandom:
    """A random source for the deterministic configuration: every draw is an error."""

    def normal(self, mean, std, shape):
        raise AssertionError("random draw in a deterministic configuration")

    randn = rand = normal


class V2EOracle:
    """EventEmulator state machine, numpy float32: output_mode 'voxel_grid' (default) or 'raw'."""

    def __init__(self, num_bins=5, pl=1.0, ps=1.0, ql=1.0, qs=1.0, pos_thres=0.2, neg_thres=0.2, sigma_thres=0.03,
                 cutoff_hz=0.0, leak_rate_hz=0.1, refractory_period_s=0.0, shot_noise_rate_hz=0.0,
                 leak_jitter_fraction=0.1, noise_rate_cov_decades=0.1, rng=None, output_mode="voxel_grid"):
        self.raw = output_mode == "raw"
        self.nb = num_bins
        self.pl, self.ps, self.ql, self.qs = pl, ps, ql, qs
        self.pos_nom, self.neg_nom = f32(pos_thres), f32(neg_thres)
        self.sigma = sigma_thres
        self.cutoff = cutoff_hz
        self.leak = leak_rate_hz
        self.refr = f32(refractory_period_s)
        self.shot = shot_noise_rate_hz
        self.jitter = leak_jitter_fraction
        self.cov = noise_rate_cov_decades
        self.rng = rng or NoRandom()
        self.base = None
        self.lp = None

    def reset(self):
        self.base = None
        self.lp = None

    # v2e_model.py:158-253
    def _init(self, frame_log, Tr_frames):
        B = frame_log.shape[0]
        self.base = frame_log.copy()
        self.lp = self.base.copy()
        shp = frame_log.shape
        if self.sigma > 0:
            pt = self.rng.normal(self.pl * self.pos_nom, self.sigma, shp).astype(f32)
            ph = self.rng.normal(self.ps * self.pos_nom, self.sigma, shp).astype(f32)
            pt[:, :, 0::2, 0::2] = ph[:, :, 0::2, 0::2]
            self.pos_thres = np.maximum(pt, f32(0.01))
            nt = self.rng.normal(self.pl * self.neg_nom, self.sigma, shp).astype(f32)
            nh = self.rng.normal(self.ps * self.neg_nom, self.sigma, shp).astype(f32)
            nt[:, :, 0::2, 0::2] = nh[:, :, 0::2, 0::2]
            self.neg_thres = np.maximum(nt, f32(0.01))
        else:
            self.pos_thres = np.full(shp, self.pos_nom, f32)
            self.neg_thres = np.full(shp, self.neg_nom, f32)
        self.pos_pre = (self.pos_thres * (f32(1) / self.pos_nom)).astype(f32)     # einsum(1/nominal, thres)
        self.neg_pre = (self.neg_thres * (f32(1) / self.neg_nom)).astype(f32)
        if self.leak > 0:
            self.noise_rate = np.exp(f32(math.log(10) * self.cov) * self.rng.randn(shp).astype(f32)).astype(f32)
        self.tmem = (np.zeros(shp, f32) - Tr_frames).astype(f32)

    def _lowpass(self, log_new, inten01, dt):
        """emulator_utils.py:49-101 (first-order, 0::2 pixels use qs)."""
        return low_pass_filter(log_new, self.lp, inten01, dt, self.cutoff, self.ql, self.qs)

    def forward(self, frames, t_frames):
        """frames (B, F, H, W) float32 intensities 0..255; t_frames (B, 2) or (B, F) seconds.
        Returns (voxels (B, nb, H, W) float32 before event_preprocess, num_events), or in raw mode
        (rows (N, 5) float32 [t, x, y, p, b], num_events): v2e_model.py:504-518 stacks each
        iteration's events in nonzero (b, y, x) order and :527-534 sorts by t, then by b -- here
        stable sorts (the reference's torch.sort makes no tie promise), so rows of equal (b, t)
        keep their emission order."""
        frames = frames.astype(f32)
        B, F, H, W = frames.shape
        t_frames = np.asarray(t_frames, dtype=np.float64)
        if t_frames.shape[1] == 2:
            tf = torch_linspace_f32(t_frames[0, 0], t_frames[0, -1], F)
        else:
            tf = t_frames[0].astype(f32)
        nb = self.nb
        duration = (nb - 1) / (F - 1)
        time_frames = torch_linspace_f32(0, duration * (F - 1), F)
        span = (t_frames[:, -1:] - t_frames[:, 0:1]).astype(f32)
        Tr = (f32(nb - 1) * self.refr * (f32(1) / span)).astype(f32)                       # (B, 1), :322
        Tr_frames = np.broadcast_to(Tr[:, :, None, None], (B, 1, H, W)).astype(f32)
        resc = rescale_intensity_frame(frames)
        logf = lin_log(frames)
        if self.base is None:
            self._init(logf[:, 0:1], Tr_frames)
            self.t_prev = f32(t_frames[0, 0])
        else:
            self.tmem[self.tmem > 0] -= f32(nb - 1)
            neg = self.tmem < 0
            self.tmem[neg] = -Tr_frames[neg]
        # IIR (:266-289)
        filt = [self.lp]
        for n in range(1, F):
            if self.cutoff > 0:
                self.lp = self._lowpass(logf[:, n:n + 1], resc[:, n:n + 1], f32(tf[n] - tf[n - 1]))
                filt.append(self.lp)
            else:
                filt.append(logf[:, n:n + 1])
        if not tf[1] > self.t_prev:
            raise ValueError("this frame time must be later than previous frame time")
        vox = np.zeros((B, nb, H, W), f32)
        rows = []
        loops = 0
        num_events = 0
        for n in range(1, F):
            new = filt[n]
            dt = f32(tf[n] - self.t_prev)
            if self.leak > 0:
                rand = self.rng.randn((B, 1, H, W)).astype(f32)
                self.base = subtract_leak_current(self.base, self.leak, dt, self.pos_thres, self.jitter,
                                                  self.noise_rate, rand)
            diff = (new - self.base).astype(f32)
            diff[~(np.abs(diff) > f32(1e-6))] = 0
            pol = np.sign(diff).astype(f32)
            C = (self.pos_thres * (pol > 0) + self.neg_thres * (pol < 0)).astype(f32)
            counts = np.floor(np.abs(diff) / (C + f32(1e-9))).astype(np.int32)
            num_iters = counts.reshape(B, -1).max(1)
            max_iters = int(num_iters.max())
            num_iters[num_iters == 0] = 1
            ts_step = (f32(duration) / num_iters.astype(f32)).astype(f32)
            steps = np.linspace(1, max_iters, max_iters).astype(f32) if max_iters > 0 else np.zeros(0, f32)
            ts = (time_frames[n - 1] + ts_step[:, None] * steps[None, :]).astype(f32)
            for b in range(B):
                ts[b, num_iters[b]:] = 0
            if self.shot > 0:
                inten = resc[:, n:n + 1]
                factor = (f32(self.shot / 2) * dt / num_iters.astype(f32))[:, None, None, None] * \
                    ((f32(0.25) - 1) * inten + 1)
                on_thr = (f32(1) - factor * self.pos_pre).astype(f32)
                off_thr = (factor * self.neg_pre).astype(f32)
                r01 = self.rng.rand((max_iters, B, 1, H, W)).astype(f32)
                itmask = np.zeros_like(r01)
                for b in range(B):
                    itmask[:num_iters[b], b] = 1
                shot_on = itmask * (r01 > on_thr[None])
                shot_off = itmask * (r01 < off_thr[None])
                shot_cord = shot_on * (pol > 0) + shot_off * (pol < 0)
            final = np.zeros((B, 1, H, W), np.int32)
            refr_on = bool((Tr > ts_step[None, :]).any())        # (B, 1) > (B,) broadcasts, :447
            loops += max_iters
            for i in range(max_iters):
                mask = counts >= i + 1
                if self.shot > 0:
                    mask = np.logical_or(mask, shot_cord[i] > 0)
                tsi = np.broadcast_to(ts[:, i][:, None, None, None], (B, 1, H, W)).astype(f32)
                if refr_on:
                    since = (tsi * mask - self.tmem).astype(f32)
                    mask = since > Tr_frames
                    self.tmem[mask] = tsi[mask]
                final += mask
                t = (tsi * mask).astype(f32)
                if self.raw:                                       # :505-518
                    bb, _, yy, xx = np.nonzero(mask)
                    num_events += len(bb)
                    rows.append(np.stack([t[mask], xx.astype(f32), yy.astype(f32), pol[mask],
                                          bb.astype(f32)], 1).astype(f32))
                    continue
                ti = np.floor(t)
                dts = (t - ti).astype(f32)
                vl = (pol * (f32(1) - dts)).astype(f32)
                vr = (pol * dts).astype(f32)
                tm = mask & (ti >= 0)
                num_events += int(tm.sum())
                bb, _, yy, xx = np.nonzero(tm)
                tl = ti[tm].astype(np.int64)
                np.add.at(vox, (bb, tl, yy, xx), vl[tm])
                tm2 = tm & ((ti + 1) < nb)
                bb, _, yy, xx = np.nonzero(tm2)
                np.add.at(vox, (bb, ti[tm2].astype(np.int64) + 1, yy, xx), vr[tm2])
            self.t_prev = tf[n]
            self.base = (self.base + pol * final.astype(f32) * C).astype(f32)
        if self.raw:
            if loops == 0:                                         # torch.tensor([]) (:347)
                return np.zeros(0, f32), 0
            ev = np.concatenate(rows, 0) if rows else np.zeros((0, 5), f32)
            ev = ev[np.argsort(ev[:, 0], kind="stable")]           # :530-531
            ev = ev[np.argsort(ev[:, 4], kind="stable")]           # :533-534
            return ev, num_events
        return vox, num_events


def preprocess_whole(vox):
    """event_preprocess_pytorch(mode='std', filter_hot_pixel=False) as v2e_model.py:526 calls it:
    statistics over the WHOLE (B, nb, H, W) tensor, float32 (utils/event_process.py:157-176)."""
    return event_preprocess_pytorch(vox, mode="std", filter_hot_pixel=False)
