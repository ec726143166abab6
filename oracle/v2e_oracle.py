"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the V2E event emulator in voxel-grid mode
(SURVEY section 8 row f2): reference v2e/v2e_model.py:290-536 (EventEmulator.forward, _init
:158-253, IIR_temporal_filtering :266-289) and v2e/emulator_utils.py:13-207 (lin_log,
rescale_intensity_frame, low_pass_filter, subtract_leak_current, generate_shot_noise).

PARITY UNPINNED: the reference emulator cannot be imported here (v2e_model.py imports cv2 and
matplotlib, both absent) and no reference fixture exercises it.  Its random draws
(torch.normal / randn / rand) make parity statistical anyway; this restatement takes the random
arrays from a pluggable source so the deterministic configuration (sigma_thres = 0,
leak_rate_hz = 0, shot_noise_rate_hz = 0) can be compared value for value.  Only tests/ import
this module.
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


class NoRandom:
    """A random source for the deterministic configuration: every draw is an error."""

    def normal(self, mean, std, shape):
        raise AssertionError("random draw in a deterministic configuration")

    randn = rand = normal


class V2EOracle:
    """EventEmulator(output_mode='voxel_grid') state machine, numpy float32."""

    def __init__(self, num_bins=5, pl=1.0, ps=1.0, ql=1.0, qs=1.0, pos_thres=0.2, neg_thres=0.2, sigma_thres=0.03,
                 cutoff_hz=0.0, leak_rate_hz=0.1, refractory_period_s=0.0, shot_noise_rate_hz=0.0,
                 leak_jitter_fraction=0.1, noise_rate_cov_decades=0.1, rng=None):
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
        if self.cutoff <= 0:
            return log_new
        if self.ql > 0:
            tau0 = 1 / (math.pi * 2 * self.cutoff * self.ql)
            eps = (inten01 * (f32(dt) / f32(tau0))).astype(f32)
        else:
            eps = np.ones_like(inten01)
        if self.qs > 0:
            tau1 = 1 / (math.pi * 2 * self.cutoff * self.qs)
            eps1 = (inten01 * (f32(dt) / f32(tau1))).astype(f32)
            eps[:, :, 0::2, 0::2] = eps1[:, :, 0::2, 0::2]
        else:
            eps[:, :, 0::2, 0::2] = 1
        eps = np.minimum(eps, f32(1))
        return ((f32(1) - eps) * self.lp + eps * log_new).astype(f32)

    def forward(self, frames, t_frames):
        """frames (B, F, H, W) float32 intensities 0..255; t_frames (B, 2) or (B, F) seconds.
        Returns (voxels (B, nb, H, W) float32 before event_preprocess, num_events)."""
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
        num_events = 0
        for n in range(1, F):
            new = filt[n]
            dt = f32(tf[n] - self.t_prev)
            if self.leak > 0:
                rand = self.rng.randn((B, 1, H, W)).astype(f32)
                leak = (f32(self.leak) * self.noise_rate * (f32(1) - f32(self.jitter) * rand)).astype(f32)
                self.base = (self.base - dt * leak * self.pos_thres).astype(f32)
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
        return vox, num_events


def preprocess_whole(vox):
    """event_preprocess_pytorch(mode='std', filter_hot_pixel=False) as v2e_model.py:526 calls it:
    statistics over the WHOLE (B, nb, H, W) tensor, float32 (utils/event_process.py:157-176)."""
    v = vox.astype(f32)
    nz = v != 0
    n = int(nz.sum())
    if n == 0:
        return v
    mean = f32(v.astype(np.float64).sum() / n)
    std = f32(math.sqrt(max((v.astype(np.float64) ** 2).sum() / n - float(mean) ** 2, 0.0)))
    return (nz.astype(f32) * (v - mean) / (std + f32(1e-8))).astype(f32)
