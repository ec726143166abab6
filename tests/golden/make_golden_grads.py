"""Golden GRADIENTS from the real reference (autograd on CPU), for the BPTT backward (SURVEY
section 8 row a11).  Run in the build container only:

    PYTHONPATH=/root/reference:. python tests/golden/make_golden_grads.py

g1: one frame with leaf previous states / previous image (requires_grad), loss = sum of every
    output times a fixed random tensor -> grads of all 25 parameters and of all 5 inputs.
g2: train_e2v.py:108-120 semantics -- 3 frames, prev_img = output.clone() (no detach), states
    carried, loss = L1(last output, target) -> parameter grads (fp32 and fp64 reference).
g3 (grads_180x240_seq15.npz): config c3's frame size and sequence length -- 180x240, 15 frames,
    B=1, the g2 loss -> parameter grads of the fp32 reference and of the fp64 reference (stored
    rounded to fp32), and the fp32-vs-fp64 noise of each (up to 2.3e-3: the 15-frame recurrence
    amplifies fp32 rounding, so the GPU gradients are judged against the fp64 truth).  Its voxels
    are NOT stored: tests regenerate them with oracle/fixtures.synthetic_voxels (seed below) and
    check them against the stored checksum.

g4 (grads_180x240_b8.npz): config c3's batch -- 180x240, B=8, 5 frames, the g2 loss -> the same
    keys as g3 plus the fp32 reference's per-sample last frames.  The wgrad partial sums and the
    DDP reductions depend on B; g1/g2 pin B <= 2 only.

    PYTHONPATH=/root/reference:. python tests/golden/make_golden_grads.py [g12] [g3] [g4]
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import fixtures as fx  # noqa: E402
from tests.golden.g3_spec import G3, g3_inputs, g3_params  # noqa: E402
from tests.golden.g4_spec import G4, g4_inputs, g4_params  # noqa: E402
from e2v.e2v_model import CistaLSTCNet  # noqa: E402

torch.set_num_threads(8)


def build(C, depth, params, dtype):
    m = CistaLSTCNet([32, 32], base_channels=C, depth=depth, num_bins=5)
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}, depth)
    m.load_state_dict(sd, strict=True)
    return m.to(dtype)


def unique_grads(m, depth):
    out = {}
    for k, p in m.named_parameters():          # named_parameters() de-duplicates tied params
        key = k.replace("lista_blocks.0.", "lista.")
        out[key] = p.grad.detach().double().numpy().copy()
    return out


def main():
    C, depth, B, H, W = 64, 5, 2, 32, 48
    params = fx.stress_params(C, depth, 5, seed=21, lam=0.05)
    vox = fx.synthetic_voxels(3, B, 5, H, W, n_events=fx.density_matched_events(H, W), seed=99)
    rng = np.random.default_rng(5)
    res = {"voxels": vox}
    for dtype, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        # ---------------- g1: one frame, all outputs weighted --------------------------
        m = build(C, depth, params, dtype)
        with torch.no_grad():
            prev0, st0 = m(torch.from_numpy(vox[0]).to(dtype), torch.zeros(B, 1, H, W, dtype=dtype), None)
        leaves = [prev0.clone().requires_grad_(True), st0[0].clone().requires_grad_(True),
                  st0[1].clone().requires_grad_(True), st0[2][0].clone().requires_grad_(True),
                  st0[2][1].clone().requires_grad_(True)]
        ev1 = torch.from_numpy(vox[1]).to(dtype).requires_grad_(True)       # the events' gradient too
        rec, st = m(ev1, leaves[0], [leaves[1], leaves[2], (leaves[3], leaves[4])])
        outs = [rec, st[0], st[1], st[2][0], st[2][1]]
        if tag == "f32":
            Rs = [rng.standard_normal(o.shape).astype(np.float32) for o in outs]
            for i, r in enumerate(Rs):
                res[f"g1_R{i}"] = r
            res["g1_prev_image"] = prev0.numpy().astype(np.float32)
            for i, n in enumerate(["c_lstc", "z", "h", "c"]):
                res[f"g1_prev_{n}"] = leaves[1 + i].detach().numpy().astype(np.float32)
        loss = sum((o * torch.from_numpy(res[f"g1_R{i}"]).to(dtype)).sum() for i, o in enumerate(outs))
        loss.backward()
        for k, v in unique_grads(m, depth).items():
            res[f"g1_{tag}_param_{k}"] = v.astype(np.float32) if tag == "f32" else v
        for i, n in enumerate(["prev_image", "c_lstc", "z", "h", "c"]):
            g = leaves[i].grad.detach().numpy()
            res[f"g1_{tag}_grad_{n}"] = g.astype(np.float32) if tag == "f32" else g
        g = ev1.grad.detach().numpy()
        res[f"g1_{tag}_grad_events"] = g.astype(np.float32) if tag == "f32" else g
        # ---------------- g2: 3-frame BPTT, L1 on the last frame -------------------------
        m = build(C, depth, params, dtype)
        target = torch.from_numpy(np.random.default_rng(6).uniform(0, 1, (B, 1, H, W))).to(dtype)
        prev = torch.zeros(B, 1, H, W, dtype=dtype)
        state = None
        for s in range(3):
            out, state = m(torch.from_numpy(vox[s]).to(dtype), prev, state)
            prev = out.clone()
        loss = torch.nn.functional.l1_loss(out, target)
        loss.backward()
        res[f"g2_{tag}_loss"] = np.float64(loss.item())
        for k, v in unique_grads(m, depth).items():
            res[f"g2_{tag}_param_{k}"] = v.astype(np.float32) if tag == "f32" else v
    res["g2_target"] = np.random.default_rng(6).uniform(0, 1, (B, 1, H, W)).astype(np.float32)
    # keep the fp64 truth only as per-tensor noise levels of the fp32 reference (size)
    for k in [k for k in res if "_f64_" in k]:
        v64 = res.pop(k)
        k32 = k.replace("_f64_", "_f32_")
        if isinstance(v64, np.ndarray) and v64.ndim > 0:
            res[k.replace("_f64_", "_noise32_")] = np.float64(
                np.abs(res[k32].astype(np.float64) - v64).max() / max(np.abs(v64).max(), 1e-30))
        else:
            res[k] = v64
    np.savez_compressed(os.path.join(HERE, "grads_32x48.npz"), **res)
    print("wrote", os.path.join(HERE, "grads_32x48.npz"))


def main_g3(c=G3, params_fn=g3_params, inputs_fn=g3_inputs, name="grads_180x240_seq15.npz"):
    params = params_fn()
    vox, target = inputs_fn()
    res = {"vox_sum": np.float64(vox.astype(np.float64).sum()),
           "vox_abs_sum": np.float64(np.abs(vox.astype(np.float64)).sum())}
    grads = {}
    for dtype, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        m = CistaLSTCNet([c["H"], c["W"]], base_channels=c["C"], depth=c["depth"], num_bins=5)
        sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}, c["depth"])
        m.load_state_dict(sd, strict=True)
        m = m.to(dtype)
        prev = torch.zeros(c["B"], 1, c["H"], c["W"], dtype=dtype)
        state = None
        for s in range(c["L"]):
            out, state = m(torch.from_numpy(vox[s]).to(dtype), prev, state)
            prev = out.clone()
        loss = torch.nn.functional.l1_loss(out, torch.from_numpy(target).to(dtype))
        loss.backward()
        res[f"{tag}_loss"] = np.float64(loss.item())
        res[f"{tag}_last_frame"] = out.detach().double().numpy().astype(np.float32)
        grads[tag] = unique_grads(m, c["depth"])
        del m, out, state, prev, loss                       # free the autograd graph (B=8: ~13 / 27 GB)
    for k, v in grads["f32"].items():
        res[f"f32_param_{k}"] = v.astype(np.float32)
        v64 = grads["f64"][k]
        res[f"f64_param_{k}"] = v64.astype(np.float32)       # the truth, rounded to fp32 (2^-24)
        res[f"noise32_param_{k}"] = np.float64(np.abs(v - v64).max() / max(np.abs(v64).max(), 1e-30))
    for k, v in c.items():
        res[f"cfg_{k}"] = np.float64(v)
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **res)
    print("wrote", path)


if __name__ == "__main__":
    which = sys.argv[1:] or ["g12", "g3", "g4"]
    if "g12" in which:
        main()
    if "g3" in which:
        main_g3()
    if "g4" in which:
        main_g3(G4, g4_params, g4_inputs, "grads_180x240_b8.npz")
