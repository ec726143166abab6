"""Generate the golden fixtures under tests/golden/ by running the REAL reference on CPU.

Run in the build container only (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference:. python tests/golden/make_golden.py

It imports ``e2v.e2v_model.CistaLSTCNet`` (reference ``e2v/e2v_model.py:5-90``) and
``utils.event_process`` (reference ``utils/event_process.py:15-63,132-154``) unmodified, and
writes data only (inputs, weights, outputs, per-layer intermediates) -- no reference source.

Fixture sets:

* ``f1_*``  C=64 depth 5 bins 5, 64x64, B=2, 3 frames; default init (seed 0, saved as a
  ``{'epoch', 'state_dict'}`` .pth.tar -- the reference checkpoint layout) and stress init;
  per-layer intermediates of frame 1 (the first frame that carries states), sample 0.
* ``f2_*``  C=32 depth 2 bins 5, 32x48, B=2, 4 frames, stress init.
* ``f3_*``  C=64 depth 5, 180x240, B=1, 2 frames, stress init (frames + state checksums).
* ``f4_*``  C=64 depth 5, 64x64, B=1, 15 frames, stress init: recurrent drift, with fp64 shadow.
* ``vox_*`` one 180x240 voxel built by the reference voxeliser from committed events.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import fixtures as fx  # noqa: E402

from e2v.e2v_model import CistaLSTCNet  # noqa: E402  (reference, PYTHONPATH=/root/reference)
from utils import event_process as ref_ev  # noqa: E402

torch.set_num_threads(8)


def load_unique(model, params):
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()},
                        model.depth)
    model.load_state_dict(sd, strict=True)


def run_sequence(model, voxels, dtype=torch.float32, hooks=None):
    """voxels [F,B,nb,H,W] -> list of (rec, states) per frame; prev_image starts at zeros
    (reference test_e2v.py:110-117)."""
    model = model.to(dtype)
    F_, B, nb, H, W = voxels.shape
    prev = torch.zeros(B, 1, H, W, dtype=dtype)
    states = None
    outs = []
    with torch.no_grad():
        for f in range(F_):
            if hooks is not None:
                hooks["frame"] = f
            ev = torch.from_numpy(voxels[f]).to(dtype)
            rec, states = model(ev, prev, states)
            prev = rec
            outs.append((rec.clone(), [states[0].clone(), states[1].clone(),
                                       (states[2][0].clone(), states[2][1].clone())]))
    return outs


def states_np(st):
    return {"c_lstc": st[0].float().numpy(), "z": st[1].float().numpy(),
            "h": st[2][0].float().numpy(), "c": st[2][1].float().numpy()}


def add_hooks(model, store, frame_to_keep):
    """Forward hooks recording per-layer intermediates of one frame (sample 0)."""
    def keep(name, t):
        if store.get("frame") == frame_to_keep:
            store.setdefault(name, []).append(t.detach()[0].float().numpy().copy())

    def hook(fn):
        # a forward hook that returns non-None REPLACES the module output: always return None
        def h(m, i, o):
            fn(m, i, o)
            return None
        return h

    model.We.register_forward_hook(hook(lambda m, i, o: keep("x_E", o)))
    model.Wi.register_forward_hook(hook(lambda m, i, o: keep("x_I", o)))
    model.W0.register_forward_hook(hook(lambda m, i, o: keep("x1", o)))
    model.P0.P0.register_forward_hook(hook(lambda m, i, o: keep("z0", o)))
    model.P0.gates.register_forward_hook(hook(lambda m, i, o: keep("lstc_gates", o)))
    model.P0.out_gates.register_forward_hook(hook(lambda m, i, o: keep("lstc_out_gates", o)))
    model.P0.register_forward_hook(hook(lambda m, i, o: (keep("z_lstc", o[0]), keep("c_lstc", o[1]))))
    blk = model.lista_blocks[0]
    blk.D.register_forward_hook(hook(lambda m, i, o: (keep("ista_z_in", i[0]), keep("ista_D", o))))
    blk.P.register_forward_hook(hook(lambda m, i, o: keep("ista_P", o)))
    model.Dg.conv.register_forward_hook(hook(lambda m, i, o: (keep("z_final", i[0]), keep("dg_y", o))))
    model.Dg.recurrent_block.Gates.register_forward_hook(hook(lambda m, i, o: keep("lstm_gates", o)))
    model.Dg.register_forward_hook(hook(lambda m, i, o: (keep("h", o[1][0]), keep("c", o[1][1]))))
    model.upsamp_conv.register_forward_hook(hook(lambda m, i, o: keep("u", o)))
    model.final_conv.register_forward_hook(hook(lambda m, i, o: keep("pre_sigmoid", o)))


def main():
    out_dir = HERE

    # ---------------- voxeliser KAT (reference utils/event_process.py) ----------------
    rng = np.random.default_rng(99)
    ev = fx.synthetic_events(15000, 180, 240, rng)
    vox_raw = ref_ev.events_to_voxel_grid(ev.copy(), 5, 240, 180).astype(np.float32)
    vox_norm = np.asarray(ref_ev.event_preprocess(vox_raw.copy(), filter_hot_pixel=True), np.float32)
    np.savez_compressed(os.path.join(out_dir, "vox_180x240.npz"), events=ev, voxel_raw=vox_raw,
                        voxel=vox_norm)

    # ---------------- F1: 64x64, C=64, depth 5, B=2, 3 frames ----------------
    H, W, B, NF = 64, 64, 2, 3
    vox = fx.synthetic_voxels(NF, B, 5, H, W, n_events=fx.density_matched_events(H, W), seed=1234)
    torch.manual_seed(0)
    np.random.seed(0)
    m = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=5)
    torch.save({"epoch": 0, "state_dict": m.state_dict()}, os.path.join(out_dir, "f1_default.pth.tar"))
    res = {"voxels": vox}
    for tag, init in (("default", None), ("stress", fx.stress_params(64, 5, 5))):
        torch.manual_seed(0)
        np.random.seed(0)
        model = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=5)
        if init is not None:
            load_unique(model, init)
        store = {}
        add_hooks(model, store, frame_to_keep=1)
        outs = run_sequence(model, vox, hooks=store)
        for f, (rec, st) in enumerate(outs):
            res[f"{tag}_rec{f}"] = rec.numpy()
        for k, v in states_np(outs[-1][1]).items():
            res[f"{tag}_state_{k}"] = v
        if tag == "stress":   # frame-0 states = inputs of the frame-1 per-layer KAT
            for k, v in states_np(outs[0][1]).items():
                res[f"{tag}_state0_{k}"] = v
        if tag == "stress":
            for k, v in store.items():
                if k in ("frame", "z_lstc"):   # z_lstc == ista_z_in[0]
                    continue
                res[f"inter_{k}"] = np.stack(v, 0)
        # fp64 shadow
        model64 = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=5)
        model64.load_state_dict(model.state_dict())
        outs64 = run_sequence(model64, vox, dtype=torch.float64)
        for f, (rec, st) in enumerate(outs64):
            res[f"{tag}_rec{f}_f64"] = rec.numpy()
    np.savez_compressed(os.path.join(out_dir, "f1_64x64.npz"), **res)

    # ---------------- F2: 32x48, C=32, depth 2, B=2, 4 frames, stress ----------------
    H, W, B, NF = 32, 48, 2, 4
    vox = fx.synthetic_voxels(NF, B, 5, H, W, n_events=fx.density_matched_events(H, W), seed=4321)
    model = CistaLSTCNet([H, W], base_channels=32, depth=2, num_bins=5)
    load_unique(model, fx.stress_params(32, 2, 5, seed=11))
    outs = run_sequence(model, vox)
    res = {"voxels": vox}
    for f, (rec, st) in enumerate(outs):
        res[f"rec{f}"] = rec.numpy()
    for k, v in states_np(outs[-1][1]).items():
        res[f"state_{k}"] = v
    np.savez_compressed(os.path.join(out_dir, "f2_32x48_c32_d2.npz"), **res)

    # ---------------- F3: 180x240, C=64, depth 5, B=1, 2 frames, stress ----------------
    H, W, B, NF = 180, 240, 1, 2
    vox = fx.synthetic_voxels(NF, B, 5, H, W, n_events=15000, seed=2024)
    model = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=5)
    load_unique(model, fx.stress_params(64, 5, 5))
    outs = run_sequence(model, vox)
    res = {"voxels": vox}
    for f, (rec, st) in enumerate(outs):
        res[f"rec{f}"] = rec.numpy()
        for k, v in states_np(st).items():
            res[f"state{f}_{k}_sum"] = np.float64(v.astype(np.float64).sum())
            res[f"state{f}_{k}_abssum"] = np.float64(np.abs(v.astype(np.float64)).sum())
            res[f"state{f}_{k}_row"] = v[0, :, v.shape[2] // 2, :].copy()   # one row, all channels
    np.savez_compressed(os.path.join(out_dir, "f3_180x240.npz"), **res)

    # ---------------- F4: 64x64, B=1, 15 frames, stress; drift vs fp64 ----------------
    H, W, B, NF = 64, 64, 1, 15
    vox = fx.synthetic_voxels(NF, B, 5, H, W, n_events=fx.density_matched_events(H, W), seed=777)
    model = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=5)
    load_unique(model, fx.stress_params(64, 5, 5))
    outs = run_sequence(model, vox)
    model64 = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=5)
    model64.load_state_dict(model.state_dict())
    outs64 = run_sequence(model64, vox, dtype=torch.float64)
    res = {"voxels": vox,
           "rec": np.stack([o[0].numpy() for o in outs]),
           "rec_f64": np.stack([o[0].numpy() for o in outs64])}
    for k, v in states_np(outs[-1][1]).items():
        res[f"state_{k}"] = v
    np.savez_compressed(os.path.join(out_dir, "f4_64x64_seq15.npz"), **res)
    print("golden fixtures written to", out_dir)


if __name__ == "__main__":
    main()
