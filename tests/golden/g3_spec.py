"""Inputs of the c3-size gradient fixture (grads_180x240_seq15.npz): shared by the generator
(make_golden_grads.py, which imports the reference) and the GPU test, which must not."""
import numpy as np

from oracle import fixtures as fx

G3 = dict(C=64, depth=5, B=1, L=15, H=180, W=240, param_seed=21, lam=0.05, vox_seed=2024, target_seed=7)


def g3_params():
    return fx.stress_params(G3["C"], G3["depth"], 5, seed=G3["param_seed"], lam=G3["lam"])


def g3_inputs():
    """(voxels (L, B, 5, H, W) float32, L1 target (B, 1, H, W) float32)."""
    c = G3
    vox = fx.synthetic_voxels(c["L"], c["B"], 5, c["H"], c["W"], n_events=15000, seed=c["vox_seed"])
    target = np.random.default_rng(c["target_seed"]).uniform(0, 1, (c["B"], 1, c["H"], c["W"])).astype(np.float32)
    return vox, target
