"""Inputs of the config-c3 batch gradient fixture (grads_180x240_b8.npz): BASELINE config c3 is
BPTT at 180x240 with batch 8; c4's per-rank shape is the same (8 GPUs x 8).  Shared by the
generator (make_golden_grads.py g4, which imports the reference) and the GPU tests, which must
not.  Sequence length 5: the fp64 autograd pass of 8 x 15 frames would hold ~80 GB of saved
activations on the generating host (~334 MB per frame and sample in fp32)."""
import numpy as np

from oracle import fixtures as fx

G4 = dict(C=64, depth=5, B=8, L=5, H=180, W=240, param_seed=21, lam=0.05, vox_seed=2025, target_seed=8)


def g4_params():
    return fx.stress_params(G4["C"], G4["depth"], 5, seed=G4["param_seed"], lam=G4["lam"])


def g4_inputs():
    """(voxels (L, B, 5, H, W) float32, L1 target (B, 1, H, W) float32)."""
    c = G4
    vox = fx.synthetic_voxels(c["L"], c["B"], 5, c["H"], c["W"], n_events=15000, seed=c["vox_seed"])
    target = np.random.default_rng(c["target_seed"]).uniform(0, 1, (c["B"], 1, c["H"], c["W"])).astype(np.float32)
    return vox, target
