"""Forward accuracy of one library build against fp64 references: F4 (15 frames, 64x64, B=1)
and the c3 gradient fixture's forward (180x240, 15 frames, B=1; its last frame, fp64)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from oracle import fixtures as fx
from tests.conftest import rel_err
from tests.golden.g3_spec import g3_inputs, g3_params
from v2e2v_amd import CistaLSTCNet


def run(params, vox):
    F_, B, nb, H, W = vox.shape
    m = CistaLSTCNet([H, W])
    m.load_state_dict(fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}, 5))
    m = m.cuda().eval()
    prev = torch.zeros(B, 1, H, W, device="cuda")
    st = None
    recs = []
    with torch.no_grad():
        for f in range(F_):
            prev, st = m(torch.from_numpy(vox[f]).cuda(), prev, st)
            recs.append(prev.cpu().numpy())
    return np.stack(recs)


d = np.load("tests/golden/f4_64x64_seq15.npz")
r = run(fx.stress_params(64, 5, 5), d["voxels"])
print("F4 vs f32 ref", rel_err(r, d["rec"]), "vs f64", rel_err(r, d["rec_f64"]))
g = np.load("tests/golden/grads_180x240_seq15.npz")
vox, _ = g3_inputs()
r = run(g3_params(), vox)
print("c3 last frame vs f32 ref", rel_err(r[-1], g["f32_last_frame"]))
