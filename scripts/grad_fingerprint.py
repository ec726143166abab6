"""Every parameter and input gradient of one BPTT step (180x240, B=2, 2 frames, stress weights)
into an npz, to compare two builds of the library bit for bit:
  CISTA_HIP_LIB=a.so python scripts/grad_fingerprint.py out_a.npz
  CISTA_HIP_LIB=b.so python scripts/grad_fingerprint.py out_b.npz
  python scripts/grad_fingerprint.py --compare out_a.npz out_b.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def compare(a, b):
    x, y = np.load(a), np.load(b)
    diff = [k for k in x.files if not np.array_equal(x[k], y[k])]
    print(f"{len(x.files)} arrays, {len(diff)} differ" + (": " + ", ".join(diff[:8]) if diff else ""))
    return 1 if diff else 0


def main(path):
    import torch
    from oracle import fixtures as fx
    from v2e2v_amd import CistaLSTCNet
    dev = "cuda"
    B, L, H, W = 2, 2, 180, 240
    m = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=5)
    p = fx.stress_params(64, 5, 5, seed=47, lam=0.05)
    m.load_state_dict(fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in p.items()}, 5))
    m = m.to(dev)
    rng = np.random.default_rng(3)
    evs = [torch.from_numpy(rng.standard_normal((B, 5, H, W)).astype(np.float32)).to(dev).requires_grad_(True)
           for _ in range(L)]
    target = torch.from_numpy(rng.random((B, 1, H, W)).astype(np.float32)).to(dev)
    prev, state = torch.zeros(B, 1, H, W, device=dev), None
    for f in range(L):
        out, state = m(evs[f], prev, state)
        prev = out.clone()
    (out - target).abs().mean().backward()
    torch.cuda.synchronize()
    res = {k: v.grad.detach().cpu().numpy() for k, v in m.named_parameters()}
    res.update({f"events{f}": e.grad.detach().cpu().numpy() for f, e in enumerate(evs)})
    np.savez(path, **res)


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    main(sys.argv[1])
