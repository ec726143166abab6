"""Experiment: does running the batch as k concurrent half/quarter batches on k HIP streams
(each its own whole-sequence hipGraph and workspace) beat one stream over the whole batch?
Different kernels of the frame then share the CUs, so one sequence's HBM-heavy phases
(staging, epilogue stores) can overlap another's MFMA phases.
usage: python scripts/stream_split.py [B] [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from v2e2v_amd import CistaLSTCNet  # noqa: E402
from v2e2v_amd.sequence import CistaSequence  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    H, W, L = 180, 240, 15
    dev = torch.device("cuda", 0)
    model = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=5)
    bench.he_init_(torch, model, seed=7)
    model = model.to(dev).eval()
    vox = bench.synth_voxels(torch, L, B, 5, H, W, 15000, seed=1000, device=dev)
    out = {}
    ref = None
    with torch.no_grad():
        for k in (1, 2, 4):
            Bk = B // k
            models = [model]
            for _ in range(k - 1):
                m2 = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=5).to(dev).eval()
                m2.load_state_dict(model.state_dict())
                models.append(m2)
            seqs = [CistaSequence(models[i], vox[:, i * Bk:(i + 1) * Bk].contiguous()) for i in range(k)]
            streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(k - 1)]

            def run():
                cur = torch.cuda.current_stream(dev)
                for s in streams[1:]:
                    s.wait_stream(cur)
                res = []
                for s, q in zip(streams, seqs):
                    with torch.cuda.stream(s):
                        res.append(q.run()[0])
                for s in streams[1:]:
                    cur.wait_stream(s)
                return res

            run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                res = run()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            recs = torch.cat([r[-1] for r in res], 0)
            if ref is None:
                ref = recs.clone()
            out[k] = {"frames_per_s": round(B * L * steps / dt, 1),
                      "max_abs_diff_vs_k1": float((recs - ref).abs().max())}
            print(k, out[k], flush=True)
            for q in seqs:
                q.close()
            del seqs, models
    print(json.dumps(out))


if __name__ == "__main__":
    main()
