"""Writes tests/golden/train_tiny/: a tiny training set in the reference's train_e2v.txt format
(data_readers/train_data_loaders.py:112-140: 'video_id num_events t0 t1 image next_image
events.npz' per line; '.npz' with fields t, x, y, p, :205-206) for the data-parallel loader tests.
Three videos of 24 x 32 frames: 40, 23 and 44 lines of 100-199 events; num_events 300 and
len_sequence 6 give 6 sequences, the third a video's 5-reconstruction tail (kept by the split
rule: the ragged case).  Run from the repo root: python tests/golden/make_train_tiny.py"""
import os

import numpy as np
from PIL import Image

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "train_tiny")
H, W = 24, 32


def main():
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(4)
    counts = [[int(rng.integers(100, 200)) for _ in range(n)] for n in (40, 23, 44)]
    lines, k = [], 0
    for vid, n_lines in enumerate([40, 23, 44]):
        for i in range(n_lines):
            n = counts[vid][i]
            t0 = float(k)
            # the first event time encodes (video, line): the tests read it back
            t = np.sort(np.concatenate([[t0], rng.uniform(t0 + 1e-3, t0 + 1, n - 1)]))
            np.savez(os.path.join(OUT, f"ev{k:03d}.npz"), t=t, x=rng.integers(0, W, n).astype(np.int16),
                     y=rng.integers(0, H, n).astype(np.int16), p=rng.integers(0, 2, n).astype(np.int8))
            Image.fromarray(rng.integers(0, 256, (H, W), dtype=np.uint8)).save(os.path.join(OUT, f"im{k:03d}.png"))
            lines.append(f"{vid} {n} {t0:.1f} {t0 + 1:.1f} im{k:03d}.png im{k + 1:03d}.png ev{k:03d}.npz")
            k += 1
    Image.fromarray(rng.integers(0, 256, (H, W), dtype=np.uint8)).save(os.path.join(OUT, f"im{k:03d}.png"))
    with open(os.path.join(OUT, "train_e2v.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
