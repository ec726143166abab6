"""Readers of SURVEY section 8 row f4 (host side): file formats and the sequence split of
reference data_readers/train_data_loaders.py:149-184, checked on hand-built known answers."""
import os
import types

import numpy as np
import pytest
import torch

from v2e2v_amd import data


def test_split_sequences_known_answer():
    # video 0: 14 lines of 6000 events -> reconstructions of 3 lines (18000 >= 15000) ... wait for
    # the 0.8 rule: a single line > 12000 closes a reconstruction alone
    video = [0] * 7 + [1] * 3 + [2] * 12
    nev = [13000, 5000, 5000, 6000, 20000, 1000, 1000] + [16000] * 3 + [16000] * 12
    seqs = data.split_sequences(video, nev, 15000, 5)
    # video 0: [0] (single > 12000), [1,2,3] (16000), [4] (single), [5,6] unfinished -> 3 recs < 5: dropped
    # video 1: 3 recs -> dropped when video 2 starts; video 2: 12 single-line recs -> one full
    # sequence of 5, a second of 5, tail of 2 dropped at the end (no later video to flush it)
    assert seqs == [[[10], [11], [12], [13], [14]], [[15], [16], [17], [18], [19]]]
    # a video change flushes a >= 5-reconstruction tail together with its open reconstruction
    video = [0] * 6 + [1]
    nev = [16000] * 5 + [100, 100]
    assert data.split_sequences(video, nev, 15000, 10) == [[[0], [1], [2], [3], [4], [5]]]


def test_readers_roundtrip(tmp_path):
    ts = tmp_path / "timestamps.txt"
    ts.write_text("0 1.5\n1 2.5\n")
    assert data.read_timestamps_file(str(ts)) == [1.5, 2.5]
    other = tmp_path / "ts_us.txt"
    other.write_text("1000000\n3000000\n")
    assert data.read_timestamps_file(str(other), unit="us") == [1.0, 3.0]
    rng = np.random.default_rng(0)
    t = np.sort(rng.uniform(0, 1, 50))
    np.savez(tmp_path / "e0.npz", t=t, x=rng.integers(0, 10, 50), y=rng.integers(0, 8, 50), p=rng.integers(0, 2, 50))
    ev = next(data.SingleEventReaderNpz([str(tmp_path / "e0.npz")]))
    assert ev.shape == (50, 4) and ev.dtype == np.float64 and np.array_equal(ev[:, 0], t)
    txt = tmp_path / "ev.txt"
    with open(txt, "w") as f:
        for i in range(20):
            f.write(f"{0.1 * i:.6f} {i % 5} {i % 3} {i % 2}\n")
    wins = list(data.RefTimeEventReaderZip(str(txt), [0.0, 0.5, 1.0, 1.5]))
    assert [len(w) for w in wins] == [5, 5, 5]
    assert abs(wins[1][0, 0] - 0.5) < 1e-9


def make_dataset(tmp_path, n_lines=12, H=24, W=32):
    from PIL import Image
    rng = np.random.default_rng(1)
    lines = []
    for i in range(n_lines):
        n = int(rng.integers(300, 900))
        np.savez(tmp_path / f"ev{i}.npz", t=np.sort(rng.uniform(i, i + 1, n)), x=rng.integers(0, W, n),
                 y=rng.integers(0, H, n), p=rng.integers(0, 2, n))
        Image.fromarray(rng.integers(0, 256, (H, W), dtype=np.uint8)).save(tmp_path / f"im{i}.png")
        Image.fromarray(rng.integers(0, 256, (H, W), dtype=np.uint8)).save(tmp_path / f"im{i + 1}n.png")
        lines.append(f"0 {n} {i}.0 {i + 1}.0 im{i}.png im{i + 1}n.png ev{i}.npz")
    (tmp_path / "train_e2v.txt").write_text("\n".join(lines) + "\n")
    cfgs = types.SimpleNamespace(path_to_train_data=str(tmp_path), num_bins=5, image_dim=[H, W], num_events=1000,
                                 len_sequence=5, add_noise=False)
    return data.TrainFixNEventData(str(tmp_path / "train_e2v.txt"), cfgs)


def test_train_dataset_items(tmp_path):
    ds = make_dataset(tmp_path)
    assert len(ds) >= 1
    events, sizes, img, gt = ds[0]
    seq = ds.sequence_line_id[0]
    assert len(sizes) == len(seq) == 5
    first = data.load_npz_events(str(tmp_path / ds.event_paths[seq[0][0]]))
    assert np.array_equal(events[: len(first)].numpy(), first.astype(np.float64))
    assert int(sizes.sum()) == events.shape[0]
    assert img.shape == (1, 24, 32) and img.dtype == torch.float32 and float(img.max()) <= 1.0


def test_ragged_batch_refused_like_default_collate():
    # a video's tail sequence (>= 5 reconstructions but < len_sequence) next to a full one:
    # the reference's default collate raises; truncating would mislabel the full-length item
    full = (torch.zeros(0, 4), torch.tensor([10] * 8), None, None)
    tail = (torch.zeros(0, 4), torch.tensor([10] * 5), None, None)
    assert data.GpuVoxelLoader.batch_length([full, full]) == 8
    with pytest.raises(RuntimeError, match="equal size"):
        data.GpuVoxelLoader.batch_length([full, tail])
