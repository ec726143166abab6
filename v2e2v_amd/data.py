"""Event / frame readers feeding the CISTA-LSTC path.

Host-side file IO mirrors the reference's readers (same names, arguments and file formats);
the voxelisation they end in runs on the GPU through the batched HIP voxelizer
(v2e2v_amd/event_process.py), one launch sequence for every window of a batch of sequences:

* ``read_timestamps_file``     <- data_readers/video_readers.py:11-39
* ``SingleEventReaderNpz``     <- data_readers/event_readers.py:60-84 ('.npz' with t, x, y, p)
* ``RefTimeEventReaderZip``    <- data_readers/event_readers.py:6-57 (space-separated t x y p)
* ``TrainFixNEventData``       <- data_readers/train_data_loaders.py:106-223: the train_e2v.txt
  line format, the sequence split by event count (``split_sequences``) and the per-item event
  windows; ``__getitem__`` returns the RAW windows of a sequence (so DataLoader workers never
  touch the GPU) and ``GpuVoxelLoader`` turns a batch of them into exactly what the reference
  loader yields -- ``(seq_events, img, gt_img)`` with ``seq_events[s]`` a (B, num_bins, H, W)
  voxel tensor -- voxelised on the GPU (event_preprocess(filter_hot_pixel=False), :187-193).
* ``SequenceShardSampler``     -- data-parallel training (config c4): the reference's
  ``DataLoader(shuffle=cfgs.shuffle)`` (train_e2v.py:60-61) becomes one rank-disjoint shard of
  the sequences per process; ``GpuVoxelLoader(..., rank, world_size)`` builds it (by default from
  the initialised torch.distributed group), so ``batch_size`` is the PER-RANK batch.

Images are read with PIL (the reference uses cv2.IMREAD_GRAYSCALE; cv2 is not installed):
8-bit grayscale / 255, float32.
"""
from __future__ import annotations

import os
from os.path import splitext

import numpy as np
import torch

from . import event_process as ep


def read_timestamps_file(path_to_timestamps, unit="s"):
    """video_readers.py:11-39: second column of a 'timestamps.txt', else first column; 'us'/'ns'
    rescaled to seconds."""
    col = 1 if path_to_timestamps.split("/")[-1] == "timestamps.txt" else 0
    ts = []
    with open(path_to_timestamps, "r") as f:
        for line in f:
            ts.append(float(line.strip().split()[col]))
    ts = np.array(ts)
    if unit in ["us"]:
        ts /= 1e6
    elif unit in ["ns"]:
        ts /= 1e9
    return list(ts)


def load_npz_events(path):
    """event_readers.py:81-82 / train_data_loaders.py:205-206: (N, 4) rows (t, x, y, p)."""
    ev = np.load(path)
    return np.stack((ev["t"], ev["x"], ev["y"], ev["p"]), axis=1)


class SingleEventReaderNpz:
    """event_readers.py:60-84: iterate over a list of '.npz' event windows."""

    def __init__(self, path_to_events):
        self.path_to_events = path_to_events
        self.len = len(self.path_to_events)
        self.frame_id = 0

    def __iter__(self):
        return self

    def __next__(self):
        if self.frame_id >= self.len:
            raise StopIteration
        window = load_npz_events(self.path_to_events[self.frame_id])
        self.frame_id += 1
        return window


class RefTimeEventReaderZip:
    """event_readers.py:6-57: one text file of events 't x y p', cut into windows at the
    reference image timestamps T_image."""

    def __init__(self, path_to_event_file, T_image):
        import pandas as pd
        if splitext(path_to_event_file)[1] not in [".txt", ".csv", ".zip"]:
            raise AssertionError("event file must be .txt, .csv or .zip")
        self.iterator = pd.read_csv(path_to_event_file, iterator=False, delimiter=" ", names=["t", "x", "y", "p"],
                                    dtype={"t": np.float64, "x": np.int16, "y": np.int16, "p": np.int16},
                                    engine="c", index_col=False)
        self.T_image = np.array(T_image) - T_image[0]
        self.len = len(T_image) - 1
        timestamps = self.iterator.loc[:, ["t"]].values
        self.t0 = T_image[0]
        timestamps -= T_image[0]
        self.bound_index = []
        for t in self.T_image:
            idx = np.where(timestamps >= t)[0]
            self.bound_index.append(len(timestamps) - 1 if len(idx) == 0 else idx[0])
        self.frame_id = 0

    def __iter__(self):
        return self

    def __next__(self):
        if self.frame_id >= self.len:
            raise StopIteration
        a, b = self.bound_index[self.frame_id], self.bound_index[self.frame_id + 1]
        window = self.iterator.values[a:b]
        window[:, 0] -= self.t0
        self.frame_id += 1
        return window


def split_sequences(video_cnt, num_events_list, limit_num_events, len_sequence):
    """train_data_loaders.py:149-184, verbatim semantics: group the txt lines into
    reconstructions of >= limit_num_events events (or a single line above 80 % of it) and those
    into sequences of len_sequence reconstructions; a video's unfinished tail sequence is kept if
    it has >= 5 reconstructions."""
    prev_video_id = -1
    sum_num_events = 0
    sequence_line_id = []
    per_rec, per_seq = [], []
    frame_cnt, single_frame_cnt = 0, 0
    for line_id, video_id in enumerate(video_cnt):
        if video_id != prev_video_id:
            if len(per_seq) >= 5:
                if per_rec:
                    per_seq.append(per_rec)
                sequence_line_id.append(per_seq)
            per_seq, per_rec = [], []
            prev_video_id = video_id
            sum_num_events = 0
            single_frame_cnt = 0
            frame_cnt = 0
        cur = num_events_list[line_id]
        sum_num_events += cur
        per_rec.append(line_id)
        single_frame_cnt += 1
        if sum_num_events >= limit_num_events or (single_frame_cnt == 1 and sum_num_events > 0.8 * limit_num_events):
            per_seq.append(per_rec)
            frame_cnt += 1
            sum_num_events = 0
            single_frame_cnt = 0
            per_rec = []
        if frame_cnt >= len_sequence:
            sequence_line_id.append(per_seq)
            per_seq, per_rec = [], []
            frame_cnt = 0
    return sequence_line_id


def _read_gray(path):
    from PIL import Image
    return np.asarray(Image.open(path).convert("L"), dtype=np.float32) / 255.0


class TrainFixNEventData(torch.utils.data.Dataset):
    """train_data_loaders.py:106-223 with GPU voxelisation moved out of the item (see module
    docstring).  cfgs needs path_to_train_data, num_bins, image_dim, num_events, len_sequence,
    add_noise -- the reference's fields."""

    def __init__(self, train_data_txt, cfgs):
        self.txt_file = train_data_txt
        self.path_to_train_data = cfgs.path_to_train_data
        self.num_bins = cfgs.num_bins
        self.height, self.width = cfgs.image_dim
        self.limit_num_events = cfgs.num_events
        self.len_sequence = cfgs.len_sequence
        self.add_noise = cfgs.add_noise
        self.video_cnt, self.event_paths, self.image_paths = [], [], []
        self.next_image_paths, self.num_events_list = [], []
        with open(self.txt_file, "rb") as f:
            for line in f:
                s = line.strip().split()
                self.video_cnt.append(int(s[0]))
                self.num_events_list.append(int(s[1]))
                self.image_paths.append(str(s[4], encoding="utf-8"))
                self.next_image_paths.append(str(s[5], encoding="utf-8"))
                self.event_paths.append(str(s[6], encoding="utf-8"))
        self.sequence_line_id = split_sequences(self.video_cnt, self.num_events_list, self.limit_num_events,
                                                self.len_sequence)

    def __len__(self):
        return len(self.sequence_line_id)

    def __getitem__(self, index):
        """(events (N, 4) float64 of all windows concatenated, window sizes (L,), img, gt_img):
        a window is the concatenation of its lines' npz files (:198-206)."""
        seq = self.sequence_line_id[index]
        windows = []
        for rec in seq:
            parts = [np.empty((0, 4), dtype=np.float32)]
            for line_id in rec:
                parts.append(load_npz_events(os.path.join(self.path_to_train_data, self.event_paths[line_id])))
            windows.append(np.concatenate(parts, 0).astype(np.float64))
        sizes = np.array([len(w) for w in windows], dtype=np.int64)
        events = np.concatenate(windows, 0) if windows else np.zeros((0, 4))
        img = _read_gray(os.path.join(self.path_to_train_data, self.image_paths[seq[0][0]]))[None]
        gt = _read_gray(os.path.join(self.path_to_train_data, self.next_image_paths[seq[-1][-1]]))[None]
        return torch.from_numpy(events), torch.from_numpy(sizes), torch.from_numpy(img), torch.from_numpy(gt)


class SequenceShardSampler(torch.utils.data.Sampler):
    """The sequences of one rank of a data-parallel job.  Every epoch the same permutation is
    drawn on all ranks (torch.randperm seeded with seed + epoch when shuffle, else identity), cut
    to a multiple of world_size, and rank r takes positions r, r + world, r + 2 world, ...: the
    shards are disjoint, every rank yields the same number of sequences (so DDP ranks run the
    same number of steps and meet in every gradient all-reduce), and together they cover the
    epoch except its last n % world_size sequences (a different few each shuffled epoch).
    Unlike torch's DistributedSampler no sequence is duplicated to pad the epoch."""

    def __init__(self, n_sequences: int, rank: int, world_size: int, shuffle: bool = False, seed: int = 0):
        if world_size < 1 or not 0 <= rank < world_size:
            raise ValueError(f"rank {rank} outside world_size {world_size}")
        self.n, self.rank, self.world = int(n_sequences), int(rank), int(world_size)
        self.shuffle, self.seed, self.epoch = bool(shuffle), int(seed), 0

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def __iter__(self):
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g).tolist()
        else:
            order = list(range(self.n))
        used = (self.n // self.world) * self.world
        return iter(order[self.rank:used:self.world])

    def __len__(self):
        return self.n // self.world


class GpuVoxelLoader:
    """Iterate a DataLoader over TrainFixNEventData and voxelise each batch on the GPU:
    yields (seq_events, img, gt_img) like the reference loader (train_e2v.py:104-107), with every
    B x L window of the batch voxelised in one cista_voxelize call (mode 'std', no hot-pixel
    filter, train_data_loaders.py:192).  add_noise (``add_noise_to_voxel`` with std 0.1, fraction
    1, :209-210) is applied on the device with torch's RNG, as the reference does with torch.

    Data parallel (config c4): with world_size > 1 -- given, or taken from the initialised
    torch.distributed group -- the loader reads only this rank's SequenceShardSampler shard and
    ``batch_size`` is the per-rank batch (global batch = world_size x batch_size).  ``shuffle``
    then goes to the sampler (same permutation on every rank); call ``set_epoch`` each epoch.

    ``strict`` (default): an event file with events outside the frame fails like the reference's
    dataset does (IndexError from np.add.at; see event_process.events_to_voxel_batch) -- one
    stream synchronisation per batch."""

    def __init__(self, dataset: TrainFixNEventData, device, rank: int | None = None, world_size: int | None = None,
                 shuffle: bool = False, seed: int = 0, strict: bool = True, **loader_kwargs):
        self.ds = dataset
        self.device = torch.device(device)
        self.strict = bool(strict)
        dd = torch.distributed
        pg = dd.is_available() and dd.is_initialized()
        if world_size is None:
            world_size = dd.get_world_size() if pg else 1
        if rank is None:
            if int(world_size) > 1 and not pg:
                # every process would otherwise take rank 0 and read the same shard
                raise ValueError("GpuVoxelLoader: world_size > 1 needs rank= (or an initialised process group)")
            rank = dd.get_rank() if int(world_size) > 1 else 0
        if not 0 <= int(rank) < int(world_size):
            raise ValueError(f"GpuVoxelLoader: rank {rank} outside world_size {world_size}")
        self.rank, self.world_size = int(rank), int(world_size)
        self.sampler = None
        if self.world_size > 1:
            if "sampler" in loader_kwargs or loader_kwargs.get("shuffle"):
                raise ValueError("data-parallel GpuVoxelLoader: pass shuffle=/seed= to the loader, not a sampler")
            self.sampler = SequenceShardSampler(len(dataset), self.rank, self.world_size, shuffle, seed)
            loader_kwargs["sampler"] = self.sampler
        else:
            loader_kwargs.setdefault("shuffle", shuffle)
        loader_kwargs.setdefault("collate_fn", self._collate)
        self.loader = torch.utils.data.DataLoader(dataset, **loader_kwargs)

    def set_epoch(self, epoch: int):
        """Reshuffle the rank shards for this epoch (no-op single-process: the DataLoader's own
        shuffle draws a new order every epoch)."""
        if self.sampler is not None:
            self.sampler.set_epoch(epoch)

    @staticmethod
    def _collate(items):
        return items

    def __len__(self):
        return len(self.loader)

    @staticmethod
    def batch_length(items):
        """Sequence length of a batch.  split_sequences keeps a video's tail sequence when it
        has enough reconstructions, so lengths can differ; the reference's default collate
        refuses such a batch (torch default_collate: 'each element in list of batch should be
        of equal size'), and so does this loader -- truncating would pair the full-length items'
        frames with a ground truth from a later window."""
        lens = {len(it[1]) for it in items}
        if len(lens) != 1:
            raise RuntimeError(f"each element in list of batch should be of equal size (sequence "
                               f"lengths {sorted(lens)} in one batch)")
        return lens.pop()

    def __iter__(self):
        for items in self.loader:
            L = self.batch_length(items)
            evs, sizes = [], []
            for s in range(L):                       # window order: (step, sequence)
                for events, sz, _, _ in items:
                    off = int(sz[:s].sum())
                    evs.append(events[off:off + int(sz[s])])
                    sizes.append(int(sz[s]))
            events = torch.cat(evs, 0) if evs else torch.zeros(0, 4, dtype=torch.float64)
            offsets = torch.tensor(np.concatenate([[0], np.cumsum(sizes)]), dtype=torch.int64)
            vox = ep.events_to_voxel_batch((events.to(self.device), offsets), self.ds.num_bins, self.ds.width,
                                           self.ds.height, mode="std", filter_hot_pixel=False, device=self.device,
                                           strict=self.strict)
            B = len(items)
            vox = vox.view(L, B, self.ds.num_bins, self.ds.height, self.ds.width)
            if self.ds.add_noise:
                vox = vox + 0.1 * torch.randn_like(vox)
            img = torch.stack([it[2] for it in items]).to(self.device)
            gt = torch.stack([it[3] for it in items]).to(self.device)
            yield [vox[s] for s in range(L)], img, gt
