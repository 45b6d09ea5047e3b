"""CIFAR-10 data layer: dataset sources, the DistributedSampler-equivalent shard sampler, and a
device-resident loader whose augmentation runs as one HIP kernel per batch.

Reference (main.py:71-98, main_gather.py:109-136): torchvision CIFAR10 + RandomCrop(32, pad 4)
+ RandomHorizontalFlip + ToTensor + Normalize, DataLoader(batch 256, 2 workers), train sharded by
DistributedSampler(shuffle=True, seed=0, drop_last=False), test set NOT sharded.

Here the whole uint8 dataset (150 MB) is uploaded once; each batch is (index slice → K10 augment
kernel → NHWC fp32 with a zero 4th channel), so no worker processes and no per-batch H2D copy sit
in the training loop.  Sources: the CIFAR-10 binary release (``cifar-10-batches-bin``), the
python release (``cifar-10-batches-py``), or deterministic synthetic data of the same shape
(no network on the GPU boxes; BASELINE.json asks for synthetic data).
"""
from __future__ import annotations

import math
import os
import pickle
from typing import Iterator, List, Optional, Tuple

import numpy as np
import torch

MEAN = [x / 255.0 for x in [125.3, 123.0, 113.9]]  # main.py:71
STD = [x / 255.0 for x in [63.0, 62.1, 66.7]]      # main.py:72


class ImageSet:
    """uint8 images [N, H, W, 3] (HWC) + int64 labels [N]."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, name: str = ""):
        assert images.dtype == torch.uint8 and images.dim() == 4 and images.shape[-1] == 3
        self.images = images
        self.labels = labels.to(torch.int64)
        self.name = name

    def __len__(self):
        return self.images.shape[0]

    def to(self, device) -> "ImageSet":
        return ImageSet(self.images.to(device), self.labels.to(device), self.name)


def synthetic_cifar(n: int, seed: int = 0, num_classes: int = 10, hw: int = 32) -> ImageSet:
    """Deterministic, *learnable* CIFAR-shaped data: each class has a random low-frequency colour
    template; an image is its class template plus per-image noise and a random shift.  Loss
    decreases and test accuracy rises above chance, so the logs are meaningful."""
    g = torch.Generator().manual_seed(1234 + seed)
    tmpl = torch.rand(num_classes, 3, 8, 8, generator=g)
    tmpl = torch.nn.functional.interpolate(tmpl, size=(hw, hw), mode="bilinear", align_corners=False)
    labels = torch.randint(0, num_classes, (n,), generator=g)
    out = torch.empty(n, hw, hw, 3, dtype=torch.uint8)
    bs = 4096
    for s in range(0, n, bs):
        lb = labels[s:s + bs]
        base = tmpl[lb]
        noise = torch.rand(base.shape, generator=g) * 0.6 - 0.3
        img = (base * 0.8 + noise + 0.1).clamp(0, 1)
        out[s:s + bs] = (img * 255).round().to(torch.uint8).permute(0, 2, 3, 1)
    return ImageSet(out, labels, "synthetic")


def _read_bin_batches(files: List[str]) -> ImageSet:
    recs = []
    for f in files:
        raw = np.fromfile(f, dtype=np.uint8).reshape(-1, 3073)
        recs.append(raw)
    raw = np.concatenate(recs, 0)
    labels = torch.from_numpy(raw[:, 0].astype(np.int64))
    imgs = torch.from_numpy(raw[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1).copy())
    return ImageSet(imgs, labels, "cifar10")


class _CifarUnpickler(pickle.Unpickler):
    """The python release of CIFAR-10 is pickled dicts of numpy arrays, lists and bytes.  A plain
    ``pickle.load`` would run whatever callable a tampered file names, so only the numpy array
    reconstruction hooks are admitted; any other global in the stream is refused."""

    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"), ("numpy", "dtype"),
        ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from a CIFAR-10 batch file")


def safe_load_batch(path: str) -> dict:
    with open(path, "rb") as fh:
        d = _CifarUnpickler(fh, encoding="bytes").load()
    if not isinstance(d, dict):
        raise pickle.UnpicklingError(f"{path}: expected a dict, got {type(d).__name__}")
    return d


def _read_py_batches(files: List[str]) -> ImageSet:
    # The user's own torchvision-format CIFAR-10 download (pickled dicts, as torchvision reads it),
    # read with a restricted unpickler.
    xs, ys = [], []
    for f in files:
        d = safe_load_batch(f)
        xs.append(np.asarray(d[b"data"], dtype=np.uint8))
        ys += list(d[b"labels"])
    x = np.concatenate(xs, 0).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1).copy()
    return ImageSet(torch.from_numpy(x), torch.tensor(ys, dtype=torch.int64), "cifar10")


def load_cifar10(root: str, train: bool) -> ImageSet:
    """Load CIFAR-10 from ``root`` (binary or python release); raises FileNotFoundError."""
    b = os.path.join(root, "cifar-10-batches-bin")
    if os.path.isdir(b):
        files = [os.path.join(b, f"data_batch_{i}.bin") for i in range(1, 6)] if train else [
            os.path.join(b, "test_batch.bin")]
        return _read_bin_batches(files)
    p = os.path.join(root, "cifar-10-batches-py")
    if os.path.isdir(p):
        files = [os.path.join(p, f"data_batch_{i}") for i in range(1, 6)] if train else [os.path.join(p, "test_batch")]
        return _read_py_batches(files)
    raise FileNotFoundError(f"no CIFAR-10 under {root} (expected cifar-10-batches-bin/ or cifar-10-batches-py/)")


def get_datasets(data_root: Optional[str], synthetic: bool, train_size: int = 50000, test_size: int = 10000):
    if not synthetic and data_root:
        try:
            return load_cifar10(data_root, True), load_cifar10(data_root, False)
        except FileNotFoundError:
            pass
    return synthetic_cifar(train_size, 0), synthetic_cifar(test_size, 1)


class ShardSampler:
    """Exact ``torch.utils.data.DistributedSampler`` semantics (shuffle with a generator seeded
    ``seed + epoch``; pad by repeating the head so every replica gets ``ceil(N/W)`` samples;
    rank-strided subsample).  Unlike the reference (which never calls it) ``set_epoch`` is used
    so each epoch reshuffles."""

    def __init__(self, n: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False):
        self.n, self.num_replicas, self.rank = n, num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        if drop_last and n % num_replicas:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def indices(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g)
        else:
            idx = torch.arange(self.n)
        if not self.drop_last:
            pad = self.total_size - idx.numel()
            if pad > 0:
                reps = math.ceil(pad / idx.numel())
                idx = torch.cat([idx, idx.repeat(reps)[:pad]])
        else:
            idx = idx[:self.total_size]
        return idx[self.rank:self.total_size:self.num_replicas]

    def __len__(self):
        return self.num_samples


class DeviceLoader:
    """Iterates (x [n,H,W,4] fp32 NHWC, target [n] int64) batches produced on-device.

    The returned tensors are views of persistent buffers that the NEXT batch overwrites —
    consume a batch before requesting the next one (the training loop does)."""

    def __init__(self, dataset: ImageSet, batch_size: int, device, sampler: Optional[ShardSampler] = None,
                 train: bool = True, seed: int = 0, pad: int = 4, backend=None, drop_last: bool = False):
        self.device = torch.device(device)
        self.ds = dataset.to(self.device)
        self.batch_size = batch_size
        self.sampler = sampler
        self.train = train
        self.seed = seed
        self.pad = pad
        self.drop_last = drop_last
        self.epoch = 0
        if backend is None:
            if self.device.type == "cuda":
                from .. import _ext

                backend = _ext.require()
            else:
                from ..ops import cpu_ref as backend
        self.K = backend
        hw = self.ds.images.shape[1]
        self.x = torch.zeros(batch_size, hw, hw, 4, device=self.device)
        self.t = torch.zeros(batch_size, dtype=torch.int64, device=self.device)
        self._idx = None

    def set_epoch(self, epoch: int):
        self.epoch = epoch
        if self.sampler is not None:
            self.sampler.set_epoch(epoch)

    def _epoch_indices(self) -> torch.Tensor:
        if self.sampler is not None:
            idx = self.sampler.indices()
        else:
            idx = torch.arange(len(self.ds))
        return idx.to(self.device, torch.int64)

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.ds)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    @property
    def dataset_len(self) -> int:
        return len(self.ds)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        return self.iterate(0)

    def iterate(self, start_batch: int = 0) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        idx = self._epoch_indices()
        n = idx.numel()
        for b, s in enumerate(range(0, n, self.batch_size)):
            if b < start_batch:
                continue
            bi = idx[s:s + self.batch_size]
            m = bi.numel()
            if self.drop_last and m < self.batch_size:
                break
            salt = (self.epoch * 1_000_003 + b) & 0x7FFFFFFFFFFF
            self.K.augment(self.ds.images, bi, self.ds.labels, self.x[:m], self.t[:m], self.pad, self.train,
                           self.seed, salt, MEAN, STD)
            yield self.x[:m], self.t[:m]
