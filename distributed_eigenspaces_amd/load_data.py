"""CIFAR-10 batch loader with the reference's API (load_data.py:8-50).

``load_CIFAR_10_data(data_dir, negatives=False) -> (data, filenames, labels)``:
every file in ``data_dir`` except ``readme.html`` and ``batches.meta`` is a
CIFAR python batch (a pickled dict with b'data' (N x 3072 uint8, channel-major
32x32 planes), b'filenames', b'labels'); batches are stacked in directory
order, reshaped to (N, 3, 32, 32) and moved to channels-last (N, 32, 32, 3)
as uint8, or as float32 when ``negatives`` is True (load_data.py:28-29).

Like the reference, the train batches and ``test_batch`` are all loaded (so the
real dataset gives 60000 rows, NB:41).  ``grayscale_flatten`` is the
distributed.py:170-173 preprocessing (mean over RGB, flatten to R^1024), here as
one device op so it can run next to the covariance.

Note: CIFAR batches are Python pickles by format; only load datasets you trust.
"""
from __future__ import annotations

import glob
import os
import pickle

import numpy as np

__all__ = ["load_CIFAR_10_data", "load_data", "unpickle", "grayscale_flatten"]

UNUSED_FILES = ("readme.html", "batches.meta")


def unpickle(path):
    with open(path, "rb") as fh:
        return pickle.load(fh, encoding="bytes")


def load_data(paths, negatives: bool = False):
    if not paths:
        raise FileNotFoundError("no CIFAR batch files found")
    parts, names, labels = [], [], []
    for p in paths:
        batch = unpickle(p)
        parts.append(np.asarray(batch[b"data"]))
        names.extend(batch[b"filenames"])
        labels.extend(batch[b"labels"])
    raw = np.concatenate(parts, axis=0).reshape(-1, 3, 32, 32)
    img = raw.transpose(0, 2, 3, 1)
    img = img.astype(np.float32) if negatives else np.ascontiguousarray(img)
    return img, np.array(names), np.array(labels)


def load_CIFAR_10_data(data_dir, negatives: bool = False):
    paths = [p for p in glob.glob(os.path.join(data_dir, "*"))
             if os.path.basename(p) not in UNUSED_FILES]
    return load_data(paths, negatives)


def grayscale_flatten(images):
    """(N, 32, 32, 3) -> (N, 1024) float32 on the GPU: mean over channels, flatten.

    Same values as ``data.mean(axis=3).reshape(N, -1)`` (distributed.py:171-173)
    rounded once to fp32: the channel sum is exact and the division is done in
    float64 on the device, then rounded (fp32 division on the device is not
    correctly rounded)."""
    import torch

    from .linalg import require_device_tensor
    if isinstance(images, np.ndarray):
        images = torch.from_numpy(np.ascontiguousarray(images))
    if not torch.cuda.is_available():
        raise RuntimeError("grayscale_flatten runs on the GPU (no CPU fallback)")
    x = images.to(device=torch.device("cuda", torch.cuda.current_device()))
    x = (x.to(torch.float64).sum(dim=3) / 3.0).to(torch.float32)
    return require_device_tensor(x.reshape(x.shape[0], -1), "images")
