"""Image federated datasets: CIFAR-10/100, FEMNIST, ImageNet (reference on-disk
formats) and synthetic look-alikes.

All in-memory image datasets keep their training images as ONE uint8
``[N, H, W, C]`` array in natural-client-major order (client 0's images, then
client 1's, ...) and expose it through ``arrays()`` so the device loader can
place the whole dataset in HBM and assemble batches on the GPU.

Formats (reference files):
* CIFAR10/100 (data_utils/fed_cifar.py:45-96): ``stats.json``
  ``{"images_per_client": [...], "num_val_images": N}``, ``client{i}.npy``
  uint8 [n,32,32,3] (one class per file), ``test.npz`` {test_images, test_targets}.
* EMNIST/FEMNIST (fed_emnist.py:82-138): ``train/client{i}.pt`` {"x": [n,28,28],
  "y": [n]}, ``test/test.pt``, ``stats.json``.  Loaded with
  ``torch.load(weights_only=True)``.
* ImageNet (fed_imagenet.py:21-64): class-per-client; ``stats.json`` with
  per-class counts; images read from ``train/<wnid>/*`` and ``val/<wnid>/*``.

``prepare_datasets`` converts the raw releases already on disk (no network,
no torchvision here): the CIFAR binary release (``cifar-10-batches-bin`` /
``cifar-100-binary``), LEAF FEMNIST JSON, the ImageNet folder layout; the
synthetic datasets need nothing.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Optional, Tuple

import numpy as np
import torch

from .fed_dataset import FedDataset


class ArrayImageFedDataset(FedDataset):
    """Base for datasets whose images live in memory as uint8 NHWC arrays."""

    mean: Tuple[float, ...] = (0.5, 0.5, 0.5)
    std: Tuple[float, ...] = (0.5, 0.5, 0.5)
    train_images: np.ndarray
    train_targets: np.ndarray
    test_images: np.ndarray
    test_targets: np.ndarray

    def arrays(self):
        """(images uint8 [N,H,W,C], targets int64 [N]) for this split."""
        if self.type == "train":
            return self.train_images, self.train_targets
        return self.test_images, self.test_targets

    def _get_train_item(self, nat_client, idx_within_client):
        start = int(np.concatenate([[0], np.cumsum(self.images_per_client)])[nat_client])
        row = start + idx_within_client
        return self.train_images[row], int(self.train_targets[row])

    def _get_val_item(self, idx):
        return self.test_images[idx], int(self.test_targets[idx])


# ----------------------------------------------------------------- CIFAR
class FedCIFAR10(ArrayImageFedDataset):
    mean = (0.4914, 0.4822, 0.4465)
    std = (0.2471, 0.2435, 0.2616)

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if self.type == "train":
            parts = [np.load(self.client_fn(i)) for i in range(len(self.images_per_client))]
            self.train_images = np.ascontiguousarray(np.concatenate(parts))
            self.train_targets = np.repeat(np.arange(len(parts)), [len(p) for p in parts])
        else:
            with np.load(self.test_fn()) as t:
                self.test_images = np.ascontiguousarray(t["test_images"])
                self.test_targets = np.asarray(t["test_targets"]).astype(np.int64)

    # the CIFAR binary release (raw bytes: no pickles), cs.toronto.edu/~kriz
    BIN_DIR, BIN_TRAIN, BIN_TEST, LABEL_BYTES, NUM_CLASSES = (
        "cifar-10-batches-bin", [f"data_batch_{i}.bin" for i in range(1, 6)], ["test_batch.bin"],
        1, 10)

    def prepare_datasets(self, download=False):
        """Reference layout (fed_cifar.py:28-75: one natural client per class)
        from the binary release unpacked under ``dataset_dir``; the reference
        downloads through torchvision, which is not available here."""
        src = os.path.join(self.dataset_dir, self.BIN_DIR)
        if not os.path.isdir(src):
            raise FileNotFoundError(
                f"{self.stats_fn()} not found and no {src}: unpack the CIFAR binary release "
                "there, provide the reference layout (client{i}.npy, test.npz, stats.json), "
                "or run with --synthetic.")
        tr_x, tr_y = read_cifar_bin([os.path.join(src, f) for f in self.BIN_TRAIN],
                                    self.LABEL_BYTES)
        te_x, te_y = read_cifar_bin([os.path.join(src, f) for f in self.BIN_TEST],
                                    self.LABEL_BYTES)
        self.write_split(self.dataset_dir, tr_x, tr_y, te_x, te_y, self.NUM_CLASSES)

    def client_fn(self, client_id):
        return os.path.join(self.dataset_dir, f"client{client_id}.npy")

    def test_fn(self):
        return os.path.join(self.dataset_dir, "test.npz")

    @staticmethod
    def write_split(dataset_dir, train_images, train_targets, test_images, test_targets,
                    num_classes):
        """Write the reference on-disk layout from arrays (fed_cifar.py:28-75)."""
        os.makedirs(dataset_dir, exist_ok=True)
        ipc = []
        for c in range(num_classes):
            sel = np.where(train_targets == c)[0]
            np.save(os.path.join(dataset_dir, f"client{c}.npy"), train_images[sel])
            ipc.append(int(len(sel)))
        np.savez(os.path.join(dataset_dir, "test.npz"), test_images=test_images,
                 test_targets=test_targets)
        with open(os.path.join(dataset_dir, "stats.json"), "w") as f:
            json.dump({"images_per_client": ipc, "num_val_images": int(len(test_targets))}, f)


def read_cifar_bin(files, label_bytes: int):
    """(images uint8 [N,32,32,3], fine labels int64 [N]) of CIFAR binary files:
    records of ``label_bytes`` label bytes (CIFAR-100: coarse, fine) and 3072
    pixel bytes (R, G, B planes of 32x32)."""
    xs, ys = [], []
    rec = label_bytes + 3072
    for fn in files:
        raw = np.fromfile(fn, dtype=np.uint8)
        if raw.size % rec:
            raise ValueError(f"{fn}: size {raw.size} is not a multiple of {rec}-byte records")
        raw = raw.reshape(-1, rec)
        ys.append(raw[:, label_bytes - 1].astype(np.int64))
        xs.append(raw[:, label_bytes:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1))
    return np.ascontiguousarray(np.concatenate(xs)), np.concatenate(ys)


class FedCIFAR100(FedCIFAR10):
    mean = (0.5071, 0.4867, 0.4408)
    std = (0.2675, 0.2565, 0.2761)
    BIN_DIR, BIN_TRAIN, BIN_TEST, LABEL_BYTES, NUM_CLASSES = (
        "cifar-100-binary", ["train.bin"], ["test.bin"], 2, 100)


# ----------------------------------------------------------------- FEMNIST
class FedEMNIST(ArrayImageFedDataset):
    mean = (0.9637,)
    std = (0.1597,)

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if self.type == "train":
            xs, ys = [], []
            for i in range(len(self.images_per_client)):
                d = torch.load(os.path.join(self.dataset_dir, "train", f"client{i}.pt"),
                               weights_only=True)
                xs.append(_to_u8(d["x"]))
                ys.append(np.asarray(d["y"]).astype(np.int64))
            self.train_images = np.ascontiguousarray(np.concatenate(xs))[..., None]
            self.train_targets = np.concatenate(ys)
        else:
            d = torch.load(os.path.join(self.dataset_dir, "test", "test.pt"), weights_only=True)
            self.test_images = np.ascontiguousarray(_to_u8(d["x"]))[..., None]
            self.test_targets = np.asarray(d["y"]).astype(np.int64)

    def prepare_datasets(self, download=False):
        """LEAF FEMNIST JSON (``train/*.json``, ``test/*.json``: {"users",
        "user_data": {user: {"x": [[784 floats]], "y": [...]}}}) -> one
        ``train/client{i}.pt`` per writer, ``test/test.pt`` and ``stats.json``
        (fed_emnist.py:82-138; torch files read ~25x faster than the JSON)."""
        if os.path.exists(self.stats_fn()):
            raise RuntimeError("won't overwrite existing stats file")
        train = read_leaf_json(os.path.join(self.dataset_dir, "train"))
        ipc = []
        for cid, cdata in enumerate(train.values()):
            x = torch.tensor(cdata["x"], dtype=torch.float32).view(-1, 28, 28)
            y = torch.tensor(cdata["y"], dtype=torch.int64)
            ipc.append(int(y.numel()))
            fn = os.path.join(self.dataset_dir, "train", f"client{cid}.pt")
            if not os.path.exists(fn):
                torch.save({"x": x, "y": y}, fn)
        test = read_leaf_json(os.path.join(self.dataset_dir, "test"))
        xs = [torch.tensor(c["x"], dtype=torch.float32).view(-1, 28, 28) for c in test.values()]
        ys = [torch.tensor(c["y"], dtype=torch.int64) for c in test.values()]
        torch.save({"x": torch.cat(xs), "y": torch.cat(ys)},
                   os.path.join(self.dataset_dir, "test", "test.pt"))
        with open(self.stats_fn(), "w") as f:
            json.dump({"images_per_client": ipc, "num_val_images": int(sum(len(y) for y in ys))},
                      f)


def read_leaf_json(data_dir):
    """{user: {"x": [...], "y": [...]}} merged over the LEAF .json files of a
    directory, in file then user order (fed_emnist.py:11-34)."""
    if not os.path.isdir(data_dir):
        raise FileNotFoundError(f"{data_dir}: LEAF FEMNIST json files expected (or use --synthetic)")
    out = {}
    for fn in sorted(f for f in os.listdir(data_dir) if f.endswith(".json")):
        with open(os.path.join(data_dir, fn)) as f:
            out.update(json.load(f)["user_data"])
    return out


def _to_u8(x):
    x = x.numpy() if torch.is_tensor(x) else np.asarray(x)
    if x.dtype != np.uint8:  # LEAF stores floats in [0, 1]
        x = np.clip(np.rint(x * 255.0), 0, 255).astype(np.uint8)
    return x


# ----------------------------------------------------------------- ImageNet
class FedImageNet(FedDataset):
    """Class-per-client ImageNet read from ``train/<wnid>/*`` image folders
    (decoded with PIL on the host; the device path is for in-memory sets)."""

    mean = (0.485, 0.456, 0.406)
    std = (0.229, 0.224, 0.225)

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        split = "train" if self.type == "train" else "val"
        wnids = sorted(os.listdir(os.path.join(self.dataset_dir, split)))
        self.files = []
        self.labels = []
        for c, w in enumerate(wnids):
            fs = sorted(glob.glob(os.path.join(self.dataset_dir, split, w, "*")))
            self.files += fs
            self.labels += [c] * len(fs)

    def prepare_datasets(self, download=False):
        root = os.path.join(self.dataset_dir, "train")
        if not os.path.isdir(root):
            raise FileNotFoundError(f"{root} not found (ImageNet folder layout) -- or use --synthetic")
        wnids = sorted(os.listdir(root))
        ipc = [len(os.listdir(os.path.join(root, w))) for w in wnids]
        vroot = os.path.join(self.dataset_dir, "val")
        nval = sum(len(os.listdir(os.path.join(vroot, w))) for w in sorted(os.listdir(vroot)))
        with open(self.stats_fn(), "w") as f:
            json.dump({"images_per_client": ipc, "num_val_images": nval}, f)

    def _load(self, i):
        from PIL import Image
        return Image.open(self.files[i]).convert("RGB"), self.labels[i]

    def _get_train_item(self, nat, idx_within):
        start = int(np.concatenate([[0], np.cumsum(self.images_per_client)])[nat])
        return self._load(start + idx_within)

    def _get_val_item(self, idx):
        return self._load(idx)


# ----------------------------------------------------------------- synthetic
class SyntheticImageFedDataset(ArrayImageFedDataset):
    """Deterministic synthetic images with a class-dependent low-frequency
    pattern plus noise (learnable, so convergence smoke tests mean something).
    Natural clients = classes, like CIFAR."""

    def __init__(self, dataset_name="CIFAR10", transform=None, do_iid=False, num_clients=None,
                 train=True, num_classes=10, hw=32, channels=3, n_train=50000, n_val=10000,
                 seed=0, mean=None, std=None, hard=False, **kw):
        self.dataset_name = dataset_name
        self._nc, self._hw, self._ch = num_classes, hw, channels
        self._n_train, self._n_val, self._seed = n_train, n_val, seed
        if mean is not None:
            self.mean, self.std = tuple(mean), tuple(std)
        super().__init__(dataset_dir="", dataset_name=dataset_name, transform=transform,
                         do_iid=do_iid, num_clients=num_clients, train=train, seed=seed)
        rng = np.random.RandomState(seed + (0 if train else 1))
        n = n_train if train else n_val
        per = np.full(num_classes, n // num_classes)
        per[: n % num_classes] += 1
        targets = np.repeat(np.arange(num_classes), per)
        base = np.random.RandomState(seed + 7).randint(40, 216, size=(num_classes, 4, 4, channels))
        base = np.kron(base, np.ones((1, hw // 4, hw // 4, 1), dtype=np.int64))[:, :hw, :hw]
        imgs = np.empty((n, hw, hw, channels), dtype=np.uint8)
        step = 8192
        for s in range(0, n, step):
            t = targets[s:s + step]
            if hard:
                # 0.25 x own class pattern + 0.2 x a random other class's + noise
                # of std 60: the classes overlap (a matched filter that knows
                # the patterns is right ~94.6 % of the time on CIFAR-10 shape)
                d = (t + 1 + rng.randint(0, num_classes - 1, size=len(t))) % num_classes
                x = (128.0 + 0.25 * (base[t] - 128.0) + 0.2 * (base[d] - 128.0)
                     + rng.normal(0.0, 60.0, size=(len(t), hw, hw, channels)))
            else:
                x = base[t] + rng.randint(-40, 41, size=(len(t), hw, hw, channels))
            imgs[s:s + step] = np.clip(x, 0, 255).astype(np.uint8)
        if train:
            self.train_images, self.train_targets = imgs, targets.astype(np.int64)
        else:
            self.test_images, self.test_targets = imgs, targets.astype(np.int64)

    def _meta_ready(self):
        return True

    def _load_meta(self, train):
        per = np.full(self._nc, self._n_train // self._nc)
        per[: self._n_train % self._nc] += 1
        self.images_per_client = per
        self.num_val_images = self._n_val


SYNTHETIC_SHAPES = {
    # name: (num_classes, hw, channels, n_train, n_val, mean, std)
    "CIFAR10": (10, 32, 3, 50000, 10000, FedCIFAR10.mean, FedCIFAR10.std),
    "CIFAR100": (100, 32, 3, 50000, 10000, FedCIFAR100.mean, FedCIFAR100.std),
    "EMNIST": (62, 28, 1, 80000, 8000, FedEMNIST.mean, FedEMNIST.std),
    "ImageNet": (1000, 224, 3, 64000, 5000, FedImageNet.mean, FedImageNet.std),
}


def make_synthetic(name, train=True, do_iid=False, num_clients=None, size=None, seed=0,
                   transform=None, hard=False):
    nc, hw, ch, ntr, nva, mean, std = SYNTHETIC_SHAPES[name]
    if size is not None:
        ntr = size
        nva = max(nc, min(nva, size // 5))
    return SyntheticImageFedDataset(name, transform=transform, do_iid=do_iid,
                                    num_clients=num_clients, train=train, num_classes=nc, hw=hw,
                                    channels=ch, n_train=ntr, n_val=nva, seed=seed, mean=mean,
                                    std=std, hard=hard)
