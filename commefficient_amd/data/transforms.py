"""Host-side image transforms (torchvision is not available in this image).

Same pipelines as /root/reference/CommEfficient/data_utils/transforms.py:1-75:
CIFAR RandomCrop(32, pad 4, reflect) + hflip + normalise; FEMNIST crop /
RandomResizedCrop(28, scale .8-1.2, ratio 4/5-5/4) / RandomRotation(5);
ImageNet RandomResizedCrop(224) + hflip for train, Resize(255) +
CenterCrop(224) for val.  Inputs are PIL images or uint8 HWC arrays; outputs
float32 CHW tensors.  The GPU path does the CIFAR pipeline in a HIP kernel
(ops.augment_u8_nhwc); these are for host-decoded datasets.
"""
from __future__ import annotations

import math
import random

import numpy as np
import torch
from PIL import Image


def _to_pil(x):
    if isinstance(x, Image.Image):
        return x
    x = np.asarray(x)
    if x.ndim == 3 and x.shape[2] == 1:
        x = x[..., 0]
    return Image.fromarray(x)


def to_tensor(img) -> torch.Tensor:
    a = np.asarray(img, dtype=np.float32) / 255.0
    if a.ndim == 2:
        a = a[..., None]
    return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))


class Compose:
    def __init__(self, ts):
        self.ts = ts

    def __call__(self, x):
        for t in self.ts:
            x = t(x)
        return x


class Normalize:
    def __init__(self, mean, std):
        self.mean = torch.tensor(mean).view(-1, 1, 1)
        self.std = torch.tensor(std).view(-1, 1, 1)

    def __call__(self, t):
        return (t - self.mean) / self.std


class ToTensor:
    def __call__(self, img):
        return to_tensor(_to_pil(img))


class RandomCrop:
    def __init__(self, size, padding=0, padding_mode="constant", fill=0):
        self.size, self.padding, self.mode, self.fill = size, padding, padding_mode, fill

    def __call__(self, img):
        a = np.asarray(_to_pil(img))
        p = self.padding
        if p:
            pad = ((p, p), (p, p)) + (((0, 0),) if a.ndim == 3 else ())
            if self.mode == "reflect":
                a = np.pad(a, pad, mode="reflect")
            else:
                fill = int(self.fill * 255) if isinstance(self.fill, float) else self.fill
                a = np.pad(a, pad, mode="constant", constant_values=fill)
        h, w = a.shape[:2]
        y = random.randint(0, h - self.size)
        x = random.randint(0, w - self.size)
        return Image.fromarray(a[y:y + self.size, x:x + self.size])


class RandomHorizontalFlip:
    def __call__(self, img):
        img = _to_pil(img)
        return img.transpose(Image.FLIP_LEFT_RIGHT) if random.random() < 0.5 else img


class RandomResizedCrop:
    def __init__(self, size, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3)):
        self.size, self.scale, self.ratio = size, scale, ratio

    def __call__(self, img):
        img = _to_pil(img)
        W, H = img.size
        area = W * H
        for _ in range(10):
            ta = area * random.uniform(*self.scale)
            ar = math.exp(random.uniform(math.log(self.ratio[0]), math.log(self.ratio[1])))
            w = int(round(math.sqrt(ta * ar)))
            h = int(round(math.sqrt(ta / ar)))
            if 0 < w <= W and 0 < h <= H:
                x = random.randint(0, W - w)
                y = random.randint(0, H - h)
                return img.resize((self.size, self.size), Image.BILINEAR, box=(x, y, x + w, y + h))
        s = min(W, H)
        x, y = (W - s) // 2, (H - s) // 2
        return img.resize((self.size, self.size), Image.BILINEAR, box=(x, y, x + s, y + s))


class RandomRotation:
    def __init__(self, degrees, fill=0):
        self.degrees, self.fill = degrees, fill

    def __call__(self, img):
        img = _to_pil(img)
        fill = int(self.fill * 255) if isinstance(self.fill, float) else self.fill
        return img.rotate(random.uniform(-self.degrees, self.degrees), fillcolor=fill)


class Resize:
    def __init__(self, size):
        self.size = size

    def __call__(self, img):
        img = _to_pil(img)
        W, H = img.size
        s = self.size / min(W, H)
        return img.resize((max(1, round(W * s)), max(1, round(H * s))), Image.BILINEAR)


class CenterCrop:
    def __init__(self, size):
        self.size = size

    def __call__(self, img):
        img = _to_pil(img)
        W, H = img.size
        x, y = (W - self.size) // 2, (H - self.size) // 2
        return img.crop((x, y, x + self.size, y + self.size))


cifar10_mean, cifar10_std = (0.4914, 0.4822, 0.4465), (0.2471, 0.2435, 0.2616)
cifar100_mean, cifar100_std = (0.5071, 0.4867, 0.4408), (0.2675, 0.2565, 0.2761)
femnist_mean, femnist_std = (0.9637,), (0.1597,)
imagenet_mean, imagenet_std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)

cifar10_train_transforms = Compose([RandomCrop(32, 4, "reflect"), RandomHorizontalFlip(),
                                    ToTensor(), Normalize(cifar10_mean, cifar10_std)])
cifar10_test_transforms = Compose([ToTensor(), Normalize(cifar10_mean, cifar10_std)])
cifar100_train_transforms = Compose([RandomCrop(32, 4, "reflect"), RandomHorizontalFlip(),
                                     ToTensor(), Normalize(cifar100_mean, cifar100_std)])
cifar100_test_transforms = Compose([ToTensor(), Normalize(cifar100_mean, cifar100_std)])
femnist_train_transforms = Compose([RandomCrop(28, 2, "constant", 1.0),
                                    RandomResizedCrop(28, (0.8, 1.2), (4 / 5, 5 / 4)),
                                    RandomRotation(5, 1.0), ToTensor(),
                                    Normalize(femnist_mean, femnist_std)])
femnist_test_transforms = Compose([ToTensor(), Normalize(femnist_mean, femnist_std)])
imagenet_train_transforms = Compose([RandomResizedCrop(224), RandomHorizontalFlip(), ToTensor(),
                                     Normalize(imagenet_mean, imagenet_std)])
imagenet_val_transforms = Compose([Resize(int(224 * 1.14)), CenterCrop(224), ToTensor(),
                                   Normalize(imagenet_mean, imagenet_std)])


def host_transforms(name):
    return {"CIFAR10": (cifar10_train_transforms, cifar10_test_transforms),
            "CIFAR100": (cifar100_train_transforms, cifar100_test_transforms),
            "EMNIST": (femnist_train_transforms, femnist_test_transforms),
            "ImageNet": (imagenet_train_transforms, imagenet_val_transforms)}[name]
