"""Image + box transforms of the ODVG training pipeline (PIL images, torch
targets; no torchvision in this image).

Semantics follow the reference's datasets/transforms.py (DETR-style):
  hflip      :60-75    boxes (x0,y0,x1,y1) -> (w-x1, y0, w-x0, y1)
  resize     :77-134   shorter side -> size, longer side capped at max_size
                       (sizes truncated like the reference's int()), boxes and
                       target["size"] rescaled; bilinear (PIL), the
                       interpolation torchvision's PIL path uses
  crop       :16-57    boxes shifted, clipped to the crop, degenerate boxes
                       and their labels dropped
  ToTensor / Normalize :237-268  [0,1] CHW float, ImageNet mean/std, boxes
                       xyxy absolute -> cxcywh normalised by the image size
  make_transforms      :make_coco_transforms in datasets/odvg.py:275-371 with
                       the standard multi-scale augmentation
"""
from __future__ import annotations

import random
from typing import Optional, Sequence

import numpy as np
import torch
from PIL import Image

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _xyxy_to_cxcywh(b: torch.Tensor) -> torch.Tensor:
    x0, y0, x1, y1 = b.unbind(-1)
    return torch.stack(((x0 + x1) / 2, (y0 + y1) / 2, x1 - x0, y1 - y0), dim=-1)


def crop(image: Image.Image, target: dict, region):
    """region = (top, left, height, width)."""
    i, j, h, w = region
    out = image.crop((j, i, j + w, i + h))
    target = dict(target)
    target["size"] = torch.tensor([h, w])
    if "boxes" in target:
        b = target["boxes"] - torch.as_tensor([j, i, j, i], dtype=torch.float32)
        b = torch.minimum(b.reshape(-1, 2, 2), torch.as_tensor([w, h], dtype=torch.float32)).clamp(min=0)
        keep = (b[:, 1, :] > b[:, 0, :]).all(dim=1)
        target["area"] = (b[:, 1, :] - b[:, 0, :]).prod(dim=1)[keep]
        target["boxes"] = b.reshape(-1, 4)[keep]
        if "labels" in target:
            target["labels"] = target["labels"][keep]
    return out, target


def hflip(image: Image.Image, target: dict):
    w, _ = image.size
    out = image.transpose(Image.FLIP_LEFT_RIGHT)
    target = dict(target)
    if "boxes" in target:
        b = target["boxes"]
        target["boxes"] = torch.stack((w - b[:, 2], b[:, 1], w - b[:, 0], b[:, 3]), dim=-1)
    return out, target


def resize_size(image_size, size, max_size=None):
    """(w, h), shorter-side size, cap -> (oh, ow); the reference's rule."""
    if isinstance(size, (list, tuple)):
        return tuple(size[::-1])
    w, h = image_size
    if max_size is not None:
        lo, hi = float(min(w, h)), float(max(w, h))
        if hi / lo * size > max_size:
            size = int(round(max_size * lo / hi))
    if (w <= h and w == size) or (h <= w and h == size):
        return h, w
    if w < h:
        return int(size * h / w), size
    return size, int(size * w / h)


def resize(image: Image.Image, target: Optional[dict], size, max_size=None):
    oh, ow = resize_size(image.size, size, max_size)
    out = image.resize((ow, oh), Image.BILINEAR)
    if target is None:
        return out, None
    rw, rh = ow / image.size[0], oh / image.size[1]
    target = dict(target)
    if "boxes" in target:
        target["boxes"] = target["boxes"] * torch.as_tensor([rw, rh, rw, rh], dtype=torch.float32)
    if "area" in target:
        target["area"] = target["area"] * (rw * rh)
    target["size"] = torch.tensor([oh, ow])
    return out, target


class Compose:
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, image, target):
        for t in self.transforms:
            image, target = t(image, target)
        return image, target


class RandomHorizontalFlip:
    def __init__(self, p=0.5, rng: Optional[random.Random] = None):
        self.p, self.rng = p, rng or random

    def __call__(self, image, target):
        return hflip(image, target) if self.rng.random() < self.p else (image, target)


class RandomResize:
    def __init__(self, sizes: Sequence, max_size=None, rng: Optional[random.Random] = None):
        self.sizes, self.max_size, self.rng = list(sizes), max_size, rng or random

    def __call__(self, image, target=None):
        return resize(image, target, self.rng.choice(self.sizes), self.max_size)


class RandomSizeCrop:
    def __init__(self, min_size: int, max_size: int, rng: Optional[random.Random] = None):
        self.min_size, self.max_size, self.rng = min_size, max_size, rng or random

    def __call__(self, image, target):
        w = self.rng.randint(self.min_size, min(image.width, self.max_size))
        h = self.rng.randint(self.min_size, min(image.height, self.max_size))
        i = self.rng.randint(0, image.height - h)
        j = self.rng.randint(0, image.width - w)
        return crop(image, target, (i, j, h, w))


class RandomSelect:
    def __init__(self, t1, t2, p=0.5, rng: Optional[random.Random] = None):
        self.t1, self.t2, self.p, self.rng = t1, t2, p, rng or random

    def __call__(self, image, target):
        return self.t1(image, target) if self.rng.random() < self.p else self.t2(image, target)


class ToTensor:
    def __call__(self, image, target):
        arr = np.asarray(image.convert("RGB"), dtype=np.float32) / 255.0
        return torch.from_numpy(arr).permute(2, 0, 1).contiguous(), target


class Normalize:
    def __init__(self, mean=IMAGENET_MEAN, std=IMAGENET_STD):
        self.mean = torch.tensor(mean).view(-1, 1, 1)
        self.std = torch.tensor(std).view(-1, 1, 1)

    def __call__(self, image, target=None):
        image = (image - self.mean) / self.std
        if target is None:
            return image, None
        target = dict(target)
        h, w = image.shape[-2:]
        if "boxes" in target:
            target["boxes"] = _xyxy_to_cxcywh(target["boxes"]) / torch.tensor([w, h, w, h], dtype=torch.float32)
        return image, target


SCALES = [480, 512, 544, 576, 608, 640, 672, 704, 736, 768, 800]
MAX_SIZE = 1333


def make_transforms(image_set: str, args=None, rng: Optional[random.Random] = None, reference_fork=False):
    """The GroundingDINO training / evaluation pipelines.

    train: flip + (multi-scale resize | resize, random crop, resize) +
    normalize; val: resize to 800 (max 1333) + normalize.  data_aug_*
    fields of ``args`` override the scales as in the reference.
    ``reference_fork=True`` reproduces this fork's pipeline, whose
    augmentations are commented out (odvg.py:344-354, 367-369): normalize only.
    """
    normalize = Compose([ToTensor(), Normalize()])
    if reference_fork:
        return normalize
    scales = list(getattr(args, "data_aug_scales", SCALES))
    max_size = getattr(args, "data_aug_max_size", MAX_SIZE)
    scales2_resize = list(getattr(args, "data_aug_scales2_resize", [400, 500, 600]))
    scales2_crop = list(getattr(args, "data_aug_scales2_crop", [384, 600]))
    overlap = getattr(args, "data_aug_scale_overlap", None)
    if overlap:
        scales = [int(s * overlap) for s in scales]
        max_size = int(max_size * overlap)
        scales2_resize = [int(s * overlap) for s in scales2_resize]
        scales2_crop = [int(s * overlap) for s in scales2_crop]
    if image_set == "train":
        if getattr(args, "fix_size", False):
            return Compose([RandomHorizontalFlip(rng=rng), RandomResize([(max_size, max(scales))], rng=rng),
                            normalize])
        return Compose([
            RandomHorizontalFlip(rng=rng),
            RandomSelect(RandomResize(scales, max_size=max_size, rng=rng),
                         Compose([RandomResize(scales2_resize, rng=rng), RandomSizeCrop(*scales2_crop, rng=rng),
                                  RandomResize(scales, max_size=max_size, rng=rng)]), rng=rng),
            normalize,
        ])
    if image_set in ("val", "test", "eval_debug", "train_reg"):
        return Compose([RandomResize([max(scales)], max_size=max_size, rng=rng), normalize])
    raise ValueError(f"unknown image_set {image_set}")
