"""ODVG datasets, collate and worker-side text preprocessing.

``ODVGDataset`` reads the ODVG jsonl format (one record per image). Its
behaviour follows the reference's datasets/odvg.py:135-272.

**OD mode** (a label map is given): ``record["detection"]["instances"]``,
each with bbox (xyxy, pixels), label (int) and category.
  * The caption is the image's positive labels plus negatives sampled up to
    ``max_labels``: ``random.sample(sorted(negatives))``, then a
    Fisher–Yates shuffle. Names are joined with " . " and the caption ends
    with " .".
  * A box's label is the index of its category in that list.

**VG mode**: ``record["grounding"]["regions"]``, each with bbox and phrase.
  * Regions are shuffled.
  * The caption joins the unique phrases.
  * A box's label is the index of its phrase.

The target holds size, cap_list, caption, boxes and labels. After the
transforms, boxes are normalised cxcywh. The fork's extras are not carried:
a second untransformed image tensor, a car-box field and a dataset length
capped at 10 000 (odvg.py:185-274).

``collate_fn`` matches util/misc.py's collate (images -> NestedTensor).
``ODVGCollator(text=TextPreprocessor(...))`` additionally tokenizes the
batch's captions and builds the phrase masks inside the DataLoader workers
(SURVEY 8f rank 2). The model then takes them as
``model(samples, captions=..., prepared_text=batch_text)``, taking that host
work off the training thread.
"""
from __future__ import annotations

import json
import os
import random
from typing import Callable, List, Optional

import torch
from PIL import Image

from ..misc import nested_tensor_from_tensor_list


class ODVGDataset(torch.utils.data.Dataset):
    def __init__(self, root: str, anno: str, label_map_anno: Optional[str] = None, max_labels: int = 80,
                 transforms: Optional[Callable] = None, seed: Optional[int] = None):
        self.root = root
        self.mode = "OD" if label_map_anno else "VG"
        self.max_labels = max_labels
        self.transforms = transforms
        # a per-dataset RNG when seeded (reproducible captions); otherwise the
        # global `random` module, like the reference
        self.rng = random.Random(seed) if seed is not None else random
        self.label_map = {}
        if self.mode == "OD":
            with open(label_map_anno) as f:
                self.label_map = {str(k): v for k, v in json.load(f).items()}
        with open(anno) as f:
            self.metas = [json.loads(line) for line in f if line.strip()]

    def __len__(self) -> int:
        return len(self.metas)

    def _od(self, meta):
        inst = meta["detection"]["instances"]
        boxes = [o["bbox"] for o in inst]
        pos = sorted(set(str(o["label"]) for o in inst))
        neg = sorted(set(self.label_map) - set(pos))
        labels = list(pos)
        k = min(len(neg), self.max_labels - len(pos))
        if k > 0:
            labels.extend(self.rng.sample(neg, k))
        for i in range(len(labels) - 1, 0, -1):  # Fisher-Yates, as the reference
            j = self.rng.randint(0, i)
            labels[i], labels[j] = labels[j], labels[i]
        cap_list = [self.label_map[lb] for lb in labels]
        index = {name: i for i, name in enumerate(cap_list)}
        classes = [index[self.label_map[str(o["label"])]] for o in inst]
        return boxes, classes, cap_list

    def _vg(self, meta):
        regions = list(meta["grounding"]["regions"])
        self.rng.shuffle(regions)
        boxes = [r["bbox"] for r in regions]
        phrases = [r["phrase"] for r in regions]
        cap_list = list(dict.fromkeys(phrases))  # unique, first-occurrence order
        index = {p: i for i, p in enumerate(cap_list)}
        return boxes, [index[p] for p in phrases], cap_list

    def __getitem__(self, index: int):
        meta = self.metas[index]
        path = os.path.join(self.root, meta["filename"])
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} not found.")
        image = Image.open(path).convert("RGB")
        w, h = image.size
        boxes, classes, cap_list = self._od(meta) if self.mode == "OD" else self._vg(meta)
        target = {"size": torch.as_tensor([int(h), int(w)]), "cap_list": cap_list,
                  "caption": " . ".join(cap_list) + " .",
                  "boxes": torch.as_tensor(boxes, dtype=torch.float32).reshape(-1, 4),
                  "labels": torch.as_tensor(classes, dtype=torch.int64)}
        if self.transforms is not None:
            image, target = self.transforms(image, target)
        return image, target


def build_odvg(image_set: str, args, datasetinfo: dict, seed: Optional[int] = None, reference_fork=False):
    """datasets/odvg.py build_odvg: datasetinfo = {"root", "anno"[, "label_map"]}."""
    from .transforms import make_transforms
    return ODVGDataset(datasetinfo["root"], datasetinfo["anno"], datasetinfo.get("label_map"),
                       max_labels=getattr(args, "max_labels", 80),
                       transforms=make_transforms(image_set, args, reference_fork=reference_fork), seed=seed)


def collate_fn(batch):
    """(images, targets) -> (NestedTensor, targets), util/misc.py collate_fn."""
    images, targets = zip(*batch)
    return nested_tensor_from_tensor_list(list(images)), list(targets)


class TextPreprocessor:
    """Picklable text preparation for DataLoader workers: the model's
    prepare_text_host with the same tokenizer, special tokens and
    max_text_len (the tokenizer is created lazily in each worker)."""

    def __init__(self, text_encoder_type: str = "bert-base-uncased", max_text_len: int = 256):
        self.text_encoder_type = text_encoder_type
        self.max_text_len = max_text_len
        self._tok = None

    def __call__(self, captions: List[str]):
        from models.GroundingDINO.groundingdino import prepare_text_host
        from ..tokenizer import get_tokenlizer
        if self._tok is None:
            self._tok = get_tokenlizer(self.text_encoder_type)
            self._special = self._tok.convert_tokens_to_ids(["[CLS]", "[SEP]", ".", "?"])
        return prepare_text_host(self._tok, self._special, self.max_text_len, captions)

    def __getstate__(self):
        return {"text_encoder_type": self.text_encoder_type, "max_text_len": self.max_text_len, "_tok": None}


class ODVGCollator:
    """collate_fn + (optionally) worker-side text preparation:
    -> (NestedTensor, targets[, prepared_text])."""

    def __init__(self, text: Optional[TextPreprocessor] = None):
        self.text = text

    def __call__(self, batch):
        samples, targets = collate_fn(batch)
        if self.text is None:
            return samples, targets
        return samples, targets, self.text([t["caption"] for t in targets])
