"""Golden vectors for the ODVG caption / label construction, produced by the
REFERENCE's own datasets/odvg.py (ODVGDataset.__getitem__, :185-272).

Run in the build container (where /root/reference exists):
    PYTHONHASHSEED=0 python tests/golden/make_odvg_golden.py

The reference module is imported by path.  torchvision is not installed and
the name ``datasets`` belongs to the HF package here, so three in-memory
stand-ins are registered first: ``torchvision.datasets.vision.VisionDataset``
(stores root / transforms, as published), ``torchvision.transforms``
(Compose / PILToTensor, only used for the fork's second image tensor) and
``datasets.transforms`` (unused with transforms=None).  Images are tiny PNGs
written to a temporary directory (the test writes the same files).

The fork's VG branch raises UnboundLocalError on ``car_bboxes`` (only the OD
branch defines it, odvg.py:206 vs :261); its caption / label / box results
are read from the raising frame's locals, which hold everything the branch
computed (:236-252).

Both branches draw from the global ``random`` module: each record is run
after ``random.seed(seed)``.  ``list(set(...))`` orders (OD positives, VG
unique phrases) depend on the string hash seed, so the generator pins
PYTHONHASHSEED=0 and the test compares those parts as sets (see
tests/test_data_odvg.py).  Output: tests/golden/odvg_ref.json (data only).
"""
from __future__ import annotations

import importlib.util
import json
import os
import random
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

LABEL_MAP = {str(i): name for i, name in enumerate(
    ["person", "bicycle", "car", "motorcycle", "dog", "cat", "umbrella", "traffic light", "bench", "bird",
     "kite", "cup"])}


def records():
    """(mode, meta) cases: OD with one / several distinct positives, repeated
    labels, max_labels below and above the label count; VG with repeated and
    unique phrases."""
    od = []
    specs = [[4], [4, 7, 4], [0, 2, 5, 11], [1], [3, 3, 3, 9, 10]]
    for i, labels in enumerate(specs):
        inst = [{"bbox": [1.0 + j, 2.0 + 2 * j, 20.0 + 3 * j, 24.0 + j], "label": lb,
                 "category": LABEL_MAP[str(lb)], "car_bbox": [0.0, 0.0, 4.0, 4.0]} for j, lb in enumerate(labels)]
        od.append({"filename": f"img{i % 3}.png", "height": 40, "width": 48, "detection": {"instances": inst}})
    vg = []
    phrase_sets = [["a man", "an umbrella", "a man"], ["red car", "tree", "sky", "road", "tree"],
                   ["one phrase"], ["a", "b", "c", "d", "e", "f", "a", "b"]]
    for i, ph in enumerate(phrase_sets):
        regions = [{"bbox": [float(j), float(2 * j), 10.0 + j, 12.0 + j], "phrase": p} for j, p in enumerate(ph)]
        vg.append({"filename": f"img{i % 3}.png", "height": 40, "width": 48,
                   "grounding": {"caption": " ".join(ph), "regions": regions}})
    return od, vg


def write_images(d):
    import numpy as np
    from PIL import Image
    rng = np.random.default_rng(0)
    for i in range(3):
        Image.fromarray(rng.integers(0, 255, (40, 48, 3), dtype=np.uint8)).save(os.path.join(d, f"img{i}.png"))


def _stubs():
    tv = types.ModuleType("torchvision")
    tv_ds = types.ModuleType("torchvision.datasets")
    tv_vis = types.ModuleType("torchvision.datasets.vision")

    class VisionDataset:
        def __init__(self, root, transforms=None, transform=None, target_transform=None):
            self.root, self.transforms = root, transforms
            self.transform, self.target_transform = transform, target_transform

    tv_vis.VisionDataset = VisionDataset
    tv_tr = types.ModuleType("torchvision.transforms")

    class Compose:
        def __init__(self, ts):
            self.ts = ts

        def __call__(self, x):
            for t in self.ts:
                x = t(x)
            return x

    class PILToTensor:
        def __call__(self, img):
            import numpy as np
            import torch
            return torch.as_tensor(np.asarray(img)).permute(2, 0, 1).contiguous()

    tv_tr.Compose, tv_tr.PILToTensor = Compose, PILToTensor
    tv.datasets, tv.transforms = tv_ds, tv_tr
    tv_ds.vision = tv_vis
    ds = types.ModuleType("datasets")
    ds.__path__ = []
    ds_tr = types.ModuleType("datasets.transforms")
    ds.transforms = ds_tr
    sys.modules.update({"torchvision": tv, "torchvision.datasets": tv_ds, "torchvision.datasets.vision": tv_vis,
                        "torchvision.transforms": tv_tr, "datasets": ds, "datasets.transforms": ds_tr})


def load_reference():
    _stubs()
    spec = importlib.util.spec_from_file_location("_ref_odvg", os.path.join(REF, "datasets", "odvg.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def run_case(mod, root, anno_path, label_map_path, meta, seed, max_labels):
    with open(anno_path, "w") as f:
        f.write(json.dumps(meta) + "\n")
    ds = mod.ODVGDataset(root, anno_path, label_map_path, max_labels=max_labels)
    random.seed(seed)
    try:
        _, _, target = ds[0]
        out = {"caption": target["caption"], "cap_list": list(target["cap_list"]),
               "boxes": target["boxes"].tolist(), "labels": target["labels"].tolist()}
    except UnboundLocalError:  # the fork's VG branch (car_bboxes), see module docstring
        tb = sys.exc_info()[2]
        while tb.tb_next is not None:
            tb = tb.tb_next
        loc = tb.tb_frame.f_locals
        out = {"caption": loc["caption"], "cap_list": list(loc["caption_list"]),
               "boxes": loc["boxes"].tolist(), "labels": loc["classes"].tolist(), "fork_vg_raises": True}
    return out


def main():
    if os.environ.get("PYTHONHASHSEED") != "0":
        raise SystemExit("run with PYTHONHASHSEED=0 (set orders in the reference depend on it)")
    mod = load_reference()
    od, vg = records()
    cases = []
    with tempfile.TemporaryDirectory() as d:
        write_images(d)
        lm = os.path.join(d, "label_map.json")
        with open(lm, "w") as f:
            json.dump(LABEL_MAP, f)
        anno = os.path.join(d, "anno.jsonl")
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):  # the reference prints per item
            for i, meta in enumerate(od):
                for max_labels in (4, 80):
                    for seed in (0, 1):
                        cases.append({"mode": "OD", "meta": meta, "seed": seed, "max_labels": max_labels,
                                      "out": run_case(mod, d, anno, lm, meta, seed, max_labels)})
            for i, meta in enumerate(vg):
                for seed in (0, 1, 2):
                    cases.append({"mode": "VG", "meta": meta, "seed": seed, "max_labels": 80,
                                  "out": run_case(mod, d, anno, None, meta, seed, 80)})
    with open(os.path.join(HERE, "odvg_ref.json"), "w") as f:
        json.dump({"label_map": LABEL_MAP, "pythonhashseed": 0, "cases": cases}, f, indent=0)
    print(f"wrote {len(cases)} cases")


if __name__ == "__main__":
    main()
