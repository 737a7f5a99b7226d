"""Hungarian matching (reference models/GroundingDINO/matcher.py:25-217).

Cost = set_cost_bbox * L1(cxcywh) + set_cost_class * token-focal cost
against each target's normalised positive token map + set_cost_giou * -GIoU,
NaN/Inf entries zeroed, then scipy's linear_sum_assignment on the host.

``HungarianMatcher.forward`` keeps the reference's per-call contract
(outputs of one image, [targets], label_map).  ``match_many`` runs a whole
list of such problems (all decoder layers x images of a step) with the cost
matrices built on the device and ONE device->host copy, instead of one copy
per (layer, image) as the reference's SetCriterion loop does.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch
from scipy.optimize import linear_sum_assignment
from torch import nn

from gdino_amd import box_ops
from gdino_amd.box_ops import box_cxcywh_to_xyxy, generalized_box_iou


def _focal_token_cost(logits, label_map, alpha, gamma):
    """[Q, 256] logits x [n_tgt, 256] token maps -> [Q, n_tgt]."""
    p = logits.float().sigmoid()
    neg = (1 - alpha) * (p ** gamma) * (-(1 - p + 1e-8).log())
    pos = alpha * ((1 - p) ** gamma) * (-(p + 1e-8).log())
    m = label_map.float()
    m = m / m.sum(-1, keepdim=True)  # an empty map gives NaN -> zeroed below, as the reference
    return (pos - neg) @ m.t()


class HungarianMatcher(nn.Module):
    # SetCriterion may batch all heads' problems (match_batched) and match on
    # the device (gdino_amd.lsap: scipy's algorithm)
    batched = True
    device_matching = True

    def __init__(self, cost_class: float = 1, cost_bbox: float = 1, cost_giou: float = 1, focal_alpha=0.25):
        super().__init__()
        self.cost_class = cost_class
        self.cost_bbox = cost_bbox
        self.cost_giou = cost_giou
        assert cost_class != 0 or cost_bbox != 0 or cost_giou != 0, "all costs cant be 0"
        self.focal_alpha = focal_alpha

    @torch.no_grad()
    def cost_matrix(self, pred_logits, pred_boxes, tgt_labels, tgt_boxes, label_map):
        """pred [Q, 256] / [Q, 4] of one image -> C [Q, n_tgt] on the device."""
        q = pred_logits.shape[0]
        n = tgt_boxes.shape[0]
        if n == 0:
            return pred_boxes.new_zeros((q, 0), dtype=torch.float32)
        maps = label_map.to(pred_logits.device)[tgt_labels.to(pred_logits.device)]
        c_cls = _focal_token_cost(pred_logits, maps, self.focal_alpha, 2.0)
        ob, tb = pred_boxes.float(), tgt_boxes.float()
        c_box = torch.cdist(ob, tb, p=1)
        c_giou = -generalized_box_iou(box_cxcywh_to_xyxy(ob), box_cxcywh_to_xyxy(tb))
        c = self.cost_bbox * c_box + self.cost_class * c_cls + self.cost_giou * c_giou
        return torch.nan_to_num(c, nan=0.0, posinf=0.0, neginf=0.0)

    @torch.no_grad()
    def match_many(self, problems: Sequence[Tuple]) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        """problems: [(pred_logits [Q,256], pred_boxes [Q,4], tgt_labels, tgt_boxes, label_map)]."""
        costs = [self.cost_matrix(*p) for p in problems]
        sizes = [c.shape[1] for c in costs]
        flat = torch.cat([c.reshape(-1) for c in costs]) if costs else torch.zeros(0)
        host = flat.cpu().numpy()  # one device->host copy for all problems
        out, off = [], 0
        for c, n in zip(costs, sizes):
            qn = c.shape[0] * n
            mat = host[off:off + qn].reshape(c.shape[0], n)
            off += qn
            try:
                i, j = linear_sum_assignment(mat)
            except ValueError:  # reference falls back to min-sum (matcher.py:109-119)
                i, j = mat.argmin(0), np.arange(n)
            out.append((torch.as_tensor(i, dtype=torch.int64), torch.as_tensor(j, dtype=torch.int64)))
        return out

    @torch.no_grad()
    def cost_batched(self, logits, boxes, tgt_boxes, maps, valid):
        """All heads and images at once.

        logits [H, B, Q, 256], boxes [H, B, Q, 4]; per image b the targets are
        padded to K: tgt_boxes [B, K, 4], maps [B, K, 256] (raw positive-token
        maps of each target's label), valid [B, K].  Returns C [H, B, Q, K];
        entries of padded targets are garbage and must be ignored.  Same cost
        as cost_matrix per (head, image)."""
        p = logits.float().sigmoid()
        a = self.focal_alpha
        cls = a * ((1 - p) ** 2.0) * (-(p + 1e-8).log()) - (1 - a) * (p ** 2.0) * (-(1 - p + 1e-8).log())
        m = maps.float()
        m = m / m.sum(-1, keepdim=True)  # empty map -> NaN -> zeroed below, as the reference
        m = torch.where(valid[..., None], m, torch.zeros((), device=m.device))
        c_cls = torch.einsum("hbqt,bkt->hbqk", cls, m)
        ob, tb = boxes.float(), tgt_boxes.float()
        c_box = (ob[:, :, :, None, :] - tb[None, :, None, :, :]).abs().sum(-1)
        c_giou = -box_ops.generalized_box_iou_batched(box_cxcywh_to_xyxy(ob), box_cxcywh_to_xyxy(tb)[None])
        c = self.cost_bbox * c_box + self.cost_class * c_cls + self.cost_giou * c_giou
        return torch.nan_to_num(c, nan=0.0, posinf=0.0, neginf=0.0)

    @torch.no_grad()
    def match_batched(self, logits, boxes, tgt_boxes, maps, valid, sizes):
        """-> [[(src, tgt)] * B] * H, int64 CPU index tensors; one D2H copy."""
        host = self.cost_batched(logits, boxes, tgt_boxes, maps, valid).cpu().numpy()
        out = []
        for h in range(host.shape[0]):
            per = []
            for b, n in enumerate(sizes):
                mat = host[h, b, :, :n]
                try:
                    i, j = linear_sum_assignment(mat)
                except ValueError:  # reference falls back to min-sum (matcher.py:109-119)
                    i, j = mat.argmin(0), np.arange(n)
                per.append((torch.as_tensor(i, dtype=torch.int64), torch.as_tensor(j, dtype=torch.int64)))
            out.append(per)
        return out

    @torch.no_grad()
    def forward(self, outputs, targets, label_map):
        bs = outputs["pred_logits"].shape[0]
        logits = outputs["pred_logits"]
        boxes = outputs["pred_boxes"]
        tgt_ids = torch.cat([v["labels"] for v in targets])
        tgt_bbox = torch.cat([v["boxes"] for v in targets])
        sizes = [len(v["boxes"]) for v in targets]
        # one cost block per image against the concatenated targets, split
        # per image like the reference (:98-110)
        problems, offs = [], np.cumsum([0] + sizes)
        for i in range(bs):
            problems.append((logits[i], boxes[i], tgt_ids[offs[i]:offs[i + 1]], tgt_bbox[offs[i]:offs[i + 1]],
                             label_map))
        return self.match_many(problems)


class SimpleMinsumMatcher(HungarianMatcher):
    """Per-target argmin over queries (reference matcher.py:123-201)."""
    batched = False  # match_batched / the device solver are Hungarian
    device_matching = False

    @torch.no_grad()
    def forward(self, outputs, targets, label_map=None):
        bs, q = outputs["pred_logits"].shape[:2]
        p = outputs["pred_logits"].flatten(0, 1).float().sigmoid()
        ob = outputs["pred_boxes"].flatten(0, 1).float()
        tgt_ids = torch.cat([v["labels"] for v in targets])
        tb = torch.cat([v["boxes"] for v in targets]).float()
        a, g = self.focal_alpha, 2.0
        neg = (1 - a) * (p ** g) * (-(1 - p + 1e-8).log())
        pos = a * ((1 - p) ** g) * (-(p + 1e-8).log())
        c = (self.cost_bbox * torch.cdist(ob, tb, p=1) + self.cost_class * (pos[:, tgt_ids] - neg[:, tgt_ids])
             + self.cost_giou * -generalized_box_iou(box_cxcywh_to_xyxy(ob), box_cxcywh_to_xyxy(tb)))
        c = c.view(bs, q, -1)
        sizes = [len(v["boxes"]) for v in targets]
        out = []
        for i, blk in enumerate(c.split(sizes, -1)):
            out.append((blk[i].min(0)[1].cpu(), torch.arange(sizes[i])))
        return out


def build_matcher(args):
    assert args.matcher_type in ["HungarianMatcher", "SimpleMinsumMatcher"], \
        f"Unknown args.matcher_type: {args.matcher_type}"
    cls = HungarianMatcher if args.matcher_type == "HungarianMatcher" else SimpleMinsumMatcher
    return cls(cost_class=args.set_cost_class, cost_bbox=args.set_cost_bbox, cost_giou=args.set_cost_giou,
               focal_alpha=args.focal_alpha)
