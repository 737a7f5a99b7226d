"""Box geometry for the matcher and the losses (contract of
groundingdino/util/box_ops.py / util/box_ops.py).  Pure torch, runs on the
device the boxes live on."""
import torch


def box_cxcywh_to_xyxy(x):
    cx, cy, w, h = x.unbind(-1)
    hw, hh = 0.5 * w, 0.5 * h
    return torch.stack((cx - hw, cy - hh, cx + hw, cy + hh), dim=-1)


def box_xyxy_to_cxcywh(x):
    x0, y0, x1, y1 = x.unbind(-1)
    return torch.stack(((x0 + x1) / 2, (y0 + y1) / 2, x1 - x0, y1 - y0), dim=-1)


def _wh_area(wh):
    """w * h of [..., 2] extents, as the reference's wh[..., 0] * wh[..., 1]
    (util/box_ops.py) -- not a prod() reduction, whose backward checks the
    input for zeros on the host (a device->host sync that HIP refuses inside
    a graph capture: the whole-step graph's criterion backward)."""
    return wh[..., 0] * wh[..., 1]


def box_area(boxes):
    return (boxes[..., 2] - boxes[..., 0]) * (boxes[..., 3] - boxes[..., 1])


def box_iou(boxes1, boxes2):
    """Pairwise IoU and union, [N, M]; union gets +1e-6 as the reference."""
    a1, a2 = box_area(boxes1), box_area(boxes2)
    lt = torch.maximum(boxes1[:, None, :2], boxes2[None, :, :2])
    rb = torch.minimum(boxes1[:, None, 2:], boxes2[None, :, 2:])
    inter = _wh_area((rb - lt).clamp(min=0))
    union = a1[:, None] + a2[None, :] - inter
    return inter / (union + 1e-6), union


def generalized_box_iou(boxes1, boxes2):
    """Pairwise GIoU [N, M] of xyxy boxes (https://giou.stanford.edu/)."""
    iou, union = box_iou(boxes1, boxes2)
    lt = torch.minimum(boxes1[:, None, :2], boxes2[None, :, :2])
    rb = torch.maximum(boxes1[:, None, 2:], boxes2[None, :, 2:])
    hull = _wh_area((rb - lt).clamp(min=0))
    return iou - (hull - union) / (hull + 1e-6)


def paired_generalized_box_iou(boxes1, boxes2):
    """GIoU of row-aligned pairs [N] (= diag of generalized_box_iou without
    building the N x N matrix)."""
    a1, a2 = box_area(boxes1), box_area(boxes2)
    lt = torch.maximum(boxes1[:, :2], boxes2[:, :2])
    rb = torch.minimum(boxes1[:, 2:], boxes2[:, 2:])
    inter = _wh_area((rb - lt).clamp(min=0))
    union = a1 + a2 - inter
    iou = inter / (union + 1e-6)
    lt2 = torch.minimum(boxes1[:, :2], boxes2[:, :2])
    rb2 = torch.maximum(boxes1[:, 2:], boxes2[:, 2:])
    hull = _wh_area((rb2 - lt2).clamp(min=0))
    return iou - (hull - union) / (hull + 1e-6)


def generalized_box_iou_batched(boxes1, boxes2):
    """GIoU of xyxy boxes with leading batch dims: boxes1 [..., N, 4],
    boxes2 [..., M, 4] (broadcastable leading dims) -> [..., N, M]; same
    formula and epsilons as generalized_box_iou."""
    a1, a2 = box_area(boxes1), box_area(boxes2)
    b1, b2 = boxes1[..., :, None, :], boxes2[..., None, :, :]
    inter = _wh_area((torch.minimum(b1[..., 2:], b2[..., 2:]) - torch.maximum(b1[..., :2], b2[..., :2])).clamp(min=0))
    union = a1[..., :, None] + a2[..., None, :] - inter
    iou = inter / (union + 1e-6)
    hull = _wh_area((torch.maximum(b1[..., 2:], b2[..., 2:]) - torch.minimum(b1[..., :2], b2[..., :2])).clamp(min=0))
    return iou - (hull - union) / (hull + 1e-6)
