"""oracle/blocks.py — TEST INFRASTRUCTURE ONLY.

Literal CPU restatements (plain torch, materialising every intermediate the
way the reference does) of the attention-family ops that the product routes
through fused kernels.  Tests compare the product's kernels against these,
and these are pinned against reference-generated fixtures where the
reference module imports here (tests/golden/make_block_golden.py).

  bi_attention_ref     fuse_modules.py:162-246 (global max shift, +-5e4
                       clamps, column-max shift, -inf masks, two softmaxes)
  window_attention_ref swin_transformer.py:134-174
  window_attention_packed_ref  the same on the packed qkv + bias table (:113-114, :171)
  window_attention_image_ref   + SwinTransformerBlock's pad / roll / partition
                               and reverse / roll back / crop (:238-292)
  attention_ref        masked softmax(q k^T * scale) v (additive / bool mask)
  contrastive_ref      utils.py:242-273
  phrase_masks_ref     bertwarper.py:224-273 (per-special-token loop)
"""
from __future__ import annotations

import torch


def bi_attention_ref(q, k, v_v, v_l, pad_v=None, pad_l=None):
    """q [B,H,S,hd] (pre-scaled), k/v_l [B,H,T,hd], v_v [B,H,S,hd] ->
    (out_v [B,H,S,hd], out_l [B,H,T,hd]).  Statement order follows
    fuse_modules.py:174-217."""
    b, h, s, hd = q.shape
    t = k.shape[2]
    qf, kf = q.reshape(b * h, s, hd), k.reshape(b * h, t, hd)
    w = torch.bmm(qf, kf.transpose(1, 2))
    w = w - w.max()
    w = torch.clamp(w, min=-50000)
    w = torch.clamp(w, max=50000)
    wt = w.transpose(1, 2)
    wl = wt - torch.max(wt, dim=-1, keepdim=True)[0]
    wl = torch.clamp(wl, min=-50000)
    wl = torch.clamp(wl, max=50000)
    if pad_v is not None:
        m = pad_v[:, None, None, :].repeat(1, h, 1, 1).flatten(0, 1)
        wl = wl.masked_fill(m, float("-inf"))
    wl = wl.softmax(dim=-1)
    if pad_l is not None:
        m = pad_l[:, None, None, :].repeat(1, h, 1, 1).flatten(0, 1)
        w = w.masked_fill(m, float("-inf"))
    wv = w.softmax(dim=-1)
    out_v = torch.bmm(wv, v_l.reshape(b * h, t, hd)).view(b, h, s, hd)
    out_l = torch.bmm(wl, v_v.reshape(b * h, s, hd)).view(b, h, t, hd)
    return out_v, out_l


def window_attention_ref(q, k, v, bias, mask, scale):
    """q/k/v [B_, nH, N, hd]; bias [nH, N, N]; mask [nW, N, N] or None."""
    attn = (q * scale) @ k.transpose(-2, -1)
    attn = attn + bias.unsqueeze(0)
    if mask is not None:
        nw = mask.shape[0]
        b_, nh, n, _ = attn.shape
        attn = attn.view(b_ // nw, nw, nh, n, n) + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, nh, n, n)
    return torch.softmax(attn, dim=-1) @ v


def window_attention_packed_ref(qkv, table, rel_index, mask, scale):
    """WindowAttention.forward core (swin_transformer.py:134-174) on the packed
    qkv [B_, N, 3, nH, hd] with the bias table [(2Wh-1)(2Ww-1), nH] and
    rel_index [N*N] (:113-114) -> [B_, N, nH*hd] (:171)."""
    b_, n, _, nh, hd = qkv.shape
    q, k, v = qkv.permute(2, 0, 3, 1, 4)
    bias = table[rel_index.view(-1)].view(n, n, -1).permute(2, 0, 1).contiguous()
    out = window_attention_ref(q, k, v, bias, mask, scale)
    return out.transpose(1, 2).reshape(b_, n, nh * hd)


def window_attention_image_ref(qkv, qkv_bias, table, rel_index, mask, hw, ws, shift, scale):
    """SwinTransformerBlock.forward between its qkv and proj Linears
    (swin_transformer.py:250-290 around :134-174), restated on the qkv Linear
    output of the unpartitioned image qkv [B, H*W, 3C] -> [B, H*W, C]: the
    normed tokens are zero-padded to multiples of ws (:255-257; a pad row's
    qkv is the Linear bias), rolled by -shift (:262), partitioned (:269),
    attended, reversed (:281), rolled back (:285) and cropped (:290)."""
    b, _, c3 = qkv.shape
    h, w = hw
    nh = table.shape[1]
    hp, wp = -(-h // ws) * ws, -(-w // ws) * ws
    x = qkv.new_zeros(b, hp, wp, c3)
    if qkv_bias is not None:
        x = x + qkv_bias.to(qkv.dtype)
    x = torch.cat([torch.cat([qkv.view(b, h, w, c3), x[:, :h, w:]], 2), x[:, h:]], 1)
    if shift > 0:
        x = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2))
    win = x.view(b, hp // ws, ws, wp // ws, ws, c3).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws, 3, nh,
                                                                                     c3 // (3 * nh))
    out = window_attention_packed_ref(win, table, rel_index, mask if shift > 0 else None, scale)
    x = out.view(b, hp // ws, wp // ws, ws, ws, -1).permute(0, 1, 3, 2, 4, 5).reshape(b, hp, wp, -1)
    if shift > 0:
        x = torch.roll(x, shifts=(shift, shift), dims=(1, 2))
    return x[:, :h, :w].reshape(b, h * w, -1)


def attention_ref(q, k, v, mask=None, scale=None):
    """q [B,H,Lq,hd], k/v [B,H,Lk,hd]; mask bool (True = attend) or additive."""
    scale = q.shape[-1] ** -0.5 if scale is None else scale
    s = (q @ k.transpose(-2, -1)) * scale
    if mask is not None:
        if mask.dtype == torch.bool:
            s = s.masked_fill(~mask, float("-inf"))
        else:
            s = s + mask
    return torch.softmax(s, dim=-1) @ v


def contrastive_ref(x, text, text_token_mask, max_text_len=256):
    res = x @ text.transpose(-1, -2)
    res.masked_fill_(~text_token_mask[:, None, :], float("-inf"))
    new = torch.full((*res.shape[:-1], max_text_len), float("-inf"), device=res.device)
    new[..., : res.shape[-1]] = res
    return new


def phrase_masks_ref(input_ids, special_tokens):
    """Loop over every special token in row-major order, previous column
    carried across rows (bertwarper.py:240-262)."""
    bs, n = input_ids.shape
    special = torch.zeros((bs, n), dtype=torch.bool)
    for tok in special_tokens:
        special |= input_ids == tok
    idxs = torch.nonzero(special)
    mask = torch.eye(n, dtype=torch.bool).unsqueeze(0).repeat(bs, 1, 1)
    pos = torch.zeros((bs, n), dtype=torch.long)
    prev = 0
    for i in range(idxs.shape[0]):
        r, c = int(idxs[i, 0]), int(idxs[i, 1])
        if c == 0 or c == n - 1:
            mask[r, c, c] = True
            pos[r, c] = 0
        else:
            mask[r, prev + 1:c + 1, prev + 1:c + 1] = True
            pos[r, prev + 1:c + 1] = torch.arange(0, c - prev)
        prev = c
    return mask, pos
