"""Text tokenizer / language model loading (reference
groundingdino/util/get_tokenlizer.py:4-29).

The reference calls ``AutoTokenizer.from_pretrained("bert-base-uncased")`` — a
remote fetch by model name.  There is no network on this pipeline, so:

* if ``text_encoder_type`` is a local directory (a saved bert-base-uncased),
  the real HF tokenizer / weights are loaded from it (local files only);
* otherwise ``OfflineBertTokenizer`` is used: bert-base-uncased's id layout for
  the special tokens ([PAD]=0, [UNK]=100, [CLS]=101, [SEP]=102, '.'=1012,
  '?'=1029, ...) and one deterministic id in [1999, 29611] per lower-cased word
  (a stable hash).  It keeps everything the model and the loss use from the
  tokenizer: ``__call__(..., padding="longest", return_tensors="pt")`` with
  input_ids / token_type_ids / attention_mask, ``convert_tokens_to_ids``,
  per-example ``char_to_token`` (create_positive_map), ``.to(device)``.
  Word-piece splitting of rare words is not reproduced (every word is one
  token); with real weights, point ``text_encoder_type`` at a local copy.
"""
from __future__ import annotations

import os
import zlib
from typing import Dict, List, Optional

import torch

_SPECIAL = {"[PAD]": 0, "[UNK]": 100, "[CLS]": 101, "[SEP]": 102, "[MASK]": 103}
# bert-base-uncased ids of ASCII punctuation (vocab rows 999..1036 are the
# punctuation block in that vocab)
_PUNCT = {c: 999 + i for i, c in enumerate("!\"#$%&'()*+,-./0123456789:;<=>?@[\\]^_`{|}~")}
_WORD_LO, _WORD_HI = 1999, 29612


def _is_punct(ch: str) -> bool:
    return ch in _PUNCT and not ch.isdigit()


class _ItemEncoding:
    """One example's offsets: ``char_to_token(char_pos)`` like
    tokenizers.Encoding (used per sample by create_positive_map)."""

    def __init__(self, char_map: Dict[int, int]):
        self._char_map = char_map

    def char_to_token(self, char_index: int) -> Optional[int]:
        return self._char_map.get(int(char_index))


class TokenBatch(dict):
    """BatchEncoding-like: tensors by key, examples by int index."""

    def __init__(self, data, items: List[_ItemEncoding]):
        super().__init__(data)
        self._items = items

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __getitem__(self, k):
        if isinstance(k, int):
            return self._items[k]
        return super().__getitem__(k)

    def to(self, device):
        return TokenBatch({k: v.to(device) for k, v in self.items()}, self._items)

    def pin_memory(self):
        return TokenBatch({k: v.pin_memory() for k, v in self.items()}, self._items)

    def char_to_token(self, batch_or_char_index: int, char_index: Optional[int] = None):
        if char_index is None:
            return self._items[0].char_to_token(batch_or_char_index)
        return self._items[batch_or_char_index].char_to_token(char_index)


class OfflineBertTokenizer:
    vocab_size = 30522
    model_max_length = 512

    def __init__(self):
        self.pad_token_id = _SPECIAL["[PAD]"]
        self.cls_token_id = _SPECIAL["[CLS]"]
        self.sep_token_id = _SPECIAL["[SEP]"]

    def word_id(self, word: str) -> int:
        if word in _SPECIAL:
            return _SPECIAL[word]
        if len(word) == 1 and _is_punct(word):
            return _PUNCT[word]
        return _WORD_LO + zlib.crc32(word.encode("utf-8")) % (_WORD_HI - _WORD_LO)

    def convert_tokens_to_ids(self, tokens):
        if isinstance(tokens, str):
            return self.word_id(tokens)
        return [self.word_id(t) for t in tokens]

    def _split(self, text: str):
        """-> [(token, char_start, char_end)] on the lower-cased text."""
        out, i, n = [], 0, len(text)
        low = text.lower()
        while i < n:
            ch = low[i]
            if ch.isspace():
                i += 1
            elif _is_punct(ch):
                out.append((ch, i, i + 1))
                i += 1
            else:
                j = i
                while j < n and not low[j].isspace() and not _is_punct(low[j]):
                    j += 1
                out.append((low[i:j], i, j))
                i = j
        return out

    def encode_one(self, text: str, max_length: Optional[int] = None):
        toks = self._split(text)
        if max_length is not None:
            toks = toks[: max(0, max_length - 2)]
        ids = [self.cls_token_id] + [self.word_id(t) for t, _, _ in toks] + [self.sep_token_id]
        char_map = {}
        for ti, (_, a, b) in enumerate(toks):
            for c in range(a, b):
                char_map[c] = ti + 1
        return ids, _ItemEncoding(char_map)

    def __call__(self, text, padding="longest", truncation=False, max_length=None,
                 return_tensors="pt", **_):
        texts = [text] if isinstance(text, str) else list(text)
        enc = [self.encode_one(t, max_length if truncation else None) for t in texts]
        if padding == "max_length" and max_length:
            width = max_length
        else:
            width = max(len(ids) for ids, _ in enc)
        input_ids = torch.full((len(enc), width), self.pad_token_id, dtype=torch.long)
        attn = torch.zeros((len(enc), width), dtype=torch.long)
        for i, (ids, _) in enumerate(enc):
            input_ids[i, : len(ids)] = torch.as_tensor(ids)
            attn[i, : len(ids)] = 1
        data = {"input_ids": input_ids, "token_type_ids": torch.zeros_like(input_ids),
                "attention_mask": attn}
        return TokenBatch(data, [e for _, e in enc])


def get_tokenlizer(text_encoder_type: str):
    """Reference name kept (get_tokenlizer.py:4)."""
    if os.path.isdir(str(text_encoder_type)):
        from transformers import AutoTokenizer
        return AutoTokenizer.from_pretrained(text_encoder_type, local_files_only=True)
    return OfflineBertTokenizer()


def get_pretrained_language_model(text_encoder_type: str):
    """A HF BertModel: local weights if ``text_encoder_type`` is a directory,
    else random init with the bert-base-uncased config (BASELINE: random
    weights, no network)."""
    from transformers import BertConfig, BertModel
    if os.path.isdir(str(text_encoder_type)):
        return BertModel.from_pretrained(text_encoder_type, local_files_only=True)
    return BertModel(BertConfig())
