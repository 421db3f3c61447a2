"""Synthetic LAION-shaped image-text pairs.

The reference streams ``laion/laion_100m_vqgan_f8`` (T5 caption ids truncated to 256, 1024 int16
VQGAN-f8 codes per image, ``data.py:11-47``). There is no network here, so training and benchmarks
use pairs of the same shape and value ranges:

* ``input_ids``: caption length drawn from [3, text_seq_len], ids in [2, vocab) (0 = pad of the
  unique-pad trick is never produced by the T5 tokenizer without special tokens, 1 = eos = pad),
  right-padded with ``pad_id = 1`` (``task.py:59``, ``DataCollatorWithPadding(max_length=256)``).
* ``attention_mask``: 1 on caption tokens, 0 on padding.
* ``image``: VQGAN codes uniform in [0, num_image_tokens).
"""
from __future__ import annotations

from typing import Dict, Iterator, Optional

import torch
from torch.utils.data import IterableDataset


def synthetic_batch(batch_size: int, text_seq_len: int, image_seq_len: int, vocab_size: int,
                    num_image_tokens: int, generator: Optional[torch.Generator] = None, device="cpu",
                    pad_id: int = 1) -> Dict[str, torch.Tensor]:
    g = generator
    lengths = torch.randint(3, text_seq_len + 1, (batch_size,), generator=g)
    ids = torch.randint(2, vocab_size, (batch_size, text_seq_len), generator=g)
    pos = torch.arange(text_seq_len)[None, :]
    mask = pos < lengths[:, None]
    ids = torch.where(mask, ids, torch.full_like(ids, pad_id))
    image = torch.randint(0, num_image_tokens, (batch_size, image_seq_len), generator=g)
    out = {"input_ids": ids, "attention_mask": mask.long(), "image": image}
    return {k: v.to(device, non_blocking=True) for k, v in out.items()}


class SyntheticLAION(IterableDataset):
    """Infinite stream of single examples, shuffled per ``seed`` (per-peer data order)."""

    def __init__(self, text_seq_len: int = 256, image_seq_len: int = 1024, vocab_size: int = 32100,
                 num_image_tokens: int = 8192, seed: int = 0, length: Optional[int] = None):
        self.text_seq_len, self.image_seq_len = text_seq_len, image_seq_len
        self.vocab_size, self.num_image_tokens = vocab_size, num_image_tokens
        self.seed, self.length = seed, length

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        g = torch.Generator().manual_seed(self.seed)
        i = 0
        while self.length is None or i < self.length:
            b = synthetic_batch(1, self.text_seq_len, self.image_seq_len, self.vocab_size, self.num_image_tokens, g)
            n = int(b["attention_mask"].sum())
            yield {"input_ids": b["input_ids"][0, :n], "attention_mask": b["attention_mask"][0, :n], "image": b["image"][0]}
            i += 1


class PadCollator:
    """``DataCollatorWithPadding(padding='max_length', max_length=text_seq_len)`` with pad id 1."""

    def __init__(self, max_length: int = 256, pad_id: int = 1):
        self.max_length, self.pad_id = max_length, pad_id

    def __call__(self, examples):
        B = len(examples)
        ids = torch.full((B, self.max_length), self.pad_id, dtype=torch.long)
        mask = torch.zeros((B, self.max_length), dtype=torch.long)
        for i, ex in enumerate(examples):
            t = ex["input_ids"][: self.max_length]
            ids[i, : len(t)] = t
            mask[i, : len(t)] = 1
        image = torch.stack([torch.as_tensor(ex["image"]) for ex in examples])
        return {"input_ids": ids, "attention_mask": mask, "image": image}
