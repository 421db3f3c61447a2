"""Caption tokenizer adapter (``T5TokenizerFast('t5-small')``, ``pad = eos = 1``).

Uses a real tokenizer when its files are available locally (a ``tokenizer.json`` for the native
``tokenizers`` library, or a SentencePiece ``spiece.model``); no network fetch is ever attempted.
Otherwise a deterministic hashing tokenizer with the same vocabulary size (32100), the same
special ids (pad = eos = 1, unk = 2) and the same call signature stands in -- enough for
throughput and plumbing runs on synthetic data.
"""
from __future__ import annotations

import os
import re
import zlib
from typing import Dict, List, Sequence, Union


class HashingTokenizer:
    def __init__(self, vocab_size: int = 32100, pad_id: int = 1, eos_id: int = 1, unk_id: int = 2):
        self.vocab_size = vocab_size
        self.pad_token_id, self.eos_token_id, self.unk_token_id = pad_id, eos_id, unk_id
        self.eos_token = "</s>"
        self.pad_token = "</s>"

    def _encode(self, text: str) -> List[int]:
        pieces = re.findall(r"\w+|[^\w\s]", text.lower())
        return [3 + zlib.crc32(p.encode()) % (self.vocab_size - 3) for p in pieces]

    def __call__(self, texts: Union[str, Sequence[str]], add_special_tokens: bool = False, max_length: int = None,
                 truncation: bool = False, **kw) -> Dict[str, list]:
        single = isinstance(texts, str)
        batch = [texts] if single else list(texts)
        ids = []
        for t in batch:
            x = self._encode(t)
            if add_special_tokens:
                x = x + [self.eos_token_id]
            if truncation and max_length is not None:
                x = x[:max_length]
            ids.append(x)
        out = {"input_ids": ids, "attention_mask": [[1] * len(x) for x in ids]}
        if single:
            out = {k: v[0] for k, v in out.items()}
        return out


class _TokenizersAdapter(HashingTokenizer):
    def __init__(self, tok, vocab_size: int):
        super().__init__(vocab_size=vocab_size)
        self.tok = tok

    def _encode(self, text: str) -> List[int]:
        return self.tok.encode(text, add_special_tokens=False).ids


class _SentencePieceAdapter(HashingTokenizer):
    def __init__(self, sp):
        super().__init__(vocab_size=sp.get_piece_size() + 100)  # T5 adds 100 sentinel ids
        self.sp = sp

    def _encode(self, text: str) -> List[int]:
        return self.sp.encode(text)


def load_tokenizer(path: str = "t5-small", vocab_size: int = 32100):
    if path and os.path.isdir(path):
        tj = os.path.join(path, "tokenizer.json")
        if os.path.exists(tj):
            from tokenizers import Tokenizer

            return _TokenizersAdapter(Tokenizer.from_file(tj), vocab_size)
        sp = os.path.join(path, "spiece.model")
        if os.path.exists(sp):
            import sentencepiece

            return _SentencePieceAdapter(sentencepiece.SentencePieceProcessor(model_file=sp))
    return HashingTokenizer(vocab_size=vocab_size)
