"""Caption tokenizers (``T5TokenizerFast('t5-small')``, ``pad = eos = 1``; reference
task.py:58-59, data.py:24, inference/run_inference.py:47,81).

Order of preference when a tokenizer directory is available locally (no network fetch is ever
attempted):

1. ``NativeUnigramTokenizer``: the in-tree C++ pipeline (``csrc/tokenizer``, module
   ``dalle_amd._tokenizer``) configured from ``tokenizer.json`` -- SentencePiece precompiled-charsmap
   normalisation, whitespace / metaspace pre-tokenisation, unigram Viterbi, ``</s>`` template,
   truncation -- batch-encoded on host threads without the GIL. This replaces the reference's Rust
   ``tokenizers`` dependency; parity with it is tested on locally trained SentencePiece
   models (tests/test_tokenizer_cpu.py).
2. the ``tokenizers`` library on the same ``tokenizer.json`` (pipelines the native one does not cover),
3. ``sentencepiece`` on ``spiece.model``.

Without tokenizer files a deterministic hashing tokenizer with the same vocabulary size (32100), the
same special ids (pad = eos = 1, unk = 2) and the same call signature stands in -- enough for
throughput and plumbing runs on synthetic data.
"""
from __future__ import annotations

import base64
import json
import os
import re
import unicodedata
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

    def __call__(self, texts: Union[str, Sequence[str]], add_special_tokens: bool = True, max_length: int = None,
                 truncation: bool = False, **kw) -> Dict[str, list]:
        single = isinstance(texts, str)
        batch = [texts] if single else list(texts)
        ids = []
        for t in batch:
            x = self._encode(t)
            if truncation and max_length is not None:
                # the library truncates the sequence and keeps room for the appended </s>
                x = x[:max(0, max_length - (1 if add_special_tokens else 0))]
            if add_special_tokens:
                x = x + [self.eos_token_id]
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


class UnsupportedPipeline(ValueError):
    """The tokenizer.json uses a component the native pipeline does not implement."""


_UNICODE_FORMS = {"NFC", "NFD", "NFKC", "NFKD"}


class NativeUnigramTokenizer(HashingTokenizer):
    """``tokenizer.json`` (unigram model) run by the native C++ pipeline. Unicode-table normalisers
    (NFKC & co.) are applied in Python when they come before every native step; anything else the
    native pipeline lacks raises ``UnsupportedPipeline`` so the caller can fall back to the library."""

    def __init__(self, tokenizer_json: str, threads: int = 4):
        from .. import _tokenizer

        with open(tokenizer_json, encoding="utf-8") as f:
            spec = json.load(f)
        model = spec.get("model") or {}
        if model.get("type") != "Unigram":
            raise UnsupportedPipeline(f"model type {model.get('type')}")
        if model.get("byte_fallback"):
            raise UnsupportedPipeline("byte_fallback")
        vocab = [(str(p), float(sc)) for p, sc in model["vocab"]]
        unk = model.get("unk_id")
        super().__init__(vocab_size=len(vocab), unk_id=0 if unk is None else int(unk))
        self.threads = threads
        pipe = _tokenizer.Pipeline()
        self._py_forms = []
        self._configure_normalizer(pipe, spec.get("normalizer"))
        self._configure_pretokenizer(pipe, spec.get("pre_tokenizer"))
        pipe.set_model(vocab, self.unk_token_id if unk is not None else 0, unk is not None)
        added = []
        for t in spec.get("added_tokens") or []:
            if t.get("normalized") or t.get("lstrip") or t.get("rstrip") or t.get("single_word"):
                raise UnsupportedPipeline(f"added token options of {t['content']!r}")
            added.append((t["content"], int(t["id"])))
        pipe.set_added(added)
        self._configure_post(pipe, spec.get("post_processor"))
        ids = dict((c, i) for c, i in added)
        self.eos_token = "</s>"
        if "</s>" in ids:
            self.eos_token_id = self.pad_token_id = ids["</s>"]
        self.pipe = pipe

    def _configure_normalizer(self, pipe, spec):
        steps = [] if spec is None else (spec["normalizers"] if spec.get("type") == "Sequence" else [spec])
        native = False
        for st in steps:
            kind = st.get("type")
            if kind in _UNICODE_FORMS:
                if native:
                    raise UnsupportedPipeline(f"{kind} after a native normaliser step")
                self._py_forms.append(kind)
            elif kind == "Precompiled":
                if st.get("precompiled_charsmap"):
                    pipe.add_charsmap(base64.b64decode(st["precompiled_charsmap"]))
                    native = True
            elif kind == "Strip":
                pipe.add_strip(bool(st.get("strip_left", False)), bool(st.get("strip_right", True)))
                native = True
            elif kind == "Replace":
                pat = st["pattern"]
                if "Regex" in pat:
                    pipe.add_replace(pat["Regex"], st["content"], True)
                else:
                    pipe.add_replace(pat["String"], st["content"], False)
                native = True
            else:
                raise UnsupportedPipeline(f"normalizer {kind}")

    @staticmethod
    def _configure_pretokenizer(pipe, spec):
        steps = [] if spec is None else (spec["pretokenizers"] if spec.get("type") == "Sequence" else [spec])
        ws = meta = False
        rep, prepend, split = "\u2581", 0, True
        for st in steps:
            kind = st.get("type")
            if kind == "WhitespaceSplit" and not meta:
                ws = True
            elif kind == "Metaspace" and not meta:
                meta = True
                rep = st.get("replacement", rep)
                scheme = st.get("prepend_scheme")
                if scheme is None:  # older files: add_prefix_space
                    scheme = "always" if st.get("add_prefix_space", True) else "never"
                prepend = {"always": 0, "first": 1, "never": 2}[scheme]
                split = bool(st.get("split", True))
            else:
                raise UnsupportedPipeline(f"pre_tokenizer {kind}")
        pipe.set_pretokenizer(ws, meta, rep, prepend, split)

    @staticmethod
    def _configure_post(pipe, spec):
        if spec is None:
            pipe.set_suffix([])
            return
        if spec.get("type") != "TemplateProcessing":
            raise UnsupportedPipeline(f"post_processor {spec.get('type')}")
        single = spec["single"]
        if not single or "Sequence" not in single[0]:
            raise UnsupportedPipeline("template with a prefix")
        suffix = []
        for piece in single[1:]:
            if "SpecialToken" not in piece:
                raise UnsupportedPipeline("template with a second sequence")
            suffix += list(spec["special_tokens"][piece["SpecialToken"]["id"]]["ids"])
        pipe.set_suffix(suffix)

    def _prep(self, text: str) -> str:
        for form in self._py_forms:
            text = unicodedata.normalize(form, text)
        return text

    def _encode(self, text: str) -> List[int]:
        return self.pipe.encode(self._prep(text))

    def __call__(self, texts: Union[str, Sequence[str]], add_special_tokens: bool = True, max_length: int = None,
                 truncation: bool = False, **kw) -> Dict[str, list]:
        single = isinstance(texts, str)
        batch = [self._prep(t) for t in ([texts] if single else texts)]
        ids = self.pipe.encode_batch(batch, bool(add_special_tokens), -1 if max_length is None else int(max_length),
                                     bool(truncation and max_length is not None), self.threads)
        out = {"input_ids": ids, "attention_mask": [[1] * len(x) for x in ids]}
        if single:
            out = {k: v[0] for k, v in out.items()}
        return out


def load_tokenizer(path: str = "t5-small", vocab_size: int = 32100):
    if path and os.path.isdir(path):
        tj = os.path.join(path, "tokenizer.json")
        if os.path.exists(tj):
            try:
                return NativeUnigramTokenizer(tj)
            except (UnsupportedPipeline, ImportError):
                pass
            from tokenizers import Tokenizer

            return _TokenizersAdapter(Tokenizer.from_file(tj), vocab_size)
        sp = os.path.join(path, "spiece.model")
        if os.path.exists(sp):
            import sentencepiece

            return _SentencePieceAdapter(sentencepiece.SentencePieceProcessor(model_file=sp))
    return HashingTokenizer(vocab_size=vocab_size)
