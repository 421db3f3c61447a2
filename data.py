"""LAION-VQGAN data pipeline (reference ``data.py:11-47``).

Same filtering (caption length >= 3, ``NSFW == 'UNLIKELY'``, positive dims, aspect ratio <= 2),
tokenisation (no special tokens, truncation to ``max_sequence_length``) and int16 -> int64 code
decoding as the reference's ``preprocess_batch``. Sources, in order of preference:

* ``dataset_path``: a local directory of parquet / jsonl shards with the
  ``laion/laion_100m_vqgan_f8`` columns (``caption, NSFW, original_width, original_height, code``),
  streamed record batch by record batch; or a ``datasets`` streaming source -- the reference's Hub id
  (network needed) or ``parquet:<glob>`` / ``json:<glob>``;
* otherwise synthetic LAION-shaped pairs (there is no network for the streamed dataset).

Per-peer shuffling uses a seeded shuffle buffer (``shuffle_buffer_size``, ``shuffle_seed``).
"""
import glob
import itertools
import json
import os
import random
from typing import Iterator, Optional

import numpy as np
import torch
from torch.utils.data import IterableDataset

from dalle_amd.data.synthetic import SyntheticLAION
from dalle_amd.utils.logging import get_logger

logger = get_logger(__name__)


def _keep_example(caption, nsfw, width, height) -> bool:
    """The reference run's LAION filter: a caption of >= 3 characters, rated SFW, and an image with
    positive dimensions whose long side is at most twice its short side."""
    if caption is None or len(caption) < 3 or nsfw != "UNLIKELY":
        return False
    if not (width > 0 and height > 0):
        return False
    return max(width, height) <= 2 * min(width, height)


def preprocess_batch(batch, tokenizer, max_sequence_length: int):
    """Filter a column batch, tokenise the kept captions (no special tokens, truncated) and decode the
    kept VQGAN code bytes (int16) into int64 token ids."""
    columns = zip(batch["caption"], batch["NSFW"], batch["original_width"], batch["original_height"])
    kept = [i for i, row in enumerate(columns) if _keep_example(*row)]
    logger.debug(f"filter kept {len(kept)} of {len(batch['caption'])} examples")
    captions = [batch["caption"][i] for i in kept]
    if captions:  # an empty list would make the tokenizer raise
        enc = tokenizer(captions, add_special_tokens=False, max_length=max_sequence_length, truncation=True)
        out = {"input_ids": list(enc["input_ids"]), "attention_mask": list(enc["attention_mask"])}
    else:
        out = {"input_ids": [], "attention_mask": []}
    out["image"] = [np.frombuffer(batch["code"][i], dtype=np.int16).astype(np.int64) for i in kept]
    return out


_COLUMNS = ("caption", "NSFW", "original_width", "original_height", "code")


def _iter_rows(path: str) -> Iterator[dict]:
    files = sorted(glob.glob(os.path.join(path, "*.parquet")) + glob.glob(os.path.join(path, "*.jsonl")))
    if not files:
        raise FileNotFoundError(f"no *.parquet / *.jsonl shards in {path}")
    for f in files:
        if f.endswith(".parquet"):
            import pyarrow.parquet as pq

            # streamed record batch by record batch: a shard is never materialised whole
            pf = pq.ParquetFile(f)
            cols = [c for c in _COLUMNS if c in pf.schema_arrow.names]
            for batch in pf.iter_batches(batch_size=1024, columns=cols):
                d = batch.to_pydict()
                for i in range(batch.num_rows):
                    yield {c: d[c][i] for c in cols}
        else:
            with open(f) as fh:
                for line in fh:
                    row = json.loads(line)
                    if isinstance(row.get("code"), list):
                        row["code"] = np.asarray(row["code"], dtype=np.int16).tobytes()
                    yield row


class LocalLAIONDataset(IterableDataset):
    def __init__(self, path, tokenizer, shuffle_buffer_size, shuffle_seed, preprocessing_batch_size, max_sequence_length):
        self.path, self.tokenizer = path, tokenizer
        self.shuffle_buffer_size, self.shuffle_seed = shuffle_buffer_size, shuffle_seed
        self.bs, self.max_len = preprocessing_batch_size, max_sequence_length

    def _examples(self):
        rows = _iter_rows(self.path)
        while True:
            chunk = list(itertools.islice(rows, self.bs))
            if not chunk:
                return
            batch = {k: [r.get(k) for r in chunk] for k in ("caption", "NSFW", "original_width", "original_height", "code")}
            out = preprocess_batch(batch, self.tokenizer, self.max_len)
            for ids, am, img in zip(out["input_ids"], out["attention_mask"], out["image"]):
                yield {"input_ids": torch.tensor(ids), "attention_mask": torch.tensor(am), "image": torch.from_numpy(img)}

    def __iter__(self):
        rng = random.Random(self.shuffle_seed)
        buf = []
        for ex in self._examples():
            if len(buf) < self.shuffle_buffer_size:
                buf.append(ex)
                continue
            i = rng.randrange(len(buf))
            yield buf[i]
            buf[i] = ex
        rng.shuffle(buf)
        yield from buf


class HFStreamingLAION(IterableDataset):
    """The reference's source (``data.py:34-47``): a ``datasets`` streaming dataset -- a Hub id such as
    ``laion/laion_100m_vqgan_f8`` (needs network) or ``parquet:<glob>`` / ``json:<glob>`` for local
    shards -- shuffled with a seeded buffer and mapped through :func:`preprocess_batch` in batches."""

    def __init__(self, spec: str, tokenizer, shuffle_buffer_size, shuffle_seed, preprocessing_batch_size, max_sequence_length):
        import datasets

        builder, _, files = spec.partition(":")
        if builder in ("parquet", "json") and files:
            ds = datasets.load_dataset(builder, data_files=sorted(glob.glob(files)), split="train", streaming=True)
        else:
            ds = datasets.load_dataset(spec, split="train", streaming=True)
        ds = ds.shuffle(seed=shuffle_seed, buffer_size=shuffle_buffer_size)
        keep = [c for c in _COLUMNS]
        self.ds = ds.map(lambda b: preprocess_batch(b, tokenizer, max_sequence_length), batched=True,
                         batch_size=preprocessing_batch_size, remove_columns=[c for c in (ds.column_names or keep)])

    def __iter__(self):
        for ex in self.ds:
            yield {"input_ids": torch.as_tensor(ex["input_ids"]), "attention_mask": torch.as_tensor(ex["attention_mask"]),
                   "image": torch.as_tensor(np.asarray(ex["image"], dtype=np.int64))}


def make_dataset(
    tokenizer,
    *,
    shuffle_buffer_size: int = 8192,
    shuffle_seed: Optional[int],
    preprocessing_batch_size: int = 256,
    max_sequence_length: int,
    dataset_path: Optional[str] = None,
    image_seq_len: int = 1024,
    num_image_tokens: int = 8192,
):
    if dataset_path and os.path.isdir(dataset_path):
        return LocalLAIONDataset(dataset_path, tokenizer, shuffle_buffer_size, shuffle_seed,
                                 preprocessing_batch_size, max_sequence_length)
    if dataset_path:  # a `datasets` streaming source (Hub id, or parquet:/json: globs)
        return HFStreamingLAION(dataset_path, tokenizer, shuffle_buffer_size, shuffle_seed,
                                preprocessing_batch_size, max_sequence_length)
    logger.info("no dataset_path given: streaming synthetic LAION-shaped pairs")
    return SyntheticLAION(text_seq_len=max_sequence_length, image_seq_len=image_seq_len,
                          vocab_size=getattr(tokenizer, "vocab_size", 32100), num_image_tokens=num_image_tokens,
                          seed=int(shuffle_seed or 0))
