"""LAION-VQGAN data pipeline (reference ``data.py:11-47``).

Same filtering (caption length >= 3, ``NSFW == 'UNLIKELY'``, positive dims, aspect ratio <= 2),
tokenisation (no special tokens, truncation to ``max_sequence_length``) and int16 -> int64 code
decoding as the reference's ``preprocess_batch``. Sources, in order of preference:

* ``dataset_path``: a local directory of parquet / jsonl shards with the
  ``laion/laion_100m_vqgan_f8`` columns (``caption, NSFW, original_width, original_height, code``);
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


def _iter_rows(path: str) -> Iterator[dict]:
    files = sorted(glob.glob(os.path.join(path, "*.parquet")) + glob.glob(os.path.join(path, "*.jsonl")))
    if not files:
        raise FileNotFoundError(f"no *.parquet / *.jsonl shards in {path}")
    for f in files:
        if f.endswith(".parquet"):
            import pyarrow.parquet as pq

            table = pq.read_table(f)
            cols = table.column_names
            for batch in table.to_batches(1024):
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
    if dataset_path:
        return LocalLAIONDataset(dataset_path, tokenizer, shuffle_buffer_size, shuffle_seed,
                                 preprocessing_batch_size, max_sequence_length)
    logger.info("no dataset_path given: streaming synthetic LAION-shaped pairs")
    return SyntheticLAION(text_seq_len=max_sequence_length, image_seq_len=image_seq_len,
                          vocab_size=getattr(tokenizer, "vocab_size", 32100), num_image_tokens=num_image_tokens,
                          seed=int(shuffle_seed or 0))
