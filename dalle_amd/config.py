"""Model recipes for the DALL-E family.

The reference builds its model inline in ``task.py:61-83`` (and a copy in
``inference/run_inference.py:46-76``); the architecture itself lives in the pinned
``dalle-pytorch`` fork. Here the recipe is a plain dataclass so that every entrypoint,
test and benchmark builds the model from one place.

Presets:
  * ``reference()``  -- the reference recipe: 64 layers, 5 shared attn + 5 shared FF blocks,
    reversible, rotary, token shift, tied input/output embeddings (``task.py:61-83``).
  * ``bench24()``    -- BASELINE config 2: d_model=1024, 24 layers, 256 text + 32x32 image tokens.
  * ``tiny()``       -- BASELINE config 1: 2 layers, 64 text + 16x16 image tokens (CPU plumbing).
  * ``large_1p3b()`` -- BASELINE config 4: ~1.3B unique params, reversible.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field, asdict
from itertools import cycle, islice
from typing import List, Union

AttnId = Union[int, str]


def reference_attn_types(depth: int) -> List[str]:
    """cycle(axial_row, axial_col, axial_row, axial_row) for depth-1 layers + conv_like (task.py:63-64)."""
    types = list(islice(cycle(["axial_row", "axial_col", "axial_row", "axial_row"]), depth - 1))
    types.append("conv_like")
    return types


def reference_shared_ids(depth: int) -> List[AttnId]:
    """cycle(0,1,2,3) for depth-1 layers + 'w_conv' (task.py:65-66)."""
    ids: List[AttnId] = list(islice(cycle(range(4)), depth - 1))
    ids.append("w_conv")
    return ids


@dataclass
class DALLEConfig:
    # tokenizer / data geometry
    num_text_tokens: int = 32100  # tokenizer vocab (t5-small); the model adds text_seq_len unique pad ids
    text_seq_len: int = 256
    image_size: int = 256
    vae_num_layers: int = 3  # downsampling factor f = 2**vae_num_layers
    num_image_tokens: int = 8192
    # transformer
    dim: int = 1024
    depth: int = 64
    heads: int = 16
    dim_head: int = 64
    ff_mult: int = 4
    attn_types: List[str] = field(default_factory=lambda: reference_attn_types(64))
    shared_attn_ids: List[AttnId] = field(default_factory=lambda: reference_shared_ids(64))
    shared_ff_ids: List[AttnId] = field(default_factory=lambda: reference_shared_ids(64))
    attn_dropout: float = 0.0
    ff_dropout: float = 0.0
    rotary_emb: bool = True
    shift_tokens: bool = True
    reversible: bool = True
    # reversible blocks rebuild their inputs in backward (the reference's O(1)-in-depth activation memory);
    # False keeps the activations instead -- same coupling math, one forward less per step (HBM permitting)
    reversible_recompute: Union[bool, str] = True  # True | False | "auto" (keep what fits in HBM)
    share_input_output_emb: bool = True
    loss_img_weight: float = 7.0
    conv_kernel_size: int = 5

    def __post_init__(self):
        assert len(self.attn_types) == self.depth, "attn_types must have one entry per layer"
        assert len(self.shared_attn_ids) == self.depth and len(self.shared_ff_ids) == self.depth
        assert self.ff_dropout == 0.0 and self.attn_dropout == 0.0, "dropout is compile-time off (task.py:76-77)"
        assert self.rotary_emb, "only rotary positional embeddings are supported (task.py:80)"
        known = {"axial_row", "axial_col", "conv_like", "full"}
        for t in self.attn_types:
            assert t in known, f"unknown attention type {t}"
        assert (self.image_fmap_size ** 2) % 32 == 0, "image token grid must be a multiple of 32 tokens"

    # ---- derived geometry (dalle_pytorch.DALLE.__init__ semantics) ----
    @property
    def image_fmap_size(self) -> int:
        return self.image_size // (2 ** self.vae_num_layers)

    @property
    def image_seq_len(self) -> int:
        return self.image_fmap_size ** 2

    @property
    def total_text_tokens(self) -> int:
        """num_text_tokens + text_seq_len: unique padding id per text position (D1)."""
        return self.num_text_tokens + self.text_seq_len

    @property
    def total_tokens(self) -> int:
        return self.total_text_tokens + self.num_image_tokens

    @property
    def seq_len(self) -> int:
        """Model sequence length: BOS + text + image - last image token."""
        return self.text_seq_len + self.image_seq_len

    @property
    def text_len(self) -> int:
        """Number of text positions incl. BOS (257 at the reference config)."""
        return self.text_seq_len + 1

    @property
    def inner_dim(self) -> int:
        return self.heads * self.dim_head

    def to_dict(self):
        return asdict(self)

    # ---- parameter / FLOP accounting ----
    def unique_param_count(self) -> int:
        d, inner = self.dim, self.inner_dim
        attn = d * 3 * inner + inner * d + d
        ff = d * 2 * self.ff_mult * d + 2 * self.ff_mult * d + self.ff_mult * d * d + d
        n_attn = len(set(map(str, self.shared_attn_ids)))
        n_ff = len(set(map(str, self.shared_ff_ids)))
        per_layer = 2 * d + 2 * 2 * d  # 2 LayerScale + 2 LayerNorm
        head = self.total_tokens * d + self.total_tokens + 2 * d
        return n_attn * attn + n_ff * ff + self.depth * per_layer + head

    def train_flops_per_sample(self, include_recompute: bool = False) -> float:
        """Matmul FLOPs of one training sample: forward + backward (3x forward) = MODEL FLOPs, the MFU
        convention. ``include_recompute`` adds the reversible stack's extra forward recompute (the
        HARDWARE FLOPs actually executed when the activations are rebuilt instead of stored)."""
        d, inner, n = self.dim, self.inner_dim, self.seq_len
        per_layer = 2 * n * (d * 3 * inner + inner * d + d * 2 * self.ff_mult * d + self.ff_mult * d * d)
        # sparse attention scores: image queries see text + local keys, text is causal
        t, i = self.text_len, self.image_seq_len
        per_layer += 4 * self.heads * self.dim_head * (t * t / 2 + i * (t + self.image_fmap_size))
        head = 2 * (self.text_seq_len * self.total_text_tokens + self.image_seq_len * self.num_image_tokens) * d
        layer_mult = 4.0 if (self.reversible and self.reversible_recompute is True and include_recompute) else 3.0
        return layer_mult * self.depth * per_layer + 3.0 * head


def reference(text_seq_len: int = 256, num_text_tokens: int = 32100) -> DALLEConfig:
    return DALLEConfig(num_text_tokens=num_text_tokens, text_seq_len=text_seq_len)


def bench24() -> DALLEConfig:
    """BASELINE config 2: d_model=1024, 24 layers, 256 text + 32x32 image tokens.

    Same layer recipe as the reference (attention cycle + final conv_like, ALBERT-style sharing
    cycle(4) + 'w_conv', rotary, token shift, tied embeddings). Activations are stored (not
    reversible): with 288 GB of HBM per GPU the recompute is not needed at this depth.
    """
    depth = 24
    return DALLEConfig(
        depth=depth,
        attn_types=reference_attn_types(depth),
        shared_attn_ids=reference_shared_ids(depth),
        shared_ff_ids=reference_shared_ids(depth),
        reversible=False,
    )


def bench24_unshared() -> DALLEConfig:
    """BASELINE config 2 without weight sharing: 24 layers with their own attention / FF weights
    (~444M unique parameters), so the data-parallel gradient all-reduce moves every layer's bytes
    (bench24 shares 5 blocks, 126M gradients, which flatters a scaling curve's comm/compute overlap)."""
    depth = 24
    return DALLEConfig(
        depth=depth,
        attn_types=reference_attn_types(depth),
        shared_attn_ids=list(range(depth)),
        shared_ff_ids=list(range(depth)),
        reversible=False,
    )


def tiny(reversible: bool = True) -> DALLEConfig:
    """BASELINE config 1: 2 layers, 64 text + 16x16 image tokens."""
    depth = 2
    return DALLEConfig(
        num_text_tokens=1000,
        text_seq_len=64,
        image_size=128,
        vae_num_layers=3,
        num_image_tokens=512,
        dim=256,
        depth=depth,
        heads=4,
        dim_head=64,
        attn_types=["axial_row", "conv_like"],
        shared_attn_ids=[0, "w_conv"],
        shared_ff_ids=[0, "w_conv"],
        reversible=reversible,
    )


def large_1p3b() -> DALLEConfig:
    """BASELINE config 4: ~1.3B unique parameters (1.29B: d_model 2048, 18 unshared layers of
    67.1M + the 83M tied head), reversible blocks, no weight sharing."""
    depth = 18
    return DALLEConfig(
        dim=2048,
        depth=depth,
        heads=32,
        dim_head=64,
        attn_types=reference_attn_types(depth),
        shared_attn_ids=list(range(depth)),
        shared_ff_ids=list(range(depth)),
        reversible=True,
    )


PRESETS = {
    "reference": reference,
    "dalle-1024-64l": reference,
    "bench24": bench24,
    "dalle-1024-24l": bench24,
    "dalle-1024-24l-unshared": bench24_unshared,
    "tiny": tiny,
    "dalle-1.3b": large_1p3b,
}


def get_config(name: str) -> DALLEConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; choose from {sorted(PRESETS)}")
    return PRESETS[name]()


def ceil_to(x: int, m: int) -> int:
    return int(math.ceil(x / m) * m)
