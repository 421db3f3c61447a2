"""dalle_amd -- an MI355X-native collaborative DALL-E training and inference engine.

Layers: ``models`` (DALL-E, patterns, rotary, reversible engine, VQGAN decoder), ``ops`` (HIP
kernel bindings + reference ops), ``optim`` (8-bit LAMB, blockwise quantisation, schedules),
``parallel`` (collaborative optimizer on RCCL/gloo, compression, PowerSGD, KV store / DHT facade),
``train`` (trainer loop + callbacks), ``data`` (synthetic LAION-shaped data, collator), ``utils``.
"""
from .config import DALLEConfig, get_config  # noqa: F401

__version__ = "0.1.0"
