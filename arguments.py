"""Command-line schema of the training, TPU-style and auxiliary peers.

Every flag of the reference (``arguments.py:8-165``) keeps its name, default and syntax
(``--name value``, booleans as ``--name True``; parsed by ``dalle_amd.utils.argparse``), so existing
launch scripts run unchanged. ``HFTrainerArguments`` does not derive from ``transformers``' class any
more: it declares the inherited fields the reference reads (``seed``, ``run_name``, ``output_dir``,
``local_rank``, ``do_eval`` ...) itself. Flags that exist only in this engine say so in their help.
"""
from dataclasses import dataclass, field
from typing import List, Optional

import torch


def flag(default, doc: str = "", factory=None):
    """A dataclass field carrying its ``--help`` text (list defaults via ``factory``)."""
    if factory is not None:
        return field(default_factory=factory, metadata={"help": doc})
    return field(default=default, metadata={"help": doc})


@dataclass
class HFTrainerArguments:
    """Micro-batching, the LAMB recipe and the inner trainer loop of one peer."""

    # --- batches and sequence
    per_device_train_batch_size: int = flag(2, "micro-batch per GPU")
    per_device_eval_batch_size: int = flag(2, "evaluation micro-batch per GPU")
    gradient_accumulation_steps: int = flag(1, "micro-batches summed into one optimizer.step() call")
    text_seq_length: int = flag(256, "caption tokens per sample (padded / truncated)")
    dataloader_num_workers: int = flag(1, "data loader worker processes")

    # --- LAMB + schedule (one scheduler step per collaborative epoch)
    learning_rate: float = flag(0.0025, "peak learning rate")
    warmup_steps: int = flag(3125, "linear warm-up length, in collaborative epochs")
    total_steps: int = flag(31250, "epochs until the linear decay reaches zero")
    adam_beta1: float = flag(0.9)
    adam_beta2: float = flag(0.96)
    adam_epsilon: float = flag(1e-6)
    weight_decay: float = flag(0.045, "decoupled weight decay (biases are exempt)")
    max_grad_norm: float = flag(4.0, "global clip applied to the averaged gradient inside LAMB")
    clamp_value: float = flag(10000.0, "upper clamp of the LAMB weight norm in the trust ratio")

    # --- trainer loop bookkeeping
    fp16: bool = flag(False, "fp16 autocast with the collaborative (deferred-unscale) grad scaler")
    do_train: bool = flag(True)
    do_eval: bool = flag(False)
    logging_steps: int = flag(100)
    max_steps: int = flag(10 ** 20, "mini-step budget of this peer")
    save_steps: int = flag(10 ** 20)
    save_total_limit: int = flag(2)
    output_dir: str = flag("outputs", "checkpoints and snapshots of this peer")
    seed: int = flag(42, "model-initialisation seed")
    run_name: Optional[str] = flag(None)
    local_rank: int = flag(-1, "set by torchrun")
    report_to: List[str] = flag(None, factory=list)

    # --- engine-only flags
    model_preset: str = flag("reference", "engine only: dalle_amd.config preset (reference, bench24, tiny, dalle-1.3b)")
    reversible_recompute: str = flag("auto", "engine only: reversible blocks rebuild activations in backward (true), "
                                           "keep them (false: ~30% faster for the 64-layer recipe, ~4 GB per sample "
                                           "of HBM) or keep as many blocks as the free HBM holds (auto)")
    dataset_path: Optional[str] = flag(None, "engine only: directory of LAION-VQGAN parquet/jsonl shards (default: synthetic)")
    optimizer_bits: int = flag(8, "engine only: LAMB moment storage, 8 (CPULAMB8Bit layout) or 32")
    grad_averaging: str = flag("size_adaptive", "engine only: none | fp16 | 8bit | size_adaptive | powersgd")
    powersgd_rank: int = flag(4, "engine only: rank of the PowerSGD factors")
    backend: Optional[str] = flag(None, "engine only: torch.distributed backend (nccl = RCCL on MI355X, gloo on CPU)")
    offload_optimizer_to_host: bool = flag(False, "engine only: optimizer master copy + state in pinned host memory, "
                                                   "stepped on the CPU (default: in HBM, fused HIP LAMB)")

    @property
    def device(self) -> torch.device:
        if not torch.cuda.is_available():
            return torch.device("cpu")
        return torch.device("cuda", max(self.local_rank, 0) % torch.cuda.device_count())

    @property
    def n_gpu(self) -> int:
        return int(torch.cuda.is_available())

    @property
    def batch_size_per_step(self) -> int:
        """Samples one ``optimizer.step()`` of this peer adds to the collaboration.

        A peer is one process on one GPU, so there is no ``torch.cuda.device_count()`` factor (the
        reference's factor would over-count 8x on a node where every process sees all GPUs)."""
        return self.per_device_train_batch_size * self.gradient_accumulation_steps


@dataclass
class TPUTrainerArguments(HFTrainerArguments):
    num_tpus: int = flag(8, "local devices driven by run_trainer_tpu.py (one worker process each)")
    wandb_project: str = flag("huggingface")

    @property
    def batch_size_per_step(self) -> int:
        return super().batch_size_per_step * self.num_tpus


@dataclass
class CollaborativeArguments:
    """Knobs of the collaborative optimizer (epoch size and averaging deadlines)."""

    target_batch_size: int = flag(4096, "global samples per collaborative epoch (one optimizer update)")
    matchmaking_time: float = flag(15.0, "seconds an averaging round waits for late peers")
    allreduce_timeout: float = flag(60, "seconds before one all-reduce round is abandoned")
    averaging_timeout: float = flag(180, "seconds before the whole averaging step is abandoned")
    reuse_grad_buffers: bool = flag(True, "accumulate micro-batch gradients directly in the .grad buffers")


@dataclass
class BasePeerArguments:
    """Identity, tokenizer and key-value-store connectivity shared by all peer kinds."""

    experiment_prefix: str = flag("my-model", "run id: prefix of every key this run stores")
    tokenizer_path: Optional[str] = flag("t5-small", "tokenizer name or directory")
    cache_dir: Optional[str] = flag("./cache", "cache directory (accepted; unused, as in the reference)")
    authorize: bool = flag(True, "obtain an authority-signed access token before joining")
    client_mode: bool = flag(False, "accept no inbound connections (never hosts the store or a reduce shard)")
    initial_peers: List[str] = flag(None, "multiaddr of the store host, e.g. /ip4/127.0.0.1/tcp/31337", factory=list)
    use_ipfs: bool = flag(False, "accepted for compatibility; there is no public DHT")
    host_maddrs: List[str] = flag(None, "listen multiaddrs (the first peer hosts the store)",
                                  factory=lambda: ["/ip4/0.0.0.0/tcp/0"])
    announce_maddrs: List[str] = flag(None, "multiaddrs to advertise instead of the bound ones", factory=list)
    identity_path: Optional[str] = flag(None, "file with this peer's persistent id")
    elastic_coordinator: Optional[str] = flag(
        None, "engine only: host:port of the elastic coordinator store (run_aux_peer.py --host_elastic_coordinator "
              "True); trainers then build their communicator through it, survive peer death and admit late joiners")


@dataclass
class TrainingPeerArguments(BasePeerArguments):
    statistics_expiration: float = flag(600, "seconds a published metrics record stays alive")
    backup_every_steps: Optional[int] = flag(None, "write a state backup every this many epochs (None: never)")
    state_path: str = flag("state.zip", "backup file, loaded at start-up and after NaN parameters")


@dataclass
class AuxiliaryPeerArguments(BasePeerArguments):
    """The monitoring / checkpointing peer: aggregates metrics, snapshots and uploads state."""

    refresh_period: float = flag(10, "seconds between two polls of the metrics records")
    wandb_project: Optional[str] = flag(None, "Weights & Biases project for the aggregated curves")
    save_checkpoint_step_interval: int = flag(2, "fetch the collaboration state every this many epochs")
    repo_url: Optional[str] = flag(None, "Hugging Face Hub repository receiving the checkpoints")
    local_path: Optional[str] = flag("Repo", "local directory (clone) for model_state.pt / optimizer_state.pt")
    upload_interval: Optional[float] = flag(None, "seconds between two uploads to the Hub")
    store_checkpoints: bool = flag(True, "enable the checkpoint handler")
    assist_in_averaging: bool = flag(False, "serve as an extra averaging peer (not implemented, as in the reference)")
    assist_refresh: float = flag(1.0, "seconds between two averaging-assist attempts")
    host_elastic_coordinator: bool = flag(False, "engine only: host the elastic coordinator at --elastic_coordinator")
    metrics_log: Optional[str] = flag(None, "engine only: JSON-lines file receiving the aggregated metrics")
    max_iterations: Optional[int] = flag(None, "engine only: stop after this many polls (tests)")
