"""Flag schema of the training / auxiliary peers -- field-for-field compatible with the reference
(``arguments.py:8-165``): same names, defaults and CLI syntax (``--flag value``, ``--flag True``).

``HFTrainerArguments`` no longer subclasses ``transformers.TrainingArguments``; it carries the
inherited fields the reference actually reads (``seed``, ``run_name``, ``output_dir``, ``local_rank``,
``do_eval`` ...) plus a few MI355X-engine extensions marked [new].
"""
from dataclasses import dataclass, field
from typing import List, Optional

import torch


@dataclass
class HFTrainerArguments:
    """Arguments for the collaborative trainer loop (formerly huggingface/transformers.Trainer)"""
    dataloader_num_workers: int = 1
    per_device_train_batch_size: int = 2
    per_device_eval_batch_size: int = 2
    gradient_accumulation_steps: int = 1
    text_seq_length: int = 256

    # DALLE-specific params
    learning_rate: float = 0.0025
    adam_beta1: float = 0.9
    adam_beta2: float = 0.96
    max_grad_norm: float = 4.0
    weight_decay: float = 0.045

    total_steps: int = 31250  # total number of collaborative SGD updates, used for learning rate schedule
    warmup_steps: int = 3125
    adam_epsilon: float = 1e-6
    clamp_value: float = 10000.0

    fp16: bool = False
    do_train: bool = True
    do_eval: bool = False

    logging_steps: int = 100
    max_steps: int = 10 ** 20
    save_steps: int = 10 ** 20
    save_total_limit: int = 2

    output_dir: str = "outputs"

    # inherited TrainingArguments fields used by the reference
    seed: int = 42
    run_name: Optional[str] = None
    local_rank: int = -1
    report_to: List[str] = field(default_factory=list)

    # [new] MI355X engine extensions
    model_preset: str = field(default="reference", metadata={"help": "dalle_amd.config preset (reference, bench24, tiny, dalle-1.3b)"})
    dataset_path: Optional[str] = field(default=None, metadata={"help": "local LAION-VQGAN shard dir (parquet/jsonl); default synthetic"})
    optimizer_bits: int = field(default=8, metadata={"help": "LAMB moment precision: 8 (CPULAMB8Bit) or 32"})
    grad_averaging: str = field(default="size_adaptive", metadata={"help": "none | fp16 | 8bit | size_adaptive | powersgd"})
    powersgd_rank: int = 4
    backend: Optional[str] = field(default=None, metadata={"help": "torch.distributed backend (nccl=RCCL on GPU, gloo on CPU)"})

    @property
    def device(self) -> torch.device:
        if torch.cuda.is_available():
            idx = max(self.local_rank, 0)
            return torch.device("cuda", idx % torch.cuda.device_count())
        return torch.device("cpu")

    @property
    def n_gpu(self) -> int:
        return 1 if torch.cuda.is_available() else 0

    @property
    def batch_size_per_step(self):
        """Training sequences contributed by each .step() of this peer.

        One process drives one GPU (one peer per MI355X), so -- unlike the reference, which multiplied
        by ``torch.cuda.device_count()`` (SURVEY §5.9 gotcha) -- the local device count is 1."""
        return self.per_device_train_batch_size * self.gradient_accumulation_steps


@dataclass
class TPUTrainerArguments(HFTrainerArguments):
    num_tpus: int = 8  # the total number of TPU cores in use
    wandb_project: str = "huggingface"

    @property
    def batch_size_per_step(self):
        return self.per_device_train_batch_size * self.gradient_accumulation_steps * self.num_tpus


@dataclass
class CollaborativeArguments:
    """Configuration for CollaborativeOptimizer and its internals"""
    target_batch_size: int = field(
        default=4096,
        metadata={"help": "Perform optimizer step after all peers collectively accumulate this many samples"},
    )
    matchmaking_time: float = field(
        default=15.0, metadata={"help": "Averaging group will wait for stragglers for at most this many seconds"}
    )
    allreduce_timeout: float = field(
        default=60, metadata={"help": "Give up on a given all-reduce round after this many seconds"}
    )
    averaging_timeout: float = field(
        default=180, metadata={"help": "Give up on averaging step after this many seconds"}
    )
    reuse_grad_buffers: bool = field(default=True, metadata={
        "help": "Whether or not to use model's .grad buffers for accumulating gradients across local steps."})


@dataclass
class BasePeerArguments:
    """Base arguments that are used for both trainers and for auxiliary peers such as training monitor"""
    experiment_prefix: str = field(default="my-model", metadata={"help": "A unique experiment name, used as prefix for all DHT keys"})
    tokenizer_path: Optional[str] = field(default="t5-small", metadata={"help": "Path to the tokenizer"})
    cache_dir: Optional[str] = field(default="./cache", metadata={"help": "Path to the cache"})

    authorize: bool = field(default=True, metadata={"help": "Whether or not to use HF authorizer"})
    client_mode: bool = field(
        default=False,
        metadata={"help": "Of True, runs training without incoming connections, in a firewall-compatible mode"},
    )
    initial_peers: List[str] = field(
        default_factory=list,
        metadata={"help": "Multiaddrs of the key-value store host, e.g. /ip4/127.0.0.1/tcp/31337"},
    )
    use_ipfs: bool = field(default=False, metadata={"help": "Accepted for compatibility; there is no public DHT"})
    host_maddrs: List[str] = field(
        default_factory=lambda: ["/ip4/0.0.0.0/tcp/0"],
        metadata={"help": "Multiaddrs to listen on (the first peer hosts the key-value store)"},
    )
    announce_maddrs: List[str] = field(
        default_factory=list,
        metadata={"help": "Visible multiaddrs the host announces for external connections"},
    )
    identity_path: Optional[str] = field(default=None, metadata={"help": "File holding this peer's persistent id"})
    elastic_coordinator: Optional[str] = field(
        default=None,
        metadata={"help": "host:port of the elastic coordinator store (hosted by run_aux_peer.py "
                          "--host_elastic_coordinator True). When set, trainers form their communicator through "
                          "it and survive peer death / admit late joiners (SURVEY 5.3)"},
    )


@dataclass
class TrainingPeerArguments(BasePeerArguments):
    statistics_expiration: float = field(
        default=600, metadata={"help": "Statistics will be removed if not updated in this many seconds"}
    )
    backup_every_steps: Optional[int] = field(
        default=None, metadata={"help": "Update training state backup on disk once in this many global steps "
                                        "(default = do not update local state)"}
    )
    state_path: str = field(
        default="state.zip", metadata={"help": "Load this state upon init and when recovering from NaN parameters"})


@dataclass
class AuxiliaryPeerArguments(BasePeerArguments):
    """
    Arguments for run_aux_peer.py that is responsible for connecting peers to one another, tracking
    learning curves, assisting in all-reduce and uploading checkpoints to the hub
    """
    refresh_period: float = field(default=10, metadata={"help": "Period (in seconds) for fetching the keys from DHT"})
    wandb_project: Optional[str] = field(
        default=None, metadata={"help": "Name of Weights & Biases project to report the training progress to"}
    )
    save_checkpoint_step_interval: int = field(
        default=2, metadata={"help": "Frequency (in steps) of fetching and saving state from peers"}
    )
    repo_url: Optional[str] = field(
        default=None, metadata={"help": "URL of Hugging Face Hub repository to upload the model and optimizer states"}
    )
    local_path: Optional[str] = field(
        default="Repo", metadata={"help": "Path to local repository to store the model and optimizer states"}
    )
    upload_interval: Optional[float] = field(
        default=None, metadata={"help": "Frequency (in seconds) of uploading the model to Hub"}
    )
    store_checkpoints: bool = field(default=True, metadata={"help": "If True, enables CheckpointHandler"})
    host_elastic_coordinator: bool = field(
        default=False, metadata={"help": "Host the elastic coordinator store at --elastic_coordinator host:port"})
    assist_in_averaging: bool = field(
        default=False, metadata={"help": "If True, this peer will facilitate averaging for other (training) peers"})
    assist_refresh: float = field(default=1.0, metadata={"help": "Period (in seconds) for tryin to assist averaging"})
    metrics_log: Optional[str] = field(default=None, metadata={"help": "[new] JSON-lines file for the aggregated metrics"})
    max_iterations: Optional[int] = field(default=None, metadata={"help": "[new] stop after this many polls (tests)"})
