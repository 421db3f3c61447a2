"""TrainingTask: model + tokenizer + key-value store + collaborative optimizer + dataset (reference ``task.py:45-181``).

The model recipe (64 layers, axial row/col + final conv-like attention, 5 shared attention and 5
shared FF blocks, rotary, reversible, tied embeddings) comes from ``dalle_amd.config`` presets
(``--model_preset reference`` by default). Peers are the ranks of a torch.distributed group (one
process per MI355X, RCCL over xGMI; gloo for CPU peers) launched with torchrun; the key-value store
replaces the public DHT for metrics / progress records.
"""
import os
import socket
from datetime import timedelta
from pathlib import Path

import torch
import torch.distributed as dist
import torch.nn as nn

import utils
from arguments import BasePeerArguments, CollaborativeArguments, HFTrainerArguments
from dalle_amd.config import get_config
from dalle_amd.data.synthetic import PadCollator
from dalle_amd.data.tokenizer import load_tokenizer
from dalle_amd.models.dalle import DALLE
from dalle_amd.optim import FlatArena, LAMB8bit, get_linear_schedule_with_warmup
from dalle_amd.parallel.compression import Float16Compression, NoCompression, SizeAdaptiveCompression, Uniform8BitQuantization
from dalle_amd.parallel.dht import DHT
from dalle_amd.parallel.optimizer import CollaborativeOptimizer
from dalle_amd.utils.logging import get_logger
from data import make_dataset
from huggingface_auth import authorize_with_huggingface

logger = get_logger(__name__)


class VQGanParams(nn.Module):
    """Parameter-only VQGAN stub: lets DALL-E size itself without loading a checkpoint (task.py:25-32)."""

    def __init__(self, *, num_layers=3, image_size=256, num_tokens=8192, is_gumbel=True):
        super().__init__()
        self.num_layers = num_layers
        self.image_size = image_size
        self.num_tokens = num_tokens
        self.is_gumbel = is_gumbel


class ModelWrapper(nn.Module):
    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, input_ids, attention_mask, image):
        loss = self.model.forward(text=input_ids, image=image, mask=attention_mask, return_loss=True)
        return {'loss': loss}


def make_averaging_compression(kind: str):
    if kind == "none" or kind == "powersgd":
        return NoCompression()
    if kind == "fp16":
        return Float16Compression()
    if kind == "8bit":
        return Uniform8BitQuantization()
    return SizeAdaptiveCompression(threshold=2 ** 16 + 1, less=Float16Compression(), greater_equal=Uniform8BitQuantization())


class TrainingTask:
    """Everything one collaborative peer trains with, built lazily: the DALL-E recipe, tokenizer, key/value
    store, process group, collaborative optimizer (fused 8-bit LAMB + schedule), dataset and collator."""
    _authorizer = _dht = _collaborative_optimizer = _training_dataset = _process_group = _arena = _elastic = None

    def __init__(self, peer_args: BasePeerArguments, trainer_args: HFTrainerArguments, collab_args: CollaborativeArguments):
        self.peer_args, self.trainer_args, self.collab_args = peer_args, trainer_args, collab_args
        if self.authorizer is not None:  # the reference dereferenced it unconditionally (task.py:53)
            self.trainer_args.run_name = self.authorizer.username

        self.validators, self.local_public_key = utils.make_validators(self.peer_args.experiment_prefix)
        torch.manual_seed(trainer_args.seed)  # seed used for initialization

        cfg = get_config(trainer_args.model_preset)
        self.tokenizer = load_tokenizer(peer_args.tokenizer_path, vocab_size=cfg.num_text_tokens)
        self.tokenizer.pad_token = self.tokenizer.eos_token
        if cfg.text_seq_len != trainer_args.text_seq_length:
            cfg = type(cfg)(**{**cfg.to_dict(), "text_seq_len": trainer_args.text_seq_length})
        rr = str(trainer_args.reversible_recompute).lower()
        cfg.reversible_recompute = "auto" if rr == "auto" else rr not in ("false", "0", "no")
        self.config = cfg

        logger.info(f"Creating model ({trainer_args.model_preset}: depth {cfg.depth}, dim {cfg.dim})")
        vae = VQGanParams(num_layers=cfg.vae_num_layers, image_size=cfg.image_size, num_tokens=cfg.num_image_tokens)
        dalle = DALLE(cfg, vae=None)
        dalle.vae_params = vae
        n_trainable = sum(p.numel() for p in dalle.parameters() if p.requires_grad)
        logger.info(f"{n_trainable / 1e6:.1f}M trainable parameters ({n_trainable})")
        self.model = ModelWrapper(dalle)

        output_dir = Path(trainer_args.output_dir)
        # resume: the newest checkpoint* directory (by creation time) that holds a model_state.pt
        candidates = sorted(output_dir.glob("checkpoint*"), key=os.path.getctime)
        newest = candidates[-1] if candidates else None
        if newest is not None and (newest / "model_state.pt").exists():
            logger.info(f"resuming model weights from {newest / 'model_state.pt'}")
            state = torch.load(newest / "model_state.pt", map_location="cpu", weights_only=True)
            self.model.load_state_dict(state)

    @property
    def authorizer(self):
        if self._authorizer is None and self.peer_args.authorize:
            self._authorizer = authorize_with_huggingface()
        return self._authorizer

    @property
    def process_group(self):
        """torch.distributed default group (torchrun launch, or an elastic generation formed through the
        coordinator store), or None for a single peer."""
        coord = getattr(self.peer_args, "elastic_coordinator", None)
        if coord and self._elastic is None:
            from dalle_amd.parallel.elastic import ElasticGroup, coordinator_store
            host, port = coord.rsplit(":", 1)
            backend = self.trainer_args.backend or ("nccl" if torch.cuda.is_available() else "gloo")
            if backend == "nccl":
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
            store = coordinator_store(host, int(port), is_master=False, timeout=self.collab_args.averaging_timeout)
            peer_id = f"{socket.gethostname()}-{os.getpid()}"
            self._elastic = ElasticGroup(store, peer_id, backend=backend, matchmaking_time=self.collab_args.matchmaking_time,
                                         allreduce_timeout=self.collab_args.allreduce_timeout,
                                         device=torch.device("cuda") if backend == "nccl" else torch.device("cpu"))
            self._elastic.join()
        if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not dist.is_initialized():
            backend = self.trainer_args.backend or ("nccl" if torch.cuda.is_available() else "gloo")
            if backend == "nccl":
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
            timeout = timedelta(seconds=self.collab_args.averaging_timeout)
            attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
            if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True" and attempt not in ("", "0"):
                # torchrun --max-restarts with a static rendezvous: the agent's store still holds the previous
                # attempt's process-group keys (a dead rank's address), so a restarted rank could read a stale
                # one before its peer overwrites it -- rendezvous under a per-attempt prefix instead
                base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), is_master=False,
                                     timeout=timeout)
                dist.init_process_group(backend, store=dist.PrefixStore(f"dalle_pg/attempt{attempt}", base),
                                        rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]), timeout=timeout)
            else:
                dist.init_process_group(backend, timeout=timeout)
        return dist.group.WORLD if dist.is_initialized() else None

    @property
    def dht(self):
        if self._dht is None:
            initial_peers = list(self.peer_args.initial_peers)
            host_maddrs = list(self.peer_args.host_maddrs)
            rank = int(os.environ.get("RANK", "0"))
            if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not initial_peers:
                # torchrun job without an external store: rank 0 starts one that lives as long as the torchrun
                # agent, so the metrics outlive a dead rank 0 (dalle_amd/parallel/dht_host.py)
                from dalle_amd.parallel.dht_host import torchrun_endpoints

                initial_peers, hm = torchrun_endpoints(rank)
                host_maddrs = hm or host_maddrs
            self._dht = DHT(
                start=True,
                initial_peers=initial_peers,
                client_mode=self.peer_args.client_mode,
                host_maddrs=host_maddrs,
                announce_maddrs=self.peer_args.announce_maddrs,
                use_ipfs=self.peer_args.use_ipfs,
                record_validators=self.validators,
                identity_path=self.peer_args.identity_path,
                authorizer=self.authorizer,
            )
            if self._dht is not None:
                if self.peer_args.client_mode:
                    logger.info(f"client-mode peer {self._dht.peer_id} (no inbound connections)")
                else:
                    utils.log_visible_maddrs(self._dht.get_visible_maddrs(), only_p2p=self.peer_args.use_ipfs)
        return self._dht

    @property
    def collaborative_optimizer(self):
        if self._collaborative_optimizer is None:
            group = self.process_group
            params, opt, scheduler = self._get_local_optimizer_and_scheduler(self.trainer_args)
            ta = self.trainer_args
            averaging_compression = make_averaging_compression(ta.grad_averaging)
            self._collaborative_optimizer = CollaborativeOptimizer(
                dht=self.dht, run_id=self.peer_args.experiment_prefix,
                params=params, optimizer=opt, scheduler=scheduler,
                offload_optimizer=True, delay_grad_averaging=False, delay_optimizer_step=True,
                batch_size_per_step=ta.batch_size_per_step,
                grad_compression=averaging_compression, state_averaging_compression=averaging_compression,
                client_mode=self.peer_args.client_mode, verbose=True, process_group=group, arena=self._arena,
                powersgd_rank=ta.powersgd_rank if ta.grad_averaging == "powersgd" else None, elastic=self._elastic,
                offload_device="cpu" if getattr(ta, "offload_optimizer_to_host", False) else None,
                **{k: v for k, v in vars(self.collab_args).items()})
        return self._collaborative_optimizer

    def _get_local_optimizer_and_scheduler(self, training_args: HFTrainerArguments):
        device = next(self.model.parameters()).device
        self._arena = FlatArena(self.model.parameters(), device=device)
        self.model.model.grad_arena = self._arena
        no_decay = ["bias", "LayerNorm.weight"]
        params = [
            {"params": [p for n, p in self.model.named_parameters() if not any(nd in n for nd in no_decay) and p.requires_grad],
             "weight_decay": training_args.weight_decay},
            {"params": [p for n, p in self.model.named_parameters() if any(nd in n for nd in no_decay) and p.requires_grad],
             "weight_decay": 0.0},
        ]

        def opt(params):
            return LAMB8bit(params, lr=training_args.learning_rate, betas=(training_args.adam_beta1, training_args.adam_beta2),
                            eps=training_args.adam_epsilon, weight_decay=training_args.weight_decay,
                            max_grad_norm=training_args.max_grad_norm, clamp_value=training_args.clamp_value,
                            reuse_grad_buffers=True, optim_bits=training_args.optimizer_bits)

        def scheduler(opt):
            return get_linear_schedule_with_warmup(opt, num_warmup_steps=training_args.warmup_steps,
                                                   num_training_steps=training_args.total_steps)

        return params, opt, scheduler

    @property
    def training_dataset(self):
        if self._training_dataset is None:
            seed = int.from_bytes(__import__("hashlib").sha256(self.local_public_key).digest()[:4], "little")
            self._training_dataset = make_dataset(
                self.tokenizer, shuffle_seed=seed, max_sequence_length=self.trainer_args.text_seq_length,
                dataset_path=self.trainer_args.dataset_path, image_seq_len=self.config.image_seq_len,
                num_image_tokens=self.config.num_image_tokens)
        return self._training_dataset

    @property
    def data_collator(self):
        return PadCollator(max_length=self.trainer_args.text_seq_length, pad_id=self.tokenizer.pad_token_id)
