"""Per-peer metric records, their validators and a few logging helpers.

Reference counterpart: ``utils.py:1-63``. A training peer publishes one :class:`LocalMetrics` record
per optimizer epoch under ``{experiment_prefix}_metrics`` with its RSA owner marker as the subkey; the
aux peer reads them all back. Records are checked twice: by the pydantic schema (field types and
ranges) and by the owner signature (``dalle_amd.parallel.validation``).
"""
from typing import Dict, List, Sequence, Tuple

from pydantic import BaseModel, Field, StrictFloat, StrictInt

from dalle_amd.parallel.dht import choose_ip_address
from dalle_amd.parallel.validation import BytesWithPublicKey, RecordValidatorBase, RSASignatureValidator, SchemaValidator
from dalle_amd.utils.logging import get_logger

logger = get_logger(__name__)

_BOLD_BLUE, _PLAIN = "\033[1m\033[34m", "\033[0m"


class LocalMetrics(BaseModel):
    """What one peer reports for one optimizer epoch (all counters non-negative)."""

    step: StrictInt = Field(ge=0, description="local epoch the numbers belong to")
    samples_per_second: float = Field(ge=0.0, strict=True, description="EMA throughput of this peer")
    samples_accumulated: StrictInt = Field(ge=0, description="samples contributed to the epoch")
    loss: StrictFloat = Field(description="sum of the mini-step losses")
    mini_steps: StrictInt = Field(ge=0, description="number of mini-steps summed in `loss`")


class MetricSchema(BaseModel):
    metrics: Dict[BytesWithPublicKey, LocalMetrics]


def make_validators(experiment_prefix: str) -> Tuple[List[RecordValidatorBase], bytes]:
    """(validators for the DHT, this peer's owner marker). The marker is the subkey a peer must use
    for its own metrics record, so only it can sign (and therefore overwrite) that record."""
    owner = RSASignatureValidator()
    return [SchemaValidator(MetricSchema, prefix=experiment_prefix), owner], owner.local_public_key


def _peer_suffixes(maddrs: Sequence[str]) -> List[str]:
    return sorted({"/p2p/" + str(m).rsplit("/p2p/", 1)[-1] for m in maddrs})


def log_visible_maddrs(visible_maddrs: Sequence[str], only_p2p: bool) -> None:
    """Print the ``--initial_peers`` value other peers should use to join this one."""
    if only_p2p:
        to_share = _peer_suffixes(visible_maddrs)
    else:
        host = choose_ip_address(visible_maddrs)
        to_share = [str(m) for m in visible_maddrs if host in str(m)] or [str(m) for m in visible_maddrs]
    logger.info(f"Key-value store peer is up; join it with {_BOLD_BLUE}--initial_peers {' '.join(to_share)}{_PLAIN}")
    logger.info("All visible multiaddresses: " + " ".join(map(str, visible_maddrs)))


def log_process_rank(training_args) -> None:
    distributed = training_args.local_rank != -1
    logger.info(f"Process rank {training_args.local_rank} on {training_args.device} (n_gpu={training_args.n_gpu}); "
                f"distributed={distributed}, fp16={training_args.fp16}")
