"""Metrics schema + DHT record validators + logging helpers (reference ``utils.py:1-63``)."""
from typing import Dict, List, Tuple

from pydantic import BaseModel, StrictFloat, confloat, conint

from dalle_amd.parallel.dht import choose_ip_address
from dalle_amd.parallel.validation import BytesWithPublicKey, RecordValidatorBase, RSASignatureValidator, SchemaValidator
from dalle_amd.utils.logging import get_logger

logger = get_logger(__name__)


class LocalMetrics(BaseModel):
    step: conint(ge=0, strict=True)
    samples_per_second: confloat(ge=0.0, strict=True)
    samples_accumulated: conint(ge=0, strict=True)
    loss: StrictFloat
    mini_steps: conint(ge=0, strict=True)


class MetricSchema(BaseModel):
    metrics: Dict[BytesWithPublicKey, LocalMetrics]


def make_validators(experiment_prefix: str) -> Tuple[List[RecordValidatorBase], bytes]:
    signature_validator = RSASignatureValidator()
    validators = [SchemaValidator(MetricSchema, prefix=experiment_prefix), signature_validator]
    return validators, signature_validator.local_public_key


class TextStyle:
    BOLD = "\033[1m"
    BLUE = "\033[34m"
    RESET = "\033[0m"


def log_visible_maddrs(visible_maddrs: List[str], only_p2p: bool) -> None:
    if only_p2p:
        unique = {str(a).split("/p2p/")[-1] for a in visible_maddrs}
        initial_peers_str = " ".join(f"/p2p/{a}" for a in unique)
    else:
        preferred = choose_ip_address(visible_maddrs)
        selected = [a for a in visible_maddrs if preferred in str(a)] or list(visible_maddrs)
        initial_peers_str = " ".join(str(a) for a in selected)
    logger.info(
        f"Running a key-value store peer. To connect other peers to this one, use "
        f"{TextStyle.BOLD}{TextStyle.BLUE}--initial_peers {initial_peers_str}{TextStyle.RESET}"
    )
    logger.info(f"Full list of visible multiaddresses: {' '.join(str(a) for a in visible_maddrs)}")


def log_process_rank(training_args):
    logger.info(
        f"Process rank: {training_args.local_rank}, device: {training_args.device}, n_gpu: {training_args.n_gpu}, "
        f"distributed training: {bool(training_args.local_rank != -1)}, 16-bits training: {training_args.fp16}"
    )
