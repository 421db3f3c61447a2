"""Argument schema: the reference's dataclasses through the HF-compatible parser from the
command line, a dict, a JSON file and a YAML file give the same configuration."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from arguments import CollaborativeArguments, HFTrainerArguments, TrainingPeerArguments  # noqa: E402
from dalle_amd.utils.argparse import HfArgumentParser  # noqa: E402


def _parser():
    return HfArgumentParser((TrainingPeerArguments, HFTrainerArguments, CollaborativeArguments))


def test_cli_dict_json_yaml_agree(tmp_path):
    cfg = {"experiment_prefix": "demo", "per_device_train_batch_size": 48, "learning_rate": 0.002,
           "target_batch_size": 1024, "authorize": False, "initial_peers": ["/ip4/127.0.0.1/tcp/1", "/ip4/127.0.0.1/tcp/2"]}
    cli = ["--experiment_prefix", "demo", "--per_device_train_batch_size", "48", "--learning_rate", "0.002",
           "--target_batch_size", "1024", "--authorize", "False", "--initial_peers", "/ip4/127.0.0.1/tcp/1",
           "/ip4/127.0.0.1/tcp/2"]
    a = _parser().parse_args_into_dataclasses(cli)
    b = _parser().parse_dict(cfg)
    (tmp_path / "c.json").write_text(json.dumps(cfg))
    c = _parser().parse_cli_or_file([str(tmp_path / "c.json")])
    import yaml

    (tmp_path / "c.yaml").write_text(yaml.safe_dump(cfg))
    d = _parser().parse_cli_or_file([str(tmp_path / "c.yaml")])
    assert a == b == c == d
    peer, trainer, collab = a
    assert trainer.per_device_train_batch_size == 48 and collab.target_batch_size == 1024
    assert peer.authorize is False and len(peer.initial_peers) == 2


def test_unknown_keys_rejected():
    with pytest.raises(ValueError):
        _parser().parse_dict({"no_such_flag": 1})
    assert _parser().parse_dict({"no_such_flag": 1}, allow_extra_keys=True)
