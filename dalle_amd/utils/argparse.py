"""Dataclass -> CLI parser compatible with ``transformers.HfArgumentParser`` as the reference uses it
(``run_trainer.py:27``, ``run_aux_peer.py:86``): every field becomes ``--field value``; ``bool``
fields take ``--flag True/False`` (or bare ``--flag``); ``List[str]`` fields take space-separated
values; ``Optional[T]`` accepts the string ``None``. As with the HF parser, a run can also be configured
from a dict or a JSON / YAML file (``parse_dict`` / ``parse_json_file`` / ``parse_yaml_file``; the
entrypoints accept a single ``*.json`` / ``*.yaml`` argument), with the same type conversions and
defaults as the command line.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import sys
import typing
from typing import Any, List, Sequence, Tuple


def _str2bool(v: str) -> bool:
    if isinstance(v, bool):
        return v
    s = v.lower()
    if s in ("yes", "true", "t", "y", "1"):
        return True
    if s in ("no", "false", "f", "n", "0"):
        return False
    raise argparse.ArgumentTypeError(f"boolean value expected, got {v!r}")


def _unwrap_optional(tp):
    origin = typing.get_origin(tp)
    if origin is typing.Union:
        args = [a for a in typing.get_args(tp) if a is not type(None)]
        if len(args) == 1:
            return args[0], True
    return tp, False


def _none_or(conv):
    def f(v):
        return None if v in ("None", "none", "null") else conv(v)
    return f


class DataclassArgumentParser(argparse.ArgumentParser):
    def __init__(self, dataclass_types: Sequence[type], **kwargs):
        super().__init__(**kwargs)
        self.dataclass_types = list(dataclass_types)
        seen = set()
        for dtype in self.dataclass_types:
            hints = typing.get_type_hints(dtype)
            for f in dataclasses.fields(dtype):
                if not f.init or f.name in seen:
                    continue
                seen.add(f.name)
                self._add(f, hints.get(f.name, f.type))

    def _add(self, f: dataclasses.Field, tp: Any):
        name = "--" + f.name
        kw = {"help": f.metadata.get("help")}
        if f.default is not dataclasses.MISSING:
            kw["default"] = f.default
        elif f.default_factory is not dataclasses.MISSING:  # type: ignore[misc]
            kw["default"] = f.default_factory()  # type: ignore[misc]
        else:
            kw["required"] = True
        base, optional = _unwrap_optional(tp)
        origin = typing.get_origin(base)
        if base is bool:
            kw.update(type=_str2bool, nargs="?", const=True)
        elif origin in (list, List):
            inner = typing.get_args(base)[0] if typing.get_args(base) else str
            kw.update(type=inner if inner in (int, float, str) else str, nargs="*")
        elif base in (int, float, str):
            kw["type"] = _none_or(base) if optional else base
        else:
            kw["type"] = str
        aliases = [name]
        if "_" in f.name:
            aliases.append("--" + f.name.replace("_", "-"))
        self.add_argument(*aliases, dest=f.name, **kw)

    def parse_args_into_dataclasses(self, args: Sequence[str] = None, return_remaining_strings: bool = False) -> Tuple:
        ns, remaining = self.parse_known_args(args if args is not None else sys.argv[1:])
        if remaining and not return_remaining_strings:
            raise ValueError(f"unknown arguments: {remaining}")
        outputs = []
        for dtype in self.dataclass_types:
            names = {f.name for f in dataclasses.fields(dtype) if f.init}
            outputs.append(dtype(**{k: v for k, v in vars(ns).items() if k in names}))
        if return_remaining_strings:
            outputs.append(remaining)
        return tuple(outputs)


    def parse_dict(self, args: dict, allow_extra_keys: bool = False) -> Tuple:
        """Dataclasses from a ``{field: value}`` mapping; values may be native (JSON / YAML) or strings,
        and go through the same conversions as their command-line form."""
        known = {a.dest: a for a in self._actions}
        unknown = [k for k in args if k not in known]
        if unknown and not allow_extra_keys:
            raise ValueError(f"unknown keys: {sorted(unknown)}")
        argv: List[str] = []
        for k, v in args.items():
            if k not in known:
                continue
            flag = "--" + k
            if isinstance(v, (list, tuple)):
                argv += [flag, *[str(x) for x in v]]
            elif v is None:
                argv += [flag, "None"]
            else:
                argv += [flag, str(v)]
        return self.parse_args_into_dataclasses(argv)

    def parse_json_file(self, path: str, allow_extra_keys: bool = False) -> Tuple:
        with open(path, encoding="utf-8") as fh:
            return self.parse_dict(json.load(fh), allow_extra_keys=allow_extra_keys)

    def parse_yaml_file(self, path: str, allow_extra_keys: bool = False) -> Tuple:
        import yaml

        with open(path, encoding="utf-8") as fh:
            return self.parse_dict(yaml.safe_load(fh) or {}, allow_extra_keys=allow_extra_keys)

    def parse_cli_or_file(self, argv: Sequence[str] = None) -> Tuple:
        """``script.py config.json`` / ``config.yaml`` (one argument) or the usual ``--flag value`` list."""
        argv = list(argv if argv is not None else sys.argv[1:])
        if len(argv) == 1 and argv[0].endswith(".json"):
            return self.parse_json_file(argv[0])
        if len(argv) == 1 and argv[0].endswith((".yaml", ".yml")):
            return self.parse_yaml_file(argv[0])
        return self.parse_args_into_dataclasses(argv)


HfArgumentParser = DataclassArgumentParser
