"""Configuration: the reference's typed config objects, defaults and strict override semantics.

Mirrors /root/reference/src/common/utils.ts:157-234:

* ``DEFAULT_CLIENT_HYPERPARAMS``  = {examplesPerUpdate: 5, learningRate: 0.001, batchSize: 32, epochs: 5}
* ``DEFAULT_SERVER_HYPERPARAMS``  = {aggregation: 'mean', minUpdatesPerVersion: 20}
  (+ ``maximumStaleness`` — the README's bounded-staleness knob, /root/reference/README.md:27,
  which the reference never implemented; default -1 = unbounded, i.e. the reference's behaviour)
* ``DEFAULT_DATASET_HYPERPARAMS`` = {batchSize: 32, epochs: 5, smallLastBatch: False}
* ``DEFAULT_DISTRIBUTED_COMPILE_ARGS`` = {loss: 'meanSquaredError', learningRate: 0.001, metrics: ['accuracy']}

``override(defaults, choices)`` keeps the reference semantics exactly: every default key is taken
from ``choices`` unless the choice is *falsy* (so 0 / False / '' fall back to the default — a
reference quirk) and unknown keys raise.  ``strict_override`` is the fixed
variant (only ``None`` falls back).  Keys may be given in the reference's camelCase or snake_case.

Environment overrides: ``DISTRIFLOW_<SNAKE_KEY>`` (e.g. DISTRIFLOW_MIN_UPDATES_PER_VERSION=4) are
applied by :func:`env_overrides`; ``VERBOSE`` switches server logging on as in
/root/reference/src/server/federated_server.ts:45-47.
"""
from __future__ import annotations

import copy
import os
import re
from typing import Any, Optional

DEFAULT_CLIENT_HYPERPARAMS: dict = {
    "examplesPerUpdate": 5,
    "learningRate": 0.001,
    "batchSize": 32,
    "epochs": 5,
}

DEFAULT_SERVER_HYPERPARAMS: dict = {
    "aggregation": "mean",
    "minUpdatesPerVersion": 20,
    "maximumStaleness": -1,
}

DEFAULT_DATASET_HYPERPARAMS: dict = {
    "batchSize": 32,
    "epochs": 5,
    "smallLastBatch": False,
}

DEFAULT_DISTRIBUTED_COMPILE_ARGS: dict = {
    "loss": "meanSquaredError",
    "learningRate": 0.001,
    "metrics": ["accuracy"],
}

_CAMEL_RE = re.compile(r"_([a-z])")


def to_camel(key: str) -> str:
    return _CAMEL_RE.sub(lambda m: m.group(1).upper(), key)


def to_snake(key: str) -> str:
    return re.sub(r"([A-Z])", lambda m: "_" + m.group(1).lower(), key)


def _normalise(choices: Optional[dict]) -> dict:
    out = {}
    for k, v in (choices or {}).items():
        out[to_camel(k) if "_" in k else k] = v
    return out


def override(defaults: dict, choices: Optional[dict]) -> dict:
    """Reference semantics (utils.ts:206-218): falsy choices fall back to the default, unknown keys raise."""
    ch = _normalise(choices)
    result = {}
    for key, dv in defaults.items():
        v = ch.get(key)
        result[key] = v if v else copy.deepcopy(dv)
    for key in ch:
        if key not in defaults:
            raise ValueError(f'Unrecognized key "{key}"')
    return result


def strict_override(defaults: dict, choices: Optional[dict]) -> dict:
    """Like :func:`override` but only ``None`` falls back (0 / False are honoured)."""
    ch = _normalise(choices)
    result = {}
    for key, dv in defaults.items():
        v = ch.get(key)
        result[key] = copy.deepcopy(dv) if v is None else v
    for key in ch:
        if key not in defaults:
            raise ValueError(f'Unrecognized key "{key}"')
    return result


def client_hyperparams(hps: Optional[dict] = None) -> dict:
    try:
        return env_overrides(strict_override(DEFAULT_CLIENT_HYPERPARAMS, hps), "CLIENT")
    except ValueError as err:
        raise ValueError(f"Error setting clientHyperparams: {err}") from None


def server_hyperparams(hps: Optional[dict] = None) -> dict:
    try:
        return env_overrides(strict_override(DEFAULT_SERVER_HYPERPARAMS, hps), "SERVER")
    except ValueError as err:
        raise ValueError(f"Error setting serverHyperparams: {err}") from None


def dataset_config(cfg: Optional[dict] = None) -> dict:
    try:
        return strict_override(DEFAULT_DATASET_HYPERPARAMS, cfg)
    except ValueError as err:
        raise ValueError(f"Error setting dataset config: {err}") from None


def compile_args(cfg: Optional[dict] = None) -> dict:
    try:
        return strict_override(DEFAULT_DISTRIBUTED_COMPILE_ARGS, cfg)
    except ValueError as err:
        raise ValueError(f"Error setting compile args: {err}") from None


def _coerce(v: str, like: Any):
    if isinstance(like, bool):
        return v.lower() in ("1", "true", "yes", "on")
    if isinstance(like, int):
        return int(v)
    if isinstance(like, float):
        return float(v)
    if isinstance(like, list):
        return [s for s in v.split(",") if s]
    return v


def env_overrides(cfg: dict, scope: str = "") -> dict:
    """Apply DISTRIFLOW_[<SCOPE>_]<SNAKE_KEY> environment variables (scoped wins over unscoped)."""
    out = dict(cfg)
    for key, dv in cfg.items():
        sk = to_snake(key).upper()
        for name in ([f"DISTRIFLOW_{scope}_{sk}"] if scope else []) + [f"DISTRIFLOW_{sk}"]:
            if name in os.environ:
                out[key] = _coerce(os.environ[name], dv)
                break
    return out


def verbose_from_env(explicit: Optional[bool]) -> bool:
    if explicit:
        return True
    return bool(os.environ.get("VERBOSE"))
