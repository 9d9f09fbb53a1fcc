"""Offload section parsing at the reference's import path (deepspeed/runtime/zero/offload_config.py).

Returns the same key -> value dicts (defaults filled in) the ZeRO config builds."""

from .. import key_schema as _ks
from .config import _OFFLOAD_OPT_DEFAULTS, _OFFLOAD_PARAM_DEFAULTS


def _section(param_dict, key, defaults):
    d = dict(defaults)
    d.update((param_dict or {}).get("zero_optimization", {}).get(key, {}) or {})
    return d


def get_offload_param_config(param_dict):
    return _section(param_dict, "offload_param", _OFFLOAD_PARAM_DEFAULTS)


def get_default_offload_param_config():
    return dict(_OFFLOAD_PARAM_DEFAULTS)


def get_offload_optimizer_config(param_dict):
    d = _section(param_dict, "offload_optimizer", _OFFLOAD_OPT_DEFAULTS)
    d["pipeline"] = bool(d.get("pipeline_read") or d.get("pipeline_write"))
    return d


def get_default_offload_optimizer_config():
    return dict(_OFFLOAD_OPT_DEFAULTS)


OFFLOAD_KEYS = _ks.defaults(_ks.OFFLOAD)
