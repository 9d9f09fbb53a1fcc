"""`module_inject` at the reference's import path (deepspeed/module_inject/inject.py):
recursively swap HuggingFace-style BERT layers for DeepSpeedTransformerLayer (implementation
in module_inject/replace_module.py, which shares the weight-copy helpers with
replace_transformer_layer / revert_transformer_layer)."""

from .replace_module import module_inject  # noqa: F401
