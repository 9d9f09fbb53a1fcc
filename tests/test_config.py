"""Config parsing (reference analogue: tests/unit/test_config.py, test_ds_config.py, test_ds_arguments.py)."""

import argparse
import json

import pytest
import torch

from deeperspeed_amd.runtime.config import DeepSpeedConfig
from deeperspeed_amd.runtime.config_utils import dict_raise_error_on_duplicate_keys


@pytest.mark.parametrize("tb,mb,ga,ok", [(32, 16, 2, True), (32, 8, 2, False), (None, 16, 2, True), (32, None, 2, True),
                                          (32, 16, None, True), (None, None, 2, False), (32, None, None, True),
                                          (None, 16, None, True)])
def test_batch_triple(tb, mb, ga, ok):
    d = {}
    if tb is not None:
        d["train_batch_size"] = tb
    if mb is not None:
        d["train_micro_batch_size_per_gpu"] = mb
    if ga is not None:
        d["gradient_accumulation_steps"] = ga
    if ok:
        c = DeepSpeedConfig(None, param_dict=d)
        assert c.train_batch_size == c.train_micro_batch_size_per_gpu * c.gradient_accumulation_steps
    else:
        with pytest.raises(AssertionError):
            DeepSpeedConfig(None, param_dict=d)


def test_bf16_semantics():
    c = DeepSpeedConfig(None, param_dict={"train_batch_size": 4, "fp16": {"enabled": True, "type": "bfloat16"}})
    assert c.precision == torch.bfloat16 and c.bfloat16_enabled
    assert c.loss_scale == 1.0  # static scale 1 for bf16 (DeeperSpeed)
    assert c.allreduce_always_fp32 is True  # fp32 comm default for bf16
    c2 = DeepSpeedConfig(None, param_dict={"train_batch_size": 4, "fp16": {"enabled": True}})
    assert c2.precision == torch.half and c2.loss_scale == 0 and c2.allreduce_always_fp32 is False
    assert c2.dynamic_loss_scale_args["init_scale"] == 2 ** 32


def test_zero_config_variants():
    c = DeepSpeedConfig(None, param_dict={"train_batch_size": 4, "fp16": {"enabled": True},
                                          "zero_optimization": True})
    assert c.zero_optimization_stage == 1
    c = DeepSpeedConfig(None, param_dict={"train_batch_size": 4, "fp16": {"enabled": True},
                                          "zero_optimization": {"stage": 2, "cpu_offload": True, "allgather_size": 7}})
    assert c.zero_config.offload_optimizer["device"] == "cpu"
    assert c.zero_config.allgather_bucket_size == 7
    c = DeepSpeedConfig(None, param_dict={"train_batch_size": 4, "fp16": {"enabled": True},
                                          "zero_optimization": {"stage": 3}})
    assert c.zero_config.overlap_comm is True
    with pytest.raises(AssertionError):
        DeepSpeedConfig(None, param_dict={"train_batch_size": 4, "zero_optimization": {"stage": 2}})


def test_duplicate_keys_rejected(tmp_path):
    p = tmp_path / "cfg.json"
    p.write_text('{"train_batch_size": 2, "train_batch_size": 4}')
    with pytest.raises(ValueError):
        DeepSpeedConfig(str(p))
    with pytest.raises(ValueError):
        json.loads('{"a": 1, "a": 2}', object_pairs_hook=dict_raise_error_on_duplicate_keys)


def test_sparse_attention_and_pipeline_sections():
    c = DeepSpeedConfig(None, param_dict={"train_batch_size": 4, "sparse_attention": {"mode": "bigbird", "block": 32}})
    assert c.sparse_attention["mode"] == "bigbird" and c.sparse_attention["block"] == 32
    assert c.sparse_attention["num_random_blocks"] == 1
    assert c.pipeline == {"stages": "auto", "partition": "best", "seed_layers": False,
                          "activation_checkpoint_interval": 0}
    with pytest.raises(NotImplementedError):
        DeepSpeedConfig(None, param_dict={"train_batch_size": 4, "sparse_attention": {"mode": "nope"}})


def test_checkpoint_tag_validation_modes():
    for mode, en, fail in (("Ignore", False, False), ("Warn", True, False), ("FAIL", True, True)):
        c = DeepSpeedConfig(None, param_dict={"train_batch_size": 4, "checkpoint": {"tag_validation": mode}})
        assert c.checkpoint_tag_validation_enabled == en and c.checkpoint_tag_validation_fail == fail


def test_add_config_arguments():
    import deeperspeed_amd as ds
    parser = ds.add_config_arguments(argparse.ArgumentParser())
    args = parser.parse_args(["--deepspeed", "--deepspeed_config", "foo.json"])
    assert args.deepspeed and args.deepspeed_config == "foo.json" and not args.deepspeed_mpi


def test_elasticity_override():
    d = {"elasticity": {"enabled": True, "max_train_batch_size": 1000, "micro_batch_sizes": [2, 4, 6],
                        "ignore_non_elastic_batch_info": True}, "train_batch_size": 3}
    c = DeepSpeedConfig(None, param_dict=d)
    assert c.train_batch_size % c.train_micro_batch_size_per_gpu == 0
    assert c.train_batch_size == c.train_micro_batch_size_per_gpu * c.gradient_accumulation_steps
