"""Collective-order verification and replicated-bucket checksums (race/consistency debug mode,
SURVEY §5.2), on gloo."""

import os

import pytest
import torch

from common import run_distributed


def _train_debug():
    import deeperspeed_amd as ds
    from deeperspeed_amd.utils import comm
    from simple_model import SimpleModel, base_config, random_batches
    comm.set_debug(True)
    torch.manual_seed(0)
    model = SimpleModel(32)
    cfg = base_config(stage=3, mb=4, ga=2, reduce_bucket_size=500, stage3_unit_max_numel=600,
                      stage3_param_persistence_threshold=10)
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
    for x, y in random_batches(4, 4, 32, seed=3):
        loss = engine(x.to(torch.bfloat16), y)
        engine.backward(loss)
        engine.step()  # verify_collective_order runs inside every optimizer step
    assert comm.collective_log() == [] or len(comm.collective_log()) < 1000


def test_debug_mode_consistent_training():
    run_distributed(_train_debug, 2)


def _divergent():
    import torch.distributed as dist
    from deeperspeed_amd.utils import comm
    comm.set_debug(True)
    comm.reset_log()
    t = torch.ones(8)
    comm.all_reduce(t)
    if dist.get_rank() == 1:
        comm._record("rogue", torch.ones(3))  # rank 1 believes it issued an extra collective
    with pytest.raises(RuntimeError, match="diverged"):
        comm.verify_collective_order()


def test_divergent_collective_order_detected():
    run_distributed(_divergent, 2)


def _replica():
    import torch.distributed as dist
    from deeperspeed_amd.utils import comm
    comm.set_debug(True)
    t = torch.arange(10.0)
    assert comm.check_replicated(t)
    if dist.get_rank() == 1:
        t[3] += 1
    with pytest.raises(RuntimeError, match="differs"):
        comm.check_replicated(t, name="bucket")


def test_replica_checksum_detects_mismatch():
    run_distributed(_replica, 2)
