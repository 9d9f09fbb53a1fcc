"""Pipeline p2p issue order per rank pair.

RCCL runs the send/recv of a rank pair in issue order on one communicator stream: if rank i's
k-th transfer towards rank i+1 is not the mirror (send <-> recv, same shape and dtype) of rank
i+1's k-th transfer towards rank i, the pair can deadlock on the GPU.  gloo queues the two
directions independently, so the gloo equivalence tests (test_pipe_async_p2p.py) cannot see
such a bug.  Here every transfer each rank issues is recorded (runtime/pipe/p2p.py op log) for
TrainSchedule (train_batch) and InferenceSchedule (eval_batch), blocking and async-prefetch
p2p, at 2 and 4 stages x 1..8 micro-batches, and the pairwise invariant is asserted.  A negative
control lets the prefetch planner hoist receives over sends (the classic 1F1B ordering bug):
the checker must flag it.
Reference: deepspeed/runtime/pipe/schedule.py:182-289, deepspeed/runtime/pipe/engine.py:939-1070.
"""

import os

import pytest
import torch
import torch.nn as nn

from common import run_distributed

HID = 8


def _bad_plan(flat):
    """Like PipelineEngine._plan_prefetch, but a receive may also move over send instructions."""
    from deeperspeed_amd.runtime.pipe import schedule
    compute = (schedule.ForwardPass, schedule.BackwardPass)
    movable = compute + (schedule.LoadMicroBatch, schedule.SendActivation, schedule.SendGrad)
    plan = {}
    for j, cmd in enumerate(flat):
        if not isinstance(cmd, (schedule.RecvActivation, schedule.RecvGrad)):
            continue
        k, target = j - 1, None
        while k >= 0 and isinstance(flat[k], movable):
            if isinstance(flat[k], compute):
                target = k
            k -= 1
        if target is not None:
            if isinstance(cmd, schedule.RecvGrad) and isinstance(flat[target], schedule.ForwardPass) and \
                    flat[target].kwargs["buffer_id"] == cmd.kwargs["buffer_id"]:
                continue
            plan.setdefault(target, []).append(j)
    return plan


def _body(out_dir, stages, micro_batches, bad):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from deeperspeed_amd.runtime.pipe import p2p
    from deeperspeed_amd.runtime.pipe.engine import PipelineEngine
    from deeperspeed_amd.runtime.pipe.module import LayerSpec, PipelineModule
    if bad:
        PipelineEngine._plan_prefetch = staticmethod(_bad_plan)
    results = {}
    for mb in micro_batches:
        for async_p2p in (False, True):
            os.environ["DSA_PIPE_ASYNC_P2P"] = "1" if async_p2p else "0"
            torch.manual_seed(0)
            specs = []
            for _ in range(2 * stages):
                specs += [LayerSpec(nn.Linear, HID, HID), LayerSpec(nn.ReLU)]
            model = PipelineModule(layers=specs, num_stages=stages, loss_fn=nn.CrossEntropyLoss(),
                                   partition_method="uniform")
            cfg = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": mb,
                   "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "steps_per_print": 10**6}
            engine, _, _, _ = ds.initialize(model=model, model_parameters=list(model.parameters()),
                                            config_params=cfg)
            g = torch.Generator().manual_seed(5)
            data = [(torch.randn(2, HID, generator=g), torch.randint(0, HID, (2,), generator=g)) for _ in range(mb)]
            for kind in ("train", "eval"):
                p2p.record_ops(True)
                if kind == "train":
                    engine.train_batch(iter(data))
                    engine.train_batch(iter(data))
                else:
                    engine.eval_batch(iter(data))
                log = p2p.op_log()
                p2p.record_ops(False)
                gathered = [None] * dist.get_world_size()
                dist.all_gather_object(gathered, log)
                results[(mb, async_p2p, kind)] = {r: l for r, l in enumerate(gathered)}
    if dist.get_rank() == 0:
        torch.save(results, os.path.join(out_dir, f"s{stages}_bad{int(bad)}.pt"))


def _violations(results):
    from deeperspeed_amd.runtime.pipe.p2p import check_pair_order
    out = {}
    for key, logs in results.items():
        assert any(logs.values()), key  # transfers were recorded at all
        errs = check_pair_order(logs)
        if errs:
            out[key] = errs
    return out


@pytest.mark.parametrize("stages", [2, 4])
def test_p2p_issue_order_is_pairwise_complementary(tmp_path, stages):
    run_distributed(_body, stages, str(tmp_path), stages, list(range(1, 9)), False, timeout=600)
    res = torch.load(tmp_path / f"s{stages}_bad0.pt", weights_only=False)
    assert len(res) == 8 * 2 * 2
    bad = _violations(res)
    assert not bad, bad


def test_p2p_order_checker_catches_hoisted_receive(tmp_path):
    """Negative control: receives hoisted over sends produce mirror mismatches."""
    run_distributed(_body, 2, str(tmp_path), 2, [4], True, timeout=300)
    res = torch.load(tmp_path / "s2_bad1.pt", weights_only=False)
    bad = _violations(res)
    assert any(k[1] for k in bad), bad  # the async-prefetch runs are flagged
    assert not any(not k[1] for k in bad), bad  # blocking runs never prefetch


def test_check_pair_order_unit():
    from deeperspeed_amd.runtime.pipe.p2p import check_pair_order
    a = [("send", 1, (2, 8), "torch.float32"), ("recv", 1, (2, 8), "torch.float32")]
    b = [("recv", 0, (2, 8), "torch.float32"), ("send", 0, (2, 8), "torch.float32")]
    assert check_pair_order({0: a, 1: b}) == []
    assert check_pair_order({0: a, 1: b[::-1]})  # swapped order
    assert check_pair_order({0: a, 1: [b[0], ("send", 0, (2, 4), "torch.float32")]})  # shape mismatch
    assert check_pair_order({0: a, 1: b[:1]})  # missing op
