"""Activation-checkpointing memory modes on a world of 2 (gloo) with a model-parallel mpu
(reference deepspeed/runtime/activation_checkpointing/checkpointing.py:418-478,604-614):
`partition_activations` keeps 1/mp of each checkpointed input per rank and all-gathers it
before the recompute, `contiguous_memory_optimization` stores the shards in one pre-sized
buffer, `cpu_checkpointing` parks them in pinned host memory.  Each mode must give exactly the
gradients of the un-checkpointed model."""

import os

import pytest
import torch
import torch.nn as nn

from common import run_distributed


class _MPU:
    """Both ranks form one model-parallel group (tensor-parallel replicas of the activations)."""

    def get_model_parallel_group(self):
        import torch.distributed as dist
        return dist.group.WORLD

    def get_model_parallel_world_size(self):
        import torch.distributed as dist
        return dist.get_world_size()

    def get_model_parallel_rank(self):
        import torch.distributed as dist
        return dist.get_rank()


def _net():
    torch.manual_seed(0)
    return nn.ModuleList([nn.Sequential(nn.Linear(24, 40), nn.GELU(), nn.Dropout(0.2), nn.Linear(40, 24))
                          for _ in range(3)])


def _run(net, x, ckpt):
    from deeperspeed_amd.runtime.activation_checkpointing import checkpointing as ck
    h = x
    for blk in net:
        h = ck.checkpoint(blk, h) if ckpt else blk(h)
    return h.square().mean()


def _modes(out, mode):
    import torch.distributed as dist
    from deeperspeed_amd.runtime.activation_checkpointing import checkpointing as ck
    net = _net()
    x = torch.randn(5, 7, 24, generator=torch.Generator().manual_seed(1), requires_grad=True)
    # reference grads (dropout replayed by the checkpoint RNG capture: seed per iteration)
    torch.manual_seed(42)
    loss = _run(net, x, ckpt=False)
    loss.backward()
    ref = [p.grad.clone() for p in net.parameters()] + [x.grad.clone()]
    for p in net.parameters():
        p.grad = None
    x.grad = None
    kw = dict(partition_activations=True, contiguous_checkpointing=mode in ("contiguous",),
              checkpoint_in_cpu=mode == "cpu", num_checkpoints=3)
    ck.configure(_MPU(), **kw)
    parts = []
    orig = ck._partition

    def spy(t):
        rec = orig(t)
        parts.append((rec[0].numel(), t.numel(), rec[0].device.type, rec[0].is_pinned() if rec[0].device.type == "cpu"
                      else False))
        return rec
    ck._partition = spy
    try:
        torch.manual_seed(42)
        loss2 = _run(net, x, ckpt=True)
        loss2.backward()
    finally:
        ck._partition = orig
        ck.configure(None, partition_activations=False, contiguous_checkpointing=False, checkpoint_in_cpu=False)
        ck.reset()
    got = [p.grad for p in net.parameters()] + [x.grad]
    assert torch.allclose(loss, loss2)
    for a, b in zip(ref, got):
        assert torch.allclose(a, b, atol=1e-6), (mode, (a - b).abs().max())
    assert len(parts) == 3
    for kept, full, dev, _ in parts:
        assert kept == -(-full // dist.get_world_size())  # 1/mp of each activation
    if mode == "contiguous":
        assert len(ck._contiguous_buffers) == 1 and ck._contiguous_buffers[0]["tensor"].numel() >= 3 * parts[0][0]
    if dist.get_rank() == 0:
        torch.save({"ok": True}, os.path.join(out, f"{mode}.pt"))


@pytest.mark.parametrize("mode", ["partition", "contiguous", "cpu"])
def test_checkpoint_modes_world2(tmp_path, mode):
    run_distributed(_modes, 2, str(tmp_path), mode)
    assert (tmp_path / f"{mode}.pt").exists()
