"""bench.py --emulate-world N (utils/comm.py emulated world): one process that runs rank 0 of an
N-rank ZeRO-3 job must build the same shards / units / buckets and issue the SAME collective
sequence (tag, element count, dtype) as rank 0 of a real world-N gloo job of the same model and
config -- only then is its memory peak and kernel trace the real rank's, which is what the
emulation is for (projecting the 8-GPU plan from one GPU)."""

import os

import pytest
import torch

from common import run_distributed

CONF = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2,
        "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "fp16": {"enabled": True, "type": "bfloat16"},
        "gradient_clipping": 1.0,
        "zero_optimization": {"stage": 3, "stage3_unit_max_numel": 20000, "stage3_param_persistence_threshold": 100,
                              "reduce_bucket_size": 4096, "stage3_max_live_parameters": 0,
                              "stage3_max_reuse_distance": 0}}


def _run(out_path, emulate, resident=False):
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    from deeperspeed_amd.utils import comm
    import copy
    conf = copy.deepcopy(CONF)
    if resident:
        conf["zero_optimization"].update(resident_grads=True, stage3_max_live_parameters=10**9,
                                         stage3_max_reuse_distance=10**9)
    comm.set_emulated_world(emulate)
    try:
        torch.manual_seed(0)
        model = GPTNeoX(get_config("tiny", num_layers=2), dtype=torch.bfloat16)
        engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
        ids = torch.randint(0, 256, (2, 32), generator=torch.Generator().manual_seed(3))
        comm.start_trace()
        comm.reset_bytes()
        for _ in range(2):  # two optimizer steps of two micro-batches
            for _ in range(2):
                loss = engine(ids, labels=ids)
                engine.backward(loss)
                engine.step()
        trace = comm.stop_trace()
        nbytes = comm.bytes_by_kind()
    finally:
        comm.set_emulated_world(0)
    import torch.distributed as dist
    if dist.get_rank() == 0:
        torch.save({"trace": trace, "bytes": nbytes,
                    "shard": sum(g.shard_param.numel() for g in engine.optimizer.groups)}, out_path)


@pytest.mark.parametrize("world,resident", [(2, False), (4, False), (4, True)])
def test_emulated_rank_issues_the_real_collective_sequence(tmp_path, world, resident):
    real, emu = str(tmp_path / "real.pt"), str(tmp_path / "emu.pt")
    run_distributed(_run, world, real, 0, resident)
    run_distributed(_run, 1, emu, world, resident)
    a, b = torch.load(real), torch.load(emu)
    assert len(a["trace"]) > 10
    # the norm / overflow all-reduces are collectives too: the whole sequence must match
    assert a["trace"] == b["trace"]
    assert a["bytes"] == b["bytes"]
    assert a["shard"] == b["shard"]


def test_emulated_standins_write_the_collective_bytes():
    from deeperspeed_amd.utils import comm
    comm.set_emulated_world(4)
    try:
        chunk = torch.arange(6, dtype=torch.float32)
        full = torch.empty(24)
        comm.all_gather_into_tensor(full, chunk, async_op=True).wait()
        assert torch.equal(full.view(4, 6), chunk.expand(4, 6))
        src = torch.arange(24, dtype=torch.float32)
        out = torch.empty(6)
        comm.reduce_scatter_tensor(out, src)
        assert torch.equal(out, src.view(4, 6).sum(0))
        assert comm.world_size() == 4 and comm.rank() == 0
    finally:
        comm.set_emulated_world(0)
    assert comm.world_size() == 1


def test_bench_emulate_world_cpu():
    """The bench mode itself (CPU plumbing): one process, an emulated-world record with the comm
    table and a projection that is labelled as one."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--model", "tiny", "--seq", "64",
                        "--steps", "2", "--warmup", "1", "--emulate-world", "4"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["emulated_world"] == 4 and out["n_gpus"] == 1
    assert out["metric"].startswith("EMULATED per-rank")
    assert "PROJECTION" in out["projection"]["label"]
    c = out["comm_per_rank_per_step"]
    assert c["assumed_xgmi_gbps_per_rank"] > 0 and "xgmi_gbps_needed_for_full_overlap" in c
