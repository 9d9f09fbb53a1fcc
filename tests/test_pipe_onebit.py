"""BASELINE config 4 rehearsal on gloo: GPT-NeoX as a PipelineModule, PP=2 x DP=2, trained with
1-bit Adam (warm-up, then error-compensated compressed momentum all-reduce over the data-parallel
group while the pipeline engine's own gradient all-reduce is switched off).

Reference analogue: tests/onebit/test_nccl_perf.py + tests/unit/test_pipe.py (pipeline with a
non-ZeRO optimizer); the reference has no combined test."""

import os

import torch

from common import run_distributed


def _body(out_dir, steps=8, freeze=3, ckpt_interval=1):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.gpt_neox import get_config, to_pipeline
    from deeperspeed_amd.runtime.pipe.topology import PipeDataParallelTopology
    torch.manual_seed(0)
    cfg = get_config("tiny", num_layers=4, max_seq_len=32)
    topo = PipeDataParallelTopology(num_pp=2, num_dp=2)
    # per-block activation checkpointing as in the bench (the embedding stage must not be
    # checkpointed: its only input is integer token ids)
    model = to_pipeline(cfg, num_stages=None, topology=topo, partition_method="uniform", seed_layers=True,
                        base_seed=11, activation_checkpoint_interval=ckpt_interval)
    conf = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2,
            "optimizer": {"type": "OneBitAdam", "params": {"lr": 2e-3, "freeze_step": freeze, "betas": [0.9, 0.9],
                                                            "comm_backend_name": "nccl"}},
            "fp16": {"enabled": True, "type": "bfloat16"}, "fp32_allreduce": False, "steps_per_print": 1000}
    engine, opt, _, _ = ds.initialize(model=model, model_parameters=[p for p in model.parameters()],
                                      config_params=conf)
    dp_rank = engine.grid.get_data_parallel_id()
    g = torch.Generator()
    g.manual_seed(5 + dp_rank)
    batch = [torch.randint(0, cfg.vocab_size, (2, 32), generator=g) for _ in range(2)]
    it = iter([(b, b) for b in batch] * steps)
    losses = [float(engine.train_batch(it)) for _ in range(steps)]
    inner = getattr(engine.optimizer, "optimizer", engine.optimizer)
    assert inner.adam_freeze_key, "compression stage never reached"
    # replicas of the same stage must hold identical weights after compressed steps
    flat = torch.cat([p.detach().float().reshape(-1) for p in engine.module.parameters()])
    peers = [None] * dist.get_world_size()
    dist.all_gather_object(peers, (engine.grid.get_pipe_parallel_rank(), flat))
    for stage, f in peers:
        if stage == engine.grid.get_pipe_parallel_rank():
            assert torch.equal(f, flat)
    if dist.get_rank() == 0:
        torch.save(losses, os.path.join(out_dir, "losses.pt"))


def test_pipeline_onebit_adam(tmp_path):
    run_distributed(_body, 4, str(tmp_path), timeout=600)
    losses = torch.load(os.path.join(tmp_path, "losses.pt"), weights_only=True)
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0], losses
