"""Per-layer HBM trace of the first training steps of a GPT-NeoX-20B-width model under ZeRO-3,
bound single-rank path vs forced sharded path (world-1 RCCL).  Diagnostic only.

    python scripts/diag_zero3_mem.py --layers 6 [--force-sharded]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--force-sharded", action="store_true")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--ckpt", type=int, default=1)
    a = ap.parse_args()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29617", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    ds.init_distributed(dist_backend="nccl")
    torch.cuda.set_device(0)
    cfg = get_config("gpt-neox-20b", num_layers=a.layers, checkpoint_activations=bool(a.ckpt))
    model = GPTNeoX(cfg, device="cuda", dtype=torch.bfloat16)
    z = {"stage": 3, "overlap_comm": True, "reduce_scatter": True, "reduce_bucket_size": int(2e8),
         "stage3_prefetch_bucket_size": int(5e8), "stage3_param_persistence_threshold": int(1e6),
         "stage3_unit_max_numel": int(2e8), "stage3_max_live_parameters": 0, "compact_master": True}
    if a.force_sharded:
        z.update(stage3_force_sharded=True, grad_accum_dtype="param")
    conf = {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": 2,
            "optimizer": {"type": "Adam", "params": {"lr": 1e-4}}, "fp16": {"enabled": True, "type": "bfloat16"},
            "fp32_allreduce": False, "gradient_clipping": 1.0, "zero_optimization": z, "steps_per_print": 10**6}
    eng, *_ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    del model
    opt = eng.optimizer
    G = 2**30
    base = torch.cuda.memory_allocated()
    print(f"states {base / G:.2f} GiB", flush=True)

    def mark(name):
        def hook(m, i, o):
            torch.cuda.synchronize()
            pool = getattr(opt, "_pool", None)
            print(f"  {name}: alloc {(torch.cuda.memory_allocated() - base) / G:6.2f} GiB reserved "
                  f"{torch.cuda.memory_reserved() / G:6.2f} pool {pool.held * 2 / G if pool else 0:5.2f} GiB "
                  f"live {getattr(opt, '_live_numel', 0) / 1e6:.0f}M", flush=True)
        return hook
    for i, l in enumerate(eng.module.layers):
        l.register_forward_hook(mark(f"layer {i} fwd"))
    x = torch.randint(0, cfg.vocab_size, (4, 2048), device="cuda")
    for st in range(a.steps):
        for mb in range(2):
            loss = eng(x, labels=x)
            mark(f"step {st} mb {mb} after fwd")(None, None, None)
            eng.backward(loss)
            mark(f"step {st} mb {mb} after bwd")(None, None, None)
            eng.step()
        print(f"step {st} peak {(torch.cuda.max_memory_allocated() - base) / G:.2f} GiB over states", flush=True)


if __name__ == "__main__":
    main()
