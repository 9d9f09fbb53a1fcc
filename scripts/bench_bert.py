"""BERT pre-training throughput (the reference's "fastest BERT training"
numbers, BERT-Large on one V100: seq 128 -> 272 samples/s, 64 TFLOPS; seq 512 -> 52 samples/s,
53 TFLOPS).

BERT-Large, pre-LN DeepSpeedTransformerLayer encoder (HIP kernels + hipBLASLt), dropout 0.1,
MLM over 15 % masked positions (20 per 128 tokens) + NSP, LAMB (FusedLamb HIP kernel) through
deeperspeed_amd.initialize, bf16.  Synthetic token ids / random-init weights.

    python scripts/bench_bert.py --seq 128 --batch 64
    python scripts/bench_bert.py --seq 512 --batch 16
"""

import argparse
import contextlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REF = {128: (272.0, 64.0), 512: (52.0, 53.0)}  # samples/s, TFLOPS on 1x V100


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-large")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--torch-profile", default="", help="write a torch.profiler op table of one step here")
    ap.add_argument("--loss-trace", action="store_true",
                    help="report every step's loss (read back once at the end) in the JSON line")
    ap.add_argument("--host-sleep-ms", type=float, default=0.0,
                    help="diagnostic: sleep this long on the host after issuing each step (a GPU-bound "
                         "step absorbs it up to its host slack; a host-bound one slows by it)")
    ap.add_argument("--hip-graphs", choices=["on", "off", "step", "step-eager"], default="off",
                    help="on: capture every encoder layer's forward / backward as HIP graphs "
                         "(ops/transformer make_graphed_encoder); step: capture the WHOLE training step "
                         "(forward, backward, batched weight gradients, clipping, LAMB) as one graph "
                         "replayed per step; both draw dropout from device RNG state; step-eager: the step "
                         "mode's setup (device RNG / step counter, persistent gradients, side stream) without "
                         "the capture, for A/B runs")
    ap.add_argument("--overlap-step", choices=["on", "off"], default="off",
                    help="run the LAMB step on a side stream overlapped with the next forward "
                         "(zero_optimization.overlap_step; identical math)")
    ap.add_argument("--pld", type=float, default=0.0,
                    help="progressive layer dropping with this theta (BASELINE.md row 20; 0 = off)")
    ap.add_argument("--pld-gamma", type=float, default=1.0,
                    help="PLD decay rate; the default reaches theta within the warmup steps, so the timed "
                         "steps measure the steady state (the reference's default 0.001 gets there after ~5k steps)")
    args = ap.parse_args()
    if args.hip_graphs.startswith("step") and args.overlap_step == "on":
        raise SystemExit("--hip-graphs step captures the plain step (the overlapped step's hooks are host-driven)")
    if args.pld and (args.hip_graphs != "off" or args.overlap_step == "on"):
        raise SystemExit("--pld runs the eager encoder (graphs / overlapped-step hooks assume every layer runs)")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.bert import BertForPreTraining, get_config

    dev = torch.device(args.device)
    ds.init_distributed(dist_backend="nccl" if dev.type == "cuda" else "gloo")
    over = {"vocab_size": 512, "max_position": args.seq} if args.model == "tiny" else {}
    cfg = get_config(args.model, **over)
    torch.manual_seed(0)
    model = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16).train()
    conf = {"train_micro_batch_size_per_gpu": args.batch, "gradient_accumulation_steps": 1,
            "optimizer": {"type": "Lamb", "params": {"lr": 1e-3, "weight_decay": 0.01}},
            "fp16": {"enabled": True, "type": "bfloat16"}, "steps_per_print": 10**9,
            # the reference's BERT configs clip at 1.0 (tests/model/BingBertSquad/*_config.json)
            "gradient_clipping": 1.0,
            "zero_optimization": {"stage": 0, "overlap_step": args.overlap_step == "on"}}
    if args.pld:
        conf["progressive_layer_drop"] = {"enabled": True, "theta": args.pld, "gamma": args.pld_gamma}
    B, S = args.batch, args.seq
    if args.hip_graphs == "on" and dev.type == "cuda":
        # captured before initialize: overlap_step registers forward pre-hooks, which
        # make_graphed_callables refuses on the modules it captures (hooks added later are fine)
        from deeperspeed_amd.ops.transformer.transformer import make_graphed_encoder
        ext = torch.zeros(B, 1, 1, S, device=dev, dtype=torch.bfloat16)  # all-ones attention mask
        make_graphed_encoder(model.layers, torch.randn(B, S, cfg.hidden_size, device=dev, dtype=torch.bfloat16), ext)
        for p in model.parameters():  # the capture's warmup iterations accumulated into the buffers
            if p.grad is not None:
                p.grad.zero_()
        torch.cuda.synchronize()
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    npred = max(1, round(0.15 * S / 8) * 8 // 1) if S != 128 else 20
    npred = 20 if S == 128 else (80 if S == 512 else npred)
    g = torch.Generator(device=dev).manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g)
    tt = (torch.arange(S, device=dev)[None] >= S // 2).long().expand(B, S).contiguous()
    am = torch.ones(B, S, device=dev, dtype=torch.long)
    pos = torch.stack([torch.randperm(S, device=dev, generator=g)[:npred].sort().values for _ in range(B)])
    lab = torch.randint(0, cfg.vocab_size, (B, npred), device=dev, generator=g)
    nsp = torch.randint(0, 2, (B,), device=dev, generator=g)

    kept = []
    trace = []

    def step():
        loss = engine(ids, tt, am, pos, lab, nsp)
        if args.loss_trace:
            trace.append(loss.detach().float())
        kept.append(len(model.pld_kept) if args.pld else cfg.num_layers)
        engine.backward(loss)
        engine.step()
        if args.host_sleep_ms > 0:
            time.sleep(args.host_sleep_ms / 1e3)
        return loss

    graph_stream = None
    if args.hip_graphs.startswith("step"):
        if dev.type != "cuda":
            raise SystemExit("--hip-graphs step needs a GPU")
        from deeperspeed_amd.runtime.step_graph import capture_step, persistent_grads
        model.enable_device_rng(1234)
        engine.basic_optimizer.enable_device_step()
        persistent_grads(model.parameters())
        # every step runs on one side stream from the first (runtime/step_graph.capture_step)
        graph_stream = torch.cuda.Stream()
        graph_stream.wait_stream(torch.cuda.current_stream())
    stream_ctx = torch.cuda.stream(graph_stream) if graph_stream is not None else contextlib.nullcontext()
    stream_ctx.__enter__()
    for _ in range(args.warmup):
        loss = step()
    if args.hip_graphs == "step":
        replay, _ = capture_step(step, stream=graph_stream)

        def step():
            loss = replay()
            if args.loss_trace:
                trace.append(loss.detach().float())
            kept.append(cfg.num_layers)
            return loss
        loss = step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
        from deeperspeed_amd.ops import native
        native.hip_ops().profile_marker(1)  # timed-region trace markers (scripts/prof_summary.py --timed)
    kept.clear()
    t0 = time.time()
    for _ in range(args.steps):
        loss = step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = (time.time() - t0) / args.steps
    if dev.type == "cuda":
        native.hip_ops().profile_marker(2)
    stream_ctx.__exit__(None, None, None)
    if args.torch_profile:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                     with_stack=True) as prof:
            step()
            torch.cuda.synchronize()
        with open(args.torch_profile, "w") as f:
            ka = prof.key_averages()
            f.write(ka.table(sort_by="self_device_time_total", row_limit=60, max_name_column_width=60) + "\n")
            f.write(prof.key_averages(group_by_input_shape=True).table(sort_by="count", row_limit=60,
                                                                        max_name_column_width=50,
                                                                        max_shapes_column_width=90))
            f.write("\n\nsmall copy / fill / memset call sites (python frames)\n")
            for e in prof.key_averages(group_by_stack_n=8):
                if any(k in e.key for k in ("copy_", "fill_", "zero_", "aten::zeros", "aten::cat", "contiguous",
                                            "aten::to", "_foreach", "aten::empty_like", "aten::add")) and e.count:
                    f.write(f"{e.key} count={e.count} device_us={e.device_time_total:.0f} "
                            f"cpu_us={e.cpu_time_total:.0f}\n")
                    for fr in e.stack:
                        f.write(f"    {fr}\n")
    sps = B / dt
    run = sum(kept[:args.steps]) / max(1, min(len(kept), args.steps))
    import dataclasses
    # FLOPs of the layers that ran (PLD skips some); linear in the layer count
    tflops = sps * dataclasses.replace(cfg, num_layers=run).flops_per_sample(S, npred) / 1e12
    ref = REF.get(S)
    print(json.dumps({"metric": f"BERT pre-training samples/s ({args.model}, seq {S})", "value": round(sps, 1),
                      "unit": "samples/s", "ms_per_step": round(dt * 1e3, 2), "batch": B, "seq": S,
                      "masked_per_seq": npred, "model_tflops": round(tflops, 1), "dtype": "bf16",
                      "optimizer": "FusedLamb", "overlap_step": args.overlap_step == "on",
                      "hip_graphs": args.hip_graphs,
                      "pld_theta": args.pld or None,
                      "mean_layers_run": round(run, 2),
                      "gradient_clipping": 1.0, "data": "synthetic", "final_loss": round(float(loss.detach()), 4),
                      **({"loss_trace": [round(x, 5) for x in torch.stack(trace).tolist()]} if trace else {}),
                      "ref_v100_samples_per_s": ref[0] if ref else None,
                      "vs_ref_v100": round(sps / ref[0], 2) if ref else None}), flush=True)


if __name__ == "__main__":
    main()
