"""Longest trainable sequence at batch 1, dense vs block-sparse attention (the
reference reports 10x (BERT-base) and 16x (BERT-large) longer sequences with sparse attention on
one 32 GB V100, docs/_posts/2020-09-09-sparse-attention.md:27).

Model: HuggingFace BertModel of the preset's shape (random init, bf16, dropout 0.1, train mode),
one forward + backward of sum(last_hidden_state) per attempt.  Variants:
  dense   HF eager attention (materialised [S, S] scores per head: the reference's dense baseline)
  sparse  the same model after SparseAttentionUtils.replace_model_self_attention_with_sparse_self_attention
          (BigBird layout: 3 sliding-window, 1 random, 1 global block of 64; one layout shared
          by the layers; fused block-sparse flash kernels)
  flash   this framework's BertForPreTraining encoder (DeepSpeedTransformerLayer, fused dense flash
          attention: O(S) memory, so dense attention is no longer the limit)

Each variant runs in its own process (a clean allocator) and tries growing sequence lengths until
the first out-of-memory; one JSON line per attempt and a summary line.

    python scripts/bench_sparse_maxseq.py [--model bert-large] [--variants dense,sparse,flash]
"""

import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PRESETS = {"bert-large": dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096),
           "bert-base": dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072)}
SEQS = {"dense": [2048, 4096, 6144, 8192, 10240, 12288, 16384, 20480, 24576, 32768],
        "sparse": [8192, 16384, 32768, 65536, 98304, 131072, 163840, 196608, 229376, 262144, 327680, 393216],
        # dense flash attention is O(S^2) work: stop at 320k (a pass there takes ~70 s)
        "flash": [8192, 16384, 32768, 65536, 131072, 196608, 262144, 327680]}


def attempt(variant, model_name, S, block):
    import torch
    dev = torch.device("cuda")
    torch.manual_seed(0)
    shape = PRESETS[model_name]
    if variant == "flash":
        from deeperspeed_amd.models.bert import BertForPreTraining, get_config
        m = BertForPreTraining(get_config(model_name, max_position=S), device=dev, dtype=torch.bfloat16).train()
        run = lambda ids: m.encode(ids)  # noqa: E731
    else:
        import transformers
        cfg = transformers.BertConfig(vocab_size=30528, max_position_embeddings=S, attn_implementation="eager",
                                      **shape)
        m = transformers.BertModel(cfg, add_pooling_layer=False).to(dev, torch.bfloat16).train()
        if variant == "sparse":
            from deeperspeed_amd.ops.sparse_attention import (BigBirdSparsityConfig, SparseAttentionUtils,
                                                              SparseSelfAttention)
            holder = type("Holder", (), {})()
            holder.bert, holder.config = m, cfg
            sc = BigBirdSparsityConfig(num_heads=shape["num_attention_heads"], block=block, num_random_blocks=1,
                                       num_sliding_window_blocks=3, num_global_blocks=1, attention="bidirectional")
            # the utils swap HF's self-attention modules (their layouts sized for 2048 positions),
            # then one SparseSelfAttention sized for S serves every layer: one [H, S/64, S/64] layout
            # and one LUT instead of 24 (host memory / build time at S ~ 300k)
            SparseAttentionUtils.replace_model_self_attention_with_sparse_self_attention(holder, 2048, sc)
            shared = SparseSelfAttention(sc, max_seq_length=S)
            for lyr in m.encoder.layer:
                lyr.attention.self.sparse_self_attention = shared
        run = lambda ids: m(ids).last_hidden_state  # noqa: E731
    ids = torch.randint(0, 30528, (1, S), device=dev)
    torch.cuda.reset_peak_memory_stats()
    torch.cuda.synchronize()
    t0 = time.time()
    run(ids).float().sum().backward()
    torch.cuda.synchronize()
    return time.time() - t0, torch.cuda.max_memory_allocated() / 2**30


def child(variant, model_name, block):
    import torch
    best = 0
    for S in SEQS[variant]:
        try:
            dt, peak = attempt(variant, model_name, S, block)
            best = S
            rec = {"variant": variant, "model": model_name, "seq": S, "ok": True, "s": round(dt, 2),
                   "peak_gib": round(peak, 1)}
        except torch.OutOfMemoryError:
            rec = {"variant": variant, "model": model_name, "seq": S, "ok": False}
        print(json.dumps(rec), flush=True)
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        if not rec["ok"]:
            break
    print(json.dumps({"variant": variant, "max_seq": best}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-large", choices=sorted(PRESETS))
    ap.add_argument("--variants", default="dense,sparse,flash")
    ap.add_argument("--block", type=int, default=64)
    ap.add_argument("--child", default="")
    args = ap.parse_args()
    if args.child:
        child(args.child, args.model, args.block)
        return
    best = {}
    for v in args.variants.split(","):
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--model", args.model, "--block",
                              str(args.block), "--child", v], stdout=subprocess.PIPE, text=True)
        for line in p.stdout:  # streamed: one line per attempt
            print(line.rstrip(), flush=True)
            if line.startswith("{"):
                rec = json.loads(line)
                if "max_seq" in rec:
                    best[v] = rec["max_seq"]
        if p.wait():
            print(json.dumps({"variant": v, "returncode": p.returncode}), flush=True)
    out = {"metric": f"longest batch-1 training sequence ({args.model})", "max_seq": best, "block": args.block,
           "sparse_layout": "BigBird(window 3, random 1, global 1 blocks, bidirectional)"}
    if best.get("dense"):
        out["sparse_vs_dense"] = round(best.get("sparse", 0) / best["dense"], 1)
        out["flash_vs_dense"] = round(best.get("flash", 0) / best["dense"], 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
