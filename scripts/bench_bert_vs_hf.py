"""BERT-Large encoder training pass, this framework's DeepSpeedTransformerLayer stack vs the
installed HuggingFace BertModel on the same GPU (the reference's transformer
kernel fine-tunes BERT "up to 1.5x" faster than the PyTorch baseline,
docs/_posts/2020-05-28-fastest-bert-training.md:27).

Same shapes, bf16, dropout 0.1, train mode, random init; one iteration = forward + backward of
sum(encoder output) (embeddings + 24 encoder layers; no optimizer, no heads).  HF runs with its
`sdpa` attention (torch's fused attention kernels) and with `eager` (materialised scores).

    python scripts/bench_bert_vs_hf.py [--shapes 384x32,128x64] [--iters 20]
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def time_it(fn, iters, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.time() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="384x32,128x64", help="seqxbatch list")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    import transformers

    from deeperspeed_amd.models.bert import BertForPreTraining, get_config
    dev = torch.device("cuda")
    for spec in args.shapes.split(","):
        S, B = (int(x) for x in spec.split("x"))
        g = torch.Generator(device=dev).manual_seed(0)
        ids = torch.randint(0, 30528, (B, S), device=dev, generator=g)
        tt = torch.zeros(B, S, dtype=torch.long, device=dev)
        am = torch.ones(B, S, dtype=torch.long, device=dev)
        res = {"seq": S, "batch": B}
        torch.manual_seed(0)
        ours = BertForPreTraining(get_config("bert-large", max_position=max(512, S)), device=dev,
                                  dtype=torch.bfloat16).train()

        def step_ours():
            ours.encode(ids, tt, am).float().sum().backward()

        res["dsa_ms"] = round(time_it(step_ours, args.iters, args.warmup), 2)
        del ours
        torch.cuda.empty_cache()
        for impl in ("sdpa", "eager"):
            cfg = transformers.BertConfig(vocab_size=30528, hidden_size=1024, num_hidden_layers=24,
                                          num_attention_heads=16, intermediate_size=4096,
                                          max_position_embeddings=max(512, S), attn_implementation=impl)
            hf = transformers.BertModel(cfg, add_pooling_layer=False).to(dev, torch.bfloat16).train()

            def step_hf():
                hf(input_ids=ids, token_type_ids=tt, attention_mask=am).last_hidden_state.float().sum().backward()

            res[f"hf_{impl}_ms"] = round(time_it(step_hf, args.iters, args.warmup), 2)
            res[f"speedup_vs_hf_{impl}"] = round(res[f"hf_{impl}_ms"] / res["dsa_ms"], 2)
            del hf
            torch.cuda.empty_cache()
        res["transformers"] = transformers.__version__
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
