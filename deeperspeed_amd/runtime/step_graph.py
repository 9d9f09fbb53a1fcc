"""Whole-training-step HIP graph capture.

`capture_step(step)` records one call of a user step function (engine forward, backward,
optimizer step) as ONE HIP graph and returns a function that replays it.  On a kernel-bound step
with hundreds of short kernels (BERT-Large: ~775 launches per step) the host launch path and the
per-launch gaps go away; only the graph launch remains.

Requirements, all met by the BERT path (`scripts/bench_bert.py --hip-graphs step`):
  * static inputs: the tensors the step reads keep their storage (copy new batches into them);
  * no host synchronisation inside the step (the sync-free FP16_UnfusedOptimizer step: gradient
    norm, clip factor and overflow skip stay on the device);
  * step-dependent scalars on the device: dropout seeds (`enable_device_rng`) and LAMB's bias
    correction (`FusedLamb.enable_device_step`), or every replay would reuse the captured values.

The reference has no graph capture (CUDA graphs postdate DeepSpeed v0.3.15); its BERT step is
the per-kernel launch sequence of csrc/transformer/ds_transformer_cuda.cpp.
"""

import torch


def persistent_grads(params):
    """Give every trainable parameter a .grad buffer that lives across steps (zeroed in place by
    the fp16 optimizer's zero_grad, accumulated into in place by backward), so the gradient
    addresses a captured graph and the optimizers' multi-tensor tables hold never change.
    The engine already binds the large weights and the 1-D parameters into layer stacks
    (ops/wgrad_batch.bind_grad_stacks); this covers the rest (embeddings, heads)."""
    n = 0
    for p in params:
        if not p.requires_grad or getattr(p, "_dsa_persistent_grad", False):
            continue
        if p.grad is None:
            p.grad = torch.zeros_like(p)
        p._dsa_persistent_grad = True
        n += 1
    return n


def capture_step(step, stream=None, warmup: int = 1):
    """Run `warmup` eager calls of `step` on a side stream (torch.cuda.graph's whole-network
    recipe: lazily created workspaces and optimizer state exist before capture), then capture one
    call.  Returns (replay, warm_out): replay() launches the graph and returns the captured
    step's output (the same tensor, refreshed by every replay); warm_out is the last eager
    output.  The captured call itself does not execute.

    stream: the non-default stream every earlier step ran on.  Autograd binds each leaf's
    gradient accumulation to the stream of its first backward; one bound to the legacy default
    stream makes the capture wait on that stream, which invalidates it.  So a captured training
    loop runs on a side stream from its first step (the bench and tests do)."""
    side = stream if stream is not None else torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    warm_out = None
    with torch.cuda.stream(side):
        for _ in range(warmup):
            warm_out = step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    from ..ops import wgrad_batch
    graph = torch.cuda.CUDAGraph()
    wgrad_batch.state.whole_step_capture = True  # layer slabs + batched weight gradients stay on
    try:
        with torch.cuda.graph(graph, stream=side):
            static_out = step()
    finally:
        wgrad_batch.state.whole_step_capture = False

    def replay():
        graph.replay()
        return static_out

    replay.graph = graph
    return replay, warm_out
