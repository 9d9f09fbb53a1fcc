"""HIP-graph capture of the BERT encoder (ops/transformer/transformer.py make_graphed_encoder):
each DeepSpeedTransformerLayer's forward and backward replay as graphs, dropout masks come from
device RNG state advanced inside the graph.  Training through the engine must equal the eager
layers that use the same device RNG state, bit for bit, with dropout on."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _env():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29567")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")


def _train(graphs, steps=4):
    _env()
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.bert import BertForPreTraining, get_config
    from deeperspeed_amd.ops.transformer.transformer import make_graphed_encoder
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config("bert-large", num_layers=3, vocab_size=4096, max_position=128)  # dropout 0.1
    model = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16).train()
    conf = {"train_micro_batch_size_per_gpu": 8, "optimizer": {"type": "Lamb", "params": {"lr": 2e-3}},
            "fp16": {"enabled": True, "type": "bfloat16"}, "gradient_clipping": 1.0}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    g = torch.Generator(device=dev).manual_seed(1)
    B, S, npred = 8, 128, 20
    ids = torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g)
    am = torch.ones(B, S, device=dev, dtype=torch.long)
    am[:, 100:] = 0
    pos = torch.stack([torch.randperm(100, device=dev, generator=g)[:npred].sort().values for _ in range(B)])
    lab = torch.randint(0, cfg.vocab_size, (B, npred), device=dev, generator=g)
    nsp = torch.randint(0, 2, (B,), device=dev, generator=g)
    if graphs:
        ext = ((1.0 - am.to(torch.bfloat16)) * -10000.0)[:, None, None, :]
        make_graphed_encoder(engine.module.layers, torch.randn(B, S, cfg.hidden_size, device=dev,
                                                               dtype=torch.bfloat16), ext, seed=77)
        # make_graphed_callables' warmup / capture forwards advanced each layer's RNG step; start
        # the comparison from the same state as the eager run
        for layer in engine.module.layers:
            layer._rng[1] = 0
    else:  # eager reference with the same device RNG and the same persistent, in-place-accumulated grads
        # graphed layers keep their own input LayerNorm (no hand-over between graphs): so does the
        # reference, or the two would differ in the fp32 summation order of some bias gradients
        engine.module.chain_norms = False
        for i, layer in enumerate(engine.module.layers):
            layer.enable_device_rng(77 + 7919 * i)
            for p in layer.parameters():
                p.grad = torch.zeros_like(p)
                p._dsa_persistent_grad = True
    losses = []
    for _ in range(steps):
        loss = engine(ids, None, am, pos, lab, nsp)
        engine.backward(loss)
        engine.step()
        losses.append(float(loss))
    torch.cuda.synchronize()
    return losses, [p.detach().float().cpu() for p in engine.module.parameters()]


def test_graphed_encoder_equals_eager_with_device_rng():
    eager_l, eager_w = _train(False)
    graph_l, graph_w = _train(True)
    assert graph_l == eager_l, (graph_l, eager_l)
    for a, b in zip(eager_w, graph_w):
        assert torch.equal(a, b)
    assert len(set(eager_l)) == len(eager_l)  # the model trains (and masks change per step)


def test_device_rng_masks_change_per_step():
    """The layer's forward advances its device RNG step, so two forwards draw different masks."""
    from deeperspeed_amd.models.bert import get_config  # noqa: F401
    from deeperspeed_amd.ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer
    dev = torch.device("cuda", 0)
    cfg = DeepSpeedTransformerConfig(batch_size=-1, hidden_size=1024, intermediate_size=4096, heads=16,
                                     attn_dropout_ratio=0.1, hidden_dropout_ratio=0.1, num_hidden_layers=1,
                                     initializer_range=0.02, layer_norm_eps=1e-12, seed=1, pre_layer_norm=True,
                                     bf16=True)
    layer = DeepSpeedTransformerLayer(cfg).to(dev).train()
    layer.enable_device_rng(5)
    x = torch.randn(4, 128, 1024, device=dev, dtype=torch.bfloat16)
    a = layer(x)
    b = layer(x)
    assert not torch.equal(a, b)
    layer._rng[1] = 0
    c = layer(x)
    assert torch.equal(a, c)


def _train_whole_step(graph, steps=6, warmup=3):
    """BERT steps through the engine with device RNG and LAMB's device step counter:
    eager for every step, or eager for `warmup` steps, one side-stream step, then replays of one
    graph of the whole step (runtime/step_graph.capture_step)."""
    _env()
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.bert import BertForPreTraining, get_config
    from deeperspeed_amd.runtime.step_graph import capture_step, persistent_grads
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config("bert-large", num_layers=3, vocab_size=4096, max_position=128)  # dropout 0.1
    model = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16).train()
    conf = {"train_micro_batch_size_per_gpu": 8, "optimizer": {"type": "Lamb", "params": {"lr": 2e-3}},
            "fp16": {"enabled": True, "type": "bfloat16"}, "gradient_clipping": 1.0}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    model.enable_device_rng(55)
    engine.basic_optimizer.enable_device_step()
    persistent_grads(model.parameters())
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.Generator(device=dev).manual_seed(1)
    B, S, npred = 8, 128, 20
    ids = torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g)
    am = torch.ones(B, S, device=dev, dtype=torch.long)
    am[:, 100:] = 0
    pos = torch.stack([torch.randperm(100, device=dev, generator=g)[:npred].sort().values for _ in range(B)])
    lab = torch.randint(0, cfg.vocab_size, (B, npred), device=dev, generator=g)
    nsp = torch.randint(0, 2, (B,), device=dev, generator=g)

    def step():
        loss = engine(ids, None, am, pos, lab, nsp)
        engine.backward(loss)
        engine.step()
        return loss

    losses = []
    with torch.cuda.stream(side):  # both runs on the same kind of stream from the first step
        if not graph:
            for _ in range(steps):
                losses.append(float(step()))
        else:
            for _ in range(warmup):
                losses.append(float(step()))
            replay, warm = capture_step(step, stream=side)
            losses.append(float(warm))
            for _ in range(steps - warmup - 1):
                losses.append(float(replay()))
    torch.cuda.synchronize()
    return losses, [p.detach().float().cpu() for p in engine.module.parameters()]


def test_whole_step_graph_equals_eager():
    """One graph of forward + backward + clipping + LAMB, replayed, trains exactly like the eager
    steps: same losses and weights bit for bit (dropout masks and bias correction advance on
    the device inside the graph)."""
    eager_l, eager_w = _train_whole_step(False)
    graph_l, graph_w = _train_whole_step(True)
    assert graph_l == eager_l, (graph_l, eager_l)
    for a, b in zip(eager_w, graph_w):
        assert torch.equal(a, b)
    assert len(set(eager_l)) == len(eager_l)
