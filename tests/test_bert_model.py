"""BERT pre-training model on DeepSpeedTransformerLayer (models/bert.py): trains through the
engine with FusedLamb (loss decreases on a fixed batch), MLM head restricted to the masked
positions matches the full-sequence head gathered at those positions."""

import torch

from common import run_distributed


def test_mlm_head_on_masked_positions_matches_full():
    from deeperspeed_amd.models.bert import BertForPreTraining, get_config
    torch.manual_seed(0)
    cfg = get_config("tiny", hidden_dropout=0.0, attn_dropout=0.0)
    m = BertForPreTraining(cfg).eval()
    ids = torch.randint(0, cfg.vocab_size, (2, 16))
    pos = torch.tensor([[1, 5, 7], [0, 2, 15]])
    full = m(ids)  # [B*S, V] logits over every position
    part = m(ids, masked_positions=pos)
    idx = (pos + 16 * torch.arange(2)[:, None]).reshape(-1)
    torch.testing.assert_close(part, full[idx])


def _train(out_dir):
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.bert import BertForPreTraining, get_config
    torch.manual_seed(0)
    cfg = get_config("tiny", hidden_dropout=0.0, attn_dropout=0.0)
    model = BertForPreTraining(cfg)
    conf = {"train_micro_batch_size_per_gpu": 4, "optimizer": {"type": "Lamb", "params": {"lr": 5e-2}}}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (4, 32), generator=g)
    pos = torch.stack([torch.randperm(32, generator=g)[:5].sort().values for _ in range(4)])
    lab = torch.randint(0, cfg.vocab_size, (4, 5), generator=g)
    nsp = torch.randint(0, 2, (4,), generator=g)
    dev = engine.device
    ids, pos, lab, nsp = ids.to(dev), pos.to(dev), lab.to(dev), nsp.to(dev)
    losses = []
    for _ in range(8):
        loss = engine(ids, None, torch.ones(4, 32, dtype=torch.long, device=dev), pos, lab, nsp)
        engine.backward(loss)
        engine.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0] - 0.5 and all(b < a for a, b in zip(losses, losses[1:])), losses


def test_bert_pretraining_trains_with_lamb(tmp_path):
    run_distributed(_train, 1, str(tmp_path))


def _train_pld(out_dir, stage=0):
    import torch.distributed as dist

    import deeperspeed_amd as ds
    from deeperspeed_amd.models.bert import BertForPreTraining, get_config
    torch.manual_seed(0)
    cfg = get_config("tiny", num_layers=6, hidden_dropout=0.0, attn_dropout=0.0)
    model = BertForPreTraining(cfg, dtype=torch.bfloat16 if stage else None)
    conf = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "Lamb", "params": {"lr": 1e-2}},
            "progressive_layer_drop": {"enabled": True, "theta": 0.5, "gamma": 0.5}}
    if stage:  # skipped layers' parameters get no gradient in some micro-batches
        conf.update(gradient_accumulation_steps=2, optimizer={"type": "Adam", "params": {"lr": 1e-3}},
                    fp16={"enabled": True, "type": "bfloat16"}, zero_optimization={"stage": stage})
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    rank = dist.get_rank()
    g = torch.Generator().manual_seed(1 + rank)  # different data per rank, same layer draws
    kept, thetas = [], []
    for _ in range(12):
        ids = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
        pos = torch.stack([torch.randperm(32, generator=g)[:5].sort().values for _ in range(2)])
        lab = torch.randint(0, cfg.vocab_size, (2, 5), generator=g)
        nsp = torch.randint(0, 2, (2,), generator=g)
        thetas.append(engine.progressive_layer_drop.get_theta())
        loss = engine(ids, None, torch.ones(2, 32, dtype=torch.long), pos, lab, nsp)
        kept.append(list(model.pld_kept))
        engine.backward(loss)
        engine.step()
        assert torch.isfinite(loss)
    assert thetas[0] == 1.0 and thetas[-1] < (0.51 if not stage else 0.8), thetas
    assert kept[0] == list(range(6))  # theta 1: every layer runs
    assert any(len(k) < 6 for k in kept), kept
    everyone = [None] * dist.get_world_size()
    dist.all_gather_object(everyone, kept)
    assert all(k == everyone[0] for k in everyone)  # every rank skipped the same layers
    for p in model.parameters():  # and the replicas stayed identical
        ps = [torch.empty_like(p.data) for _ in range(dist.get_world_size())]
        dist.all_gather(ps, p.data.contiguous())
        assert all(torch.equal(ps[0], q) for q in ps)
    model.eval()
    model(ids, progressive_layer_drop=True, pld_theta=0.0)  # eval: PLD never applies
    assert model.pld_kept == kept[-1]


def test_progressive_layer_drop_skips_same_layers_on_every_rank(tmp_path):
    run_distributed(_train_pld, 2, str(tmp_path))


def test_progressive_layer_drop_with_zero3_accumulation(tmp_path):
    run_distributed(_train_pld, 2, str(tmp_path), 3)
