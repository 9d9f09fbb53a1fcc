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
