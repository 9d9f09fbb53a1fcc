"""Compact fp32 master (bf16 high half + int16 residual): exact round trip, and ZeRO stages
0-3 trained with it must match the separate-fp32-master path (gloo/CPU)."""

import os

import pytest
import torch

from common import run_distributed


def test_encode_decode_exact():
    from deeperspeed_amd.runtime.zero import compact_master as cm
    g = torch.Generator().manual_seed(0)
    x = torch.cat([torch.randn(100000, generator=g) * 10 ** torch.randint(-30, 30, (100000,), generator=g).float(),
                   torch.tensor([0.0, -0.0, 1.0, -1.0, 3.4e38, -3.4e38, 1e-45, -1e-45, 1.00390625, 1.0078125,
                                 65504.0, 2.0 - 2 ** -23, -(2.0 - 2 ** -23)])])
    hi, res = cm.encode(x)
    assert hi.dtype == torch.bfloat16 and res.dtype == torch.int16
    y = cm.decode(hi, res)
    assert torch.equal(y.view(torch.int32), x.view(torch.int32))
    # the high half is the nearest bf16 (differs from RNE on exact ties only)
    rne = x.to(torch.bfloat16).float()
    diff = (hi.float() - rne).abs()
    ulp = (rne.abs() * 2 ** -7).clamp_min(1e-38)
    fin = torch.isfinite(rne)
    assert (diff[fin] <= ulp[fin]).all()
    assert (hi.float() == rne).float().mean() > 0.999


def test_adam_compact_cpu_matches_fp32():
    from deeperspeed_amd.ops import native
    from deeperspeed_amd.runtime.zero import compact_master as cm
    torch.manual_seed(0)
    w = torch.randn(4096)
    hi, res = cm.encode(w)
    m1, v1, m2, v2 = (torch.zeros(4096) for _ in range(4))
    w_ref = w.clone()
    for step in range(1, 6):
        g = torch.randn(4096).to(torch.bfloat16)
        native.adam_flat_(w_ref, g, m1, v1, None, 1e-2, 0.9, 0.999, 1e-8, 0.01, step, True, 0.5, True)
        native.adam_compact_(hi, res, g, m2, v2, 1e-2, 0.9, 0.999, 1e-8, 0.01, step, True, 0.5, True)
    assert torch.equal(cm.decode(hi, res), w_ref)
    assert torch.equal(m1, m2) and torch.equal(v1, v2)


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
def test_zero_compact_master_matches(tmp_path, stage):
    from test_zero import _train_and_dump
    run_distributed(_train_and_dump, 2, str(tmp_path), stage, 2, None)
    run_distributed(_train_and_dump, 2, str(tmp_path), stage, 2, "compact")
    a = torch.load(os.path.join(tmp_path, f"s{stage}_ga2_None.pt"), weights_only=True)
    b = torch.load(os.path.join(tmp_path, f"s{stage}_ga2_compact.pt"), weights_only=True)
    for k in a["sd"]:
        assert torch.allclose(a["sd"][k].float(), b["sd"][k].float(), atol=1e-2, rtol=1e-2), k
    if a["masters"] is not None:
        assert torch.allclose(a["masters"], b["masters"], atol=1e-3, rtol=1e-3)


def _ckpt_body(out_dir):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from simple_model import SimpleModel, base_config, random_batches
    torch.manual_seed(1)
    cfg = base_config(stage=3, mb=4, ga=1, compact_master=True, reduce_bucket_size=500,
                      stage3_unit_max_numel=600, stage3_param_persistence_threshold=10)

    def build():
        model = SimpleModel(32)
        e, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
        return e

    e1 = build()
    for x, y in random_batches(3, 4, 32, seed=5 + dist.get_rank()):
        loss = e1(x.to(torch.bfloat16), y)
        e1.backward(loss)
        e1.step()
    e1.save_checkpoint(out_dir, tag="c")
    e2 = build()
    e2.load_checkpoint(out_dir, tag="c")
    for g1, g2 in zip(e1.optimizer.groups, e2.optimizer.groups):
        assert torch.equal(e1.optimizer.master_fp32(g1), e2.optimizer.master_fp32(g2))
        assert torch.equal(g1.shard_param, g2.shard_param)
    # the consolidated fp32 weights come out of the residual encoding too
    if dist.get_rank() == 0:
        from deeperspeed_amd.utils.zero_to_fp32 import convert_zero_chkpt_to_fp32_consolid_state_dict
        sd = convert_zero_chkpt_to_fp32_consolid_state_dict(os.path.join(out_dir, "c"), os.path.join(out_dir, "f.pt"))
        assert all(v.dtype == torch.float32 for v in sd.values())


def test_compact_master_checkpoint_roundtrip(tmp_path):
    run_distributed(_ckpt_body, 2, str(tmp_path))
