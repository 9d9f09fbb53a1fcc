"""Eight data-parallel ranks (gloo/CPU, the code that runs on RCCL across an 8-GPU node): the
ZeRO-2 / ZeRO-3 configurations `bench.py` uses at N = 8 -- ZeRO-3 with every gathered unit
retained across the micro-batches (`stage3_max_live_parameters` covering the model), with and
without resident gradients -- train to the same weights as plain data parallelism (stage 0) on
the same per-rank data."""

from common import run_distributed
from test_zero_comm_modes import ZBASE, _load, _train

RETAIN = dict(stage3_max_live_parameters=10 ** 9, stage3_max_reuse_distance=10 ** 9)


def test_world8_sharded_stages_match_plain_dp(tmp_path):
    ga, lr = 2, 1e-2
    # fp32 with Adam eps 1e-3 (test_zero_fp32_exact.py): every stage equals plain DP to 1e-6
    kw = dict(lr=lr, dtype="float32", eps=1e-3)
    run_distributed(_train, 8, str(tmp_path), "s0", 0, ga, {}, **kw)
    ref = _load(tmp_path, "s0")
    runs = {"s2": (2, dict(ZBASE)),
            "s3": (3, dict(ZBASE, stage3_max_live_parameters=0, stage3_max_reuse_distance=0)),
            "s3_retained": (3, dict(ZBASE, **RETAIN)),
            "s3_retained_resident": (3, dict(ZBASE, resident_grads=True, **RETAIN))}
    for tag, (stage, zcfg) in runs.items():
        run_distributed(_train, 8, str(tmp_path), tag, stage, ga, zcfg, **kw)
        got = _load(tmp_path, tag)
        for k in ref["sd"]:
            d = (ref["sd"][k].float() - got["sd"][k].float()).abs()
            assert float(d.max()) <= 1e-6, (tag, k, float(d.max()))
        assert abs(ref["losses"][-1] - got["losses"][-1]) < 1e-6, (tag, ref["losses"], got["losses"])
        assert got["counts"]["reduce_scatter"] > 0, tag
    # retained units are gathered once per optimizer step instead of before every forward and
    # backward use; resident gradients are reduce-scattered once per step instead of per micro-batch
    plain, kept, res = (_load(tmp_path, t) for t in ("s3", "s3_retained", "s3_retained_resident"))
    assert kept["counts"]["all_gather"] < plain["counts"]["all_gather"], (kept["counts"], plain["counts"])
    assert res["counts"]["reduce_scatter"] * ga == kept["counts"]["reduce_scatter"]
