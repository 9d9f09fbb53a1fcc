"""Dynamic loss scaling against the reference's documented update rule
(deepspeed/runtime/fp16/loss_scaler.py:150-168: hysteresis, growth window, min-scale error),
transcribed as a small state machine and compared on random overflow sequences."""

import random

import pytest

from deeperspeed_amd.runtime.fp16.loss_scaler import DynamicLossScaler, LossScaleUnderflowError


def _spec_step(st, overflow):
    if overflow:
        if st["ds"] == 1 or st["h"] == 1:
            if st["s"] == st["min"]:
                raise RuntimeError("min")
            st["s"] = max(st["s"] / 2, st["min"])
        else:
            st["h"] -= 1
        st["lo"] = st["it"]
    else:
        if st["c"]:
            st["h"] = st["ds"]
        if (st["it"] - st["lo"]) % st["w"] == 0:
            if not st["c"]:
                st["h"] = st["ds"]
            st["s"] *= 2
    st["it"] += 1


@pytest.mark.parametrize("seed", range(5))
def test_dynamic_scaler_matches_spec(seed):
    rng = random.Random(seed)
    for _ in range(60):
        ds, c, w = rng.choice([1, 2, 3]), rng.choice([False, True]), rng.choice([1, 3, 5])
        a = DynamicLossScaler(init_scale=2 ** 10, scale_window=w, min_scale=1, delayed_shift=ds,
                              consecutive_hysteresis=c)
        st = dict(s=2 ** 10, it=0, lo=-1, h=ds, ds=ds, c=c, w=w, min=1)
        for _ in range(60):
            ov = rng.random() < 0.4
            raised = spec_raised = False
            try:
                a.update_scale(ov)
            except LossScaleUnderflowError:
                raised = True
            try:
                _spec_step(st, ov)
            except RuntimeError:
                spec_raised = True
            assert raised == spec_raised
            if raised:
                break
            assert (a.cur_scale, a.cur_hysteresis, a.cur_iter) == (st["s"], st["h"], st["it"])


def test_state_dict_roundtrip():
    a = DynamicLossScaler(init_scale=2 ** 8, scale_window=2, delayed_shift=2)
    for ov in (True, False, False, True, True):
        a.update_scale(ov)
    b = DynamicLossScaler(init_scale=1.0)
    b.load_state_dict(a.state_dict())
    assert (b.cur_scale, b.cur_iter, b.last_overflow_iter, b.cur_hysteresis) == \
        (a.cur_scale, a.cur_iter, a.last_overflow_iter, a.cur_hysteresis)
