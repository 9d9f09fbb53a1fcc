"""CPU checks of the measured-solution table logic (ops/lt_tune.py, scripts/make_lt_table.py)."""

import json
import os
import sys

from deeperspeed_amd.ops import lt_tune

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_keys_are_the_column_major_problems():
    # Y[M,N] = X W^T  ->  Y^T[N,M] = W(T) X(N)
    assert lt_tune.key("fwd", 8192, 18432, 6144, bias=True) == (1, 0, 18432, 8192, 6144, 4, 0)
    # dX[M,K] = dY W  ->  dX^T[K,M] = W(N) dY(N)
    assert lt_tune.key("dgrad", 8192, 18432, 6144) == (0, 0, 6144, 8192, 18432, 1, 0)
    # dW[N,K] += dY^T X  ->  dW^T[K,N] = X(N) dY(T), accumulating
    assert lt_tune.key("wgrad", 8192, 18432, 6144) == (0, 1, 6144, 18432, 8192, 1, 1)
    assert lt_tune.key("wgradT", 8192, 18432, 6144) == (1, 0, 6144, 18432, 8192, 1, 1)


def test_make_table_matches_runtime_keys(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    try:
        import make_lt_table
    finally:
        sys.path.pop(0)
    for layout, kind, bias in (("fwd+bias", "fwd", True), ("fwd", "fwd", False), ("dgrad", "dgrad", False),
                               ("wgrad", "wgrad", False), ("wgradT", "wgradT", False)):
        c = make_lt_table.col_of(layout, 8192, 24576, 6144)
        assert (c["ta"], c["tb"], c["m"], c["n"], c["k"], c["epi"], c["beta"]) == \
            lt_tune.key(kind, 8192, 24576, 6144, bias)


def _table(tmp_path, rows):
    p = tmp_path / "t.json"
    ents = []
    for kind, M, N, K, tf in rows:
        k = lt_tune.key(kind, M, N, K)
        ents.append({"col": dict(zip(("ta", "tb", "m", "n", "k", "epi", "beta"), k)), "names": ["s"], "tflops": tf})
    p.write_text(json.dumps({"entries": ents}))
    return str(p)


def test_shipped_table_parses():
    t = lt_tune.load_table(lt_tune.TABLE_PATH)
    assert t, "ops/lt_table.json missing or empty"
    for k, e in t.items():
        assert len(k) == 7 and e["names"] and e["tflops"] > 0


def test_routes_gated_by_measured_gain(tmp_path, monkeypatch):
    p = tmp_path / "g.json"
    ents = []
    for kind, bias, tf, h in (("fwd", True, 1100.0, 900.0), ("wgradT", False, 1000.0, 990.0)):
        k = lt_tune.key(kind, 8192, 3072, 1024, bias)
        ents.append({"col": dict(zip(("ta", "tb", "m", "n", "k", "epi", "beta"), k)), "names": ["s"], "tflops": tf,
                     "heuristic_tflops": h})
    p.write_text(json.dumps({"entries": ents}))
    monkeypatch.setattr(lt_tune, "_table", lt_tune.load_table(str(p)))
    monkeypatch.setattr(lt_tune, "ENABLED", True)
    monkeypatch.setattr(lt_tune, "FWD", True)
    assert lt_tune.use_fwd(8192, 3072, 1024, True)  # +22 %
    assert not lt_tune.use_fwd(8192, 1024, 1024, True)  # no record
