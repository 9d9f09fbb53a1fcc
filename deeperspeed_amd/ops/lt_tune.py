"""Measured hipBLASLt solutions for the transformer GEMMs, and the layout choices they imply.

hipBLASLt's heuristic returns a handful of algorithms per problem; on gfx950 the fastest kernel
for the GPT-NeoX shapes is often not among them.  `scripts/lt_sweep.cpp` times EVERY solution
`hipblaslt_ext::getAllAlgos` lists for the problems of a linear layer (forward with bias, input
gradient untransposed "NN", weight gradient token-major "NT", and both gradients after operand
transposes "TN") and `scripts/make_lt_table.py` keeps the fastest few per problem in
`ops/lt_table.json` (source data: `profiles/r4i_lt_sweep*.jsonl`).

At run time (`ops/csrc/gemm_lt.cpp`):
- the table's solutions (by hipBLASLt solution name; indices differ between processes) join the
  heuristic candidates that the wrapper times on the first call of each problem (a stale name is
  checked with matmulIsAlgoSupported and can only lose the timing);
- `ops/linear.py` routes a linear's forward through the wrapper for the problems where the
  table's best solution beats the heuristic's by MIN_GAIN.  The table's input- and weight-gradient
  records (untransposed NN / NT, transposed TN) were measured too; routing them lost in the step
  (20B N=1 -0.8 %, 1.3B ZeRO-2 -0.2 %, profiles/r4u_notes.md, r4m_notes.md), so those GEMMs keep
  torch's hipBLASLt call on transposed operands (ops/linear.py).

Reference counterpart: the reference calls cuBLAS with the default heuristic
(`csrc/includes/cublas_wrappers.h`, `cublasGemmEx(..., CUBLAS_GEMM_DEFAULT_TENSOR_OP)`); the
per-shape algorithm choice is an MI355X addition.

DSA_LT=0 disables the route; DSA_LT_TABLE names another table file.
"""

from __future__ import annotations

import json
import os
import threading
from typing import Dict, Optional, Tuple

ENABLED = os.environ.get("DSA_LT", "1") != "0"
# forward GEMMs with a measured solution >= MIN_GAIN over the heuristic (BERT-Large QKV projection
# +22 %, the seq-128 step +1.2 %, profiles/r4u_notes.md)
FWD = ENABLED
TABLE_PATH = os.environ.get("DSA_LT_TABLE", os.path.join(os.path.dirname(__file__), "lt_table.json"))

EPI_DEFAULT, EPI_BIAS = 1, 4

Key = Tuple[int, int, int, int, int, int, int]  # column-major (ta, tb, m, n, k, epilogue, beta)

_lock = threading.Lock()
_table: Optional[Dict[Key, dict]] = None
_registered = False


def key(kind: str, M: int, N: int, K: int, bias: bool = False) -> Key:
    """Column-major hipBLASLt problem of a row-major linear over M tokens, N outputs, K inputs:
    fwd    Y[M,N]   = X[M,K] W[N,K]^T (+ b)
    dgrad  dX[M,K]  = dY[M,N] W[N,K]
    wgrad  dW[N,K] += dY[M,N]^T X[M,K]          (token-major operands)
    wgradT dW[N,K] += dYt[N,M] Xt[K,M]^T        (operands transposed first)"""
    if kind == "fwd":
        return (1, 0, N, M, K, EPI_BIAS if bias else EPI_DEFAULT, 0)
    if kind == "dgrad":
        return (0, 0, K, M, N, EPI_DEFAULT, 0)
    if kind == "wgrad":
        return (0, 1, K, N, M, EPI_DEFAULT, 1)
    if kind == "wgradT":
        return (1, 0, K, N, M, EPI_DEFAULT, 1)
    raise ValueError(kind)


def load_table(path: Optional[str] = None) -> Dict[Key, dict]:
    """{column-major key: {"names": [solution names], "tflops": best measured, ...}}."""
    global _table
    if path is None and _table is not None:
        return _table
    p = path or TABLE_PATH
    out: Dict[Key, dict] = {}
    if os.path.exists(p):
        with open(p) as f:
            data = json.load(f)
        for e in data.get("entries", []):
            c = e["col"]
            k = (int(c["ta"]), int(c["tb"]), int(c["m"]), int(c["n"]), int(c["k"]), int(c["epi"]), int(c["beta"]))
            out[k] = e
    if path is None:
        _table = out
    return out


def register(hip_ops) -> int:
    """Hand every table entry's solution indices to the wrapper (once per process)."""
    global _registered
    with _lock:
        if _registered:
            return 0
        _registered = True
        n = 0
        for (ta, tb, m, n_, k, epi, beta), e in load_table().items():
            if e.get("names"):
                hip_ops.lt_register(bool(ta), bool(tb), m, n_, k, epi, bool(beta), True, list(e["names"]))
                n += 1
        return n


def entry(kind: str, M: int, N: int, K: int, bias: bool = False) -> Optional[dict]:
    if not ENABLED:
        return None
    return load_table().get(key(kind, M, N, K, bias))


# a measured solution is routed only when it beats the heuristic's first choice by this factor
# (the sweep times each solution over few launches; smaller gains are within its noise)
MIN_GAIN = 1.05


def gain(kind: str, M: int, N: int, K: int, bias: bool = False) -> float:
    """Best measured rate over the heuristic's (0.0 when the table has no record)."""
    e = entry(kind, M, N, K, bias)
    if e is None or not e.get("heuristic_tflops"):
        return 0.0
    return float(e["tflops"]) / float(e["heuristic_tflops"])


def use_fwd(M: int, N: int, K: int, bias: bool) -> bool:
    return FWD and gain("fwd", M, N, K, bias) >= MIN_GAIN
