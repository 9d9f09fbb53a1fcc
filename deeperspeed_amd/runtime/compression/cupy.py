"""Import path of the reference's 1-bit compression backend (deepspeed/runtime/compression/cupy.py).

There is no CuPy on ROCm here: the name `CupyBackend` resolves to the HIP backend
(runtime/compression/hip.py: sign packing / unpacking kernels in ops/csrc/kernels/onebit.hip),
which offers the same `compress_by_chunk` surface on torch tensors (torch2cupy / cupy2torch are
identities)."""

from .hip import HipCompressionBackend as CupyBackend  # noqa: F401
