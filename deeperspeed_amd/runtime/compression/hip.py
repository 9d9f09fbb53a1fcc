"""Compression helpers (reference runtime/compression/cupy.py `CupyBackend`): sign packing
done by the HIP kernels in ops/csrc/kernels/onebit.hip instead of CuPy."""

import torch

from ...ops import native


class HipCompressionBackend:
    def compress_by_chunk(self, bool_tensor: torch.Tensor, num_chunks: int):
        """Pack a boolean tensor MSB-first into `num_chunks` equal uint8 chunks."""
        packed = native._packbits(bool_tensor.reshape(-1).to(torch.bool))
        return list(packed.chunk(num_chunks))

    def unpack(self, packed: torch.Tensor) -> torch.Tensor:
        return native._unpackbits(packed)
