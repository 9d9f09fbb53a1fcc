"""`deepspeed.ops.op_builder` import path: builders of the in-tree native extensions."""

from .builder import (ALL_OPS, AsyncIOBuilder, CPUAdamBuilder, FusedAdamBuilder, FusedLambBuilder, OpBuilder,
                      SparseAttnBuilder, StochasticTransformerBuilder, TransformerBuilder, UtilsBuilder)
