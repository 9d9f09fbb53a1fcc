"""Block-sparse attention (reference: deepspeed/ops/sparse_attention), HIP/MFMA kernels."""

from .sparsity_config import (BigBirdSparsityConfig, BSLongformerSparsityConfig, DenseSparsityConfig,
                              FixedSparsityConfig, LocalSlidingWindowSparsityConfig, SparsityConfig,
                              VariableSparsityConfig)
from .matmul import MatMul
from .softmax import Softmax
from .sparse_self_attention import SparseSelfAttention
from .bert_sparse_self_attention import BertSparseSelfAttention
from .sparse_attention_utils import SparseAttentionUtils
