from .sparsity_config import (BigBirdSparsityConfig, BSLongformerSparsityConfig, DenseSparsityConfig,
                              FixedSparsityConfig, LocalSlidingWindowSparsityConfig, SparsityConfig,
                              VariableSparsityConfig)
from .sparse_self_attention import BertSparseSelfAttention, SparseAttentionUtils, SparseSelfAttention
