"""dlrm.jl_amd — MI355X-native (gfx950) DLRM embedding + feature-interaction hot path.

A drop-in for the hot path of darchr/DLRM.jl: the embedding gather
(maplookup), the pairwise-dot interaction (DotInteraction / dot_back) and the sparse SGD
update (update!), as hand-written HIP kernels behind the C ABI in include/dlrm_hip.h.
Import name: `dlrm_jl_amd` (the directory name carries a dot; see dlrm_pkg.py).
"""
from . import _lib
from ._lib import BoundsError, DLRMError, LibraryMissing
from . import dac
from .dac import DAC_DTYPE, DACLoader, DACMaps
from .dense import DenseMLP, DLRMModel, ShardedDLRMModel, bce_loss, bce_loss_back, kaggle_mlp_sizes, random_mlp
from .embedding import (DefaultStrategy, EmbeddingTableSet, PackedIndices, PreallocationStrategy, SimpleEmbedding,
                        lookup, maplookup)
from .hotpath import HotPath
from .lazy import DeferredUpdate, HipTables, LazyGrad, LazyLookup
from .interact import (POST_INTERACTION_PAD_TO_MUL, DotInteraction, cdiv, dot_back, dot_interaction, fast_vcat,
                       interaction_sizes, rrule, rrule_dot_interaction, rrule_self_batched_mul, rrule_triangular_slice,
                       self_batched_mul, triangular_slice, triangular_slice_back, up_to_mul_of)
from .shapes import (KAGGLE_EMBEDDING_SIZES, TERABYTE_EMBEDDING_SIZES, WORKLOADS, step_chunk, step_parts, step_pipeline, zipf_perm,
                     zipf_rows)
from .update import Descent, SparseEmbeddingUpdate, SparseIndexer, maplookup_pullback, update_

__all__ = [
    "BoundsError", "DLRMError", "LibraryMissing", "DefaultStrategy", "EmbeddingTableSet", "PackedIndices",
    "PreallocationStrategy", "SimpleEmbedding", "lookup", "maplookup", "HotPath", "POST_INTERACTION_PAD_TO_MUL",
    "DotInteraction", "cdiv", "dot_back", "fast_vcat", "interaction_sizes", "rrule", "up_to_mul_of",
    "KAGGLE_EMBEDDING_SIZES", "TERABYTE_EMBEDDING_SIZES", "WORKLOADS", "Descent", "SparseEmbeddingUpdate",
    "SparseIndexer", "maplookup_pullback", "update_", "DenseMLP", "DLRMModel", "bce_loss", "bce_loss_back",
    "kaggle_mlp_sizes", "random_mlp", "dac", "DAC_DTYPE", "DACLoader", "DACMaps", "ShardedDLRMModel",
    "dot_interaction", "rrule_dot_interaction", "triangular_slice", "triangular_slice_back", "rrule_triangular_slice",
    "self_batched_mul", "rrule_self_batched_mul", "step_pipeline", "step_chunk", "step_parts", "zipf_perm", "HipTables", "LazyLookup",
    "LazyGrad", "DeferredUpdate",
]
