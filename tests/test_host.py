"""Host-side logic that needs no GPU: shapes, sizes, index packing, fail-loudly behaviour."""
import numpy as np
import pytest
import torch


def test_interaction_sizes_follow_process_batches(pkg):
    # interact.jl:449-456 with POST_INTERACTION_PAD_TO_MUL = 1 (model.jl:32)
    assert pkg.interaction_sizes(16, 8) == (16 + 28, 44, 0)     # golden: output_interaction 128 x 44
    assert pkg.interaction_sizes(128, 27) == (128 + 351, 479, 0)
    assert pkg.interaction_sizes(4, 4) == (10, 10, 0)           # model.jl KAT: 4 + 6
    assert pkg.interaction_sizes(16, 8, pad_to=8) == (44, 48, 4)
    assert pkg.up_to_mul_of(44, 8) == 48 and pkg.cdiv(44, 8) == 6


def test_top_mlp_input_size_matches_dlrm_builder(pkg):
    # model.jl:220-226: pre_triangle_size = D*T/d + 1, top input = tri + d
    D, T, d = 128, 26, 128
    F = D * T // d + 1
    assert pkg.interaction_sizes(d, F)[1] == 479


def test_packed_indices_forms(pkg):
    B, L, T = 5, 3, 4
    per_table_2d = [torch.arange(B * L).reshape(B, L) + 10 * t for t in range(T)]
    p = pkg.PackedIndices(per_table_2d)
    assert (p.T, p.B, p.L) == (T, B, L)
    assert p.data.shape == (T, B * L)
    # sample-major within a table: position b*L + k (criteo.jl:551-557 reshape(vec, :, B))
    assert p.data[2, 1 * L + 2].item() == 20 + 5
    p1 = pkg.PackedIndices([torch.arange(B) for _ in range(T)])
    assert (p1.T, p1.B, p1.L) == (T, B, 1)
    p2 = pkg.PackedIndices(torch.zeros((T, B), dtype=torch.int32))
    assert p2.data.dtype == torch.int32 and p2.stride == B
    with pytest.raises(ValueError):
        pkg.PackedIndices([torch.arange(3), torch.arange(4)])


def test_kaggle_and_terabyte_sizes(pkg):
    assert len(pkg.KAGGLE_EMBEDDING_SIZES) == 26 and sum(pkg.KAGGLE_EMBEDDING_SIZES) == 33762577
    assert len(pkg.TERABYTE_EMBEDDING_SIZES) == 26 and sum(pkg.TERABYTE_EMBEDDING_SIZES) == 882774559
    assert pkg.WORKLOADS["kaggle-d128-b2048"]["batch"] == 2048


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure mode")
def test_hot_path_fails_loudly_without_gpu(pkg):
    from dlrm_jl_amd import runtime
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        runtime.context()


def test_product_package_never_imports_the_oracle():
    import os
    import re
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dlrm.jl_amd")
    for dirpath, _, files in os.walk(root):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp")):
                text = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"\boracle\b", text.replace("oracle/", "")), f"{f} references the oracle"
