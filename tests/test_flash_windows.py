"""enable_flash=True window table (host logic, no GPU): ptv3_ops.window_table_varlen_np against the oracle's
restatement of Pointcept get_padding_and_inverse + cu_seqlens (reference pointtransformer_v3.py:121-123 selects
patch 1024 for the flash branch)."""
import numpy as np
import pytest
import torch

from oracle import ptv3_ref
from splatformer_amd import ptv3_ops as ops


@pytest.mark.parametrize("K", [1024, 128, 7])
@pytest.mark.parametrize("counts", [[700], [1024], [2500], [2048], [5, 1, 3000, 1024, 1025, 2047]])
def test_varlen_table_matches_cu_seqlens(K, counts):
    offset = torch.tensor(counts).cumsum(0)
    pad, unpad = ptv3_ref.get_padding_and_inverse(offset, K)
    cu = ptv3_ref.cu_seqlens(offset, K).tolist()
    tab = ops.window_table_varlen_np(offset.tolist(), K)
    assert tab.shape == (len(cu) - 1, 3)
    n = int(offset[-1])
    covered = np.zeros(n, np.int64)
    for (ks, qs, cnt), s, e in zip(tab.tolist(), cu[:-1], cu[1:]):
        assert cnt <= K and cnt == e - s
        # keys: the window's padded slots hold exactly the serialized positions [ks, ks + cnt)
        assert sorted(pad[s:e].tolist()) == list(range(ks, ks + cnt))
        # queries: the real points whose padded slot falls in the window are [qs, ks + cnt)
        real = np.nonzero(((unpad >= s) & (unpad < e)).numpy())[0]
        assert real.tolist() == list(range(qs, ks + cnt))
        covered[qs:ks + cnt] += 1
    assert (covered == 1).all()


def test_varlen_table_empty_batches():
    tab = ops.window_table_varlen_np([0, 0, 10, 10], 1024)
    assert tab.tolist() == [[0, 0, 10]]
    assert ops.window_table_varlen_np([], 1024).shape == (0, 3)


def test_flash_oracle_reduces_to_pinned_attention():
    """With every batch no longer than K the flash branch is one softmax over the whole batch -- the non-flash
    restatement (pinned by tests/golden/backbone_pins.npz) at patch = n gives the same numbers; with n > K the
    windows are the non-flash K-windows of a single-batch cloud."""
    g = torch.Generator().manual_seed(0)
    C, H = 32, 2
    for n, K in ((300, 1024), (1000, 128), (1000, 1000)):
        qkv = torch.randn(n, 3 * C, generator=g, dtype=torch.float64)
        order = torch.randperm(n, generator=g)
        inverse = torch.empty_like(order)
        inverse[order] = torch.arange(n)
        mk = lambda: ptv3_ref.Point(offset=torch.tensor([n]), serialized_order=order[None],
                                    serialized_inverse=inverse[None])
        eye = torch.eye(3 * C, dtype=torch.float64)  # qkv projection = identity: the input is qkv itself
        sd = {"a.qkv.weight": eye, "a.qkv.bias": torch.zeros(3 * C, dtype=torch.float64)}
        flash = ptv3_ref.serialized_attention_heads(sd, "a", mk(), C, H, K, 0, qkv, flash=True)
        plain = ptv3_ref.serialized_attention_heads(sd, "a", mk(), C, H, K, 0, qkv, flash=False)
        assert torch.allclose(flash, plain, rtol=1e-12, atol=1e-12)
