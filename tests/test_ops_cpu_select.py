"""Host-side kernel selection of the decode attention (no GPU needed)."""
import pytest

from k8s_vgpu_scheduler_amd import ops


@pytest.fixture
def cus(monkeypatch):
    state = {"n": 256}
    monkeypatch.setattr(ops, "visible_cus", lambda: state["n"])
    monkeypatch.setattr(ops, "attn_split", lambda: 256)
    monkeypatch.delenv("MIVGPU_ATTN_SPLITS", raising=False)
    monkeypatch.delenv("MIVGPU_ATTN_W12", raising=False)
    return state


def test_one_split_when_every_cu_gets_a_kv_head(cus):
    # Qwen3-8B at batch 32: 256 (b, kv-head) pairs on 256 CUs -> twelve-wave one-split workgroups
    assert ops.attn_fused_splits(32, 8, 1088, 32) == 1
    # a 64-CU slice: four pairs per CU
    cus["n"] = 64
    assert ops.attn_fused_splits(32, 8, 1088, 32) == 1


def test_splits_kept_where_the_one_split_grid_is_too_small(cus):
    assert ops.attn_fused_splits(1, 8, 1088, 32) == 5         # batch-1 serving: 8 workgroups would idle the chip
    assert ops.attn_fused_splits(31, 8, 1088, 32) == 5        # 248 < 256 CUs
    assert ops.attn_fused_splits(32, 8, 1088, 16) == 5        # two query heads per kv-head: no twelve-wave kernel
    assert ops.attn_fused_splits(32, 8, 1088) == 5            # caller did not say the head count
    # a long cache: a long row among short ones must not be one workgroup's stream
    assert ops.attn_fused_splits(32, 8, 2048, 32) == 1
    assert ops.attn_fused_splits(32, 8, 8448, 32) == 16


def test_one_split_env_overrides(cus, monkeypatch):
    monkeypatch.setenv("MIVGPU_ATTN_W12", "0")
    assert ops.attn_fused_splits(32, 8, 1088, 32) == 5
    monkeypatch.setenv("MIVGPU_ATTN_SPLITS", "3")
    assert ops.attn_fused_splits(32, 8, 1088, 32) == 3
