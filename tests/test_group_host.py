"""Host side of the in-process multi-GPU group (no GPU here): the LPT split of
nhip_group_shard covers every proof, is deterministic, balances the word count within one
proof, and a group on a machine without a GPU is an error, never a CPU fallback."""
import numpy as np
import pytest


def test_group_shard_is_lpt_balanced():
    import neptune_hip.stark as NS
    rng = np.random.default_rng(3)
    lens = [int(x) for x in rng.choice([3_000, 12_000, 25_000, 80_000, 160_000], size=257)]
    proofs = [np.zeros(n, dtype=np.uint64) for n in lens]
    for members in (1, 2, 3, 8):
        m = NS.group_shard(proofs, members)
        assert m == NS.group_shard(proofs, members)
        assert len(m) == len(proofs) and set(m) <= set(range(members))
        load = [sum(n + 1 for n, k in zip(lens, m) if k == j) for j in range(members)]
        assert max(load) - min(load) <= max(lens) + 1
    assert NS.group_shard([], 4) == []


def test_group_without_device_is_an_error():
    import neptune_hip._lib as L
    import neptune_hip.stark as NS
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    with pytest.raises(L.NhipError):
        NS.Group([0, 0])
    with pytest.raises(L.NhipError):
        NS.Group(mask=0)


def test_group_entry_points_reject_bad_arguments():
    """C-ABI argument checks of the group entry points (host only): null outputs, zero members,
    null arrays with n > 0 are NHIP_ERR_ARG; null handles are harmless."""
    import ctypes
    import neptune_hip._lib as L
    lib = L.load()
    member = (ctypes.c_uint32 * 1)()
    assert lib.nhip_group_shard(None, 0, 1, None) == L.NHIP_OK
    assert lib.nhip_group_shard(None, 1, 1, member) == L.NHIP_ERR_ARG
    p = (L.Proof * 1)()
    assert lib.nhip_group_shard(p, 1, 0, member) == L.NHIP_ERR_ARG
    assert lib.nhip_group_shard(p, 1, 1, None) == L.NHIP_ERR_ARG
    assert lib.nhip_group_create(None, 0, None) == L.NHIP_ERR_ARG
    assert lib.nhip_group_init(0, None) == L.NHIP_ERR_ARG
    assert lib.nhip_group_size(None) == 0
    assert lib.nhip_group_member(None, 0) is None
    lib.nhip_group_destroy(None)
    v = np.zeros(1, dtype=np.uint8)
    assert lib.nhip_group_verify_batch(None, None, None, None, None, 0, v, None) == L.NHIP_ERR_ARG
