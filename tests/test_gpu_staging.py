"""The staging path from pageable host memory (stark_host.cpp: copy threads bound to the GPU's NUMA
node, streaming-store copy into the context's pinned staging, DMA per 64 MB chunk): proofs handed
over as views into one large pageable array at odd 8-byte offsets (source and staging offsets not
16-byte aligned, the copy's head and tail paths), in both input forms, give the verdicts of the
same proofs passed as separate arrays, and a batch big enough to be split over several copy
threads and chunks does too (the Rust drop-in passes each `Vec`'s words as they lie:
rust/neptune-hip/src/lib.rs marshal)."""
import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def batch():
    pool4 = bench.load_pool4()
    claims, proofs, expect, _, _, _ = bench.make_config4(pool4, 512, 0.02, 1, 0)
    return pool4["air"], claims, proofs, expect


def _scattered(proofs, seed):
    """Every proof copied into one pageable array at a random odd word gap after the previous one."""
    rng = np.random.default_rng(seed)
    gaps = [1 + 2 * int(rng.integers(0, 8)) for _ in proofs]
    total = sum(len(p) for p in proofs) + sum(gaps)
    big = np.zeros(total, dtype=np.uint64)
    views, at = [], 0
    for p, g in zip(proofs, gaps):
        at += g
        big[at:at + len(p)] = p
        views.append(big[at:at + len(p)])
        at += len(p)
    return big, views


@pytest.mark.parametrize("mont", [False, True])
def test_pageable_views_at_odd_offsets(ctx, batch, mont):
    import neptune_hip.stark as NS
    air_words, claims, proofs, expect = batch
    dcl, dpr = bench.device_form(claims, proofs, mont)
    stark = NS.Stark.default().montgomery() if mont else NS.Stark.default()
    air = NS.Air([int(w) for w in air_words])
    cl = [NS.Claim(*c) for c in dcl]
    want = [bool(x) for x in expect]
    assert NS.verify_batch(ctx, air, stark, list(zip(cl, dpr))) == want
    big, views = _scattered(dpr, 0x57 + int(mont))
    assert any(v.ctypes.data % 16 for v in views) and any(v.ctypes.data % 16 == 0 for v in views)
    assert NS.verify_batch(ctx, air, stark, list(zip(cl, views))) == want
    # the same through a resident batch refilled from the views (nhip_batch_refill's staging)
    b = NS.Batch(ctx, air, stark, cl[:8], dpr[:8])
    b.refill(cl, views)
    v, ok = b.run()
    assert [bool(x) for x in v] == want and ok == all(want)
    b.close()
    del big


def test_receive_buffer_on_the_gpus_numa_node(ctx, batch):
    """nhip_host_alloc_near places the pinned receive buffer on the NUMA node of the context's GPU
    (when the platform reports one), and proofs received into it verify as they lie."""
    import ctypes
    import neptune_hip.stark as NS
    air_words, claims, proofs, expect = batch
    topo = ctx.numa()
    pinned = NS.PinnedProofs(proofs[:64], near=ctx)
    try:
        node = ctx.lib.nhip_host_page_node(ctypes.c_void_p(pinned.ptr))
        if topo["node"] >= 0 and node >= 0:
            assert node == topo["node"]
        air = NS.Air([int(w) for w in air_words])
        got = NS.verify_batch(ctx, air, NS.Stark.default(), list(zip([NS.Claim(*c) for c in claims[:64]],
                                                                      pinned.views)))
        assert got == [bool(x) for x in expect[:64]]
    finally:
        pinned.close()
