"""N > 1 host path on CPU: world-size-2 gloo ranks shard independent units, verify their shard
(with the C oracle standing in for the GPU, test-only), and exchange exactly the verdicts."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    for p in ("oracle", "neptune-core_amd"):
        sys.path.insert(0, os.path.join(ROOT, p))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import coracle as C
    from neptune_hip import shard

    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(99)  # same data on every rank
    n, depth = 128, 7
    leafs = rng.integers(0, 2**63, size=(n, 5), dtype=np.uint64)
    nodes = C.mtree_build(leafs)
    idx = np.arange(n, dtype=np.int64)
    paths = np.empty((n, depth, 5), dtype=np.uint64)
    paths[:, 0] = leafs[idx ^ 1]
    run = idx + n
    for k in range(1, depth):
        run >>= 1
        paths[:, k] = nodes[run ^ 1]
    el = leafs.copy()
    el[[5, 77]] ^= np.uint64(1)
    costs = rng.integers(1, 10, size=n)
    shards = shard.lpt_shard(costs, world)
    mine = np.asarray(shards[rank], dtype=np.int64)
    v = C.mtree_verify_batch(nodes[1], idx[mine].astype(np.uint64), el[mine], paths[mine].reshape(-1), depth)
    ok = shard.all_ok(bool(v.all()), dist)
    full = shard.gather_verdicts(v, shards, n, dist)
    q.put((rank, ok, full.tolist(), [len(s) for s in shards]))
    dist.destroy_process_group()


def test_two_rank_sharded_verdicts():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    expect = np.ones(128, dtype=np.uint8)
    expect[[5, 77]] = 0
    for rank, ok, full, sizes in res:
        assert ok is False
        assert full == expect.tolist()
        assert sum(sizes) == 128 and abs(sizes[0] - sizes[1]) <= 16


def test_lpt_shard_balances_and_covers():
    sys.path.insert(0, os.path.join(ROOT, "neptune-core_amd"))
    from neptune_hip import shard
    costs = [16, 10, 11, 12, 12, 11, 9, 9] * 32
    s = shard.lpt_shard(costs, 8)
    assert sorted(i for r in s for i in r) == list(range(len(costs)))
    loads = [sum(costs[i] for i in r) for r in s]
    assert max(loads) - min(loads) <= max(costs)
    assert shard.contiguous_shard(10, 3, 2) == range(8, 10)


def _stark_worker(rank, world, port, q):
    for p in ("oracle", "neptune-core_amd", ""):
        sys.path.insert(0, os.path.join(ROOT, p))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import bench
    import coracle as C
    import stark_ref as S
    from neptune_hip import shard

    dist.init_process_group("gloo", rank=rank, world_size=world)
    air, pool = bench.load_pool()
    total = 48
    claims, proofs, expect, _, shards, expect_all = bench.make_config4(bench.pool4_from_c3(pool), total, 0.1, world,
                                                                       rank)
    v = C.stark_verify_batch(air, S.StarkParams(), claims, proofs, threads=2)
    rng = np.random.default_rng(0xC4)
    hs = rng.choice(bench.COLLECTION_HEIGHTS, size=total)
    assert shards == shard.lpt_shard([10_000 + 600 * int(h) for h in hs], world)
    ok = shard.all_ok(bool(v.all()), dist)
    full = shard.gather_verdicts(v, shards, total, dist)
    q.put((rank, ok, full.tolist(), [bool(x) == bool(e) for x, e in zip(v, expect)], [len(s) for s in shards],
           full.astype(bool).tolist() == expect_all.tolist()))
    dist.destroy_process_group()


def test_two_rank_config4_stark_sharding():
    """bench.py config 4 on world size 2 (gloo; the C verifier stands in for the GPU): the LPT
    shards cover every proof once, each rank's verdicts are the expected ones, and the verdict
    exchange (all-reduce MIN + all-gather) reconstructs the job's verdict vector."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stark_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    fulls = [r[2] for r in res]
    assert fulls[0] == fulls[1] and sum(fulls[0]) == 48 - 5
    for rank, ok, full, matches, sizes, gathered_ok in res:
        assert ok is False and all(matches) and sum(sizes) == 48 and gathered_ok


def _exchange_worker(rank, world, port, q, depth=2):
    sys.path.insert(0, os.path.join(ROOT, "neptune-core_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from neptune_hip import shard

    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 37
    costs = [(7 * i) % 11 + 1 for i in range(n)]
    shards = shard.lpt_shard(costs, world)
    mine = np.asarray(shards[rank], dtype=np.int64)
    steps = []
    for k in range(4):  # a different verdict vector per step: exchanges must complete in order
        full = np.ones(n, dtype=np.uint8)
        full[[k, (5 * k + 3) % n]] = 0
        if k == 3:
            full[:] = 1
        steps.append(full)
    ex = shard.VerdictExchange(shards, n, dist, depth=depth)
    got = []
    for k, full in enumerate(steps):
        v = full[mine]
        ex.post(bool(v.all()), v)
        if len(ex.pending) >= depth:
            got.append(ex.complete())
    try:
        ex.post(True, steps[0][mine])
        ex.post(True, steps[0][mine])  # one posted exchange past the ring's depth is refused
        third = False
    except RuntimeError:
        third = True
    while ex.pending:
        got.append(ex.complete())
    # the two-collective form gives the same answers
    v = steps[1][mine]
    pair = (shard.all_ok(bool(v.all()), dist), shard.gather_verdicts(v, shards, n, dist).tolist())
    q.put((rank, [(ok, full.tolist()) for ok, full in got], [s.tolist() for s in steps], pair, third))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,depth", [(2, 2), (8, 2), (2, 4), (8, 4)])
def test_two_rank_verdict_exchange_one_collective(world, depth):
    """shard.VerdictExchange at world size 2 and 8 (gloo; 8 = the driver's node, every rank's LPT
    shard of 37 units): one all-gather per step carries the batch verdict (the MIN of every rank's
    leading byte) and the per-proof verdicts, exchanges posted two or four deep complete in posting
    order, and the answers equal all_ok + gather_verdicts on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q, depth)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, got, steps, pair, third in res:
        assert third
        assert len(got) == 5
        for k, full in enumerate(steps):
            assert got[k] == (all(full), full)
        assert got[4] == (True, steps[0])  # the extra post: local_ok as given, step 0's verdicts
        assert pair == (all(steps[1]), steps[1])


def _rank0_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "neptune-core_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import time
    import torch.distributed as dist
    from neptune_hip import shard

    dist.init_process_group("gloo", rank=rank, world_size=world)
    t0 = time.time()

    def leg():
        time.sleep(0.5)
        return {"ran_on": dist.get_rank()}

    got = shard.on_rank0(leg, dist, "leg_a")
    waited = time.time() - t0

    def bad():
        raise RuntimeError("leg failed")

    raised = None
    try:
        shard.on_rank0(bad, dist, "leg_b")
    except RuntimeError as e:
        raised = str(e)
    dist.barrier()
    q.put((rank, got, waited, raised))
    dist.destroy_process_group()


def test_rank0_leg_others_wait_on_the_store():
    """shard.on_rank0 (bench.py's group_stream leg at N > 1): rank 0 runs the leg, the other ranks
    wait on the host until it is done (no collective in flight meanwhile), get None, and are
    released even when the leg raises on rank 0."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank0_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    (r0, g0, w0, e0), (r1, g1, w1, e1) = res
    assert g0 == {"ran_on": 0} and g1 is None
    assert w1 >= 0.45  # rank 1 waited for rank 0's leg
    assert e0 == "leg failed" and e1 is None
