"""bench.py's multi-GPU launch (CPU): `--gpus N` with no launcher relaunches N ranks under
torch.distributed.run, a launcher's WORLD_SIZE must equal N, and the final cross-rank reduction
(shard.agreed_max) ends the same way on every rank when the RCCL attempt fails on some of them
(world-size-2 gloo).  Reference: the batch callers shard at proof granularity
(proof_collection.rs:342-388, state/mod.rs:2226-2272); the only exchange is the verdict."""
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_plan_one_gpu_runs_here():
    assert bench.launch_plan(1, {}, [])["action"] == "run"
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}, [])["action"] == "run"


@pytest.mark.parametrize("n", [2, 8])
def test_plan_relaunches_n_ranks(n):
    argv = ["--gpus", str(n), "--steps", "20", "--warmup", "5"]
    p = bench.launch_plan(n, {}, argv, n_visible=8, port=29999)
    assert p["action"] == "relaunch" and p["world"] == n
    cmd = p["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == str(n)
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29999"
    assert cmd[-len(argv) - 1].endswith("bench.py") and cmd[-len(argv):] == argv


def test_plan_under_a_launcher_is_one_rank():
    p = bench.launch_plan(8, {"WORLD_SIZE": "8", "RANK": "3"}, [])
    assert p == {"action": "run", "world": 8}


@pytest.mark.parametrize("gpus,env,visible", [(2, {"WORLD_SIZE": "4"}, None), (8, {"WORLD_SIZE": "1"}, None),
                                               (8, {}, 1), (0, {}, None)])
def test_plan_mismatch_is_an_error(gpus, env, visible):
    p = bench.launch_plan(gpus, env, [], n_visible=visible)
    assert p["action"] == "error" and p["message"]


def test_mismatch_exits_nonzero_before_any_work():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 2 and "WORLD_SIZE=2 but --gpus 3" in out.stderr
    assert out.stdout == ""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _agree_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "neptune-core_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from neptune_hip import shard

    dist.init_process_group("gloo", rank=rank, world_size=world)
    vals = [1.5 + rank, float(rank == 1), 0.0]

    def fails_on_rank1(v):
        if dist.get_rank() == 1:
            raise RuntimeError("simulated RCCL fault")
        return [x * 100 for x in v]  # a value the host path never produces: shows which path was taken

    def works(v):
        return [x + 1000 for x in v]

    a = shard.agreed_max(vals, dist, fails_on_rank1)
    b = shard.agreed_max(vals, dist, works)
    c = shard.agreed_max(vals, dist, None)
    # the collectives after the reduction still line up on every rank
    perms = shard.all_ok(True, dist)
    q.put((rank, a, b, c, perms))
    dist.destroy_process_group()


def test_agreed_fallback_when_one_rank_fails():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    (r0, a0, b0, c0, p0), (r1, a1, b1, c1, p1) = res
    want = [2.5, 1.0, 0.0]  # the MAX over ranks, on the host group
    assert a0[0] == a1[0] == want and a0[1] is False and a1[1] is False
    assert a0[2] is None and "simulated RCCL fault" in a1[2]
    assert b0[1] is True and b1[1] is True and b0[0] == [1001.5, 1000.0, 1000.0] and b1[0] == [1002.5, 1001.0, 1000.0]
    assert c0[0] == c1[0] == want and not c0[1] and not c1[1]
    assert p0 is True and p1 is True


def _pcie_worker(rank, world, port, q):
    """bench.pcie_stream's barrier protocol with host fakes: rank 1's setup raises, rank 0 streams."""
    sys.path[:0] = [os.path.join(ROOT, "neptune-core_amd"), ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch.distributed as dist
    import bench
    import neptune_hip.stark as NS

    dist.init_process_group("gloo", rank=rank, world_size=world)

    class Buf:
        def upload(self, a):
            pass

        def free(self):
            pass

    class Ctx:
        def synchronize(self):
            pass

        def alloc(self, n):
            return Buf()

    class Pinned:
        def __init__(self, proofs, near=None):
            if dist.get_rank() == 1:
                raise RuntimeError("simulated pinned-allocation fault")
            self.flat = np.zeros(8, dtype=np.uint64)
            self.views = proofs

        def close(self):
            pass

    class Batch:
        def __init__(self, *a, **k):
            self.n = len(a[4])

        def run(self):
            return [True] * self.n, True

        def refill(self, *a, **k):
            pass

        def launch(self):
            pass

        def wait(self):
            return [True] * self.n, True

        def stats(self):
            return {"ms_decode": 0.0, "ms_upload": 0.0}

        def close(self):
            pass

    NS.PinnedProofs, NS.Batch, NS.marshal = Pinned, Batch, lambda c, p: None
    NS.Claim = lambda *c: c
    claims = [((0,) * 5, 0, [], [])] * 4
    proofs = [np.zeros(16, dtype=np.uint64)] * 4
    r = bench.pcie_stream(Ctx(), None, None, claims, proofs, np.ones(4, dtype=bool), 3, dist, 8)
    from neptune_hip import shard
    shard_ok = shard.all_ok(True, dist)  # the ranks' next collective still lines up
    q.put((rank, r.get("verdicts_correct"), "error" in r, "value" in r, shard_ok))
    dist.destroy_process_group()


def test_pcie_leg_fault_on_one_rank_does_not_strand_the_others():
    """Every rank reaches every barrier of the multi-rank PCIe leg even when its own work raised: the
    faulting rank reports the error in its leg (verdicts_correct None, never fatal for the headline),
    the others finish the leg, and the next collective lines up."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pcie_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    (r0, v0, e0, val0, ok0), (r1, v1, e1, val1, ok1) = res
    assert v0 is True and not e0 and val0
    assert v1 is None and e1 and not val1
    assert ok0 is True and ok1 is True


def test_tx_stream_is_what_the_node_leg_decodes():
    """bench.tx_stream (the node leg's wire bytes): back-to-back SingleProof TransferTransactions that
    the native scanner (host only) splits back into exactly the proofs, in order."""
    sys.path.insert(0, os.path.join(ROOT, "neptune-core_amd"))
    import numpy as np
    from neptune_hip import blocks as NB
    _, pool = bench.load_pool()
    proofs = [pool[h]["proof"] for h in sorted(pool)][:3] * 2
    buf = bench.tx_stream(proofs)
    pos, got = 0, []
    while pos < buf.size:
        tt = NB.TransferTransaction.from_bytes(buf[pos:])
        got.append(tt.proof.payload)
        pos += tt.size
    assert pos == buf.size and len(got) == len(proofs)
    for a, b in zip(got, proofs):
        assert np.array_equal(np.asarray(a, dtype=np.uint64), np.asarray(b, dtype=np.uint64))
