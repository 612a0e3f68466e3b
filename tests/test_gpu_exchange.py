"""The verdict exchange's RCCL form on the GPU: shard.VerdictExchange over the "nccl" backend
(RCCL) posts all_gather_into_tensor on device buffers with async_op and completes it one step
later.  A one-GPU box holds one rank (RCCL refuses two ranks on one device), so this is world size
1 in a child process: it runs the device-buffer path bench.py takes for N > 1 (the gather of
several ranks is covered with gloo in test_multirank.py)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.path.join(sys.argv[1], "neptune-core_amd"))
from neptune_hip import shard
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + sys.argv[2], rank=0, world_size=1)
n = 300
shards = [list(range(n))]
steps = []
for k in range(9):
    v = np.ones(n, dtype=np.uint8)
    v[(17 * k) % n] = 0
    if k == 4:
        v[:] = 1
    steps.append(v)
for depth in (2, 4):  # bench.py posts 4 deep (pinned staging, on-stream copies, one event per slot)
    ex = shard.VerdictExchange(shards, n, dist, depth=depth)
    assert ex.flat and ex.dev.type == "cuda"
    got = []
    for v in steps:
        ex.post(bool(v.all()), v)
        if len(ex.pending) >= depth:
            got.append(ex.complete())
    while ex.pending:
        got.append(ex.complete())
    assert len(got) == len(steps)
    for (ok, full), v in zip(got, steps):
        assert ok == bool(v.all()) and (full == v).all()
dist.destroy_process_group()
print("exchange ok")
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_verdict_exchange_rccl_device_buffers():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(_free_port())], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "exchange ok" in r.stdout
