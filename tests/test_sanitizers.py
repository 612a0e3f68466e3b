"""The parsers of untrusted bytes under ASan + UBSan (host only): the proof-stream
walk shared by k_decode and nhip_proof_decodes (proof_codec.hpp), the bincode block-file and
TransferTransaction decoders (bincode.cpp) and the proof-file reader (ingest.cpp), each on valid
inputs, every truncation and seeded mutations (tests/native/parser_fuzz.cpp).  The build recipe is
tests/native/Makefile; a sanitizer report fails the run."""
import json
import os
import random
import shutil
import subprocess

import numpy as np
import pytest

import bincode_ref as B

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")


@pytest.fixture(scope="module")
def fuzz_bin(tmp_path_factory):
    if not shutil.which("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc absent")
    out = tmp_path_factory.mktemp("san")
    subprocess.check_call(["make", "-s", "-C", NATIVE, f"OUT={out}"])
    return os.path.join(out, "parser_fuzz")


def _write(path, data: bytes):
    with open(path, "wb") as f:
        f.write(data)
    return str(path)


def test_parsers_clean_under_asan_ubsan(fuzz_bin, tmp_path):
    args = []
    g = json.load(open(os.path.join(HERE, "golden", "stark_tiny.json")))
    for i, case in enumerate(g["cases"]):
        w = np.array([int(x) for x in case["proof"]], dtype=np.uint64)
        args.append("proof-tiny:" + _write(tmp_path / f"tiny{i}.bin", w.tobytes()))
    z = np.load(os.path.join(HERE, "golden", "c3_pool.npz"))
    args.append("proof-full:" + _write(tmp_path / "full9.bin", z["proof_9"].tobytes()))
    args.append("be:" + _write(tmp_path / "be.bin", z["proof_9"][:4096].astype(">u8").tobytes()))
    rng = random.Random(77)
    from test_blocks_host import H, _blocks, _proof_collection
    assert H == 10
    blk = b"".join(B.encode_block(b) for b in _blocks(3, 4))
    args.append("blk10:" + _write(tmp_path / "blk.dat", blk))
    for i, case in enumerate((
            {"kernel": B.random_kernel(rng), "kind": B.TT_SINGLE_PROOF, "proof": [rng.randrange(B.P) for _ in range(40)]},
            {"kernel": B.random_kernel(rng), "kind": B.TT_PROOF_COLLECTION, "proof": _proof_collection(rng, 2, 1, 3)})):
        args.append("tx:" + _write(tmp_path / f"tx{i}.bin", B.encode_transfer_transaction(case)))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([fuzz_bin, "3000"] + args, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    runs, ok, mismatch = (int(x) for x in r.stdout.split()[1::2])
    # mismatch: the arena ingest's scanner or its streaming decode disagreeing with nhip_tx_scan /
    # nhip_tx_parts / nhip_le_words on any (mutated) transaction
    assert runs > 20000 and ok > 0 and mismatch == 0, r.stdout


def test_queue_receive_ring_under_asan_ubsan(fuzz_bin):
    """The queue's pinned receive arena (pinned_ring.hpp): random takes and out-of-order releases,
    no live range overwritten or crossing the buffer end, the ring whole again at the end."""
    ring = os.path.join(os.path.dirname(fuzz_bin), "ring_check")
    for cap, iters in (("4096", "200000"), ("1000003", "50000")):
        out = subprocess.run([ring, cap, iters], capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "ring ok" in out.stdout
