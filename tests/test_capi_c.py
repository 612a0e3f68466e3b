"""The C ABI from C: neptune-core_amd/tools/abi_c_check.c is built as C99 with -pedantic -Werror
against include/neptune_hip.h and linked to libneptune_hip.so (make target build/abi_c_check),
then driven the way a non-Python host (the Rust binding of INTEGRATION.md) would.
CPU: the host-only entry points, and nhip_init without a GPU is an error code (no fallback).
GPU: verify_batch on one context and group_verify_batch over every GPU give the Python binding's
verdicts on the tiny golden proofs and mutations of them."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "neptune-core_amd")
EXE = os.path.join(PKG, "build", "abi_c_check")
GOLD = os.path.join(ROOT, "tests", "golden", "stark_tiny.json")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except ImportError:
        return False


def test_c_consumer_builds_and_host_entry_points():
    subprocess.check_call(["make", "-s", "-C", PKG, "build/abi_c_check"])
    out = subprocess.run([EXE, "host"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "host ok" in out.stdout
    if not _has_gpu():
        assert "init 1" in out.stdout  # NHIP_ERR_NO_DEVICE


def test_c_consumer_marshal_timing():
    """The harness times handing proofs over in both input forms (round 3's per-word canonical
    conversion + copy vs the Montgomery words as they lie); small here, 4,096 proofs on the GPU box."""
    subprocess.check_call(["make", "-s", "-C", PKG, "build/abi_c_check"])
    out = subprocess.run([EXE, "marshal", "64", "20000"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    tag, canon_ms, mont_ms, nbytes, _ = out.stdout.split()
    assert tag == "marshal" and int(nbytes) == 64 * 20000 * 8
    assert float(canon_ms) > float(mont_ms) >= 0


def _batch_file(path, air, stark, cases):
    w = [len(air)] + list(air)
    w += [stark.security_level, stark.log2_fri_expansion, stark.num_collinearity_checks, stark.num_main,
          stark.num_aux, stark.num_quotient_segments, len(cases)]
    for (digest, version, inp, outp), proof in cases:
        w += list(digest) + [version, len(inp)] + list(inp) + [len(outp)] + list(outp) + [len(proof)] + list(proof)
    np.asarray(w, dtype=np.uint64).tofile(path)


@pytest.mark.gpu
def test_c_consumer_verifies_like_the_python_binding(ctx, tmp_path):
    import neptune_hip.stark as NS
    assert os.path.exists(EXE), "build/abi_c_check missing: run make -C neptune-core_amd (build())"
    g = json.load(open(GOLD))
    air = [int(x) for x in g["air"]]
    stark = NS.Stark(num_collinearity_checks=8, num_main=24, num_aux=9)
    cases = []
    rng = np.random.default_rng(0xCC)
    for c in g["cases"]:
        claim = (c["claim"]["digest"], c["claim"]["version"], c["claim"]["input"], c["claim"]["output"])
        proof = [int(x) for x in c["proof"]]
        cases.append((claim, proof))
        m = list(proof)
        pos = int(rng.integers(len(m) // 4, len(m)))
        m[pos] = (m[pos] + 1) % 0xFFFFFFFF00000001
        cases.append((claim, m))
    cases.append((cases[0][0], []))  # empty proof: reject, never an error
    path = str(tmp_path / "batch.bin")
    _batch_file(path, air, stark, cases)
    want = NS.verify_batch(ctx, NS.Air(air), stark, [(NS.Claim(*c), p) for c, p in cases])
    s = "".join("1" if x else "0" for x in want)
    out = subprocess.run([EXE, "verify", path], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = dict(l.split(" ", 1) for l in out.stdout.strip().splitlines())
    assert lines["ctx"] == s
    gv, ok, members = lines["group"].split()
    assert gv == s and int(ok) == int(all(want)) and int(members) >= 1
    assert want[0] and not want[-1]
