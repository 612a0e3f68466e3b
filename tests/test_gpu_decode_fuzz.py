"""Adversarial proof streams on the device decoder (k_decode, proof_codec.hpp): a peer controls
every word of a proof (neptune-core decodes peer transactions and blocks, verifier.rs:60-63), so
every STRUCTURAL word of full-size proofs -- the stream length, the item count, each item's length
and discriminant, the dynamic items' body lengths and element counts, the FRI response's nested
lengths -- is set to boundary values (0, 1, 2, v - 1, v + 1, 2^31, 2^32 - 1, 2^32, 2^63, p - 1,
2^64 - 1, which reads as 2^32 - 2 mod p).  One batch holds every mutant: the batch completes (no
device fault), each verdict equals the C restatement's (oracle/stark_oracle.c), and the device's
FAIL_DECODE bit equals the host walk of the same codec (nhip_proof_decodes)."""
import os

import numpy as np
import pytest

import stark_ref as S

pytestmark = pytest.mark.gpu
FAIL_DECODE = 1
P = S.P

# ProofItem discriminants (stark_ref.py; the public triton-vm ProofItem order)
_DYN = {S.AUTH_STRUCTURE, S.MAIN_ROWS, S.AUX_ROWS, S.QUOT_SEGMENTS_ELEMENTS, S.FRI_CODEWORD, S.FRI_POLYNOMIAL}


def _structural_positions(w):
    """Word positions of every length / count / discriminant of a well-formed proof stream."""
    pos = [0, 1]
    n_items = int(w[1])
    at = 2
    for _ in range(n_items):
        ln = int(w[at])
        pos += [at, at + 1]  # item length, discriminant
        kind = int(w[at + 1])
        if kind in _DYN:
            pos += [at + 2, at + 3]  # body length, element count
        elif kind == S.FRI_RESPONSE:
            b = at + 2
            pos += [b]  # body length
            lrl = int(w[b + 1])
            pos += [b + 1, b + 2]  # revealed-leaf list length, leaf count
            a = b + 2 + lrl
            pos += [a, a + 1]  # authentication list length, digest count
        at += 1 + ln
    assert at == len(w), "pool proof is not a well-formed stream"
    return pos


def _boundary_values(v):
    return sorted({0, 1, 2, (v - 1) % (1 << 64), (v + 1) % (1 << 64), 1 << 31, (1 << 32) - 1, 1 << 32, 1 << 63, P - 1,
                   (1 << 64) - 1} - {v})


def test_structural_word_fuzz_device_decoder(ctx):
    import coracle as C
    import neptune_hip.stark as NS
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_pool.npz"))
    import json
    meta = json.loads(bytes(z["meta"]).decode())
    air_w = z["air"]
    claims, proofs = [], []
    for h in sorted(meta["heights"])[:2]:  # the two smallest padded heights: ~1.3k mutants each
        c = meta["claims"][str(h)]
        claim = (c["digest"], c["version"], c["input"], c["output"])
        proof = z[f"proof_{h}"]
        claims.append(claim)
        proofs.append(proof)
        for p in _structural_positions(proof):
            for v in _boundary_values(int(proof[p])):
                m = proof.copy()
                m[p] = np.uint64(v)
                claims.append(claim)
                proofs.append(m)
    assert len(proofs) > 1000
    air = NS.Air([int(w) for w in air_w])
    stark = NS.Stark.default()
    nclaims = [NS.Claim(*c) for c in claims]
    b = NS.Batch(ctx, air, stark, nclaims, proofs)
    got, _ = b.run()
    want = C.stark_verify_batch(air_w, S.StarkParams(), claims, proofs, threads=16)
    assert [bool(x) for x in got] == [bool(x) for x in want]
    n_decode_fail = 0
    for i, (c, p) in enumerate(zip(nclaims, proofs)):
        _, _, fail = b.transcript(i, max_xfe=1)
        host = NS.proof_decodes(air, stark, c, p)
        assert (fail & FAIL_DECODE == 0) == host, i
        n_decode_fail += 0 if host else 1
    b.close()
    assert bool(got[0]) and n_decode_fail > len(proofs) // 2  # clean proofs accept; most mutants fail to decode
    # the same mutants in one-stream batches of 32 (the fused small-batch launches must skip every
    # proof that failed to decode, whatever its neighbours in the launch)
    from test_gpu_payload_sweep import _one_stream_chunks
    small = _one_stream_chunks(ctx, NS, air_w, claims, proofs)
    assert small == [bool(x) for x in want]
