"""Item-stratified payload mutations at scale against the C restatement.

The random-word sweep of test_gpu_stark.py draws positions uniformly, so almost every mutant lands in
the revealed rows (the bulk of a proof).  Here every proof item of every padded height of the
config-3 pool -- Merkle roots, OOD rows, the padded-height word, authentication structures, revealed
main / aux / quotient rows, FRI codewords, the last polynomial and each FRI round's response -- gets
the same number of payload (non-structural) mutations: +1 mod p, + p (the same field element
written non-canonically: BFieldElement::new reads any u64 mod p, so the verdict must not change),
p - 1, and a random u64.  Whole items are also swapped with their neighbour, dropped and duplicated
(the stream order is the Fiat-Shamir order).  One device batch holds every mutant; each verdict
equals the C restatement's (oracle/stark_oracle.c), and the + p mutants of accepting proofs accept.
The same mutants then run again in one-stream batches of 32 (the fused small-batch launches).
"""
import json
import os

import numpy as np
import pytest

import stark_ref as S

pytestmark = pytest.mark.gpu
P = S.P
_DYN = {S.AUTH_STRUCTURE, S.MAIN_ROWS, S.AUX_ROWS, S.QUOT_SEGMENTS_ELEMENTS, S.FRI_CODEWORD, S.FRI_POLYNOMIAL}


def _items(w):
    """[(kind, item start, item end, payload positions)] of a well-formed proof stream; the item
    spans [start, end) include the item-length word."""
    out = []
    at = 2
    for _ in range(int(w[1])):
        ln = int(w[at])
        kind = int(w[at + 1])
        skip = {at, at + 1}
        if kind in _DYN:
            skip |= {at + 2, at + 3}
        elif kind == S.FRI_RESPONSE:
            b = at + 2
            lrl = int(w[b + 1])
            a = b + 2 + lrl
            skip |= {b, b + 1, b + 2, a, a + 1}
        pay = [p for p in range(at, at + 1 + ln) if p not in skip]
        out.append((kind, at, at + 1 + ln, pay))
        at += 1 + ln
    assert at == len(w)
    return out


def _restream(w, spans):
    """A proof stream made of the given item spans (each [len, disc, body...]) of w."""
    body = [np.asarray(w[a:b], dtype=np.uint64) for a, b in spans]
    n = np.uint64(len(spans))
    inner = np.concatenate([np.asarray([n], dtype=np.uint64)] + body)
    return np.concatenate([np.asarray([len(inner)], dtype=np.uint64), inner])


def _one_stream_chunks(ctx, NS, air_w, claims, proofs, size=32):
    air = NS.Air([int(w) for w in air_w])
    out = []
    b = None
    for s0 in range(0, len(proofs), size):
        cl = [NS.Claim(*c) for c in claims[s0:s0 + size]]
        pr = proofs[s0:s0 + size]
        if b is None:
            b = NS.Batch(ctx, air, NS.Stark.default(), cl, pr).set_streams(1)
        else:
            b.refill(cl, pr)
        v, _ = b.run()
        out += [bool(x) for x in v]
    b.close()
    return out


def test_item_stratified_payload_mutations_vs_c_oracle(ctx):
    import coracle as C
    import neptune_hip.stark as NS
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_pool.npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    air_w = z["air"]
    rng = np.random.default_rng(0x5EEB)
    claims, proofs, plus_p = [], [], []
    kinds_hit = set()
    for h in sorted(meta["heights"]):
        c = meta["claims"][str(h)]
        claim = (c["digest"], c["version"], c["input"], c["output"])
        proof = z[f"proof_{h}"]
        claims.append(claim)
        proofs.append(proof)
        items = _items(proof)
        for kind, _, _, pay in items:
            kinds_hit.add(kind)
            for pos in rng.choice(pay, size=min(6, len(pay)), replace=False):
                v = int(proof[pos])
                for new in ((v + 1) % P, (P - 1) if v != P - 1 else 0, int(rng.integers(0, 1 << 63)) * 2 + 1):
                    m = proof.copy()
                    m[pos] = np.uint64(new)
                    claims.append(claim)
                    proofs.append(m)
                if v + P < (1 << 64):
                    m = proof.copy()
                    m[pos] = np.uint64(v + P)
                    plus_p.append(len(proofs))
                    claims.append(claim)
                    proofs.append(m)
        spans = [(a, b) for _, a, b, _ in items]
        for i in range(len(spans)):
            rest = spans[:i] + spans[i + 1:]
            claims.append(claim)
            proofs.append(_restream(proof, rest))  # item i dropped
            claims.append(claim)
            proofs.append(_restream(proof, spans[:i + 1] + spans[i:]))  # item i duplicated
            if i + 1 < len(spans) and items[i][0] != items[i + 1][0]:
                sw = spans[:i] + [spans[i + 1], spans[i]] + spans[i + 2:]
                claims.append(claim)
                proofs.append(_restream(proof, sw))  # items i, i + 1 swapped
    assert len(kinds_hit) == 12, sorted(kinds_hit)  # every ProofItem kind carries mutations
    assert len(proofs) > 2000
    got = NS.verify_batch(ctx, NS.Air([int(w) for w in air_w]), NS.Stark.default(),
                          [(NS.Claim(*c), p) for c, p in zip(claims, proofs)])
    want = [bool(x) for x in C.stark_verify_batch(air_w, S.StarkParams(), claims, proofs, threads=16)]
    diff = [i for i in range(len(got)) if got[i] != want[i]]
    assert not diff, diff[:20]
    # the same proofs in one-stream batches of 32: the fused small-batch launches (replay + rows, plan +
    # FRI, roots + verdicts in one launch each) on the same mutants
    small = _one_stream_chunks(ctx, NS, air_w, claims, proofs)
    diff = [i for i in range(len(small)) if small[i] != want[i]]
    assert not diff, diff[:20]
    assert all(want[i] for i in plus_p)  # the same field elements, written non-canonically
    n_accept = sum(want)
    assert n_accept >= len(meta["heights"]) + len(plus_p)
    assert n_accept < len(proofs) // 2  # most value mutations reject
