"""Per-member proof arenas (nhip_arena_*): wire bytes decoded straight into
pinned memory on each member GPU's NUMA node and verified through nhip_group_stream_submit_placed.

  * peer transactions (transfer_transaction.rs:31-47): a stream of SingleProof and ProofCollection
    TransferTransactions is decoded into a 3-member arena set (three contexts on GPU 0); every
    decoded proof equals the nhip_le_words / restatement decode word for word (values >= p reduced
    like BFieldElement::new), each proof lies inside its member's arena, the members' loads are
    balanced, and the placed batch's verdicts equal the C oracle's (one proof mutated);
  * a full arena stops before the transaction that does not fit (NHIP_OK, consumed < size); after a
    reset the stream continues where it stopped, and every proof is verified exactly once;
  * a malformed transaction fails with its position; the ones before it stay decoded;
  * blk files (import_blocks_from_files.rs:100-115): every SingleProof block proof lands in the arenas
    with its block index;
  * the bench's node leg in small: two arena sets, decode of batch k + 1 beside the upload of batch k.
Reference semantics per proof: triton_vm::verify at verifier.rs:60-63."""
import random

import numpy as np
import pytest

import bench
import bincode_ref as B
import coracle as C
import stark_ref as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pool():
    air_words, pool = bench.load_pool()
    hs = sorted(pool)
    claims = [pool[h]["claim"] for h in hs]
    proofs = [np.asarray(pool[h]["proof"], dtype=np.uint64) for h in hs]
    return [int(w) for w in air_words], claims, proofs, [pool[h]["main_rows"] for h in hs]


def _stream(proofs, g):
    """SingleProof txs for `proofs` plus one ProofCollection tx of small random proofs in the middle;
    returns (bytes, [(tx index, proof words)] in stream order, index of the collection's proofs)."""
    parts, order = [], []
    mid = len(proofs) // 2
    for i, p in enumerate(proofs):
        if i == mid:
            pc = {"removal_records_integrity": [g.randrange(B.P) for _ in range(33)],
                  "collect_lock_scripts": [B.P + 5, (1 << 64) - 1, 7],  # non-canonical: reduced mod p
                  "lock_scripts_halt": [[g.randrange(B.P) for _ in range(9)]], "kernel_to_outputs": [1, 2, 3],
                  "collect_type_scripts": [4], "type_scripts_halt": [],
                  "lock_script_hashes": [[1, 2, 3, 4, 5]], "type_script_hashes": [], "kernel_mast_hash": [0] * 5,
                  "salted_inputs_hash": [0] * 5, "salted_outputs_hash": [0] * 5, "merge_bit_mast_path": []}
            parts.append(B.encode_transfer_transaction({"kernel": B.random_kernel(g), "kind": B.TT_PROOF_COLLECTION,
                                                        "proof": pc}))
            for name in ("removal_records_integrity", "collect_lock_scripts"):
                order.append(("pc", [int(x) % B.P for x in pc[name]]))
            order.append(("pc", pc["lock_scripts_halt"][0]))
            for name in ("kernel_to_outputs", "collect_type_scripts"):
                order.append(("pc", pc[name]))
        parts.append(B.encode_transfer_transaction({"kernel": B.random_kernel(g), "kind": B.TT_SINGLE_PROOF,
                                                    "proof": [int(x) for x in p]}))
        order.append((i, [int(x) for x in p]))
    return b"".join(parts), order


def test_tx_stream_into_arenas_and_placed_verdicts(pool):
    import neptune_hip.stark as NS
    air_words, claims, proofs, main_rows = pool
    proofs = list(proofs) * 2  # 10 proofs of the 5 heights
    claims = list(claims) * 2
    bad = 3
    lo, hi = main_rows[bad % 5]
    proofs[bad] = proofs[bad].copy()
    proofs[bad][(lo + hi) // 2] = np.uint64((int(proofs[bad][(lo + hi) // 2]) + 1) % S.P)
    data, order = _stream(proofs, random.Random(11))
    gair = NS.Air(air_words)
    total = sum(len(p) for p in proofs) * 8
    with NS.Group([0, 0, 0]) as g, NS.Arena(g, total // 2) as a, NS.GroupStream(g, gair, NS.Stark.default()) as st:
        pl, ntx, used = a.ingest_txs(data)
        assert ntx == len(proofs) + 1 and used == len(data) and pl.n == len(order)
        for i, (_, words) in enumerate(order):
            assert pl.words(i).tolist() == words, i
        info = [a.member_info(m) for m in range(3)]
        assert sum(x["used_words"] for x in info) == sum(len(w) for _, w in order)
        members = pl.members()
        for i in range(pl.n):  # every proof inside its member's arena part
            assert members[i] in (0, 1, 2)
        loads = [x["used_words"] for x in info]
        assert max(loads) - min(loads) <= max(len(w) for _, w in order)
        # verify the SingleProof proofs, placed (skip the collection's random proofs)
        idx = [i for i, (k, _) in enumerate(order) if k != "pc"]
        sub = NS.Placed(len(idx))
        for j, i in enumerate(idx):
            sub.proofs[j] = pl.proofs[i]
            sub.member_of[j] = pl.member_of[i]
        sub.n = len(idx)
        cm = NS.marshal([NS.Claim(*claims[order[i][0]]) for i in idx], [[] for _ in idx])
        assert st.submit_placed(cm, sub) is None
        got, all_ok = st.finish()
    want = [bool(x) for x in C.stark_verify_batch(air_words, S.StarkParams(), claims, proofs, threads=8)]
    assert got == want and want.count(False) == 1 and not want[bad] and all_ok is False


def test_full_arena_stops_before_the_tx_then_continues(pool):
    import neptune_hip.stark as NS
    air_words, claims, proofs, _ = pool
    proofs = list(proofs) * 3
    claims = list(claims) * 3
    g0 = random.Random(5)
    data = b"".join(B.encode_transfer_transaction({"kernel": B.random_kernel(g0), "kind": B.TT_SINGLE_PROOF,
                                                   "proof": [int(x) for x in p]}) for p in proofs)
    gair = NS.Air(air_words)
    cap = max(len(p) for p in proofs) * 8 * 3  # about 3-4 proofs per member
    seen, verdicts = [], []
    view = memoryview(data)
    with NS.Group([0, 0]) as g, NS.Arena(g, cap) as a, NS.GroupStream(g, gair, NS.Stark.default()) as st:
        pos, rounds = 0, 0
        while pos < len(data):
            a.reset()
            pl, ntx, used = a.ingest_txs(view[pos:])
            assert ntx >= 1 and pl.n == ntx and (pos + used == len(data) or used < len(data) - pos)
            first = len(seen)
            seen += [pl.words(i).tolist() for i in range(pl.n)]
            cm = NS.marshal([NS.Claim(*claims[first + i]) for i in range(pl.n)], [[] for _ in range(pl.n)])
            r = st.submit_placed(cm, pl)
            r = st.finish()  # the arena is reset next round: its words must be on the GPU (they are after submit)
            verdicts += r[0]
            pos += used
            rounds += 1
        assert rounds >= 3
    assert seen == [[int(x) for x in p] for p in proofs]
    assert verdicts == [True] * len(proofs)


def test_malformed_tx_reports_its_position(pool):
    import neptune_hip.stark as NS
    _, _, proofs, _ = pool
    g0 = random.Random(8)
    good = [B.encode_transfer_transaction({"kernel": B.random_kernel(g0), "kind": B.TT_SINGLE_PROOF,
                                           "proof": [int(x) for x in p[:50]]}) for p in proofs[:3]]
    bad = bytearray(good[0])
    bad[-8 * 50 - 8 - 4:-8 * 50 - 8] = (7).to_bytes(4, "little")  # TransferTransactionProof variant 7
    data = good[0] + good[1] + bytes(bad) + good[2]
    with NS.Group([0]) as g, NS.Arena(g, 1 << 20) as a:
        with pytest.raises(ValueError, match="after 2 transactions"):
            a.ingest_txs(data)
        assert a.member_info(0)["used_words"] == 100  # the two before it


def test_blk_file_block_proofs_into_arenas():
    import neptune_hip.stark as NS
    g0 = random.Random(3)
    blks, want = [], []
    for i in range(6):
        kind = B.SINGLE_PROOF if i % 3 != 1 else B.GENESIS
        proof = [g0.randrange(B.P) for _ in range(g0.randrange(1, 300))] if kind == B.SINGLE_PROOF else None
        blks.append(B.random_block(g0, [], kind, proof, 10))
        if kind == B.SINGLE_PROOF:
            want.append((i, proof))
    data = b"".join(B.encode_block(b) for b in blks)
    with NS.Group([0, 0]) as g, NS.Arena(g, 1 << 20) as a:
        pl, block_of = a.ingest_blocks(data, 10)
        assert block_of == [i for i, _ in want]
        assert [pl.words(k).tolist() for k in range(pl.n)] == [p for _, p in want]


def test_node_leg_small(pool):
    """bench.node_from_bytes on 40 proofs over 2 members: every batch's verdicts correct."""
    air_words, claims, proofs, _ = pool
    cl, pr = list(claims) * 8, list(proofs) * 8
    r = bench.node_from_bytes([0, 0], air_words, cl, pr, np.ones(len(pr), dtype=bool), 3)
    assert r["verdicts_correct"] and r["value"] > 0 and r["batches"] == 3
