"""CPU: the native bincode decoder (csrc/bincode.cpp, through neptune_hip.blocks) against the
restatement (oracle/bincode_ref.py) on synthetic block files and peer transactions — every
field the verifier reads, the BFieldCodec MAST sequences, and the reference's error behaviour
(`bincode::deserialize(..)?` fails the file) on truncated and corrupted inputs.  Parity with real
neptune-core block files is unpinned: none ship with the reference."""
import random
import struct

import numpy as np
import pytest

import bincode_ref as B

H = 10   # BlockPow tree height of the reference's test builds (pow.rs:34-35); 29 is tested once


def _claim(g, n_in, n_out):
    return {"program_digest": [g.randrange(B.P) for _ in range(5)], "version": g.getrandbits(32),
            "input": [g.randrange(B.P) for _ in range(n_in)], "output": [g.randrange(B.P) for _ in range(n_out)]}


def _blocks(seed, n, tree_height=H):
    g = random.Random(seed)
    out = []
    for i in range(n):
        kind = [B.SINGLE_PROOF, B.GENESIS, B.INVALID][i % 3] if i else B.SINGLE_PROOF
        app = [_claim(g, g.randrange(6), g.randrange(3)) for _ in range(g.randrange(4))]
        proof = [g.randrange(B.P) for _ in range(g.randrange(1, 200))]
        out.append(B.random_block(g, app, kind, proof, tree_height))
    return out


def _check_record(rec, blk, want):
    assert rec.offset == want["offset"] and rec.size == want["size"]
    assert rec.height == blk["header"]["height"] and rec.timestamp == blk["header"]["timestamp"]
    assert list(rec.prev_block_digest) == blk["header"]["prev_block_digest"]
    assert [s.tolist() for s in rec.kernel_sequences] == B.kernel_mast_sequences(blk["body"]["transaction_kernel"])
    assert [s.tolist() for s in rec.body_tail_sequences] == B.body_tail_sequences(blk["body"])
    assert [(list(c.program_digest), c.version, list(c.input), list(c.output)) for c in rec.appendix] == [
        (c["program_digest"], c["version"], c["input"], c["output"]) for c in blk["appendix"]]
    assert rec.proof_kind == blk["proof_kind"]
    if blk["proof_kind"] == B.SINGLE_PROOF:
        assert rec.proof.tolist() == blk["proof"]
    else:
        assert rec.proof is None


def test_block_file_matches_restatement(tmp_path):
    from neptune_hip import blocks as NB
    blks = _blocks(1, 7)
    data = b"".join(B.encode_block(b) for b in blks)
    want = B.blocks_from_file(data, H)
    assert len(want) == len(blks)
    path = tmp_path / "blk0.dat"
    path.write_bytes(data)
    recs = NB.blocks_from_file_without_record(str(path), H)
    assert len(recs) == len(blks)
    for rec, blk, w in zip(recs, blks, want):
        _check_record(rec, blk, w)
    # the restatement's decoder reads back what its encoder wrote
    for blk, w in zip(blks, want):
        assert {k: w[k] for k in blk} == blk


def test_production_pow_height_and_empty_file(tmp_path):
    from neptune_hip import blocks as NB
    blks = _blocks(2, 2, tree_height=B.POW_TREE_HEIGHT)
    data = b"".join(B.encode_block(b) for b in blks)
    recs = NB.blocks_from_bytes(data)  # default height 29
    for rec, blk, w in zip(recs, blks, B.blocks_from_file(data)):
        _check_record(rec, blk, w)
    (tmp_path / "empty.dat").write_bytes(b"")
    assert NB.blocks_from_file_without_record(str(tmp_path / "empty.dat")) == []
    # the wrong tree height misreads the header: it must fail, not return garbage silently
    with pytest.raises(NB.BlockFileError):
        NB.blocks_from_bytes(data, H)


def test_kernel_edge_cases():
    """Empty vectors, Option None / Some, negative fee (i128), announcements of length 0,
    removal records with and without chunks; BFE words >= p reduced as BFieldElement::new."""
    from neptune_hip import blocks as NB
    g = random.Random(3)
    kernels = [B.random_kernel(g, 0, 0, 0), B.random_kernel(g, 3, 2, 2)]
    kernels[0]["coinbase"], kernels[0]["fee"] = None, -5
    kernels[1]["coinbase"], kernels[1]["announcements"][0] = (1 << 100) + 7, []
    blks = [B.random_block(g, [], B.GENESIS, None, H, kernel=k) for k in kernels]
    data = bytearray(b"".join(B.encode_block(b) for b in blks))
    recs = NB.blocks_from_bytes(bytes(data), H)
    for rec, blk, w in zip(recs, blks, B.blocks_from_file(bytes(data), H)):
        _check_record(rec, blk, w)
    # timestamp word (offset 8 + 8 + 40) written as p + 5 -> reads 5
    struct.pack_into("<Q", data, 56, B.P + 5)
    assert NB.blocks_from_bytes(bytes(data), H)[0].timestamp == 5


def test_malformed_files_fail_like_bincode():
    from neptune_hip import blocks as NB
    blks = _blocks(4, 3)
    enc = [B.encode_block(b) for b in blks]
    data = b"".join(enc)
    # truncated inside the last block: the first two decode, then the file fails
    for cut in (1, 9, len(enc[2]) // 2, len(enc[2]) - 1):
        with pytest.raises(NB.BlockFileError) as e:
            NB.blocks_from_bytes(data[:-cut], H)
        assert e.value.n_good == 2
    with pytest.raises(B.DecodeError):
        B.blocks_from_file(data[:-1], H)
    # an invalid BlockProof variant (the last 4 + 8 + 8 * len bytes of a SingleProof block)
    b0 = bytearray(enc[0])
    n_words = len(blks[0]["proof"])
    struct.pack_into("<I", b0, len(b0) - 8 * n_words - 8 - 4, 3)
    with pytest.raises(NB.BlockFileError):
        NB.blocks_from_bytes(bytes(b0), H)
    with pytest.raises(B.DecodeError):
        B.blocks_from_file(bytes(b0), H)
    # a huge sequence length (the proof's) is rejected without allocating or reading past the end
    b0 = bytearray(enc[0])
    struct.pack_into("<Q", b0, len(b0) - 8 * n_words - 8, 1 << 60)
    with pytest.raises(NB.BlockFileError):
        NB.blocks_from_bytes(bytes(b0), H)


def test_corrupt_bool_and_option_tags():
    from neptune_hip import blocks as NB
    g = random.Random(5)
    k = B.random_kernel(g, 0, 0, 0)
    k["coinbase"], k["merge_bit"] = None, True
    blk = B.random_block(g, [], B.INVALID, None, H, kernel=k)
    enc = bytearray(B.encode_block(blk))
    # kernel layout with no inputs/outputs/announcements: 3 x u64 0, fee 16, Option tag 1,
    # timestamp 8, digest 40, merge_bit 1
    ko = 8 + 8 + 40 + 8 + 40 * (2 * H + 2) + 24 + 20 + 80
    assert NB.blocks_from_bytes(bytes(enc), H)[0].kernel_sequences[7].tolist() == [1]
    tag, mb = ko + 24 + 16, ko + 24 + 16 + 1 + 8 + 40
    for pos, bad in ((tag, 2), (mb, 2)):
        e = bytearray(enc)
        e[pos] = bad
        with pytest.raises(NB.BlockFileError):
            NB.blocks_from_bytes(bytes(e), H)
        with pytest.raises(B.DecodeError):
            B.blocks_from_file(bytes(e), H)


def _proof_collection(g, nl, nt, nmerge):
    pr = lambda: [g.randrange(B.P) for _ in range(g.randrange(1, 40))]  # noqa: E731
    dg = lambda: [g.randrange(B.P) for _ in range(5)]  # noqa: E731
    return {"removal_records_integrity": pr(), "collect_lock_scripts": pr(),
            "lock_scripts_halt": [pr() for _ in range(nl)], "kernel_to_outputs": pr(), "collect_type_scripts": pr(),
            "type_scripts_halt": [pr() for _ in range(nt)], "lock_script_hashes": [dg() for _ in range(nl)],
            "type_script_hashes": [dg() for _ in range(nt)], "kernel_mast_hash": dg(), "salted_inputs_hash": dg(),
            "salted_outputs_hash": dg(), "merge_bit_mast_path": [dg() for _ in range(nmerge)]}


def test_transfer_transactions_match_restatement():
    from neptune_hip import blocks as NB
    from neptune_hip import verifier as V
    g = random.Random(6)
    single = {"kernel": B.random_kernel(g), "kind": B.TT_SINGLE_PROOF, "proof": [g.randrange(B.P) for _ in range(77)]}
    for case in (single, {"kernel": B.random_kernel(g), "kind": B.TT_PROOF_COLLECTION,
                          "proof": _proof_collection(g, 2, 1, 3)},
                 {"kernel": B.random_kernel(g, 0, 0, 0), "kind": B.TT_PROOF_COLLECTION,
                  "proof": _proof_collection(g, 0, 0, 0)}):
        data = B.encode_transfer_transaction(case)
        want = B.decode_transfer_transaction(data + b"\x00trailing")
        assert want["size"] == len(data)
        tt = NB.TransferTransaction.from_bytes(data)
        assert tt.size == len(data)
        assert [s.tolist() for s in tt.kernel_sequences] == B.kernel_mast_sequences(case["kernel"])
        if case["kind"] == B.TT_SINGLE_PROOF:
            assert tt.proof.kind == V.SINGLE_PROOF and tt.proof.payload.tolist() == case["proof"]
            continue
        pc, w = tt.proof.payload, case["proof"]
        assert tt.proof.kind == V.PROOF_COLLECTION
        for name in ("removal_records_integrity", "collect_lock_scripts", "kernel_to_outputs", "collect_type_scripts"):
            assert getattr(pc, name).tolist() == w[name]
        for name in ("lock_scripts_halt", "type_scripts_halt"):
            assert [p.tolist() for p in getattr(pc, name)] == w[name]
        for name in ("lock_script_hashes", "type_script_hashes", "merge_bit_mast_path"):
            assert [list(d) for d in getattr(pc, name)] == w[name]
        for name in ("kernel_mast_hash", "salted_inputs_hash", "salted_outputs_hash"):
            assert list(getattr(pc, name)) == w[name]
        assert pc.num_proofs() == 4 + len(w["lock_scripts_halt"]) + len(w["type_scripts_halt"])
        for cut in (1, len(data) // 3):
            with pytest.raises(ValueError):
                NB.TransferTransaction.from_bytes(data[:-cut])
    bad = bytearray(B.encode_transfer_transaction(single))
    struct.pack_into("<I", bad, len(bad) - 8 * 77 - 8 - 4, 2)  # TransferTransactionProof has 2 variants
    with pytest.raises(ValueError):
        NB.TransferTransaction.from_bytes(bytes(bad))


def test_le_words_alignment():
    from neptune_hip import _lib
    lib = _lib.load()
    raw = bytes([0xAB]) + struct.pack("<3Q", 1, B.P, (1 << 64) - 1)
    a = np.frombuffer(raw, dtype=np.uint8)
    out = np.zeros(3, dtype=np.uint64)
    assert lib.nhip_le_words(a.ctypes.data, len(raw), 1, 3, out.ctypes.data) == 0
    assert out.tolist() == [1, 0, (1 << 64) - 1 - B.P]
    assert lib.nhip_le_words(a.ctypes.data, len(raw), 2, 3, out.ctypes.data) == _lib.NHIP_ERR_ARG
