"""GPU: block files and peer transactions end to end — a blk file of bincode blocks decoded
natively, kernel and body MAST hashes on the GPU (vs the oracle), rules 1.a-1.d with every
block proof made for exactly the BlockProgram claim the mirror builds; TransferTransactions
(SingleProof and ProofCollection) decoded and checked by Transaction::is_valid in one batch."""
import random

import numpy as np
import pytest

import bincode_ref as B
import mast_ref as M
import stark_prover_const as K
import stark_ref as S
import tip5_ref as T

pytestmark = pytest.mark.gpu
H = 10  # BlockPow tree height of the reference's test builds


def _setup(ctx):
    from neptune_hip import stark as NS
    from neptune_hip import verifier as V
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    d = lambda k: [k, 3 * k, 5 * k, 7 * k, 11 * k]  # noqa: E731
    progs = V.ConsensusPrograms(d(1001), d(1002), d(1003), d(1004), single_proof=d(1005), block_program=d(1006))
    ver = V.Verifier(ctx, NS.Air(air.to_words()))

    def prove(c, h, seed):
        return K.prove(params, air, recipe, (list(c.program_digest), c.version, list(c.input), list(c.output)),
                       h, seed=seed)[0]

    def oracle_accepts(c, proof):
        return S.verify(params, air, (list(c.program_digest), c.version, list(c.input), list(c.output)), proof)
    return NS, V, progs, ver, prove, oracle_accepts


def _cd(c):
    return {"program_digest": list(c.program_digest), "version": c.version, "input": list(c.input),
            "output": list(c.output)}


def test_block_file_validation(ctx, tmp_path):
    from neptune_hip import blocks as NB
    NS, V, progs, ver, prove, oracle_accepts = _setup(ctx)
    g = random.Random(0xB1)
    kernels = [B.random_kernel(g, 2, 2, 1), B.random_kernel(g, 1, 3, 0), B.random_kernel(g, 0, 1, 2)]
    txk = [M.mast_hash(B.kernel_mast_sequences(k)) for k in kernels]
    apps = [[V.single_proof_claim(txk[0], progs)],
            [V.single_proof_claim(txk[1], progs), NS.Claim([9, 8, 7, 6, 5], 0, [1, 2], [3])],
            [V.single_proof_claim(txk[2], progs)]]
    blks = [B.random_block(g, [_cd(c) for c in a], B.SINGLE_PROOF, [0], H, kernel=k) for a, k in zip(apps, kernels)]
    body = [M.mast_hash([list(h)] + B.body_tail_sequences(b["body"])) for h, b in zip(txk, blks)]
    bclaims = [V.BlockProgram.claim(ctx, body[i], apps[i], progs) for i in range(3)]
    proofs = [prove(bclaims[i], 9 + i % 2, seed=40 + i) for i in range(3)]
    blks[0]["proof"], blks[1]["proof"], blks[2]["proof"] = proofs[0], proofs[1], proofs[0]  # 2: another block's
    genesis = B.random_block(g, [_cd(apps[0][0])], B.GENESIS, None, H, kernel=kernels[0])
    path = tmp_path / "blk0.dat"
    path.write_bytes(b"".join(B.encode_block(b) for b in blks + [genesis]))
    recs = NB.blocks_from_file_without_record(str(path), H)
    tv = NB.blocks_to_validate(ctx, recs)
    assert [list(t.tx_kernel_mast_hash) for t in tv[:3]] == [list(h) for h in txk]
    assert [list(t.body_mast_hash) for t in tv[:3]] == [list(h) for h in body]
    out = NB.validate_block_file(ctx, str(path), ver, progs, pow_tree_height=H)
    assert out == [None, None, V.PROOF_VALIDITY, V.PROOF_QUALITY]
    # the same file with the block proofs decoded straight into a pinned arena on the GPU's node
    with NS.Group([0]) as grp, NS.Arena(grp, 32 << 20) as arena:
        out_a = NB.validate_block_file(ctx, str(path), ver, progs, pow_tree_height=H, arena=arena)
        assert arena.member_info(0)["used_words"] == sum(len(p) for p in (proofs[0], proofs[1], proofs[0]))
    assert out_a == out
    # the oracle accepts the two good block proofs for the same claims
    assert all(oracle_accepts(c, p) for c, p in zip(bclaims[:2], proofs[:2]))


def test_transfer_transactions_is_valid(ctx):
    from neptune_hip import blocks as NB
    NS, V, progs, ver, prove, oracle_accepts = _setup(ctx)
    g = random.Random(0x77)
    # SingleProof transactions
    k_sp = [B.random_kernel(g, 1, 2, 1), B.random_kernel(g, 2, 1, 0)]
    h_sp = [M.mast_hash(B.kernel_mast_sequences(k)) for k in k_sp]
    sp = [prove(V.single_proof_claim(h, progs), 9, seed=i + 1) for i, h in enumerate(h_sp)]
    txs = [{"kernel": k_sp[0], "kind": B.TT_SINGLE_PROOF, "proof": sp[0]},
           {"kernel": k_sp[1], "kind": B.TT_SINGLE_PROOF, "proof": sp[1]},
           {"kernel": k_sp[1], "kind": B.TT_SINGLE_PROOF, "proof": sp[0]}]  # other kernel's proof
    # a ProofCollection transaction, every member proven for the mirror's claim
    k_pc = B.random_kernel(g, 1, 1, 0)
    h_pc = M.mast_hash(B.kernel_mast_sequences(k_pc))
    dg = lambda k: [k, k + 1, k + 2, k + 3, k + 4]  # noqa: E731
    shell = V.ProofCollection(None, None, [None], None, None, [], [dg(70)], [], list(h_pc), dg(80), dg(90))
    members = [prove(c, 8 + i % 2, seed=100 + i) for i, (c, _) in enumerate(shell.claims_and_proofs(progs))]
    # claims_and_proofs order: rri, k2o, cls, cts, lock scripts -> proof_collection.rs field order
    pc = {"removal_records_integrity": members[0], "collect_lock_scripts": members[2],
          "lock_scripts_halt": [members[4]], "kernel_to_outputs": members[1], "collect_type_scripts": members[3],
          "type_scripts_halt": [], "lock_script_hashes": [dg(70)], "type_script_hashes": [],
          "kernel_mast_hash": list(h_pc), "salted_inputs_hash": dg(80), "salted_outputs_hash": dg(90),
          "merge_bit_mast_path": [dg(5)]}
    txs.append({"kernel": k_pc, "kind": B.TT_PROOF_COLLECTION, "proof": pc})
    bad_pc = dict(pc, lock_script_hashes=[dg(71)])  # a lock script claim the member proof is not for
    txs.append({"kernel": k_pc, "kind": B.TT_PROOF_COLLECTION, "proof": bad_pc})
    decoded = [NB.TransferTransaction.from_bytes(B.encode_transfer_transaction(t)) for t in txs]
    items = [(tt.kernel_sequences, tt.proof) for tt in decoded]
    assert V.transactions_are_valid(ctx, items, ver, progs) == [True, True, False, True, False]
    # member proofs decoded straight into a pinned arena (two members: each proof on the lighter one)
    with NS.Group([0, 0]) as grp, NS.Arena(grp, 16 << 20) as arena:
        dec_a = [NB.TransferTransaction.from_bytes(B.encode_transfer_transaction(t), arena=arena) for t in txs]
        items_a = [(tt.kernel_sequences, tt.proof) for tt in dec_a]
        assert V.transactions_are_valid(ctx, items_a, ver, progs) == [True, True, False, True, False]
        assert min(arena.member_info(m)["used_words"] for m in range(2)) > 0
