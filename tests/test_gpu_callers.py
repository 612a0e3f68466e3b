"""GPU: the batched callers and ingestion formats end to end — claim hash / proof file name vs
the oracle, proof files written and read back then verified, and ProofCollection::verify over a
collection whose member proofs are proven (constant-codeword synthetic prover) for exactly the
claims the mirror builds."""
import os

import numpy as np
import pytest

import stark_prover_const as K
import stark_ref as S
import tip5_ref as T

pytestmark = pytest.mark.gpu


def _mods():
    from neptune_hip import proof_files as PF
    from neptune_hip import stark as NS
    from neptune_hip import verifier as V
    return PF, NS, V


def test_claim_hash_and_proof_file_name(ctx):
    PF, NS, _ = _mods()
    for claim in [([1, 2, 3, 4, 5], 0, [], []), ([P_ := (1 << 64) - (1 << 32), 7, 7, 7, 7], 0, list(range(30)), [5, 6])]:
        want = T.hash_varlen(S.encode_claim(*claim))
        got = PF.claim_hash(ctx, NS.Claim(*claim))
        assert list(got) == [int(x) for x in want]
        assert PF.proof_filename(ctx, NS.Claim(*claim)) == T.digest_to_hex([int(x) for x in want]) + ".proof"


def test_proof_file_roundtrip_then_verify(ctx, tmp_path):
    PF, NS, V = _mods()
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    claim = ([3, 1, 4, 1, 5], 0, [9, 2, 6], [5])
    proof, _ = K.prove(params, air, recipe, claim, 9, seed=3)
    path = os.path.join(tmp_path, PF.proof_filename(ctx, NS.Claim(*claim)))
    PF.save_proof(path, proof)
    loaded = PF.try_load_proof_from_disk(path)
    assert loaded.tolist() == list(proof)
    ver = V.Verifier(ctx, NS.Air(air.to_words()))
    assert ver.verify(NS.Claim(*claim), loaded) is True
    with open(path, "ab") as f:
        f.write(b"\x00" * 3)
    assert PF.try_load_proof_from_disk(path) is None


def test_proof_collection_verify_on_gpu(ctx):
    _, NS, V = _mods()
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    d = lambda k: [k, 2 * k, 3 * k, 4 * k, 5 * k]  # noqa: E731
    progs = V.ConsensusPrograms(d(1001), d(1002), d(1003), d(1004))
    pc = V.ProofCollection(
        removal_records_integrity=None, collect_lock_scripts=None, lock_scripts_halt=[None, None],
        kernel_to_outputs=None, collect_type_scripts=None, type_scripts_halt=[None],
        lock_script_hashes=[d(7), d(8)], type_script_hashes=[d(9)],
        kernel_mast_hash=d(11), salted_inputs_hash=d(12), salted_outputs_hash=d(13))
    # prove every member for exactly the claim the mirror builds (heights like a 2in/2out mix)
    pairs = pc.claims_and_proofs(progs)
    heights = [10, 12, 9, 11, 8, 8, 9]
    proofs = []
    for (c, _), h in zip(pairs, heights):
        p, _ = K.prove(params, air, recipe, (c.program_digest, c.version, c.input, c.output), h, seed=h)
        proofs.append(np.asarray(p, dtype=np.uint64))
    pc.removal_records_integrity, pc.kernel_to_outputs = proofs[0], proofs[1]
    pc.collect_lock_scripts, pc.collect_type_scripts = proofs[2], proofs[3]
    pc.lock_scripts_halt, pc.type_scripts_halt = [proofs[4], proofs[5]], [proofs[6]]
    ver = V.Verifier(ctx, NS.Air(air.to_words()))
    assert pc.verify(pc.kernel_mast_hash, ver, progs) is True
    assert pc.verify(d(99), ver, progs) is False  # other transaction kernel
    bad = V.ProofCollection(**{**pc.__dict__, "type_scripts_halt": [proofs[5]]})  # wrong proof for the claim
    swapped = V.ProofCollection(**{**pc.__dict__, "lock_script_hashes": [d(8), d(7)]})
    out = V.ProofCollection.verify_many([(pc, pc.kernel_mast_hash), (bad, bad.kernel_mast_hash),
                                         (swapped, swapped.kernel_mast_hash), (pc, pc.kernel_mast_hash)], ver, progs)
    assert out == [True, False, False, True]
    # the oracle agrees member by member
    assert all(S.verify(params, air, (c.program_digest, c.version, c.input, c.output), p)
               for (c, _), p in zip(pairs, proofs))


def test_transactions_and_blocks_on_gpu(ctx):
    """Transaction::is_valid (kernel MAST hash on the GPU, then the SingleProof claim) and
    Block::validate rules 1.a-1.d over a batch of blocks, with every proof made for exactly the
    claim the mirror builds; BlockProgram's claim output equals the oracle's claim hashes."""
    import mast_ref as M
    _, NS, V = _mods()
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    rng = np.random.default_rng(0x7B)
    d = lambda k: [k, 3 * k, 5 * k, 7 * k, 11 * k]  # noqa: E731
    progs = V.ConsensusPrograms(d(1001), d(1002), d(1003), d(1004), single_proof=d(1005), block_program=d(1006))
    ver = V.Verifier(ctx, NS.Air(air.to_words()))
    prove = lambda c, h, seed: np.asarray(  # noqa: E731
        K.prove(params, air, recipe, (c.program_digest, c.version, c.input, c.output), h, seed=seed)[0], dtype=np.uint64)
    # two transactions: kernel field encodings -> MAST hash -> SingleProof claim
    kernels = [[list(rng.integers(0, T.P, size=int(rng.integers(1, 12)), dtype=np.uint64)) for _ in range(8)]
               for _ in range(2)]
    txk = [M.mast_hash(k) for k in kernels]
    sp = [prove(V.single_proof_claim(h, progs), 9, seed=i + 1) for i, h in enumerate(txk)]
    items = [(kernels[0], V.TransactionProof(V.SINGLE_PROOF, sp[0])),
             (kernels[1], V.TransactionProof(V.SINGLE_PROOF, sp[1])),
             (kernels[1], V.TransactionProof(V.SINGLE_PROOF, sp[0]))]  # proof of the other kernel
    assert V.transactions_are_valid(ctx, items, ver, progs) == [True, True, False]
    # blocks: appendix = [transaction validity claim] (+ an extra claim), BlockProgram proof
    body = [list(rng.integers(0, T.P, size=5, dtype=np.uint64)) for _ in range(2)]
    appendix = [[V.single_proof_claim(txk[0], progs)],
                [V.single_proof_claim(txk[1], progs), NS.Claim(d(77), 0, [1, 2], [3])]]
    bclaims = [V.BlockProgram.claim(ctx, body[i], appendix[i], progs) for i in range(2)]
    for bc, app in zip(bclaims, appendix):
        want = [int(x) for c in app for x in T.hash_varlen(S.encode_claim(c.program_digest, c.version, c.input, c.output))]
        assert bc.output == want
    bproofs = [prove(bclaims[i], 10, seed=20 + i) for i in range(2)]
    blocks = [V.BlockToValidate(body[0], txk[0], appendix[0], V.SINGLE_PROOF, bproofs[0]),
              V.BlockToValidate(body[1], txk[1], appendix[1], V.SINGLE_PROOF, bproofs[1]),
              V.BlockToValidate(body[1], txk[1], appendix[1], V.SINGLE_PROOF, bproofs[0]),  # other block's proof
              V.BlockToValidate(body[0], txk[1], appendix[0], V.SINGLE_PROOF, bproofs[0]),  # claim missing
              V.BlockToValidate(body[0], txk[0], appendix[0], V.GENESIS, None)]
    assert V.validate_block_proofs(ctx, blocks, ver, progs) == [
        None, None, V.PROOF_VALIDITY, V.APPENDIX_MISSING_CLAIM, V.PROOF_QUALITY]
    assert all(S.verify(params, air, (c.program_digest, c.version, c.input, c.output), p)
               for c, p in zip(bclaims, bproofs))
