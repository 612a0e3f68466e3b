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
