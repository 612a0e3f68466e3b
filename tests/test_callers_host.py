"""Host-side mirrors of the verification callers and ingestion formats (no GPU):
proof files (program.rs:374-390), the mock-proof gate (verifier.rs:44-74), and the claims of
ProofCollection::verify (proof_collection.rs:273-389)."""
import numpy as np
import pytest

from neptune_hip import proof_files as PF
from neptune_hip import verifier as V
from neptune_hip.stark import Claim

P = (1 << 64) - (1 << 32) + 1


def test_proof_file_bytes_roundtrip_and_reduction():
    words = [0, 1, P - 1, 2 ** 63, 123456789]
    data = PF.proof_to_be_bytes(words)
    assert len(data) == 40 and data[8:16] == (1).to_bytes(8, "big")
    assert PF.proof_from_be_bytes(data).tolist() == words
    # BFieldElement::new reduces non-canonical words; the writer emits value()
    raw = (P + 5).to_bytes(8, "big") + (2 ** 64 - 1).to_bytes(8, "big")
    assert PF.proof_from_be_bytes(raw).tolist() == [5, 2 ** 64 - 1 - P]
    assert PF.proof_from_be_bytes(b"").tolist() == []
    assert PF.proof_from_be_bytes(data + b"\x01\x02") is None  # trailing partial chunk -> None


def test_proof_file_save_load(tmp_path):
    rng = np.random.default_rng(1)
    w = rng.integers(0, P, size=1000, dtype=np.uint64)
    path = str(tmp_path / "x.proof")
    PF.save_proof(path, w)
    assert (PF.try_load_proof_from_disk(path) == w).all()
    assert PF.try_load_proof_from_disk(str(tmp_path / "missing.proof")) is None


def _collection(n_lock=2, n_type=1):
    d = lambda k: [k, k + 1, k + 2, k + 3, k + 4]  # noqa: E731
    return V.ProofCollection(
        removal_records_integrity=[0], collect_lock_scripts=[0], lock_scripts_halt=[[0]] * n_lock,
        kernel_to_outputs=[0], collect_type_scripts=[0], type_scripts_halt=[[0]] * n_type,
        lock_script_hashes=[d(100 + 10 * i) for i in range(n_lock)], type_script_hashes=[d(200)] * n_type,
        kernel_mast_hash=d(1), salted_inputs_hash=d(11), salted_outputs_hash=d(21))


PROGS = V.ConsensusPrograms([1] * 5, [2] * 5, [3] * 5, [4] * 5)


def test_proof_collection_claims_follow_the_reference():
    pc = _collection()
    assert pc.num_proofs() == 4 + 2 + 1
    pairs = pc.claims_and_proofs(PROGS)
    cl = [c for c, _ in pairs]
    rev = lambda k: [k + 4, k + 3, k + 2, k + 1, k]  # noqa: E731
    assert (cl[0].program_digest, cl[0].input, cl[0].output) == ([1] * 5, rev(1), [11, 12, 13, 14, 15])
    assert (cl[1].program_digest, cl[1].input, cl[1].output) == ([2] * 5, rev(1), [21, 22, 23, 24, 25])
    assert (cl[2].input, cl[2].output) == (rev(11), list(range(100, 105)) + list(range(110, 115)))
    assert (cl[3].input, cl[3].output) == (rev(11) + rev(21), list(range(200, 205)))
    assert [(c.program_digest, c.input, c.output) for c in cl[4:6]] == [
        (list(range(100, 105)), rev(1), []), (list(range(110, 115)), rev(1), [])]
    assert (cl[6].program_digest, cl[6].input) == (list(range(200, 205)), rev(1) + rev(11) + rev(21))
    # zip truncation: a missing halting proof drops the claim, as Iterator::zip does
    pc.lock_scripts_halt = [[0]]
    assert len(pc.claims_and_proofs(PROGS)) == 6


def test_mock_network_gate_never_runs_the_verifier():
    ver = V.Verifier(ctx=None, air=None, stark=V.Stark())
    pairs = [(Claim([0] * 5), [0]), (Claim([0] * 5), [1]), (Claim([0] * 5), [0, 0]), (Claim([0] * 5), [])]
    assert ver.verify_batch(pairs, V.Network.REGTEST) == [True, False, False, False]
    assert ver.verify_batch(pairs, V.Network.TESTNET_MOCK) == [True, False, False, False]
    good, bad = _collection(), _collection()
    bad.collect_type_scripts = [1]
    out = V.ProofCollection.verify_many([(good, good.kernel_mast_hash), (bad, bad.kernel_mast_hash),
                                         (good, [9] * 5)], ver, PROGS, V.Network.REGTEST)
    assert out == [True, False, False]
    with pytest.raises(AttributeError):
        ver.verify_batch(pairs, V.Network.MAIN)  # a real network needs a GPU context


PROGS6 = V.ConsensusPrograms([1] * 5, [2] * 5, [3] * 5, [4] * 5, single_proof=[5] * 5, block_program=[6] * 5)


def test_single_proof_claim_and_transaction_dispatch_mock():
    txk = [10, 11, 12, 13, 14]
    c = V.single_proof_claim(txk, PROGS6)
    assert (c.program_digest, c.version, c.input, c.output) == ([5] * 5, 0, [14, 13, 12, 11, 10], [])
    ver = V.Verifier(ctx=None, air=None, stark=V.Stark())
    pc = _collection()
    items = [(V.TransactionProof(V.SINGLE_PROOF, [0]), txk), (V.TransactionProof(V.SINGLE_PROOF, [1]), txk),
             (V.TransactionProof(V.PROOF_COLLECTION, pc), pc.kernel_mast_hash),
             (V.TransactionProof(V.PROOF_COLLECTION, pc), txk)]  # collection of another kernel
    assert V.TransactionProof.verify_many(items, ver, PROGS6, V.Network.REGTEST) == [True, False, True, False]
    with pytest.raises(ValueError):
        V.TransactionProof.verify_many([(V.TransactionProof(V.WITNESS, None), txk)], ver, PROGS6, V.Network.REGTEST)


def test_block_rules_1a_to_1d_in_reference_order_mock():
    ver = V.Verifier(ctx=None, air=None, stark=V.Stark())
    txk, body = [1, 2, 3, 4, 5], [7, 7, 7, 7, 8]
    tx_claim = V.single_proof_claim(txk, PROGS6)
    other = Claim([9] * 5, 0, [], [])

    def blk(appendix, kind=V.SINGLE_PROOF, proof=(0,)):
        return V.BlockToValidate(body, txk, appendix, kind, list(proof))

    blocks = [blk([tx_claim]),                                  # valid (mock)
              blk([other]),                                     # 1.a missing consensus claim
              blk([other] * 500 + [tx_claim]),                  # 1.b more than MAX_NUM_CLAIMS
              blk([tx_claim], kind=V.GENESIS, proof=()),        # 1.c not a SingleProof
              blk([tx_claim], proof=(1,)),                      # 1.d invalid mock
              blk([other, tx_claim]),                           # extra claims are fine
              blk([Claim(tx_claim.program_digest, 0, tx_claim.input[::-1], [])])]  # un-reversed input
    assert V.validate_block_proofs(None, blocks, ver, PROGS6, V.Network.REGTEST) == [
        None, V.APPENDIX_MISSING_CLAIM, V.APPENDIX_TOO_LARGE, V.PROOF_QUALITY, V.PROOF_VALIDITY, None,
        V.APPENDIX_MISSING_CLAIM]
