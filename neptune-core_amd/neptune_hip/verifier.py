"""Host mirror of neptune-core's verification callers, batched over the GPU verifier.

* `verify(claim, proof, network)` — neptune-core/src/protocol/proof_abstractions/verifier.rs:44-74:
  on networks that use mock proofs (RegTest, TestnetMock; application/config/network.rs:61-63) the
  verdict is `proof.is_valid_mock()` (a proof equal to the encoding of MockProofBehavior::ValidMock,
  `[0]`; neptune_proof.rs:18-21,172-187) and the verifier never runs; otherwise
  `triton_vm::verify(Stark::default(), claim, proof)`, here `nhip_verify_batch`.
* `verify_batch(pairs, network)` — the same per pair, all real verifications in one GPU batch.
* `ProofCollection.verify(txk_mast_hash, ...)` — proof_collection.rs:273-389: the kernel-hash gate,
  the claims of the four consensus programs and of every lock / type script (inputs are reversed
  digests, `Digest::reversed()`), the member proofs verified (here: one batch instead of the
  sequential awaits at :343-385, zip-truncated like the reference's `zip`) and AND-ed (:388).
  `ProofCollection.verify_many` batches many collections (a mempool batch) in one call.
* `single_proof_claim` / `TransactionProof.verify_many` — single_proof.rs:227-230,295-304 and
  transaction_proof.rs:134-153: a SingleProof is one claim (the SingleProof program with input =
  the kernel MAST hash reversed), a ProofCollection its members; any mix of transactions goes
  into one GPU batch.  `transactions_are_valid` adds `Transaction::is_valid`'s kernel MAST hash
  (transaction/mod.rs:172-177), computed on the GPU from the kernel's field encodings.
* `BlockProgram.claim` / `validate_block_proofs` — block_program.rs:45-65 (input = body MAST
  hash reversed, output = `BlockAppendix::claims_as_output`, the Tip5 hashes of the appendix
  claims; block_appendix.rs:40-47) and `Block::validate` rules 1.a-1.d (block/mod.rs:783-804)
  for a batch of blocks (bootstrap import `state/mod.rs:2226-2272`, peer block batches
  `peer_loop.rs:315-323`): every block proof of the batch in one GPU batch.
The consensus programs' digests (RemovalRecordsIntegrity, KernelToOutputs, CollectLockScripts,
CollectTypeScripts) come from tasm-lib code generation, which is not vendored, so they are
parameters (`ConsensusPrograms`).
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

from .stark import Air, Claim, Group, Stark, verify_batch as _gpu_verify_batch, verify_batch_group

MOCK_VALID = (0,)    # MockProofBehavior::ValidMock.encode()
MOCK_INVALID = (1,)  # MockProofBehavior::InvalidMock.encode()


class Network(enum.Enum):
    MAIN = "main"
    TESTNET = "testnet"
    TESTNET_MOCK = "testnet-mock"
    REGTEST = "regtest"

    def use_mock_proof(self) -> bool:
        return self in (Network.REGTEST, Network.TESTNET_MOCK)


def is_valid_mock(proof) -> bool:
    return len(proof) == 1 and (int(proof[0]),) == MOCK_VALID


def is_invalid_mock(proof) -> bool:
    return len(proof) == 1 and (int(proof[0]),) == MOCK_INVALID


class Verifier:
    """GPU-backed `verify`: the AIR descriptor and Stark parameters are fixed.  `ctx` is one GPU's
    Context, or a Group (every GPU of the node from one process: each batch is split over them)."""

    def __init__(self, ctx, air: Air, stark: Optional[Stark] = None):
        self.ctx, self.air = ctx, air
        self.stark = stark or Stark.default()

    def verify(self, claim: Claim, proof, network: Network = Network.MAIN) -> bool:
        return self.verify_batch([(claim, proof)], network)[0]

    def verify_batch(self, pairs: Sequence[Tuple[Claim, object]], network: Network = Network.MAIN) -> List[bool]:
        if network.use_mock_proof():
            return [is_valid_mock(p) for _, p in pairs]
        if not pairs:
            return []
        if isinstance(self.ctx, Group):
            return verify_batch_group(self.ctx, self.air, self.stark, list(pairs))[0]
        return _gpu_verify_batch(self.ctx, self.air, self.stark, list(pairs))


def _rev(d: Sequence[int]) -> List[int]:
    return [int(x) for x in reversed(list(d))]


@dataclass
class ConsensusPrograms:
    """Program digests of the consensus programs (tasm-lib codegen): the four ProofCollection
    programs, SingleProof and BlockProgram."""
    removal_records_integrity: Sequence[int]
    kernel_to_outputs: Sequence[int]
    collect_lock_scripts: Sequence[int]
    collect_type_scripts: Sequence[int]
    single_proof: Sequence[int] = (0, 0, 0, 0, 0)
    block_program: Sequence[int] = (0, 0, 0, 0, 0)


def single_proof_claim(txk_mast_hash: Sequence[int], programs: ConsensusPrograms) -> Claim:
    """single_proof.rs:227-230 (`SingleProof::claim`), selected for both rule sets by :295-304."""
    return Claim(list(programs.single_proof), 0, _rev(txk_mast_hash), [])


@dataclass
class ProofCollection:
    """proof_collection.rs:34-49 (field names as there)."""
    removal_records_integrity: object
    collect_lock_scripts: object
    lock_scripts_halt: List[object]
    kernel_to_outputs: object
    collect_type_scripts: object
    type_scripts_halt: List[object]
    lock_script_hashes: List[Sequence[int]]
    type_script_hashes: List[Sequence[int]]
    kernel_mast_hash: Sequence[int]
    salted_inputs_hash: Sequence[int]
    salted_outputs_hash: Sequence[int]
    merge_bit_mast_path: List[Sequence[int]] = field(default_factory=list)

    def num_proofs(self) -> int:  # proof_collection.rs:53-60
        return 4 + len(self.lock_scripts_halt) + len(self.type_scripts_halt)

    def claims_and_proofs(self, programs: ConsensusPrograms) -> List[Tuple[Claim, object]]:
        """proof_collection.rs:286-339 claims, paired with their proofs in the order of :343-385."""
        kmh, sih, soh = self.kernel_mast_hash, self.salted_inputs_hash, self.salted_outputs_hash
        flat = lambda ds: [int(x) for d in ds for x in d]  # noqa: E731
        rri = Claim(list(programs.removal_records_integrity), 0, _rev(kmh), [int(x) for x in sih])
        k2o = Claim(list(programs.kernel_to_outputs), 0, _rev(kmh), [int(x) for x in soh])
        cls = Claim(list(programs.collect_lock_scripts), 0, _rev(sih), flat(self.lock_script_hashes))
        cts = Claim(list(programs.collect_type_scripts), 0, _rev(sih) + _rev(soh), flat(self.type_script_hashes))
        lock = [Claim(list(h), 0, _rev(kmh), []) for h in self.lock_script_hashes]
        typ = [Claim(list(h), 0, _rev(kmh) + _rev(sih) + _rev(soh), []) for h in self.type_script_hashes]
        pairs = [(rri, self.removal_records_integrity), (k2o, self.kernel_to_outputs),
                 (cls, self.collect_lock_scripts), (cts, self.collect_type_scripts)]
        pairs += list(zip(lock, self.lock_scripts_halt))  # zip truncates, as the reference's does
        pairs += list(zip(typ, self.type_scripts_halt))
        return pairs

    def verify(self, txk_mast_hash: Sequence[int], verifier: Verifier, programs: ConsensusPrograms,
               network: Network = Network.MAIN) -> bool:
        return ProofCollection.verify_many([(self, txk_mast_hash)], verifier, programs, network)[0]

    @staticmethod
    def verify_many(items: Sequence[Tuple["ProofCollection", Sequence[int]]], verifier: Verifier,
                    programs: ConsensusPrograms, network: Network = Network.MAIN) -> List[bool]:
        """Many collections (e.g. a mempool batch) in ONE verifier batch; per-collection ANDs."""
        pairs, owner, gate = [], [], []
        for ci, (pc, txk) in enumerate(items):
            ok = [int(x) for x in pc.kernel_mast_hash] == [int(x) for x in txk]  # :280-282
            gate.append(ok)
            if not ok:
                continue
            for pr in pc.claims_and_proofs(programs):
                pairs.append(pr)
                owner.append(ci)
        verdicts = verifier.verify_batch(pairs, network)
        out = list(gate)
        for ci, v in zip(owner, verdicts):
            out[ci] = out[ci] and v
        return out


# ------------------------------------------------------------------ transactions
WITNESS, SINGLE_PROOF, PROOF_COLLECTION = "witness", "single_proof", "proof_collection"


@dataclass
class TransactionProof:
    """transaction_proof.rs: `Witness(PrimitiveWitness)`, `SingleProof(Proof)` or
    `ProofCollection(ProofCollection)`; `payload` is the proof words or the ProofCollection."""
    kind: str
    payload: object = None

    @staticmethod
    def verify_many(items: Sequence[Tuple["TransactionProof", Sequence[int]]], verifier: Verifier,
                    programs: ConsensusPrograms, network: Network = Network.MAIN) -> List[bool]:
        """`TransactionProof::verify(kernel_mast_hash, ..)` for many transactions in ONE verifier batch.
        A primitive witness is validated by running the consensus programs on the host
        (`PrimitiveWitness::validate`), which is not a STARK verification and not on this path."""
        pairs, owner, out = [], [], []
        for ti, (tp, txk) in enumerate(items):
            if tp.kind == SINGLE_PROOF:
                pairs.append((single_proof_claim(txk, programs), tp.payload))
                owner.append(ti)
                out.append(True)
            elif tp.kind == PROOF_COLLECTION:
                pc = tp.payload
                ok = [int(x) for x in pc.kernel_mast_hash] == [int(x) for x in txk]  # proof_collection.rs:280-282
                out.append(ok)
                if ok:
                    for pr in pc.claims_and_proofs(programs):
                        pairs.append(pr)
                        owner.append(ti)
            elif tp.kind == WITNESS:
                raise ValueError("a primitive witness is validated on the host, not by the STARK verifier")
            else:
                raise ValueError(f"unknown transaction proof kind {tp.kind!r}")
        verdicts = verifier.verify_batch(pairs, network)
        for ti, v in zip(owner, verdicts):
            out[ti] = out[ti] and v
        return out


def transactions_are_valid(ctx, items: Sequence[Tuple[Sequence[Sequence[int]], TransactionProof]],
                           verifier: Verifier, programs: ConsensusPrograms,
                           network: Network = Network.MAIN) -> List[bool]:
    """`Transaction::is_valid` (transaction/mod.rs:172-177) for many transactions: the kernel MAST
    hashes (`kernel.mast_hash()`; items carry each kernel's 8 field encodings,
    transaction_kernel.rs:246-277) in one GPU call, then every proof in one verifier batch."""
    if not items:
        return []
    from .mast import mast_hash_batch
    hashes = mast_hash_batch(ctx, [fields for fields, _ in items])
    return TransactionProof.verify_many([(tp, h) for (_, tp), h in zip(items, hashes)], verifier, programs, network)


# ------------------------------------------------------------------ blocks
MAX_NUM_CLAIMS = 500                 # block_appendix.rs:19
GENESIS, INVALID = "genesis", "invalid"   # BlockProof (block/mod.rs:114-119); SINGLE_PROOF as above


def claims_as_output(ctx, claims: Sequence[Claim]) -> List[int]:
    """`BlockAppendix::claims_as_output` (block_appendix.rs:40-47): the concatenated Tip5 hashes of
    the appendix claims (`Tip5::hash(claim)`, on the GPU)."""
    from .proof_files import claim_hash
    return [int(x) for c in claims for x in claim_hash(ctx, c)]


class BlockProgram:
    @staticmethod
    def claim(ctx, body_mast_hash: Sequence[int], appendix: Sequence[Claim], programs: ConsensusPrograms) -> Claim:
        """block_program.rs:45-49."""
        return Claim(list(programs.block_program), 0, _rev(body_mast_hash), claims_as_output(ctx, appendix))


@dataclass
class BlockToValidate:
    """What `Block::validate` rules 1.a-1.d read: the body MAST hash, the transaction kernel's MAST
    hash, the appendix claims and the block proof (`kind` GENESIS / INVALID / SINGLE_PROOF)."""
    body_mast_hash: Sequence[int]
    tx_kernel_mast_hash: Sequence[int]
    appendix: Sequence[Claim]
    proof_kind: str
    proof: object = None


# BlockValidationError variants of rules 1.a-1.d (block/mod.rs:783-804); None = passed
APPENDIX_MISSING_CLAIM, APPENDIX_TOO_LARGE, PROOF_QUALITY, PROOF_VALIDITY = (
    "AppendixMissingClaim", "AppendixTooLarge", "ProofQuality", "ProofValidity")


def _same_claim(a: Claim, b: Claim) -> bool:
    key = lambda c: ([int(x) for x in c.program_digest], int(c.version), [int(x) for x in c.input],  # noqa: E731
                     [int(x) for x in c.output])
    return key(a) == key(b)


def validate_block_proofs(ctx, blocks: Sequence[BlockToValidate], verifier: Verifier, programs: ConsensusPrograms,
                          network: Network = Network.MAIN) -> List[Optional[str]]:
    """`Block::validate` rules 1.a-1.d, in the reference's order, for a batch of blocks; the
    BlockProgram proofs of all blocks that reach 1.d are verified in ONE GPU batch."""
    out: List[Optional[str]] = []
    pairs, owner = [], []
    for bi, blk in enumerate(blocks):
        required = [single_proof_claim(blk.tx_kernel_mast_hash, programs)]  # consensus_claims, :53-61
        if not all(any(_same_claim(r, c) for c in blk.appendix) for r in required):
            out.append(APPENDIX_MISSING_CLAIM)
        elif len(blk.appendix) > MAX_NUM_CLAIMS:
            out.append(APPENDIX_TOO_LARGE)
        elif blk.proof_kind != SINGLE_PROOF:
            out.append(PROOF_QUALITY)
        else:
            out.append(None)
            claim = (Claim(list(programs.block_program), 0, [], []) if network.use_mock_proof()
                     else BlockProgram.claim(ctx, blk.body_mast_hash, blk.appendix, programs))
            pairs.append((claim, blk.proof))
            owner.append(bi)
    verdicts = verifier.verify_batch(pairs, network)
    for bi, v in zip(owner, verdicts):
        if not v:
            out[bi] = PROOF_VALIDITY
    return out
