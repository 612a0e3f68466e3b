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
The consensus programs' digests (RemovalRecordsIntegrity, KernelToOutputs, CollectLockScripts,
CollectTypeScripts) come from tasm-lib code generation, which is not vendored, so they are
parameters (`ConsensusPrograms`).
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

from .stark import Air, Claim, Stark, verify_batch as _gpu_verify_batch

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
    """GPU-backed `verify` for one device: the AIR descriptor and Stark parameters are fixed."""

    def __init__(self, ctx, air: Air, stark: Optional[Stark] = None):
        self.ctx, self.air = ctx, air
        self.stark = stark or Stark.default()

    def verify(self, claim: Claim, proof, network: Network = Network.MAIN) -> bool:
        return self.verify_batch([(claim, proof)], network)[0]

    def verify_batch(self, pairs: Sequence[Tuple[Claim, object]], network: Network = Network.MAIN) -> List[bool]:
        if network.use_mock_proof():
            return [is_valid_mock(p) for _, p in pairs]
        return _gpu_verify_batch(self.ctx, self.air, self.stark, list(pairs)) if pairs else []


def _rev(d: Sequence[int]) -> List[int]:
    return [int(x) for x in reversed(list(d))]


@dataclass
class ConsensusPrograms:
    """Program digests of the four ProofCollection consensus programs (tasm-lib codegen)."""
    removal_records_integrity: Sequence[int]
    kernel_to_outputs: Sequence[int]
    collect_lock_scripts: Sequence[int]
    collect_type_scripts: Sequence[int]


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
