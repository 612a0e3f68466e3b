"""Block files and peer transactions over the C ABI: bincode decoded
natively (csrc/bincode.cpp) straight into the verifier's inputs.

* `blocks_from_file_without_record(path)` — state/archival_state/import_blocks_from_files.rs:100-115:
  every `Block` of a blk file (bincode, back to back), as `BlockRecord`s.  A malformed block
  fails the whole file (the reference's `?`), with `BlockFileError.n_good` blocks before it.
* `blocks_to_validate(ctx, records)` — what `Block::validate` rules 1.a-1.d read
  (`verifier.BlockToValidate`): the transaction kernels' and then the bodies' MAST hashes
  (`MastHash::mast_hash`, block_body.rs:175-182, transaction_kernel.rs:246-277) in two GPU calls
  for the whole file, the appendix claims and the block proof.  `validate_block_file` then runs
  the bootstrap import's proof checks (state/mod.rs:2226-2272) for a file in ONE verifier batch.
* `TransferTransaction.from_bytes(data)` — protocol/peer/transfer_transaction.rs:31-47: the kernel's
  MAST sequences and the `TransactionProof` (SingleProof words or a `ProofCollection`), ready for
  `verifier.transactions_are_valid`.
Proof words are copied once, reduced mod p, from the file bytes into numpy buffers that the
verifier stages without further conversion, or, given an `arena` (`stark.Arena`, round 6), straight
into pinned memory on a GPU's NUMA node (nhip_arena_ingest_blocks / _spans), from where the
verifier DMAs them as they lie.
"""
from __future__ import annotations

import ctypes
import mmap
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import NHIP_ERR_DECODE, check
from .stark import Claim

POW_TREE_HEIGHT = 29   # pow.rs:33-37 (production POW_MEMORY_PARAMETER = 2^29)
GENESIS_KIND, INVALID_KIND, SINGLE_PROOF_KIND = 0, 1, 2


class BlockFileError(ValueError):
    def __init__(self, msg, n_good):
        super().__init__(msg)
        self.n_good = n_good


def _buf(data) -> Tuple[np.ndarray, int]:
    a = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, dtype=np.uint8)
    return a, len(data)


def _words(lib, a, n, offset, count) -> np.ndarray:
    out = np.zeros(max(count, 1), dtype=np.uint64)
    check(lib.nhip_le_words(a.ctypes.data, n, offset, count, out.ctypes.data), "nhip_le_words")
    return out[:count]


@dataclass
class BlockRecord:
    """One block of a blk file: header fields the callers print, the MAST sequences (kernel 8,
    body 2-4), the appendix claims and the block proof (`proof_kind` as block/mod.rs:114-119)."""
    offset: int
    size: int
    height: int
    timestamp: int
    prev_block_digest: Tuple[int, ...]
    kernel_sequences: List[np.ndarray]
    body_tail_sequences: List[np.ndarray]
    appendix: List[Claim]
    proof_kind: int
    proof: Optional[np.ndarray]


def blocks_from_bytes(data, pow_tree_height: int = POW_TREE_HEIGHT, arena=None) -> List[BlockRecord]:
    """`arena`: decode the block proofs into it (pinned, on its GPUs' nodes) instead of numpy
    buffers; each record's `proof` is then a view of the arena (valid until the arena's reset)."""
    lib = _lib.load()
    in_arena = {}
    if arena is not None:
        placed, block_of = arena.ingest_blocks(data, pow_tree_height)
        in_arena = {b: placed.words(i) for i, b in enumerate(block_of)}
    a, n = _buf(data)
    count = ctypes.c_size_t(0)
    rc = lib.nhip_blk_scan(a.ctypes.data, n, pow_tree_height, None, 0, ctypes.byref(count))
    if rc == NHIP_ERR_DECODE:
        raise BlockFileError(f"malformed block after {count.value} blocks", count.value)
    check(rc, "nhip_blk_scan")
    blocks = (_lib.BlkBlock * max(count.value, 1))()
    check(lib.nhip_blk_scan(a.ctypes.data, n, pow_tree_height, ctypes.cast(blocks, ctypes.c_void_p), count.value,
                            ctypes.byref(count)), "nhip_blk_scan")
    out = []
    for i in range(count.value):
        b = blocks[i]
        offs = np.zeros(12, dtype=np.uint64)
        words = np.zeros(max(int(b.seq_words), 1), dtype=np.uint64)
        check(lib.nhip_blk_sequences(a.ctypes.data, n, pow_tree_height, ctypes.byref(b), words.ctypes.data,
                                     words.size, offs.ctypes.data), "nhip_blk_sequences")
        seqs = [words[int(offs[j]):int(offs[j + 1])] for j in range(11)]
        cw = np.zeros(max(int(b.claim_words), 1), dtype=np.uint64)
        cl = (_lib.Claim * max(b.n_claims, 1))()
        check(lib.nhip_blk_claims(a.ctypes.data, n, ctypes.byref(b), cw.ctypes.data,
                                  ctypes.cast(cl, ctypes.c_void_p)), "nhip_blk_claims")
        claims = [Claim([int(x) for x in c.program_digest], int(c.version),
                        [int(c.input[k]) for k in range(c.input_len)],
                        [int(c.output[k]) for k in range(c.output_len)]) for c in cl[:b.n_claims]]
        proof = None
        if b.proof_kind == SINGLE_PROOF_KIND:
            proof = in_arena[i] if i in in_arena else _words(lib, a, n, int(b.proof_offset), int(b.proof_len))
        out.append(BlockRecord(int(b.offset), int(b.size), int(b.height), int(b.timestamp),
                               tuple(int(x) for x in b.prev_block_digest), seqs[:8], seqs[8:], claims,
                               int(b.proof_kind), proof))
    return out


def blocks_from_file_without_record(path: str, pow_tree_height: int = POW_TREE_HEIGHT, arena=None) -> List[BlockRecord]:
    """import_blocks_from_files.rs:100-115 (the file is memory-mapped, as there)."""
    if os.path.getsize(path) == 0:
        return []
    with open(path, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as m:
        return blocks_from_bytes(m, pow_tree_height, arena)


def blocks_to_validate(ctx, records: Sequence[BlockRecord]):
    """Kernel MAST hashes, then body MAST hashes (sequence 1 = the kernel hash's encoding), each
    for all blocks in one GPU call; returns `verifier.BlockToValidate`s."""
    from .mast import mast_hash_batch
    from .verifier import BlockToValidate, GENESIS, INVALID, SINGLE_PROOF
    if not records:
        return []
    txk = mast_hash_batch(ctx, [r.kernel_sequences for r in records])
    body = mast_hash_batch(ctx, [[list(h)] + list(r.body_tail_sequences) for h, r in zip(txk, records)])
    kinds = {GENESIS_KIND: GENESIS, INVALID_KIND: INVALID, SINGLE_PROOF_KIND: SINGLE_PROOF}
    return [BlockToValidate(list(bh), list(th), r.appendix, kinds[r.proof_kind], r.proof)
            for r, th, bh in zip(records, txk, body)]


def validate_block_file(ctx, path: str, verifier, programs, network=None,
                        pow_tree_height: int = POW_TREE_HEIGHT, arena=None) -> List[Optional[str]]:
    """Rules 1.a-1.d for every block of a blk file, all block proofs in one verifier batch;
    `arena`: the block proofs decoded straight into pinned memory (DMA'd from there)."""
    from .verifier import Network, validate_block_proofs
    recs = blocks_from_file_without_record(path, pow_tree_height, arena)
    return validate_block_proofs(ctx, blocks_to_validate(ctx, recs), verifier, programs,
                                 network if network is not None else Network.MAIN)


@dataclass
class TransferTransaction:
    """transfer_transaction.rs:31-47: `kernel_sequences` (the kernel's 8 MAST sequences) and the
    proof as a `verifier.TransactionProof`."""
    kernel_sequences: List[np.ndarray]
    proof: object
    size: int

    @staticmethod
    def from_bytes(data, arena=None) -> "TransferTransaction":
        """`arena`: the member proofs decoded straight into it (pinned, nhip_arena_ingest_spans)."""
        from .verifier import PROOF_COLLECTION, SINGLE_PROOF, ProofCollection, TransactionProof
        lib = _lib.load()
        a, n = _buf(data)
        t = _lib.Tx()
        rc = lib.nhip_tx_scan(a.ctypes.data, n, ctypes.byref(t))
        if rc == NHIP_ERR_DECODE:
            raise ValueError("malformed TransferTransaction")
        check(rc, "nhip_tx_scan")
        seq = np.zeros(max(int(t.seq_words), 1), dtype=np.uint64)
        offs = np.zeros(9, dtype=np.uint64)
        spans = np.zeros(2 * t.n_proofs, dtype=np.uint64)
        dig = np.zeros(max(5 * t.n_digests, 1), dtype=np.uint64)
        check(lib.nhip_tx_parts(a.ctypes.data, n, ctypes.byref(t), seq.ctypes.data, offs.ctypes.data,
                                spans.ctypes.data, dig.ctypes.data), "nhip_tx_parts")
        seqs = [seq[int(offs[j]):int(offs[j + 1])] for j in range(8)]
        if arena is not None:
            pl = arena.ingest_spans(a[:n], [(int(spans[2 * i]), int(spans[2 * i + 1])) for i in range(t.n_proofs)])
            proofs = [pl.words(i) for i in range(t.n_proofs)]
        else:
            proofs = [_words(lib, a, n, int(spans[2 * i]), int(spans[2 * i + 1])) for i in range(t.n_proofs)]
        if t.kind == 1:
            return TransferTransaction(seqs, TransactionProof(SINGLE_PROOF, proofs[0]), int(t.size))
        d = [tuple(int(x) for x in dig[5 * i:5 * i + 5]) for i in range(t.n_digests)]
        nl, nt = int(t.n_lock_scripts), int(t.n_type_scripts)
        lh, th = int(t.n_lock_hashes), int(t.n_type_hashes)
        pc = ProofCollection(
            removal_records_integrity=proofs[0], collect_lock_scripts=proofs[1],
            lock_scripts_halt=proofs[2:2 + nl], kernel_to_outputs=proofs[2 + nl],
            collect_type_scripts=proofs[3 + nl], type_scripts_halt=proofs[4 + nl:4 + nl + nt],
            lock_script_hashes=d[:lh], type_script_hashes=d[lh:lh + th], kernel_mast_hash=d[lh + th],
            salted_inputs_hash=d[lh + th + 1], salted_outputs_hash=d[lh + th + 2],
            merge_bit_mast_path=d[lh + th + 3:])
        return TransferTransaction(seqs, TransactionProof(PROOF_COLLECTION, pc), int(t.size))
