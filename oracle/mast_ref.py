"""MAST hashing and mutator-set absolute index sets restated — TEST ORACLE ONLY.

* mast_hash (neptune-core/src/protocol/proof_abstractions/mast_hash.rs:22-39): leaves
  hash_varlen(sequence), padded with Digest::default() to a power of two, Merkle root.
* absolute_index_set (util_types/mutator_set/removal_record/absolute_index_set.rs:86-113) with
  WINDOW_SIZE = 2^20, CHUNK_SIZE = 2^12, BATCH_SIZE = 2^3, NUM_TRIALS = 45 (shared.rs:12-15).
  u64 BFieldCodec = two u32 limbs, low limb first (twenty-first; unpinned).
Only tests/ use it.
"""
from __future__ import annotations

import tip5_ref as T

WINDOW_SIZE, CHUNK_SIZE, BATCH_SIZE, NUM_TRIALS = 1 << 20, 1 << 12, 1 << 3, 45


def mast_hash(sequences):
    leaves = [list(T.hash_varlen([int(x) for x in s])) for s in sequences]
    while len(leaves) & (len(leaves) - 1):
        leaves.append([0] * 5)
    while len(leaves) > 1:
        leaves = [list(T.hash_pair(leaves[2 * i], leaves[2 * i + 1])) for i in range(len(leaves) // 2)]
    return tuple(int(x) for x in leaves[0])


def absolute_index_set(item, sender_randomness, receiver_preimage, aocl_leaf_index: int):
    inp = [int(x) for x in item] + [int(x) for x in sender_randomness] + [int(x) for x in receiver_preimage] + \
        [aocl_leaf_index & 0xFFFFFFFF, aocl_leaf_index >> 32]
    sp = T.Tip5(fixed_length=False)
    sp.pad_and_absorb_all(inp)
    rel = sp.sample_indices(WINDOW_SIZE, NUM_TRIALS)
    mn = min(rel)
    return mn + (aocl_leaf_index // BATCH_SIZE) * CHUNK_SIZE, [x - mn for x in rel]
