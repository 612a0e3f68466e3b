"""Host mirror of neptune-core's MAST hashing and mutator-set index derivation
over the C ABI.

* `mast_hash_batch(ctx, objects)` — `MastHash::mast_hash` (neptune-core/src/protocol/
  proof_abstractions/mast_hash.rs:22-39) of many objects at once: each object is its list of field
  sequences (`mast_sequences()`, e.g. the 8 BFieldCodec encodings of a TransactionKernel,
  transaction_kernel.rs:246-277).
* `AbsoluteIndexSet.compute_batch(ctx, ...)` — `AbsoluteIndexSet::compute`
  (util_types/mutator_set/removal_record/absolute_index_set.rs:86-113) for many removal records.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import check

NUM_TRIALS = 45
WINDOW_SIZE = 1 << 20


def mast_hash_batch(ctx, objects: Sequence[Sequence[Sequence[int]]]) -> List[Tuple[int, ...]]:
    n = len(objects)
    if n == 0:
        return []
    fields = len(objects[0])
    if any(len(o) != fields for o in objects):
        raise ValueError("one field count per batch")
    seqs = [s for o in objects for s in o]
    off = np.zeros(len(seqs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(s) for s in seqs])
    data = np.zeros(max(int(off[-1]), 1), dtype=np.uint64)
    pos = 0
    for s in seqs:
        data[pos:pos + len(s)] = np.asarray([int(x) for x in s], dtype=np.uint64)
        pos += len(s)
    roots = np.zeros((n, 5), dtype=np.uint64)
    check(ctx.lib.nhip_mast_hash_batch(ctx.handle, data.ctypes.data, off.ctypes.data, fields, n, roots.ctypes.data),
          "nhip_mast_hash_batch")
    return [tuple(int(x) for x in r) for r in roots]


@dataclass
class AbsoluteIndexSet:
    minimum: int            # u128
    distances: List[int]    # NUM_TRIALS u32

    def to_array(self) -> List[int]:
        return [d + self.minimum for d in self.distances]

    @staticmethod
    def compute_batch(ctx, items, sender_randomness, receiver_preimages, aocl_leaf_indices) -> List["AbsoluteIndexSet"]:
        n = len(items)
        if n == 0:
            return []
        a = lambda x: np.ascontiguousarray(np.asarray(x, dtype=np.uint64).reshape(n, 5))  # noqa: E731
        it, sr, rp = a(items), a(sender_randomness), a(receiver_preimages)
        leaf = np.ascontiguousarray(np.asarray(aocl_leaf_indices, dtype=np.uint64).reshape(n))
        mn = np.zeros((n, 2), dtype=np.uint64)
        dist = np.zeros((n, NUM_TRIALS), dtype=np.uint32)
        check(ctx.lib.nhip_absolute_index_sets(ctx.handle, it.ctypes.data, sr.ctypes.data, rp.ctypes.data,
                                               leaf.ctypes.data, n, mn.ctypes.data, dist.ctypes.data),
              "nhip_absolute_index_sets")
        return [AbsoluteIndexSet(int(mn[i, 0]) + (int(mn[i, 1]) << 64), [int(x) for x in dist[i]]) for i in range(n)]
