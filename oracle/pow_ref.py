"""Proof-of-work Tip5 workloads restated — TEST ORACLE ONLY.

Restates neptune-core/src/protocol/consensus/block/pow.rs (in-tree reference code) on top of
tip5_ref (Tip5 pinned by KAT-V / KAT-F) and coracle (C Tip5, for speed):
  bud (:321-323), leaf (:325-331), indices (:333-343), bitreverse (:349-356), swap_indices
  (:358-363), preprocess (:365-469), guess (:471-507), validate (:509-557),
  PowMastPaths::commit / fast_mast_hash (:209-241), MTree build / path / verify (:66-180).
Only tests/ use it.  Digest ordering (`pow_digest <= target`) follows twenty-first: canonical
values compared from the last element down — unpinned (no in-tree vector).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

import coracle as CO
import tip5_ref as T

NUM_BUD_LAYERS = 5
BUDS_PER_LEAF = 1 << NUM_BUD_LAYERS
NUM_INDEX_REPETITIONS = 63
Digest = Tuple[int, int, int, int, int]
ZERO: Digest = (0, 0, 0, 0, 0)


def hp(a, b) -> Digest:
    return tuple(int(x) for x in T.hash_pair(list(a), list(b)))


def bud(commitment, index: int) -> Digest:
    return hp(commitment, [index, 0, 0, 0, 0])


def mtree_root(leafs: Sequence[Digest]) -> Digest:
    level = [tuple(d) for d in leafs]
    while len(level) > 1:
        level = [hp(level[2 * i], level[2 * i + 1]) for i in range(len(level) // 2)]
    return level[0]


def leaf(commitment, index: int, height: int) -> Digest:
    n = 1 << height
    return mtree_root([bud(commitment, (index + j) % n) for j in range(BUDS_PER_LEAF)])


def bitreverse(k: int, log2_n: int) -> int:
    return int(format(k, f"0{32}b")[::-1], 2) >> ((32 - log2_n) & 0x1F) if log2_n else 0


def commit(mast) -> Digest:
    pow_, header, kernel = mast
    words = [int(x) for d in list(pow_) + list(header) + list(kernel) for x in d]
    return tuple(int(x) for x in T.hash_varlen(words))


def preprocess(height: int, mast, reboot: bool, prev_block_digest) -> Tuple[np.ndarray, np.ndarray]:
    """(leafs, internal nodes) of the guesser buffer's MTree (nodes[1] = root)."""
    n = 1 << height
    prefix = commit(mast) if reboot else tuple(prev_block_digest)
    buds = np.array([bud(prefix, i) for i in range(n)], dtype=np.uint64)
    for i in range(NUM_BUD_LAYERS):
        sh = np.roll(buds, -(1 << i), axis=0)
        buds = np.array([CO.hash_pair(buds[k], sh[k]) for k in range(n)], dtype=np.uint64)
    leafs = buds
    if not reboot:
        perm = np.array([bitreverse(k, height) for k in range(n)])
        leafs = leafs[perm]
    nodes = CO.mtree_build(np.ascontiguousarray(leafs))
    return leafs, nodes


def path(leafs: np.ndarray, nodes: np.ndarray, index: int) -> List[Digest]:
    n = leafs.shape[0]
    out = [tuple(int(x) for x in leafs[index ^ 1])]
    run = index + n
    for _ in range(1, n.bit_length() - 1):
        run >>= 1
        out.append(tuple(int(x) for x in nodes[run ^ 1]))
    return out


def mtree_verify(root, index: int, p: Sequence[Digest], element) -> bool:
    if index > (1 << len(p)):
        return False
    run, ri = tuple(element), index
    for sib in p:
        run = hp(sib, run) if ri & 1 else hp(run, sib)
        ri >>= 1
    return run == tuple(root)


def indices(h, nonce, height: int) -> Tuple[int, int]:
    x = hp(h, nonce)
    for _ in range(1, NUM_INDEX_REPETITIONS):
        x = hp(x, ZERO)
    return x[0] % (1 << height), x[1] % (1 << height)


def encode_pow(root, path_a, path_b, nonce) -> List[int]:
    """BFieldCodec of Pow { root, path_a, path_b, nonce }: fields reversed, static sizes unprefixed."""
    return [int(x) for d in [nonce] + list(path_b) + list(path_a) + [root] for x in d]


def fast_mast_hash(mast, root, path_a, path_b, nonce) -> Digest:
    pow_, header, kernel = mast
    hv = lambda w: tuple(int(x) for x in T.hash_varlen(list(w)))  # noqa: E731
    h = hp(hv(encode_pow(root, path_a, path_b, nonce)), pow_[0])
    h = hp(h, pow_[1])
    h = hp(pow_[2], h)
    k = hp(hv(h), header[0])
    k = hp(k, header[1])
    return hp(hv(k), kernel[0])


def digest_le(a, b) -> bool:
    return list(reversed([int(x) for x in a])) <= list(reversed([int(x) for x in b]))


def guess(leafs, nodes, mast, index_picker_preimage, nonce, target):
    height = leafs.shape[0].bit_length() - 1
    ia, ib = indices(index_picker_preimage, nonce, height)
    root = tuple(int(x) for x in nodes[1])
    d = fast_mast_hash(mast, root, path(leafs, nodes, ia), path(leafs, nodes, ib), nonce)
    return d, (ia, ib), digest_le(d, target)


def validate(height, root, path_a, path_b, nonce, mast, target, reboot: bool, parent) -> bool:
    c = commit(mast)
    prefix = c if reboot else tuple(parent)
    ia, ib = indices(hp(root, c), nonce, height)
    la = leaf(prefix, ia if reboot else bitreverse(ia, height), height)
    lb = leaf(prefix, ib if reboot else bitreverse(ib, height), height)
    if not mtree_verify(root, ia, path_a, la) or not mtree_verify(root, ib, path_b, lb):
        return False
    return digest_le(fast_mast_hash(mast, root, path_a, path_b, nonce), target)
