"""GPU MAST hashing (mast_hash.rs:22-39) and mutator-set absolute index sets
(absolute_index_set.rs:86-113) bit-exact against the oracle restatement (mast_ref.py)."""
import numpy as np
import pytest

import mast_ref as M
import tip5_ref as T

pytestmark = pytest.mark.gpu


def test_mast_hash_batch_matches_oracle(ctx):
    from neptune_hip.mast import mast_hash_batch
    rng = np.random.default_rng(8)
    for fields in (1, 2, 3, 8, 11):
        objs = [[list(rng.integers(0, T.P, size=int(rng.integers(0, 40)), dtype=np.uint64)) for _ in range(fields)]
                for _ in range(25)]
        got = mast_hash_batch(ctx, objs)
        assert got == [M.mast_hash(o) for o in objs]


def test_absolute_index_sets_match_oracle(ctx):
    from neptune_hip.mast import AbsoluteIndexSet
    rng = np.random.default_rng(9)
    n = 300
    d = lambda: rng.integers(0, T.P, size=(n, 5), dtype=np.uint64)  # noqa: E731
    items, sr, rp = d(), d(), d()
    leaf = rng.integers(0, 2 ** 63, size=n, dtype=np.uint64)
    leaf[:3] = [0, 7, 2 ** 64 - 1]
    got = AbsoluteIndexSet.compute_batch(ctx, items, sr, rp, leaf)
    for i in range(n):
        mn, dist = M.absolute_index_set(items[i], sr[i], rp[i], int(leaf[i]))
        assert got[i].minimum == mn and got[i].distances == dist
        assert min(got[i].distances) == 0 and max(got[i].distances) < M.WINDOW_SIZE
