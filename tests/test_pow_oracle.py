"""PoW oracle (oracle/pow_ref.py) against the reference's own unit tests of pow.rs: bitreverse known
answers (pow.rs:696-705), leafs_agree_with_bud_trees (:618-636), guess -> validate happy path
(:721-747).  CPU only."""
import numpy as np

import pow_ref as W
import tip5_ref as T


def _mast(rng):
    d = lambda: tuple(int(x) for x in rng.integers(0, T.P, size=5, dtype=np.uint64))  # noqa: E731
    return ([d(), d(), d()], [d(), d()], [d()])


def test_bitreverse_reference_unit_test():
    assert [W.bitreverse(7, 3), W.bitreverse(7, 4), W.bitreverse(7, 2), W.bitreverse(7, 1), W.bitreverse(14, 4),
            W.bitreverse(12, 4), W.bitreverse(100, 7)] == [7, 14, 3, 1, 7, 3, 19]


def test_leafs_agree_with_bud_trees_and_happy_path():
    T.use_c_backend()
    rng = np.random.default_rng(42)
    mast = _mast(rng)
    prev = tuple(int(x) for x in rng.integers(0, T.P, size=5, dtype=np.uint64))
    h = 8
    for reboot in (True, False):
        leafs, nodes = W.preprocess(h, mast, reboot, prev)
        prefix = W.commit(mast) if reboot else prev
        for index in (0, 5, 200, 255):
            k = index if reboot else W.bitreverse(index, h)
            assert tuple(int(x) for x in leafs[index]) == W.leaf(prefix, k, h)
        root = tuple(int(x) for x in nodes[1])
        picker = W.hp(root, W.commit(mast))
        target = (2 ** 64 - 2 ** 32,) * 4 + (2 ** 62,)  # accepts ~1 in 4 (last element most significant)
        found = 0
        for nonce_i in range(12):
            nonce = (nonce_i, 7, 7, 7, 7)
            d, (ia, ib), ok = W.guess(leafs, nodes, mast, picker, nonce, target)
            pa, pb = W.path(leafs, nodes, ia), W.path(leafs, nodes, ib)
            assert W.validate(h, root, pa, pb, nonce, mast, target, reboot, prev) == ok
            found += ok
            if ok:  # a tampered path or the other rule set must fail
                bad = list(pa)
                bad[3] = W.ZERO
                assert not W.validate(h, root, bad, pb, nonce, mast, target, reboot, prev)
                assert not W.validate(h, root, pa, pb, nonce, mast, target, not reboot, prev)
        assert found >= 1
