"""GPU proof-of-work workloads (pow.rs) bit-exact against the oracle restatement (pow_ref.py):
the guesser buffer (every leaf and internal node, both consensus rule sets), MTree path / leaf /
root readback, guess over a nonce batch (digests, indices, verdicts) and validate over a block
batch with tampered paths, nonces and rule sets."""
import numpy as np
import pytest

import pow_ref as W
import tip5_ref as T

pytestmark = pytest.mark.gpu


def _mast(rng):
    d = lambda: tuple(int(x) for x in rng.integers(0, T.P, size=5, dtype=np.uint64))  # noqa: E731
    return ([d(), d(), d()], [d(), d()], [d()])


def _pm(mast):
    from neptune_hip.pow import PowMastPaths
    return PowMastPaths(*mast)


@pytest.mark.parametrize("reboot", [True, False])
def test_guesser_buffer_matches_oracle(ctx, reboot):
    from neptune_hip.pow import Pow
    T.use_c_backend()
    rng = np.random.default_rng(7 + reboot)
    mast, h = _mast(rng), 10
    prev = tuple(int(x) for x in rng.integers(0, T.P, size=5, dtype=np.uint64))
    leafs, nodes = W.preprocess(h, mast, reboot, prev)
    assert _pm(mast).commit(ctx) == W.commit(mast)
    buf = Pow.preprocess(ctx, h, _pm(mast), reboot, prev)
    assert buf.root() == tuple(int(x) for x in nodes[1])
    for i in (0, 1, 2, 511, 1023):
        assert buf.leaf(i) == tuple(int(x) for x in leafs[i])
        assert buf.path(i) == W.path(leafs, nodes, i)
    buf.close()


def test_guess_and_validate_match_oracle(ctx):
    from neptune_hip.pow import Pow
    T.use_c_backend()
    rng = np.random.default_rng(99)
    mast, h = _mast(rng), 9
    prev = tuple(int(x) for x in rng.integers(0, T.P, size=5, dtype=np.uint64))
    target = (2 ** 64 - 2 ** 32,) * 4 + (2 ** 62,)
    blocks, want = [], []
    for reboot in (True, False):
        leafs, nodes = W.preprocess(h, mast, reboot, prev)
        buf = Pow.preprocess(ctx, h, _pm(mast), reboot, prev)
        picker = buf.index_picker_preimage(_pm(mast))
        root = tuple(int(x) for x in nodes[1])
        assert picker == W.hp(root, W.commit(mast))
        nonces = rng.integers(0, T.P, size=(64, 5), dtype=np.uint64)
        dig, idx, ok = Pow.guess(ctx, buf, _pm(mast), picker, nonces, target)
        for i in range(16):
            nonce = tuple(int(x) for x in nonces[i])
            d, (ia, ib), o = W.guess(leafs, nodes, mast, picker, nonce, target)
            assert tuple(int(x) for x in dig[i]) == d and tuple(idx[i]) == (ia, ib) and bool(ok[i]) == o
            pa, pb = W.path(leafs, nodes, ia), W.path(leafs, nodes, ib)
            blk = dict(root=root, path_a=pa, path_b=pb, nonce=nonce, mast=_pm(mast), target=target, parent=prev,
                       reboot=reboot)
            blocks.append(blk)
            want.append(o)
            if i < 4:
                bad = dict(blk, path_b=list(pb[:-1]) + [W.ZERO])
                blocks.append(bad)
                want.append(False)
                blocks.append(dict(blk, reboot=not reboot))
                want.append(W.validate(h, root, pa, pb, nonce, mast, target, not reboot, prev))
                blocks.append(dict(blk, nonce=(nonce[0] ^ 1,) + nonce[1:]))
                want.append(W.validate(h, root, pa, pb, (nonce[0] ^ 1,) + nonce[1:], mast, target, reboot, prev))
        buf.close()
    got = Pow.validate(ctx, h, blocks)
    assert got == want and any(want) and not all(want)
