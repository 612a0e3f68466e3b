import sys, numpy as np
sys.path[:0] = ['oracle', 'neptune-core_amd']
import pow_ref as W, tip5_ref as T
T.use_c_backend()
import neptune_hip as nh
from neptune_hip.pow import Pow, PowMastPaths
rng = np.random.default_rng(99)
d = lambda: tuple(int(x) for x in rng.integers(0, T.P, size=5, dtype=np.uint64))
mast = ([d(), d(), d()], [d(), d()], [d()]); h = 9
prev = d()
ctx = nh.Context(0)
leafs, nodes = W.preprocess(h, mast, True, prev)
buf = Pow.preprocess(ctx, h, PowMastPaths(*mast), True, prev)
picker = buf.index_picker_preimage(PowMastPaths(*mast))
nonce = d()
dig, idx, ok = Pow.guess(ctx, buf, PowMastPaths(*mast), picker, np.array([nonce], dtype=np.uint64), (0,)*5)
ia, ib = W.indices(picker, nonce, h)
print('idx gpu', idx[0], 'oracle', ia, ib)
root = tuple(int(x) for x in nodes[1])
pa, pb = W.path(leafs, nodes, ia), W.path(leafs, nodes, ib)
print('gpu digest', dig[0])
print('oracle', W.fast_mast_hash(mast, root, pa, pb, nonce))
# variants
print('swap paths', W.fast_mast_hash(mast, root, pb, pa, nonce))
enc = W.encode_pow(root, pa, pb, nonce)
hv = ctx.hash_varlen(rows=[enc])[0]
print('gpu hv(enc)', hv, 'oracle', T.hash_varlen(enc))
