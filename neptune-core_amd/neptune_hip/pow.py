"""Host mirror of neptune-core's proof-of-work Tip5 workloads over the C ABI.

Names follow neptune-core/src/protocol/consensus/block/pow.rs: `Pow.preprocess` builds the
`GuesserBuffer` (:365-469) on the GPU, `GuesserBuffer.{root, leaf, path, index_picker_preimage}`,
`Pow.guess` over a batch of nonces (:471-507), `Pow.validate` over a batch of blocks (:509-557),
`PowMastPaths.commit` (:209-217).  Digests are canonical 5-tuples.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import check


class MastPathsC(ctypes.Structure):
    _fields_ = [("pow", (ctypes.c_uint64 * 5) * 3), ("header", (ctypes.c_uint64 * 5) * 2),
                ("kernel", (ctypes.c_uint64 * 5) * 1)]


@dataclass
class PowMastPaths:
    pow: Sequence[Sequence[int]]     # [BlockHeader::MAST_HEIGHT = 3]
    header: Sequence[Sequence[int]]  # [BlockKernel::MAST_HEIGHT = 2]
    kernel: Sequence[Sequence[int]]  # [Block::MAST_HEIGHT = 1]

    def c(self) -> MastPathsC:
        m = MastPathsC()
        for name, k in (("pow", 3), ("header", 2), ("kernel", 1)):
            arr = getattr(m, name)
            for i in range(k):
                for q in range(5):
                    arr[i][q] = int(getattr(self, name)[i][q])
        return m

    def commit(self, ctx) -> Tuple[int, ...]:
        out = np.zeros(5, dtype=np.uint64)
        m = self.c()
        check(ctx.lib.nhip_pow_mast_commit(ctx.handle, ctypes.byref(m), out.ctypes.data), "nhip_pow_mast_commit")
        return tuple(int(x) for x in out)


def _d5(v) -> np.ndarray:
    return np.ascontiguousarray(np.asarray([int(x) for x in v], dtype=np.uint64))


class GuesserBuffer:
    def __init__(self, ctx, handle, height: int):
        self.ctx, self.handle, self.height = ctx, handle, height

    def root(self) -> Tuple[int, ...]:
        out = np.zeros(5, dtype=np.uint64)
        check(self.ctx.lib.nhip_pow_buffer_root(self.ctx.handle, self.handle, out.ctypes.data), "pow root")
        return tuple(int(x) for x in out)

    def leaf(self, index: int) -> Tuple[int, ...]:
        out = np.zeros(5, dtype=np.uint64)
        check(self.ctx.lib.nhip_pow_buffer_leaf(self.ctx.handle, self.handle, index, out.ctypes.data), "pow leaf")
        return tuple(int(x) for x in out)

    def path(self, index: int) -> List[Tuple[int, ...]]:
        out = np.zeros(5 * self.height, dtype=np.uint64)
        check(self.ctx.lib.nhip_pow_buffer_path(self.ctx.handle, self.handle, index, out.ctypes.data), "pow path")
        return [tuple(int(x) for x in out[5 * j:5 * j + 5]) for j in range(self.height)]

    def index_picker_preimage(self, mast: PowMastPaths) -> Tuple[int, ...]:
        """GuesserBuffer::index_picker_preimage: hash_pair(root, mast.commit())."""
        out = self.ctx.hash_pair(np.array([self.root()], dtype=np.uint64),
                                 np.array([mast.commit(self.ctx)], dtype=np.uint64))
        return tuple(int(x) for x in out[0])

    def close(self):
        if self.handle:
            self.ctx.lib.nhip_pow_buffer_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Pow:
    @staticmethod
    def preprocess(ctx, height: int, mast: PowMastPaths, reboot: bool, prev_block_digest) -> GuesserBuffer:
        h = ctypes.c_void_p()
        m = mast.c()
        prev = _d5(prev_block_digest)  # keep the buffers alive across the call
        check(ctx.lib.nhip_pow_preprocess(ctx.handle, height, ctypes.byref(m), 1 if reboot else 0,
                                          prev.ctypes.data, ctypes.byref(h)), "nhip_pow_preprocess")
        return GuesserBuffer(ctx, h.value, height)

    @staticmethod
    def guess(ctx, buffer: GuesserBuffer, mast: PowMastPaths, index_picker_preimage, nonces, target):
        """(pow digests [n,5], indices [n,2], success [n]) for a batch of nonces."""
        nz = np.ascontiguousarray(np.asarray(nonces, dtype=np.uint64).reshape(-1, 5))
        n = nz.shape[0]
        dig = np.zeros((max(n, 1), 5), dtype=np.uint64)
        idx = np.zeros((max(n, 1), 2), dtype=np.uint64)
        ok = np.zeros(max(n, 1), dtype=np.uint8)
        m = mast.c()
        pick, tgt = _d5(index_picker_preimage), _d5(target)  # keep the buffers alive across the call
        check(ctx.lib.nhip_pow_guess_batch(ctx.handle, buffer.handle, ctypes.byref(m), pick.ctypes.data,
                                           nz.ctypes.data, n, tgt.ctypes.data, dig.ctypes.data, idx.ctypes.data,
                                           ok.ctypes.data), "nhip_pow_guess_batch")
        return dig[:n], idx[:n], ok[:n].astype(bool)

    @staticmethod
    def validate(ctx, height: int, blocks: Sequence[dict]) -> List[bool]:
        """blocks: dicts with root, path_a, path_b, nonce, mast (PowMastPaths), target, parent, reboot."""
        n = len(blocks)
        if n == 0:
            return []
        arr = lambda key: np.ascontiguousarray(np.asarray([[int(x) for x in b[key]] for b in blocks],  # noqa: E731
                                                          dtype=np.uint64))
        pa = np.ascontiguousarray(np.asarray([[int(x) for d in b["path_a"] for x in d] for b in blocks], dtype=np.uint64))
        pb = np.ascontiguousarray(np.asarray([[int(x) for d in b["path_b"] for x in d] for b in blocks], dtype=np.uint64))
        masts = (MastPathsC * n)(*[b["mast"].c() for b in blocks])
        rules = np.ascontiguousarray(np.asarray([1 if b["reboot"] else 0 for b in blocks], dtype=np.uint8))
        v = np.zeros(n, dtype=np.uint8)
        roots, nonces, targets, parents = arr("root"), arr("nonce"), arr("target"), arr("parent")
        check(ctx.lib.nhip_pow_validate_batch(ctx.handle, height, roots.ctypes.data, pa.ctypes.data, pb.ctypes.data,
                                              nonces.ctypes.data, masts, targets.ctypes.data, parents.ctypes.data,
                                              rules.ctypes.data, n, v.ctypes.data), "nhip_pow_validate_batch")
        return [bool(x) for x in v]
