"""neptune_hip — host-side mirror of the reference's Tip5 / MTree interfaces over the
MI355X C ABI (include/neptune_hip.h, libneptune_hip.so).

Reference interfaces mirrored (paths relative to /root/reference):
  * ``Tip5.hash_pair`` / ``Tip5.hash_varlen`` / ``Tip5.permutation`` — twenty-first 1.0.0
    ``Tip5`` (Cargo.lock:4297) as used by neptune-core, e.g.
    neptune-core/src/protocol/consensus/block/pow.rs:112,130 and
    neptune-core/src/protocol/proof_abstractions/mast_hash.rs:26.
  * ``MTree.build_inplace`` / ``MTree.root`` / ``MTree.path`` / ``MTree.verify`` —
    neptune-core/src/protocol/consensus/block/pow.rs:60-181.
  * ``Digest`` — 5 BFieldElements; LowerHex = little-endian bytes of each canonical value
    (pinned by the reference's KATs, tests/test_oracle_kat.py).

All arithmetic runs in the HIP kernels; this module only marshals buffers.  Batch forms
(``Context.*``) are the throughput path; the scalar mirrors exist so code written against
the reference's API reads the same.
"""
from __future__ import annotations

import ctypes
import os
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import NhipError, check

P = (1 << 64) - (1 << 32) + 1
DIGEST_LEN = 5

__all__ = ["Context", "DeviceBuffer", "Digest", "Tip5", "MTree", "NhipError", "default_context", "P"]


def _as_u64(a, shape_tail: Tuple[int, ...] = ()) -> np.ndarray:
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.uint64))
    if shape_tail and arr.shape[-len(shape_tail):] != shape_tail:
        raise ValueError(f"expected trailing shape {shape_tail}, got {arr.shape}")
    return arr


class DeviceBuffer:
    """A device allocation owned by a Context (freed on close / garbage collection)."""

    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(ctx.lib.nhip_dev_alloc(ctx.handle, self.nbytes, ctypes.byref(p)), "nhip_dev_alloc")
        self.ptr = p.value

    def free(self):
        if self.ptr is not None and self.ctx.handle:
            self.ctx.lib.nhip_dev_free(self.ctx.handle, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def upload(self, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        check(self.ctx.lib.nhip_memcpy_h2d(self.ctx.handle, self.ptr, arr.ctypes.data, arr.nbytes), "h2d")
        return self

    def download(self, dtype, shape) -> np.ndarray:
        out = np.empty(shape, dtype=dtype)
        assert out.nbytes <= self.nbytes
        check(self.ctx.lib.nhip_memcpy_d2h(self.ctx.handle, out.ctypes.data, self.ptr, out.nbytes), "d2h")
        return out


def numa_of(lib, ctx_handle) -> dict:
    node, n = ctypes.c_int(-1), ctypes.c_size_t(0)
    check(lib.nhip_device_numa(ctx_handle, ctypes.byref(node), None, 0, ctypes.byref(n)), "nhip_device_numa")
    cpus = (ctypes.c_int * max(1, n.value))()
    got = ctypes.c_size_t(0)
    check(lib.nhip_device_numa(ctx_handle, ctypes.byref(node), cpus, n.value, ctypes.byref(got)), "nhip_device_numa")
    return {"node": node.value, "cpus": list(cpus[:min(n.value, got.value)])}


class Context:
    """One GPU (one process per GPU).  Wraps an ``nhip_ctx``."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        h = ctypes.c_void_p()
        check(self.lib.nhip_init(ctypes.c_uint32(1 << device), ctypes.byref(h)), "nhip_init")
        self.handle = h.value
        self.device = device

    def close(self):
        if self.handle:
            self.lib.nhip_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ------------------------------------------------------------ host-buffer batch API
    def tip5_permutation(self, states) -> np.ndarray:
        s = _as_u64(states, (16,)).copy()
        n = s.shape[0] if s.ndim == 2 else 1
        if n:
            check(self.lib.nhip_tip5_permutation(self.handle, s.reshape(-1), n), "permutation")
        return s

    def hash_pair(self, left, right) -> np.ndarray:
        l_ = _as_u64(left, (5,)).reshape(-1, 5)
        r_ = _as_u64(right, (5,)).reshape(-1, 5)
        if l_.shape != r_.shape:
            raise ValueError("left/right batch mismatch")
        out = np.zeros_like(l_)
        if l_.shape[0]:
            check(self.lib.nhip_tip5_hash_pair(self.handle, l_.reshape(-1), r_.reshape(-1), l_.shape[0],
                                               out.reshape(-1)), "hash_pair")
        return out

    def hash_varlen(self, rows: Sequence[Sequence[int]] = None, data=None, offsets=None) -> np.ndarray:
        """Hash ragged rows: either ``rows`` (list of sequences) or flat ``data`` + ``offsets``."""
        if rows is not None:
            lens = np.array([len(r) for r in rows], dtype=np.uint64)
            offsets = np.zeros(len(rows) + 1, dtype=np.uint64)
            np.cumsum(lens, out=offsets[1:])
            data = np.array([int(v) for r in rows for v in r], dtype=np.uint64)
        data = _as_u64(data).reshape(-1)
        offsets = _as_u64(offsets).reshape(-1)
        n = offsets.shape[0] - 1
        out = np.zeros((max(n, 0), 5), dtype=np.uint64)
        if n > 0:
            d = data if data.size else np.zeros(1, dtype=np.uint64)
            check(self.lib.nhip_tip5_hash_varlen(self.handle, d, offsets, n, out.reshape(-1)), "hash_varlen")
        return out

    def mtree_build(self, leafs) -> np.ndarray:
        lv = _as_u64(leafs, (5,)).reshape(-1, 5)
        nodes = np.zeros_like(lv)
        check(self.lib.nhip_mtree_build(self.handle, lv.reshape(-1), lv.shape[0], nodes.reshape(-1)), "mtree_build")
        return nodes

    def mtree_verify(self, roots, indices, leafs, paths, depth: int) -> np.ndarray:
        rt = _as_u64(roots).reshape(-1, 5)
        idx = _as_u64(indices).reshape(-1)
        n = idx.shape[0]
        lv = _as_u64(leafs).reshape(-1)
        pt = _as_u64(paths).reshape(-1)
        v = np.zeros(max(n, 1), dtype=np.uint8)
        if n:
            if lv.size != 5 * n or pt.size != 5 * n * depth:
                raise ValueError("leafs/paths shape mismatch")
            check(self.lib.nhip_mtree_verify(self.handle, rt.reshape(-1), rt.shape[0], idx, lv,
                                             pt if pt.size else np.zeros(1, np.uint64), depth, n, v),
                  "mtree_verify")
        return v[:n]

    # ------------------------------------------------------------ device-resident API
    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def upload(self, arr) -> DeviceBuffer:
        arr = np.ascontiguousarray(arr)
        return DeviceBuffer(self, max(arr.nbytes, 1)).upload(arr)

    def synchronize(self):
        check(self.lib.nhip_synchronize(self.handle), "synchronize")

    def tip5_permutation_dev(self, d_states: DeviceBuffer, n: int):
        check(self.lib.nhip_tip5_permutation_dev(self.handle, d_states.ptr, n), "permutation_dev")

    def hash_pair_dev(self, d_l: DeviceBuffer, d_r: DeviceBuffer, n: int, d_out: DeviceBuffer):
        check(self.lib.nhip_tip5_hash_pair_dev(self.handle, d_l.ptr, d_r.ptr, n, d_out.ptr), "hash_pair_dev")

    def hash_varlen_dev(self, d_data: DeviceBuffer, d_off: DeviceBuffer, n: int, d_out: DeviceBuffer):
        check(self.lib.nhip_tip5_hash_varlen_dev(self.handle, d_data.ptr, d_off.ptr, n, d_out.ptr),
              "hash_varlen_dev")

    def mtree_build_dev(self, d_leafs: DeviceBuffer, n_leafs: int, d_nodes: DeviceBuffer):
        check(self.lib.nhip_mtree_build_dev(self.handle, d_leafs.ptr, n_leafs, d_nodes.ptr), "mtree_build_dev")

    def mtree_verify_dev(self, d_roots: DeviceBuffer, n_roots: int, d_idx: DeviceBuffer, d_leafs: DeviceBuffer,
                         d_paths: DeviceBuffer, depth: int, n: int, d_verdicts: DeviceBuffer):
        check(self.lib.nhip_mtree_verify_dev(self.handle, d_roots.ptr, n_roots, d_idx.ptr, d_leafs.ptr,
                                             d_paths.ptr, depth, n, d_verdicts.ptr), "mtree_verify_dev")

    def verdicts_all_dev(self, d_verdicts: DeviceBuffer, n: int) -> bool:
        ok = ctypes.c_uint8(0)
        check(self.lib.nhip_verdicts_all_dev(self.handle, d_verdicts.ptr, n, ctypes.byref(ok)), "verdicts_all")
        return bool(ok.value)

    # ------------------------------------------------------------ timing
    def numa(self) -> dict:
        """The NUMA node of this context's GPU and that node's CPUs (nhip_device_numa): where its
        pinned staging lives and where its staging copy threads run."""
        return numa_of(self.lib, self.handle)

    def timing(self, on: bool = True):
        check(self.lib.nhip_timing_enable(self.handle, 1 if on else 0), "timing_enable")

    def timing_read(self, reset: bool = True) -> Tuple[float, int]:
        ms = ctypes.c_double(0.0)
        n = ctypes.c_uint64(0)
        check(self.lib.nhip_timing_read(self.handle, ctypes.byref(ms), ctypes.byref(n), 1 if reset else 0),
              "timing_read")
        return ms.value, n.value


_default: Optional[Context] = None


def default_context() -> Context:
    global _default
    if _default is None:
        _default = Context(int(os.environ.get("LOCAL_RANK", "0")))
    return _default


# ---------------------------------------------------------------- reference-shaped mirror
class Digest(tuple):
    """twenty-first Digest: 5 canonical BFieldElement values."""

    def __new__(cls, values: Iterable[int]):
        vals = tuple(int(v) % P for v in values)
        if len(vals) != DIGEST_LEN:
            raise ValueError("Digest has 5 elements")
        return super().__new__(cls, vals)

    def values(self) -> Tuple[int, ...]:
        return tuple(self)

    def to_hex(self) -> str:
        return b"".join(v.to_bytes(8, "little") for v in self).hex()

    @classmethod
    def from_hex(cls, h: str) -> "Digest":
        b = bytes.fromhex(h)
        if len(b) != 40:
            raise ValueError("Digest hex is 40 bytes")
        vals = [int.from_bytes(b[8 * i:8 * i + 8], "little") for i in range(5)]
        if any(v >= P for v in vals):
            raise ValueError("non-canonical field element")
        return cls(vals)

    @classmethod
    def default(cls) -> "Digest":
        return cls([0] * 5)


class Tip5:
    """Mirror of twenty-first ``Tip5`` associated functions (GPU-backed)."""

    @staticmethod
    def hash_pair(left: Sequence[int], right: Sequence[int]) -> Digest:
        out = default_context().hash_pair(np.array([list(left)], dtype=np.uint64),
                                          np.array([list(right)], dtype=np.uint64))
        return Digest(int(x) for x in out[0])

    @staticmethod
    def hash_varlen(data: Sequence[int]) -> Digest:
        out = default_context().hash_varlen(rows=[list(data)])
        return Digest(int(x) for x in out[0])

    @staticmethod
    def permutation(state: Sequence[int]) -> List[int]:
        out = default_context().tip5_permutation(np.array([list(state)], dtype=np.uint64))
        return [int(x) for x in out[0]]


class MTree:
    """Mirror of neptune-core's ``MTree`` (pow.rs:60-181)."""

    def __init__(self, leafs: np.ndarray, internal_nodes: np.ndarray):
        self.leafs = leafs
        self.internal_nodes = internal_nodes

    @classmethod
    def build_inplace(cls, leafs) -> "MTree":
        lv = _as_u64(leafs, (5,)).reshape(-1, 5)
        return cls(lv, default_context().mtree_build(lv))

    def root(self) -> Digest:
        if self.internal_nodes.shape[0] < 2:
            return Digest.default()
        return Digest(int(x) for x in self.internal_nodes[1])

    def path(self, index: int) -> List[Digest]:
        n = self.leafs.shape[0]
        running = index + n
        path = [Digest(int(x) for x in self.leafs[index ^ 1])]
        for _ in range(1, n.bit_length() - 1):
            running >>= 1
            path.append(Digest(int(x) for x in self.internal_nodes[running ^ 1]))
        return path

    @staticmethod
    def verify(root: Sequence[int], index: int, path: Sequence[Sequence[int]], element: Sequence[int]) -> bool:
        depth = len(path)
        paths = np.array([list(d) for d in path], dtype=np.uint64).reshape(-1)
        v = default_context().mtree_verify(np.array(list(root), dtype=np.uint64), np.array([index], dtype=np.uint64),
                                           np.array(list(element), dtype=np.uint64), paths, depth)
        return bool(v[0])

    @staticmethod
    def verify_batch(root, indices, paths, elements, depth: int) -> np.ndarray:
        return default_context().mtree_verify(root, indices, elements, paths, depth)
