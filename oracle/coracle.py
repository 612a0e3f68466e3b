"""ctypes loader for the C restatement oracle (oracle/liboracle_tip5.so) — TEST ORACLE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle_tip5.so")
_lib = None

_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB):
        build()
    L = ctypes.CDLL(_LIB)
    L.oracle_init.argtypes = [_u64p]
    L.oracle_tip5_permutation.argtypes = [_u64p]
    L.oracle_hash_pair.argtypes = [_u64p, _u64p, _u64p]
    L.oracle_hash_varlen.argtypes = [_u64p, ctypes.c_size_t, _u64p]
    L.oracle_hash_varlen_batch.argtypes = [_u64p, _u64p, ctypes.c_size_t, _u64p]
    L.oracle_mtree_verify.argtypes = [_u64p, ctypes.c_uint64, _u64p, ctypes.c_uint32, _u64p]
    L.oracle_mtree_verify.restype = ctypes.c_int
    L.oracle_mtree_verify_batch.argtypes = [_u64p, ctypes.c_size_t, _u64p, _u64p, _u64p, ctypes.c_uint32,
                                            ctypes.c_size_t, _u8p, ctypes.c_int]
    L.oracle_mtree_build.argtypes = [_u64p, ctypes.c_size_t, _u64p]
    # round constants: derived independently in Python from BLAKE3 (see tip5_ref.py)
    import tip5_ref
    rc_raw = np.array([tip5_ref.to_mont(c) for c in tip5_ref.ROUND_CONSTANTS], dtype=np.uint64)
    L.oracle_init(rc_raw)
    _lib = L
    return L


_perm_buf = (ctypes.c_uint64 * 16)()
_perm_fn = None


def permutation_list(state):
    """One Tip5 permutation of a 16-element list (canonical in / out) through the C restatement;
    the drop-in for tip5_ref.permutation installed by tip5_ref.use_c_backend()."""
    global _perm_fn
    if _perm_fn is None:
        f = lib().oracle_tip5_permutation
        _perm_fn = ctypes.CFUNCTYPE(None, ctypes.c_void_p)(ctypes.cast(f, ctypes.c_void_p).value)
    for i in range(16):
        _perm_buf[i] = state[i] % 0xFFFFFFFF00000001
    _perm_fn(ctypes.addressof(_perm_buf))
    return list(_perm_buf)


def permutation_batch(states: np.ndarray) -> np.ndarray:
    L = lib()
    out = np.ascontiguousarray(states, dtype=np.uint64).copy()
    for i in range(out.shape[0]):
        row = np.ascontiguousarray(out[i])
        L.oracle_tip5_permutation(row)
        out[i] = row
    return out


def hash_pair(left, right) -> np.ndarray:
    out = np.zeros(5, dtype=np.uint64)
    lib().oracle_hash_pair(np.ascontiguousarray(left, dtype=np.uint64),
                           np.ascontiguousarray(right, dtype=np.uint64), out)
    return out


def hash_varlen_batch(data: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    n = len(offsets) - 1
    out = np.zeros((n, 5), dtype=np.uint64)
    d = np.ascontiguousarray(data, dtype=np.uint64)
    if d.size == 0:
        d = np.zeros(1, dtype=np.uint64)
    lib().oracle_hash_varlen_batch(d, np.ascontiguousarray(offsets, dtype=np.uint64), n, out)
    return out


def mtree_build(leaves: np.ndarray) -> np.ndarray:
    n = leaves.shape[0]
    nodes = np.zeros((n, 5), dtype=np.uint64)
    lib().oracle_mtree_build(np.ascontiguousarray(leaves, dtype=np.uint64), n, nodes)
    return nodes


def mtree_verify_batch(roots, indices, leaves, paths, depth: int, nthreads: int = 1) -> np.ndarray:
    roots = np.ascontiguousarray(roots, dtype=np.uint64).reshape(-1, 5)
    n = int(np.asarray(indices).shape[0])
    verdicts = np.zeros(max(n, 1), dtype=np.uint8)
    paths = np.ascontiguousarray(paths, dtype=np.uint64)
    if paths.size == 0:
        paths = np.zeros(1, dtype=np.uint64)
    lib().oracle_mtree_verify_batch(roots, roots.shape[0], np.ascontiguousarray(indices, dtype=np.uint64),
                                    np.ascontiguousarray(leaves, dtype=np.uint64).reshape(-1) if n else np.zeros(1, np.uint64),
                                    paths, depth, n, verdicts, nthreads)
    return verdicts[:n]


def set_mds_avx2(on: bool) -> bool:
    """The fast permutation's MDS form: AVX2 (where the host has it) or scalar; returns AVX2 in use."""
    return bool(lib().oracle_set_mds_avx2(1 if on else 0))


def permutation_raw_pair(states_raw: np.ndarray):
    """(reference-form perm_raw, twenty-first-MDS perm_raw_fast) of raw Montgomery states, for the
    cross-check of the two C permutations."""
    L = lib()
    for fn in ("oracle_tip5_permutation_raw", "oracle_tip5_permutation_raw_fast"):
        getattr(L, fn).argtypes = [_u64p]
    a = np.ascontiguousarray(states_raw, dtype=np.uint64).copy()
    b = a.copy()
    for i in range(a.shape[0]):
        ra, rb = np.ascontiguousarray(a[i]), np.ascontiguousarray(b[i])
        L.oracle_tip5_permutation_raw(ra)
        L.oracle_tip5_permutation_raw_fast(rb)
        a[i], b[i] = ra, rb
    return a, b


def stark_batch_args(air_words, params, claims, proofs):
    """The flat arguments of oracle_stark_verify_batch for (claim, proof) pairs, built once (the CPU
    baseline times only the C verifier over them, not this marshaling)."""
    L = lib()
    fn = L.oracle_stark_verify_batch
    fn.argtypes = [_u64p, ctypes.c_size_t, np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS"),
                   _u64p, np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS"), _u64p, _u64p, _u64p,
                   _u64p, _u64p, _u64p, ctypes.c_size_t, _u8p, ctypes.c_int]
    fn.restype = ctypes.c_int
    n = len(proofs)
    air = np.ascontiguousarray(np.asarray(air_words, dtype=np.uint64))
    import math
    pw = np.array([int(math.log2(params.fri_expansion_factor)), params.num_collinearity_checks, params.num_main,
                   params.num_aux, params.num_quotient_segments], dtype=np.uint32)
    dig = np.array([[int(x) % (2 ** 64) for x in c[0]] for c in claims] or [[0] * 5], dtype=np.uint64).reshape(-1)
    ver = np.array([int(c[1]) for c in claims] or [0], dtype=np.uint32)

    def flat(lists):
        if lists and all(isinstance(l, np.ndarray) for l in lists):
            off = np.zeros(len(lists) + 1, dtype=np.uint64)
            off[1:] = np.cumsum([l.size for l in lists])
            data = np.concatenate([np.asarray(l, dtype=np.uint64).reshape(-1) for l in lists] + [np.zeros(1, np.uint64)])
            return np.ascontiguousarray(data), off
        off = np.zeros(len(lists) + 1, dtype=np.uint64)
        for i, l in enumerate(lists):
            off[i + 1] = off[i] + len(l)
        data = np.zeros(max(int(off[-1]), 1), dtype=np.uint64)
        for i, l in enumerate(lists):
            if len(l):
                data[int(off[i]):int(off[i + 1])] = np.asarray(l, dtype=np.uint64)
        return data, off

    ind, ino = flat([list(map(int, c[2])) for c in claims])
    outd, outo = flat([list(map(int, c[3])) for c in claims])
    prd, pro = flat(proofs)
    return (air, air.size, pw, dig, ver, ind, ino, outd, outo, prd, pro, n)


def stark_verify_args(args, threads: int = 1) -> np.ndarray:
    """oracle_stark_verify_batch over stark_batch_args' arrays on `threads` host threads."""
    n = args[-1]
    v = np.zeros(max(n, 1), dtype=np.uint8)
    rc = lib().oracle_stark_verify_batch(*args, v, threads)
    if rc != 0:
        raise ValueError("oracle_stark_verify_batch: malformed AIR or parameters")
    return v[:n]


def stark_verify_batch(air_words, params, claims, proofs, threads: int = 1) -> np.ndarray:
    """C restatement of the verifier (oracle/stark_oracle.c) over (claim, proof) pairs.
    params: oracle StarkParams; claims: (digest, version, input, output) tuples; proofs: word lists."""
    return stark_verify_args(stark_batch_args(air_words, params, claims, proofs), threads)
