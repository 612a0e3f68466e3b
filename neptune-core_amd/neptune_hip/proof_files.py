"""Proof ingestion formats over the C ABI.

Mirrors neptune-core/src/protocol/proof_abstractions/tasm/program.rs:
  * `proof_filename(claim)` (:355-358): `Tip5::hash(claim).to_hex() + ".proof"`.
  * `try_load_proof_from_disk` (:374-390): 8-byte big-endian chunks, `BFieldElement::new` each;
    a trailing partial chunk -> None.
  * the writer (:565-572): `value().to_be_bytes()` per element.
The words land directly in a numpy buffer that `neptune_hip.stark.Batch` / `verify_batch` take as
a proof (no per-element Python conversion).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from . import _lib
from ._lib import NHIP_ERR_ARG, check


def proof_from_be_bytes(data: bytes) -> Optional[np.ndarray]:
    lib = _lib.load()
    n = ctypes.c_size_t(0)
    buf = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, dtype=np.uint8)
    rc = lib.nhip_proof_from_be_bytes(buf.ctypes.data, len(data), None, 0, ctypes.byref(n))
    if rc == NHIP_ERR_ARG:
        return None
    check(rc, "nhip_proof_from_be_bytes")
    out = np.zeros(max(n.value, 1), dtype=np.uint64)
    check(lib.nhip_proof_from_be_bytes(buf.ctypes.data, len(data), out.ctypes.data, out.size, ctypes.byref(n)),
          "nhip_proof_from_be_bytes")
    return out[:n.value]


def proof_to_be_bytes(words) -> bytes:
    lib = _lib.load()
    w = np.ascontiguousarray(np.asarray(words, dtype=np.uint64))
    out = np.zeros(max(8 * w.size, 1), dtype=np.uint8)
    check(lib.nhip_proof_to_be_bytes(w.ctypes.data if w.size else None, w.size, out.ctypes.data),
          "nhip_proof_to_be_bytes")
    return out[:8 * w.size].tobytes()


def claim_hash(ctx, claim) -> "Digest":
    """`Tip5::hash(claim)` (hash_varlen of the claim's BFieldCodec encoding), on the GPU."""
    from . import Digest
    from .stark import _Marshal
    m = _Marshal([claim], [[]])
    out = np.zeros(5, dtype=np.uint64)
    check(ctx.lib.nhip_claim_hash(ctx.handle, ctypes.byref(m.claims[0]), out), "nhip_claim_hash")
    return Digest(int(x) for x in out)


def proof_filename(ctx, claim) -> str:
    return f"{claim_hash(ctx, claim).to_hex()}.proof"


def try_load_proof_from_disk(path: str) -> Optional[np.ndarray]:
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    return proof_from_be_bytes(data)


def save_proof(path: str, words) -> None:
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(proof_to_be_bytes(words))
    os.replace(tmp, path)
