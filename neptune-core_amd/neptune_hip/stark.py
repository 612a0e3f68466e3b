"""Host mirror of `triton_vm::verify(stark, claim, proof) -> bool` and its batched form over the
C ABI (nhip_verify_batch / nhip_batch_*).

Reference call site: neptune-core/src/protocol/proof_abstractions/verifier.rs:60-63
(`task::spawn_blocking(move || triton_vm::verify(Stark::default(), &claim, &proof))`); batch
callers that verify sequentially today: proof_collection.rs:342-388, block_program.rs:51-65,
state/mod.rs:2226-2272.  `Stark` mirrors `Stark::default()` plus the table dimensions, `Claim` the
triton-vm Claim fields, a proof is the flat `Proof(Vec<BFieldElement>)` word vector.
"""
from __future__ import annotations

import ctypes
import dataclasses
from dataclasses import dataclass, field
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import check


@dataclass
class Stark:
    security_level: int = 160
    log2_fri_expansion: int = 2
    num_collinearity_checks: int = 80
    num_main: int = 379
    num_aux: int = 88
    num_quotient_segments: int = 4
    # how the claims' and proofs' field elements are given (nhip_stark_params.input_form): canonical
    # values, or twenty-first's in-memory Montgomery words (the drop-in hands `Proof.0` over as is)
    input_form: int = _lib.NHIP_INPUT_CANONICAL

    def c(self) -> _lib.StarkParams:
        return _lib.StarkParams(self.security_level, self.log2_fri_expansion, self.num_collinearity_checks,
                                self.num_main, self.num_aux, self.num_quotient_segments, self.input_form)

    @classmethod
    def default(cls) -> "Stark":
        lib = _lib.load()
        p = _lib.StarkParams()
        lib.nhip_stark_params_default(ctypes.byref(p))
        return cls(p.security_level, p.log2_fri_expansion, p.num_collinearity_checks, p.num_main, p.num_aux,
                   p.num_quotient_segments, p.input_form)

    def montgomery(self) -> "Stark":
        """The same parameters taking Montgomery-word input (NHIP_INPUT_MONTGOMERY)."""
        return dataclasses.replace(self, input_form=_lib.NHIP_INPUT_MONTGOMERY)


_P = (1 << 64) - (1 << 32) + 1


def to_montgomery(words) -> np.ndarray:
    """Canonical values (any u64, read mod p) -> twenty-first's in-memory BFieldElement words
    x * 2^64 mod p (goldilocks.hpp to_mont's closed form: with x = h 2^32 + l, x 2^64 == l 2^32 - h - l).
    Host-side test-data preparation: a node's proofs are in this form already."""
    x = np.asarray(words, dtype=np.uint64)
    lo = x & np.uint64(0xFFFFFFFF)
    hi = x >> np.uint64(32)
    s = hi + lo
    t = lo << np.uint64(32)
    v = t - s
    return np.where(t < s, v + np.uint64(_P), v).astype(np.uint64)


def from_montgomery(words) -> np.ndarray:
    """Inverse of to_montgomery: the canonical values of Montgomery words (any u64 read mod p),
    x * 2^-64 = -(x * 2^32) mod p with x = h 2^32 + l: x 2^32 == (h + l) 2^32 - h."""
    x = np.asarray(words, dtype=np.uint64)
    p = np.uint64(_P)
    h = x >> np.uint64(32)
    s = h + (x & np.uint64(0xFFFFFFFF))
    t1 = ((s & np.uint64(0xFFFFFFFF)) << np.uint64(32)) + (s >> np.uint64(32)) * np.uint64(0xFFFFFFFF)
    t1 = np.where(t1 >= p, t1 - p, t1)
    t = np.where(t1 >= h, t1 - h, t1 + (p - h))
    return np.where(t == 0, t, p - t).astype(np.uint64)


def montgomery_claim(c: "Claim") -> "Claim":
    """A claim's field elements (digest, input, output) as Montgomery words; version unchanged."""
    return Claim([int(v) for v in to_montgomery(list(c.program_digest))], c.version,
                 [int(v) for v in to_montgomery(list(c.input))] if len(c.input) else [],
                 [int(v) for v in to_montgomery(list(c.output))] if len(c.output) else [])


def set_fs_form(form: int) -> None:
    """Fiat-Shamir replay form of later launches (nhip_set_fs_form): -1 by batch size, 0 row, 1 pair,
    2 quad (tests / A/B runs)."""
    check(_lib.load().nhip_set_fs_form(int(form)), "nhip_set_fs_form")


@dataclass
class Claim:
    program_digest: Sequence[int]
    version: int = 0
    input: Sequence[int] = field(default_factory=list)
    output: Sequence[int] = field(default_factory=list)


class Air:
    """AIR circuit descriptor (format: DESIGN.md §9)."""

    def __init__(self, words: Sequence[int], lds_slots: int = 0, step_width: int = 0, slot_budget: int = 0):
        """lds_slots / step_width / slot_budget: the OOD program compiler's options
        (nhip_air_create_ex; 0 = default): tests of the compiler and of the global-slot path."""
        self.lib = _lib.load()
        w = np.ascontiguousarray(np.asarray(words, dtype=np.uint64))
        h = ctypes.c_void_p()
        opts = (ctypes.c_uint32 * 3)(lds_slots, step_width, slot_budget)
        check(self.lib.nhip_air_create_ex(w, w.size, ctypes.cast(opts, ctypes.c_void_p), ctypes.byref(h)),
              "nhip_air_create_ex")
        self.handle = h.value

    def info(self):
        a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        check(self.lib.nhip_air_info(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "air_info")
        lds, glob = ctypes.c_uint32(), ctypes.c_uint32()
        check(self.lib.nhip_air_slots(self.handle, ctypes.byref(lds), ctypes.byref(glob)), "air_slots")
        return {"nodes": a.value, "levels": b.value, "constraints": c.value, "lds_slots": lds.value,
                "global_slots": glob.value}

    def program(self):
        """The compiled OOD program (nhip_air_program): step offsets and an (n, 4) array of
        (op, a, b, dst) instructions."""
        ns, ni = ctypes.c_size_t(), ctypes.c_size_t()
        check(self.lib.nhip_air_program(self.handle, None, 0, None, 0, ctypes.byref(ns), ctypes.byref(ni)),
              "nhip_air_program")
        off = np.zeros(ns.value + 1, dtype=np.uint32)
        ins = np.zeros((max(ni.value, 1), 4), dtype=np.uint32)
        check(self.lib.nhip_air_program(self.handle, off.ctypes.data, off.size, ins.ctypes.data, ins.size,
                                        ctypes.byref(ns), ctypes.byref(ni)), "nhip_air_program")
        return off, ins[:ni.value]

    def __del__(self):
        try:
            if self.handle:
                self.lib.nhip_air_destroy(self.handle)
        except Exception:
            pass


class _Marshal:
    """Keeps the numpy buffers alive while the C structs point into them."""

    def __init__(self, claims: Sequence[Claim], proofs: Sequence[Sequence[int]]):
        n = len(claims)
        self.keep = []
        self.claims = (_lib.Claim * max(n, 1))()
        self.proofs = (_lib.Proof * max(n, 1))()
        u64 = ctypes.POINTER(ctypes.c_uint64)
        for i, (c, pw) in enumerate(zip(claims, proofs)):
            inp = np.ascontiguousarray(np.asarray(list(c.input), dtype=np.uint64))
            out = np.ascontiguousarray(np.asarray(list(c.output), dtype=np.uint64))
            pa = np.ascontiguousarray(np.asarray(pw, dtype=np.uint64))
            self.keep += [inp, out, pa]
            cc = self.claims[i]
            for k in range(5):
                cc.program_digest[k] = int(c.program_digest[k])
            cc.version = int(c.version)
            cc.input = inp.ctypes.data_as(u64) if inp.size else None
            cc.input_len = inp.size
            cc.output = out.ctypes.data_as(u64) if out.size else None
            cc.output_len = out.size
            self.proofs[i].words = pa.ctypes.data_as(u64) if pa.size else None
            self.proofs[i].len = pa.size
        self.n = n


def marshal(claims: Sequence[Claim], proofs: Sequence[Sequence[int]]):
    """The C claim / proof arrays over `proofs`' memory (no copy for contiguous uint64 arrays)."""
    return _Marshal(claims, proofs)


class Batch:
    """Device-resident batch: decode + upload once, run the device phases any number of times."""

    def __init__(self, ctx, air: Air, stark: Stark, claims: Sequence[Claim], proofs: Sequence[Sequence[int]]):
        self.ctx, self.air, self.stark = ctx, air, stark
        m = _Marshal(claims, proofs)
        self.n = m.n
        h = ctypes.c_void_p()
        params = stark.c()
        check(ctx.lib.nhip_batch_prepare(ctx.handle, air.handle, ctypes.byref(params), m.claims, m.proofs, m.n,
                                         ctypes.byref(h)), "nhip_batch_prepare")
        self.handle = h.value

    def refill(self, claims: Sequence[Claim], proofs: Sequence[Sequence[int]] = None, marshalled=None) -> None:
        """Replace the batch's proofs in place (`nhip_batch_refill`; the batch must be idle).
        `marshalled`: a `marshal(claims, proofs)` made once and reused (streaming the same buffers
        again without re-building the C structs in Python)."""
        m = marshalled if marshalled is not None else _Marshal(claims, proofs)
        params = self.stark.c()
        self.n = 0
        check(self.ctx.lib.nhip_batch_refill(self.ctx.handle, self.handle, self.air.handle, ctypes.byref(params),
                                             m.claims, m.proofs, m.n), "nhip_batch_refill")
        self.n = m.n

    def run(self) -> Tuple[np.ndarray, bool]:
        v = np.zeros(max(self.n, 1), dtype=np.uint8)
        ok = ctypes.c_uint8(0)
        check(self.ctx.lib.nhip_batch_run(self.ctx.handle, self.handle, v, ctypes.byref(ok)), "nhip_batch_run")
        return v[:self.n], bool(ok.value)

    def launch(self) -> None:
        """Enqueue the device phases on the batch's own streams (returns immediately)."""
        check(self.ctx.lib.nhip_batch_launch(self.ctx.handle, self.handle), "nhip_batch_launch")

    def wait(self) -> Tuple[np.ndarray, bool]:
        v = np.zeros(max(self.n, 1), dtype=np.uint8)
        ok = ctypes.c_uint8(0)
        check(self.ctx.lib.nhip_batch_wait(self.ctx.handle, self.handle, v, ctypes.byref(ok)), "nhip_batch_wait")
        return v[:self.n], bool(ok.value)

    def set_launch_timing(self, on: bool = True) -> "Batch":
        """Per-dispatch timestamps on the Merkle hash and row launches (stats ms_mp_hash_exec /
        ms_row_hash_exec); off by default (nhip_batch_set_launch_timing)."""
        check(self.ctx.lib.nhip_batch_set_launch_timing(self.handle, 1 if on else 0), "nhip_batch_set_launch_timing")
        return self

    def set_streams(self, streams: int) -> "Batch":
        """2 (default): the latency-bound chain and the hashing overlap on two streams; 1: every
        phase in order on one stream, so twice as many tiny batches fit in flight
        (nhip_batch_set_streams)."""
        check(self.ctx.lib.nhip_batch_set_streams(self.handle, int(streams)), "nhip_batch_set_streams")
        return self

    def set_graph(self, on: bool = True) -> "Batch":
        """Replay later untimed launches from a captured HIP graph (nhip_batch_set_graph): resident
        batches of at most 1,024 proofs relaunched many times; a replayed launch has no phase split."""
        check(self.ctx.lib.nhip_batch_set_graph(self.handle, 1 if on else 0), "nhip_batch_set_graph")
        return self

    def stats(self) -> dict:
        s = _lib.Stats()
        check(self.ctx.lib.nhip_batch_stats(self.handle, ctypes.byref(s)), "nhip_batch_stats")
        return s.as_dict()

    def transcript(self, i: int, max_xfe: int = 1 << 16):
        xs = np.zeros(3 * max_xfe, dtype=np.uint64)
        k = self.stark.num_collinearity_checks
        idx = (ctypes.c_uint32 * k)()
        fail = ctypes.c_uint32(0)
        nx = ctypes.c_size_t(0)
        check(self.ctx.lib.nhip_batch_transcript(self.ctx.handle, self.handle, i, xs, max_xfe, idx, k,
                                                 ctypes.byref(fail), ctypes.byref(nx)), "nhip_batch_transcript")
        n = min(nx.value, max_xfe)
        return [tuple(int(v) for v in xs[3 * j:3 * j + 3]) for j in range(n)], list(idx), fail.value

    def close(self):
        if self.handle:
            self.ctx.lib.nhip_batch_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def verify_batch(ctx, air: Air, stark: Stark, pairs: Sequence[Tuple[Claim, Sequence[int]]]) -> List[bool]:
    """`verify_batch(&[(Claim, Proof)]) -> Vec<bool>`."""
    claims = [c for c, _ in pairs]
    proofs = [p for _, p in pairs]
    m = _Marshal(claims, proofs)
    v = np.zeros(max(m.n, 1), dtype=np.uint8)
    stats = _lib.Stats()
    params = stark.c()
    check(ctx.lib.nhip_verify_batch(ctx.handle, air.handle, ctypes.byref(params), m.claims, m.proofs, m.n, v,
                                    ctypes.byref(stats)), "nhip_verify_batch")
    return [bool(x) for x in v[:m.n]]


def verify(ctx, air: Air, stark: Stark, claim: Claim, proof: Sequence[int]) -> bool:
    """`triton_vm::verify(stark, &claim, &proof) -> bool`."""
    return verify_batch(ctx, air, stark, [(claim, proof)])[0]


class Queue:
    """Coalescing verifier for concurrent callers (``nhip_queue``): ``verify(claim, proof)`` from
    any number of threads; the proofs of callers waiting at the same time are verified in one
    device batch (ctypes releases the GIL during the blocking C call)."""

    def __init__(self, ctx, air: Air, stark: Stark, max_batch: int = 0, max_wait_us: int = 200):
        self.ctx, self.air, self.stark = ctx, air, stark
        h = ctypes.c_void_p()
        params = stark.c()
        check(ctx.lib.nhip_queue_create(ctx.handle, air.handle, ctypes.byref(params), max_batch, max_wait_us,
                                        ctypes.byref(h)), "nhip_queue_create")
        self.handle = h.value

    def verify_many(self, pairs: Sequence[Tuple[Claim, Sequence[int]]]) -> List[bool]:
        m = _Marshal([c for c, _ in pairs], [p for _, p in pairs])
        v = np.zeros(max(m.n, 1), dtype=np.uint8)
        check(self.ctx.lib.nhip_queue_verify(self.handle, m.claims, m.proofs, m.n, v.ctypes.data), "nhip_queue_verify")
        return [bool(x) for x in v[:m.n]]

    def verify(self, claim: Claim, proof: Sequence[int]) -> bool:
        return self.verify_many([(claim, proof)])[0]

    def stats(self):
        b, p = ctypes.c_uint64(), ctypes.c_uint64()
        check(self.ctx.lib.nhip_queue_stats(self.handle, ctypes.byref(b), ctypes.byref(p)), "nhip_queue_stats")
        return {"batches": b.value, "proofs": p.value}

    def profile(self, reset: bool = False) -> dict:
        """Where the queue's time went (nhip_queue_profile_read): per-batch window / stage / upload /
        launch / device / wait / turnaround milliseconds summed, and the batch-size histogram."""
        pr = _lib.QueueProfile()
        check(self.ctx.lib.nhip_queue_profile_read(self.handle, ctypes.byref(pr), int(reset)), "nhip_queue_profile_read")
        return pr.as_dict()

    def latencies_ms(self, reset: bool = False) -> np.ndarray:
        """Per-request latency (arrival -> verdicts delivered) of the last <= 65,536 requests, as the
        library measured it (nhip_queue_latencies), oldest first, in milliseconds."""
        n = ctypes.c_size_t()
        check(self.ctx.lib.nhip_queue_latencies(self.handle, None, 0, ctypes.byref(n), 0), "nhip_queue_latencies")
        out = np.zeros(max(n.value, 1), dtype=np.float32)
        check(self.ctx.lib.nhip_queue_latencies(self.handle, out.ctypes.data, n.value, ctypes.byref(n), int(reset)),
              "nhip_queue_latencies")
        return out[:n.value].astype(np.float64) / 1e3

    def close(self):
        if self.handle:
            self.ctx.lib.nhip_queue_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class PinnedProofs:
    """Proofs copied back to back into one pinned host buffer (``nhip_host_alloc``): batches
    staged from them are DMA'd straight from this memory (no staging copy).  ``views`` are the
    proofs as numpy arrays over the pinned buffer."""

    def __init__(self, proofs: Sequence[Sequence[int]], near=None):
        """``near``: a Context whose GPU's NUMA node the buffer is placed on (nhip_host_alloc_near,
        the receive path of a node feeding that GPU); None: nhip_host_alloc."""
        self.lib = _lib.load()
        arrs = [np.asarray(p, dtype=np.uint64) for p in proofs]
        total = sum(a.size for a in arrs)
        h = ctypes.c_void_p()
        if near is not None:
            check(self.lib.nhip_host_alloc_near(near.handle, max(total, 1) * 8, ctypes.byref(h)), "nhip_host_alloc_near")
        else:
            check(self.lib.nhip_host_alloc(max(total, 1) * 8, ctypes.byref(h)), "nhip_host_alloc")
        self.ptr = h.value
        buf = (ctypes.c_uint64 * max(total, 1)).from_address(self.ptr)
        self.flat = np.frombuffer(buf, dtype=np.uint64, count=max(total, 1))
        self.views, off = [], 0
        for a in arrs:
            self.flat[off:off + a.size] = a
            self.views.append(self.flat[off:off + a.size])
            off += a.size

    def close(self):
        if self.ptr:
            self.views, self.flat = [], None
            self.lib.nhip_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Group:
    """Several GPUs (or several contexts on one GPU) from one process: ``nhip_group``.
    ``Group([0, 1, 2, 3])`` or ``Group(mask=0)`` (every visible device)."""

    def __init__(self, devices: Sequence[int] = None, mask: int = None):
        self.lib = _lib.load()
        h = ctypes.c_void_p()
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
            check(self.lib.nhip_group_create(arr, len(devices), ctypes.byref(h)), "nhip_group_create")
        else:
            check(self.lib.nhip_group_init(ctypes.c_uint32(mask or 0), ctypes.byref(h)), "nhip_group_init")
        self.handle = h.value

    def __len__(self) -> int:
        return int(self.lib.nhip_group_size(self.handle))

    def numa(self) -> List[dict]:
        """Per member: its GPU's NUMA node and CPUs (the member's threads and staging live there)."""
        from . import numa_of
        out = []
        for i in range(len(self)):
            h = self.lib.nhip_group_member(self.handle, i)
            d = numa_of(self.lib, h)
            d["device"] = int(self.lib.nhip_device_ordinal(h))
            out.append(d)
        return out

    def close(self):
        if self.handle:
            self.lib.nhip_group_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def group_shard(proofs: Sequence[Sequence[int]], n_members: int) -> List[int]:
    """Member of each proof under nhip_group_verify_batch's LPT split (host only)."""
    m = _Marshal([Claim([0] * 5) for _ in proofs], proofs)
    out = (ctypes.c_uint32 * max(m.n, 1))()
    check(_lib.load().nhip_group_shard(m.proofs, m.n, n_members, out), "nhip_group_shard")
    return [int(out[i]) for i in range(m.n)]


def verify_batch_group(group: Group, air: Air, stark: Stark,
                       pairs: Sequence[Tuple[Claim, Sequence[int]]]) -> Tuple[List[bool], bool]:
    """`verify_batch(&[(Claim, Proof)])` over every member of the group: (verdicts, all_ok)."""
    claims = [c for c, _ in pairs]
    proofs = [p for _, p in pairs]
    m = _Marshal(claims, proofs)
    v = np.zeros(max(m.n, 1), dtype=np.uint8)
    ok = ctypes.c_uint8(0)
    params = stark.c()
    check(group.lib.nhip_group_verify_batch(group.handle, air.handle, ctypes.byref(params), m.claims, m.proofs, m.n,
                                            v, ctypes.byref(ok)), "nhip_group_verify_batch")
    return [bool(x) for x in v[:m.n]], bool(ok.value)


class GroupStream:
    """Batch after batch over every member of a group (nhip_group_stream_*): each member's share of
    batch k is staged and uploaded while its share of batch k - 1 still runs.  ``submit(pairs)``
    returns the verdicts of the PREVIOUS batch (None for the first), ``finish()`` the last one's."""

    def __init__(self, group: Group, air: Air, stark: Stark):
        self.group, self.air, self.stark = group, air, stark
        self.lib = group.lib
        h = ctypes.c_void_p()
        params = stark.c()
        check(self.lib.nhip_group_stream_create(group.handle, air.handle, ctypes.byref(params), ctypes.byref(h)),
              "nhip_group_stream_create")
        self.handle = h.value
        self._prev = None  # (verdict array, all_ok byte) of the batch in flight

    def submit_marshalled(self, m: "_Marshal"):
        v = np.zeros(max(m.n, 1), dtype=np.uint8)
        ok = (ctypes.c_uint8 * 1)()
        check(self.lib.nhip_group_stream_submit(self.handle, m.claims, m.proofs, m.n, v.ctypes.data,
                                                ctypes.addressof(ok)), "nhip_group_stream_submit")
        prev, self._prev = self._prev, (v[:m.n], ok, m.n)
        return None if prev is None else ([bool(x) for x in prev[0]], bool(prev[1][0]))

    def submit(self, pairs: Sequence[Tuple[Claim, Sequence[int]]]):
        return self.submit_marshalled(_Marshal([c for c, _ in pairs], [p for _, p in pairs]))

    def submit_placed(self, claims: "_Marshal", placed: "Placed"):
        """nhip_group_stream_submit_placed: the proofs an Arena decoded, each to the member it was
        placed on (`claims`: marshal(claims, []) in the proofs' order)."""
        n = placed.n
        if claims.n < n:
            raise ValueError("fewer claims than placed proofs")
        v = np.zeros(max(n, 1), dtype=np.uint8)
        ok = (ctypes.c_uint8 * 1)()
        check(self.lib.nhip_group_stream_submit_placed(self.handle, claims.claims, placed.proofs,
                                                       ctypes.addressof(placed.member_of), n, v.ctypes.data,
                                                       ctypes.addressof(ok)), "nhip_group_stream_submit_placed")
        prev, self._prev = self._prev, (v[:n], ok, n)
        return None if prev is None else ([bool(x) for x in prev[0]], bool(prev[1][0]))

    def finish(self):
        check(self.lib.nhip_group_stream_finish(self.handle), "nhip_group_stream_finish")
        prev, self._prev = self._prev, None
        return None if prev is None else ([bool(x) for x in prev[0]], bool(prev[1][0]))

    def stats(self) -> dict:
        b, p = ctypes.c_uint64(), ctypes.c_uint64()
        st, up, dv = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        check(self.lib.nhip_group_stream_stats(self.handle, ctypes.byref(b), ctypes.byref(p), ctypes.byref(st),
                                               ctypes.byref(up), ctypes.byref(dv)), "nhip_group_stream_stats")
        return {"batches": b.value, "proofs": p.value, "ms_stage": st.value, "ms_upload": up.value,
                "ms_device": dv.value}

    def close(self):
        if self.handle:
            self.lib.nhip_group_stream_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Placed:
    """Proofs an Arena decoded: the C proof records (pointing into the arenas), each proof's member,
    and the wire bytes they came from (kept alive with them)."""

    def __init__(self, cap: int, data=None):
        self.proofs = (_lib.Proof * max(cap, 1))()
        self.member_of = (ctypes.c_uint32 * max(cap, 1))()
        self.n = 0
        self.data = data

    def words(self, i: int) -> np.ndarray:
        """Proof i's words (a view of the pinned arena)."""
        p = self.proofs[i]
        if not p.len:
            return np.zeros(0, dtype=np.uint64)
        return np.ctypeslib.as_array(p.words, shape=(p.len,))

    def members(self) -> List[int]:
        return [int(self.member_of[i]) for i in range(self.n)]


def _byte_buffer(data):
    a = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, dtype=np.uint8)
    return a, len(data)


class Arena:
    """Per-member pinned proof arenas of a group (nhip_arena_*): wire bytes (bincode
    TransferTransactions, blk files, or explicit word spans) decoded straight into pinned memory on
    each member GPU's NUMA node, each proof on the least-loaded member, ready for
    ``GroupStream.submit_placed``.  The words are canonical values (Stark input_form canonical)."""

    def __init__(self, group: Group, bytes_per_member: int):
        self.group = group
        self.lib = group.lib
        h = ctypes.c_void_p()
        check(self.lib.nhip_arena_create(group.handle, int(bytes_per_member), ctypes.byref(h)), "nhip_arena_create")
        self.handle = h.value

    def reset(self) -> None:
        check(self.lib.nhip_arena_reset(self.handle), "nhip_arena_reset")

    def member_info(self, i: int) -> dict:
        u, c, nd = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        check(self.lib.nhip_arena_member_info(self.handle, i, ctypes.byref(u), ctypes.byref(c), ctypes.byref(nd)),
              "nhip_arena_member_info")
        return {"used_words": u.value, "cap_words": c.value, "page_node": nd.value}

    def ingest_txs(self, data, max_txs: int = None, proof_cap: int = None):
        """Back-to-back TransferTransactions -> (Placed, transactions taken, bytes consumed); stops
        before the first transaction that does not fit (then reset after submitting, and continue)."""
        a, n = _byte_buffer(data)
        cap = proof_cap if proof_cap is not None else max(1, n // 8)
        pl = Placed(cap, a)
        nt, npf, used = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        rc = self.lib.nhip_arena_ingest_txs(self.handle, a.ctypes.data, n, max_txs if max_txs is not None else n,
                                            pl.proofs, ctypes.addressof(pl.member_of), cap, ctypes.byref(nt),
                                            ctypes.byref(npf), ctypes.byref(used))
        pl.n = npf.value
        if rc == _lib.NHIP_ERR_DECODE:
            raise ValueError(f"malformed TransferTransaction after {nt.value} transactions ({used.value} bytes)")
        check(rc, "nhip_arena_ingest_txs")
        return pl, nt.value, used.value

    def ingest_blocks(self, data, pow_tree_height: int):
        """A blk file's bytes -> (Placed, block index of each SingleProof)."""
        a, n = _byte_buffer(data)
        cnt = ctypes.c_size_t()
        check(self.lib.nhip_blk_scan(a.ctypes.data, n, pow_tree_height, None, 0, ctypes.byref(cnt)), "nhip_blk_scan")
        cap = max(cnt.value, 1)
        pl = Placed(cap, a)
        block_of = np.zeros(cap, dtype=np.uint64)
        npf, nb = ctypes.c_size_t(), ctypes.c_size_t()
        check(self.lib.nhip_arena_ingest_blocks(self.handle, a.ctypes.data, n, pow_tree_height, pl.proofs,
                                                ctypes.addressof(pl.member_of), block_of.ctypes.data, cap,
                                                ctypes.byref(npf), ctypes.byref(nb)), "nhip_arena_ingest_blocks")
        pl.n = npf.value
        return pl, [int(x) for x in block_of[:pl.n]]

    def ingest_spans(self, data, spans: Sequence[Tuple[int, int]]):
        """Proofs at (byte offset, words) of `data` -> Placed."""
        a, n = _byte_buffer(data)
        sp = np.ascontiguousarray(np.asarray(spans, dtype=np.uint64).reshape(-1))
        k = sp.size // 2
        pl = Placed(k, a)
        check(self.lib.nhip_arena_ingest_spans(self.handle, a.ctypes.data, n, sp.ctypes.data, k, pl.proofs,
                                               ctypes.addressof(pl.member_of)), "nhip_arena_ingest_spans")
        pl.n = k
        return pl

    def close(self):
        if self.handle:
            self.lib.nhip_arena_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def proof_decodes(air: Air, stark: Stark, claim: Claim, proof: Sequence[int]) -> bool:
    """Host-only structural decode of the proof stream (no GPU)."""
    m = _Marshal([claim], [proof])
    params = stark.c()
    rc = _lib.load().nhip_proof_decodes(air.handle, ctypes.byref(params), m.claims, m.proofs)
    if rc < 0:
        raise _lib.NhipError("nhip_proof_decodes: invalid argument")
    return rc == 1
