"""ctypes binding of libneptune_hip.so (C ABI: include/neptune_hip.h).

The shared library is built in-tree (``make -C neptune-core_amd``) and loaded from this
directory.  There is no CPU fallback: if the library is missing or no GPU is present the
calls raise, so a product path can never silently run on something else.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NHIP_LIB") or os.path.join(_HERE, "libneptune_hip.so")

NHIP_OK = 0
NHIP_OK, NHIP_ERR_NO_DEVICE, NHIP_ERR_HIP, NHIP_ERR_OOM, NHIP_ERR_ARG, NHIP_ERR_DECODE = range(6)
_ERRORS = {1: "no HIP device", 2: "HIP runtime error", 3: "out of device memory", 4: "invalid argument",
           5: "malformed encoding"}

_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t

class StarkParams(ctypes.Structure):
    _fields_ = [("security_level", ctypes.c_uint32), ("log2_fri_expansion", ctypes.c_uint32),
                ("num_collinearity_checks", ctypes.c_uint32), ("num_main", ctypes.c_uint32),
                ("num_aux", ctypes.c_uint32), ("num_quotient_segments", ctypes.c_uint32),
                ("input_form", ctypes.c_uint32)]


NHIP_INPUT_CANONICAL, NHIP_INPUT_MONTGOMERY = 0, 1


class Claim(ctypes.Structure):
    _fields_ = [("program_digest", ctypes.c_uint64 * 5), ("version", ctypes.c_uint32),
                ("input", ctypes.POINTER(ctypes.c_uint64)), ("input_len", ctypes.c_size_t),
                ("output", ctypes.POINTER(ctypes.c_uint64)), ("output_len", ctypes.c_size_t)]


class Proof(ctypes.Structure):
    _fields_ = [("words", ctypes.POINTER(ctypes.c_uint64)), ("len", ctypes.c_size_t)]


class Stats(ctypes.Structure):
    _fields_ = [("num_proofs", ctypes.c_uint64), ("proof_words", ctypes.c_uint64),
                ("tip5_perms_static", ctypes.c_uint64), ("tip5_perms_merkle", ctypes.c_uint64),
                ("ms_decode", ctypes.c_double),
                ("ms_upload", ctypes.c_double), ("ms_fiat_shamir", ctypes.c_double),
                ("ms_row_hash", ctypes.c_double), ("ms_merkle", ctypes.c_double),
                ("ms_ood_air", ctypes.c_double), ("ms_fri", ctypes.c_double), ("ms_deep", ctypes.c_double),
                ("ms_device_total", ctypes.c_double), ("ms_merkle_hash", ctypes.c_double),
                ("merkle_hash_launches", ctypes.c_uint64), ("ms_mp_hash_kernel", ctypes.c_double),
                ("mp_hash_kernel_launches", ctypes.c_uint64), ("mp_hash_kernel_perms", ctypes.c_uint64),
                ("ms_device_decode", ctypes.c_double), ("ms_mp_hash_exec", ctypes.c_double),
                ("ms_row_hash_exec", ctypes.c_double)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class QueueProfile(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_uint64), ("proofs", ctypes.c_uint64), ("size_hist", ctypes.c_uint64 * 8),
                ("ms_window", ctypes.c_double), ("ms_stage", ctypes.c_double), ("ms_upload", ctypes.c_double),
                ("ms_launch", ctypes.c_double), ("ms_device", ctypes.c_double), ("ms_wait", ctypes.c_double),
                ("ms_turnaround", ctypes.c_double), ("pinned_proofs", ctypes.c_uint64)]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["size_hist"] = list(self.size_hist)
        return d


class BlkBlock(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("size", ctypes.c_uint64), ("height", ctypes.c_uint64),
                ("timestamp", ctypes.c_uint64), ("prev_block_digest", ctypes.c_uint64 * 5),
                ("proof_kind", ctypes.c_uint32), ("n_claims", ctypes.c_uint32),
                ("proof_offset", ctypes.c_uint64), ("proof_len", ctypes.c_uint64),
                ("kernel_offset", ctypes.c_uint64), ("appendix_offset", ctypes.c_uint64),
                ("claim_words", ctypes.c_uint64), ("seq_words", ctypes.c_uint64)]


class Tx(ctypes.Structure):
    _fields_ = [("size", ctypes.c_uint64), ("kind", ctypes.c_uint32), ("n_proofs", ctypes.c_uint32),
                ("n_lock_scripts", ctypes.c_uint32), ("n_type_scripts", ctypes.c_uint32),
                ("n_lock_hashes", ctypes.c_uint32), ("n_type_hashes", ctypes.c_uint32),
                ("n_merge_path", ctypes.c_uint32), ("n_digests", ctypes.c_uint32), ("seq_words", ctypes.c_uint64)]


_pp = ctypes.POINTER(ctypes.c_void_p)

# (name, argtypes) for every symbol of include/neptune_hip.h
SIGNATURES = {
    "nhip_init": ([ctypes.c_uint32, ctypes.POINTER(_vp)], ctypes.c_int),
    "nhip_destroy": ([_vp], None),
    "nhip_strerror": ([ctypes.c_int], ctypes.c_char_p),
    "nhip_device_ordinal": ([_vp], ctypes.c_int),
    "nhip_abi_version": ([], ctypes.c_int),
    "nhip_tip5_permutation": ([_vp, _u64p, _sz], ctypes.c_int),
    "nhip_tip5_hash_pair": ([_vp, _u64p, _u64p, _sz, _u64p], ctypes.c_int),
    "nhip_tip5_hash_varlen": ([_vp, _u64p, _u64p, _sz, _u64p], ctypes.c_int),
    "nhip_mtree_build": ([_vp, _u64p, _sz, _u64p], ctypes.c_int),
    "nhip_mtree_verify": ([_vp, _u64p, _sz, _u64p, _u64p, _u64p, ctypes.c_uint32, _sz, _u8p], ctypes.c_int),
    "nhip_dev_alloc": ([_vp, _sz, ctypes.POINTER(_vp)], ctypes.c_int),
    "nhip_dev_free": ([_vp, _vp], ctypes.c_int),
    "nhip_memcpy_h2d": ([_vp, _vp, _vp, _sz], ctypes.c_int),
    "nhip_memcpy_d2h": ([_vp, _vp, _vp, _sz], ctypes.c_int),
    "nhip_synchronize": ([_vp], ctypes.c_int),
    "nhip_tip5_permutation_dev": ([_vp, _vp, _sz], ctypes.c_int),
    "nhip_tip5_hash_pair_dev": ([_vp, _vp, _vp, _sz, _vp], ctypes.c_int),
    "nhip_tip5_hash_varlen_dev": ([_vp, _vp, _vp, _sz, _vp], ctypes.c_int),
    "nhip_mtree_build_dev": ([_vp, _vp, _sz, _vp], ctypes.c_int),
    "nhip_mtree_verify_dev": ([_vp, _vp, _sz, _vp, _vp, _vp, ctypes.c_uint32, _sz, _vp], ctypes.c_int),
    "nhip_verdicts_all_dev": ([_vp, _vp, _sz, ctypes.POINTER(ctypes.c_uint8)], ctypes.c_int),
    "nhip_stark_params_default": ([ctypes.POINTER(StarkParams)], None),
    "nhip_air_create": ([_u64p, _sz, _pp], ctypes.c_int),
    "nhip_air_create_ex": ([_u64p, _sz, ctypes.c_void_p, _pp], ctypes.c_int),
    "nhip_air_destroy": ([_vp], None),
    "nhip_air_info": ([_vp, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                       ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
    "nhip_air_program": ([_vp, ctypes.c_void_p, _sz, ctypes.c_void_p, _sz, ctypes.POINTER(_sz), ctypes.POINTER(_sz)],
                         ctypes.c_int),
    "nhip_air_slots": ([_vp, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
    "nhip_proof_from_be_bytes": ([ctypes.c_void_p, _sz, ctypes.c_void_p, _sz, ctypes.POINTER(_sz)], ctypes.c_int),
    "nhip_proof_to_be_bytes": ([ctypes.c_void_p, _sz, ctypes.c_void_p], ctypes.c_int),
    "nhip_claim_hash": ([_vp, ctypes.POINTER(Claim), _u64p], ctypes.c_int),
    "nhip_queue_create": ([_vp, _vp, ctypes.POINTER(StarkParams), ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.POINTER(_vp)], ctypes.c_int),
    "nhip_queue_verify": ([_vp, _vp, _vp, _sz, _vp], ctypes.c_int),
    "nhip_queue_stats": ([_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "nhip_queue_profile_read": ([_vp, ctypes.POINTER(QueueProfile), ctypes.c_int], ctypes.c_int),
    "nhip_queue_destroy": ([_vp], None),
    "nhip_host_alloc": ([_sz, ctypes.POINTER(_vp)], ctypes.c_int),
    "nhip_host_free": ([_vp], ctypes.c_int),
    "nhip_host_register": ([_vp, _sz], ctypes.c_int),
    "nhip_host_alloc_near": ([_vp, _sz, ctypes.POINTER(_vp)], ctypes.c_int),
    "nhip_device_numa": ([_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), _sz,
                          ctypes.POINTER(_sz)], ctypes.c_int),
    "nhip_numa_from_sysfs": ([ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                              ctypes.POINTER(ctypes.c_int), _sz, ctypes.POINTER(_sz)], ctypes.c_int),
    "nhip_cpulist_parse": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), _sz, ctypes.POINTER(_sz)], ctypes.c_int),
    "nhip_host_page_node": ([_vp], ctypes.c_int),
    "nhip_set_host_threads": ([_vp, ctypes.c_uint], ctypes.c_int),
    "nhip_host_unregister": ([_vp], ctypes.c_int),
    "nhip_pow_mast_commit": ([_vp, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nhip_pow_preprocess": ([_vp, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                             ctypes.POINTER(_vp)], ctypes.c_int),
    "nhip_pow_buffer_destroy": ([_vp], None),
    "nhip_pow_buffer_root": ([_vp, _vp, ctypes.c_void_p], ctypes.c_int),
    "nhip_pow_buffer_leaf": ([_vp, _vp, ctypes.c_uint64, ctypes.c_void_p], ctypes.c_int),
    "nhip_pow_buffer_path": ([_vp, _vp, ctypes.c_uint64, ctypes.c_void_p], ctypes.c_int),
    "nhip_pow_guess_batch": ([_vp, _vp, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _sz, ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nhip_pow_validate_batch": ([_vp, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 _sz, ctypes.c_void_p], ctypes.c_int),
    "nhip_mast_hash_batch": ([_vp, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, _sz, ctypes.c_void_p],
                             ctypes.c_int),
    "nhip_absolute_index_sets": ([_vp, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _sz,
                                  ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nhip_proof_decodes": ([_vp, ctypes.POINTER(StarkParams), ctypes.POINTER(Claim), ctypes.POINTER(Proof)],
                           ctypes.c_int),
    "nhip_verify_batch": ([_vp, _vp, ctypes.POINTER(StarkParams), ctypes.POINTER(Claim), ctypes.POINTER(Proof),
                           _sz, _u8p, ctypes.POINTER(Stats)], ctypes.c_int),
    "nhip_group_create": ([ctypes.POINTER(ctypes.c_int), _sz, ctypes.POINTER(_vp)], ctypes.c_int),
    "nhip_group_init": ([ctypes.c_uint32, ctypes.POINTER(_vp)], ctypes.c_int),
    "nhip_group_destroy": ([_vp], None),
    "nhip_group_size": ([_vp], _sz),
    "nhip_group_member": ([_vp, _sz], _vp),
    "nhip_group_shard": ([ctypes.POINTER(Proof), _sz, _sz, ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
    "nhip_group_verify_batch": ([_vp, _vp, ctypes.POINTER(StarkParams), ctypes.POINTER(Claim), ctypes.POINTER(Proof),
                                 _sz, _u8p, ctypes.POINTER(ctypes.c_uint8)], ctypes.c_int),
    "nhip_group_stream_create": ([_vp, _vp, ctypes.POINTER(StarkParams), ctypes.POINTER(_vp)], ctypes.c_int),
    "nhip_group_stream_submit": ([_vp, ctypes.POINTER(Claim), ctypes.POINTER(Proof), _sz, _vp, _vp], ctypes.c_int),
    "nhip_group_stream_submit_placed": ([_vp, ctypes.POINTER(Claim), ctypes.POINTER(Proof), _vp, _sz, _vp, _vp],
                                        ctypes.c_int),
    "nhip_group_stream_finish": ([_vp], ctypes.c_int),
    "nhip_queue_latencies": ([_vp, _vp, _sz, ctypes.POINTER(_sz), ctypes.c_int], ctypes.c_int),
    "nhip_arena_create": ([_vp, _sz, ctypes.POINTER(_vp)], ctypes.c_int),
    "nhip_arena_destroy": ([_vp], None),
    "nhip_arena_reset": ([_vp], ctypes.c_int),
    "nhip_arena_member_info": ([_vp, _sz, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "nhip_arena_ingest_spans": ([_vp, _vp, _sz, _vp, _sz, ctypes.POINTER(Proof), _vp], ctypes.c_int),
    "nhip_arena_ingest_txs": ([_vp, _vp, _sz, _sz, ctypes.POINTER(Proof), _vp, _sz, ctypes.POINTER(_sz),
                               ctypes.POINTER(_sz), ctypes.POINTER(_sz)], ctypes.c_int),
    "nhip_arena_ingest_blocks": ([_vp, _vp, _sz, ctypes.c_uint32, ctypes.POINTER(Proof), _vp, _vp, _sz,
                                  ctypes.POINTER(_sz), ctypes.POINTER(_sz)], ctypes.c_int),
    "nhip_group_stream_stats": ([_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                 ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
    "nhip_group_stream_destroy": ([_vp], None),
    "nhip_batch_prepare": ([_vp, _vp, ctypes.POINTER(StarkParams), ctypes.POINTER(Claim), ctypes.POINTER(Proof),
                            _sz, _pp], ctypes.c_int),
    "nhip_batch_refill": ([_vp, _vp, _vp, ctypes.POINTER(StarkParams), ctypes.POINTER(Claim),
                           ctypes.POINTER(Proof), _sz], ctypes.c_int),
    "nhip_batch_run": ([_vp, _vp, _u8p, ctypes.POINTER(ctypes.c_uint8)], ctypes.c_int),
    "nhip_batch_launch": ([_vp, _vp], ctypes.c_int),
    "nhip_batch_wait": ([_vp, _vp, _u8p, ctypes.POINTER(ctypes.c_uint8)], ctypes.c_int),
    "nhip_batch_stats": ([_vp, ctypes.POINTER(Stats)], ctypes.c_int),
    "nhip_set_fs_form": ([ctypes.c_int], ctypes.c_int),
    "nhip_set_climb_from_ops": ([ctypes.c_int64], ctypes.c_int),
    "nhip_batch_set_launch_timing": ([_vp, ctypes.c_int], ctypes.c_int),
    "nhip_batch_set_streams": ([_vp, ctypes.c_int], ctypes.c_int),
    "nhip_batch_set_graph": ([_vp, ctypes.c_int], ctypes.c_int),
    "nhip_batch_transcript": ([_vp, _vp, _sz, _u64p, _sz, ctypes.POINTER(ctypes.c_uint32), _sz,
                               ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "nhip_batch_destroy": ([_vp], None),
    "nhip_blk_scan": ([_vp, _sz, ctypes.c_uint32, _vp, _sz, ctypes.POINTER(_sz)], ctypes.c_int),
    "nhip_blk_sequences": ([_vp, _sz, ctypes.c_uint32, ctypes.POINTER(BlkBlock), _vp, _sz, _vp], ctypes.c_int),
    "nhip_blk_claims": ([_vp, _sz, ctypes.POINTER(BlkBlock), _vp, _vp], ctypes.c_int),
    "nhip_le_words": ([_vp, _sz, ctypes.c_uint64, _sz, _vp], ctypes.c_int),
    "nhip_tx_scan": ([_vp, _sz, ctypes.POINTER(Tx)], ctypes.c_int),
    "nhip_tx_parts": ([_vp, _sz, ctypes.POINTER(Tx), _vp, _vp, _vp, _vp], ctypes.c_int),
    "nhip_timing_enable": ([_vp, ctypes.c_int], ctypes.c_int),
    "nhip_timing_read": ([_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64), ctypes.c_int],
                         ctypes.c_int),
}

_lib = None
_lock = threading.Lock()


class NhipError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libneptune_hip.so (raises if it has not been built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NhipError(f"{LIB_PATH} is missing: build it with `make -C neptune-core_amd` "
                            "(or __graft_entry__.build()); there is no CPU fallback")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            if os.environ.get("NHIP_LIB") and not hasattr(lib, name):
                continue  # an older build loaded for an A/B comparison
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        _lib = lib
        return lib


def check(rc: int, what: str = ""):
    if rc != NHIP_OK:
        raise NhipError(f"{what}: {_ERRORS.get(rc, f'error {rc}')}")
