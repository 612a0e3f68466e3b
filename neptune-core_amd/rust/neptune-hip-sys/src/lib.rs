//! Raw FFI of `libneptune_hip.so`, the MI355X (gfx950) batched STARK verifier for neptune-core's
//! proof-validation path.  One declaration per entry point of `include/neptune_hip.h` (the C ABI
//! is the contract; `tests/test_rust_crates.py` checks that this file declares every symbol the
//! header does).  Conventions: field elements as canonical u64 (`BFieldElement::value()`), or for
//! the STARK entry points with `input_form = NHIP_INPUT_MONTGOMERY` as twenty-first's in-memory
//! words (a `Vec<BFieldElement>` passed by pointer), caller-owned buffers borrowed for the call,
//! return 0 = ok, otherwise an infrastructure fault (never "accept").  Not compiled in the build
//! container (no Rust toolchain there).
#![allow(non_camel_case_types)]
#![no_std]

use core::ffi::{c_char, c_int, c_uint, c_void};

pub const NHIP_OK: c_int = 0;
pub const NHIP_ERR_NO_DEVICE: c_int = 1;
pub const NHIP_ERR_HIP: c_int = 2;
pub const NHIP_ERR_OOM: c_int = 3;
pub const NHIP_ERR_ARG: c_int = 4;
pub const NHIP_ERR_DECODE: c_int = 5;

pub const NHIP_BLOCK_PROOF_GENESIS: u32 = 0;
pub const NHIP_BLOCK_PROOF_INVALID: u32 = 1;
pub const NHIP_BLOCK_PROOF_SINGLE: u32 = 2;
pub const NHIP_TX_PROOF_COLLECTION: u32 = 0;
pub const NHIP_TX_SINGLE_PROOF: u32 = 1;
pub const NHIP_INPUT_CANONICAL: u32 = 0;
pub const NHIP_INPUT_MONTGOMERY: u32 = 1;
pub const NHIP_HW_QUEUES_RECOMMENDED: u32 = 8;

macro_rules! opaque {
    ($($name:ident),*) => { $( #[repr(C)] pub struct $name { _p: [u8; 0] } )* };
}
opaque!(nhip_ctx, nhip_air, nhip_batch, nhip_group, nhip_group_stream, nhip_queue, nhip_pow_buffer, nhip_arena);

/// `Stark::default()` plus the table dimensions (`nhip_stark_params_default`).
#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct nhip_stark_params {
    pub security_level: u32,
    pub log2_fri_expansion: u32,
    pub num_collinearity_checks: u32,
    pub num_main: u32,
    pub num_aux: u32,
    pub num_quotient_segments: u32,
    /// `NHIP_INPUT_CANONICAL` or `NHIP_INPUT_MONTGOMERY` (claims' and proofs' field elements)
    pub input_form: u32,
}

/// The OOD program compiler's options (`nhip_air_create_ex`; 0 = default for each).
#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct nhip_air_options {
    pub lds_slots: u32,
    pub step_width: u32,
    pub slot_budget: u32,
}

/// `triton_vm::proof::Claim { program_digest, version, input, output }`, words in the params'
/// `input_form`.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct nhip_claim {
    pub program_digest: [u64; 5],
    pub version: u32,
    pub input: *const u64,
    pub input_len: usize,
    pub output: *const u64,
    pub output_len: usize,
}

/// `triton_vm::proof::Proof(Vec<BFieldElement>)`, words in the params' `input_form`.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct nhip_proof {
    pub words: *const u64,
    pub len: usize,
}

#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct nhip_stats {
    pub num_proofs: u64,
    pub proof_words: u64,
    pub tip5_perms_static: u64,
    pub tip5_perms_merkle: u64,
    pub ms_decode: f64,
    pub ms_upload: f64,
    pub ms_fiat_shamir: f64,
    pub ms_row_hash: f64,
    pub ms_merkle: f64,
    pub ms_ood_air: f64,
    pub ms_fri: f64,
    pub ms_deep: f64,
    pub ms_device_total: f64,
    pub ms_merkle_hash: f64,
    pub merkle_hash_launches: u64,
    pub ms_mp_hash_kernel: f64,
    pub mp_hash_kernel_launches: u64,
    pub mp_hash_kernel_perms: u64,
    pub ms_device_decode: f64,
    pub ms_mp_hash_exec: f64,
    pub ms_row_hash_exec: f64,
}

#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct nhip_queue_profile {
    pub batches: u64,
    pub proofs: u64,
    pub size_hist: [u64; 8],
    pub ms_window: f64,
    pub ms_stage: f64,
    pub ms_upload: f64,
    pub ms_launch: f64,
    pub ms_device: f64,
    pub ms_wait: f64,
    pub ms_turnaround: f64,
    pub pinned_proofs: u64,
}

#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct nhip_blk_block {
    pub offset: u64,
    pub size: u64,
    pub height: u64,
    pub timestamp: u64,
    pub prev_block_digest: [u64; 5],
    pub proof_kind: u32,
    pub n_claims: u32,
    pub proof_offset: u64,
    pub proof_len: u64,
    pub kernel_offset: u64,
    pub appendix_offset: u64,
    pub claim_words: u64,
    pub seq_words: u64,
}

#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct nhip_tx {
    pub size: u64,
    pub kind: u32,
    pub n_proofs: u32,
    pub n_lock_scripts: u32,
    pub n_type_scripts: u32,
    pub n_lock_hashes: u32,
    pub n_type_hashes: u32,
    pub n_merge_path: u32,
    pub n_digests: u32,
    pub seq_words: u64,
}

#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct nhip_pow_mast_paths {
    pub pow: [[u64; 5]; 3],
    pub header: [[u64; 5]; 2],
    pub kernel: [[u64; 5]; 1],
}

extern "C" {
    pub fn nhip_init(device_mask: u32, out: *mut *mut nhip_ctx) -> c_int;
    pub fn nhip_destroy(ctx: *mut nhip_ctx);
    pub fn nhip_strerror(code: c_int) -> *const c_char;
    pub fn nhip_device_ordinal(ctx: *const nhip_ctx) -> c_int;
    pub fn nhip_abi_version() -> c_int;
    pub fn nhip_tip5_permutation(ctx: *mut nhip_ctx, states: *mut u64, n: usize) -> c_int;
    pub fn nhip_tip5_hash_pair(ctx: *mut nhip_ctx, left: *const u64, right: *const u64, n: usize,
                               out: *mut u64) -> c_int;
    pub fn nhip_tip5_hash_varlen(ctx: *mut nhip_ctx, data: *const u64, offsets: *const u64, n: usize,
                                 out: *mut u64) -> c_int;
    pub fn nhip_mtree_build(ctx: *mut nhip_ctx, leafs: *const u64, n_leafs: usize, nodes_out: *mut u64) -> c_int;
    pub fn nhip_mtree_verify(ctx: *mut nhip_ctx, roots: *const u64, n_roots: usize, indices: *const u64,
                             leafs: *const u64, paths: *const u64, depth: u32, n: usize, verdicts: *mut u8) -> c_int;
    pub fn nhip_dev_alloc(ctx: *mut nhip_ctx, bytes: usize, dptr: *mut *mut c_void) -> c_int;
    pub fn nhip_dev_free(ctx: *mut nhip_ctx, dptr: *mut c_void) -> c_int;
    pub fn nhip_memcpy_h2d(ctx: *mut nhip_ctx, dst: *mut c_void, src: *const c_void, bytes: usize) -> c_int;
    pub fn nhip_memcpy_d2h(ctx: *mut nhip_ctx, dst: *mut c_void, src: *const c_void, bytes: usize) -> c_int;
    pub fn nhip_synchronize(ctx: *mut nhip_ctx) -> c_int;
    pub fn nhip_tip5_permutation_dev(ctx: *mut nhip_ctx, d_states: *mut u64, n: usize) -> c_int;
    pub fn nhip_tip5_hash_pair_dev(ctx: *mut nhip_ctx, d_left: *const u64, d_right: *const u64, n: usize,
                                   d_out: *mut u64) -> c_int;
    pub fn nhip_tip5_hash_varlen_dev(ctx: *mut nhip_ctx, d_data: *const u64, d_offsets: *const u64, n: usize,
                                     d_out: *mut u64) -> c_int;
    pub fn nhip_mtree_build_dev(ctx: *mut nhip_ctx, d_leafs: *const u64, n_leafs: usize, d_nodes: *mut u64) -> c_int;
    pub fn nhip_mtree_verify_dev(ctx: *mut nhip_ctx, d_roots: *const u64, n_roots: usize,
                                 d_indices: *const u64, d_leafs: *const u64, d_paths: *const u64, depth: u32,
                                 n: usize, d_verdicts: *mut u8) -> c_int;
    pub fn nhip_verdicts_all_dev(ctx: *mut nhip_ctx, d_verdicts: *const u8, n: usize, all_ok: *mut u8) -> c_int;
    pub fn nhip_stark_params_default(out: *mut nhip_stark_params);
    pub fn nhip_air_create(words: *const u64, n_words: usize, out: *mut *mut nhip_air) -> c_int;
    pub fn nhip_air_create_ex(words: *const u64, n_words: usize, options: *const nhip_air_options,
                              out: *mut *mut nhip_air) -> c_int;
    pub fn nhip_air_destroy(air: *mut nhip_air);
    pub fn nhip_air_info(air: *const nhip_air, num_nodes: *mut u32, num_levels: *mut u32,
                         num_constraints: *mut u32) -> c_int;
    pub fn nhip_air_program(air: *const nhip_air, step_off: *mut u32, step_cap: usize, ins: *mut u32, ins_cap: usize,
                            n_steps: *mut usize, n_ins: *mut usize) -> c_int;
    pub fn nhip_air_slots(air: *const nhip_air, lds_slots: *mut u32, global_slots: *mut u32) -> c_int;
    pub fn nhip_proof_decodes(air: *const nhip_air, params: *const nhip_stark_params,
                              claim: *const nhip_claim, proof: *const nhip_proof) -> c_int;
    pub fn nhip_host_alloc(bytes: usize, out: *mut *mut c_void) -> c_int;
    pub fn nhip_host_free(p: *mut c_void) -> c_int;
    pub fn nhip_host_register(p: *mut c_void, bytes: usize) -> c_int;
    pub fn nhip_host_alloc_near(ctx: *mut nhip_ctx, bytes: usize, out: *mut *mut c_void) -> c_int;
    pub fn nhip_device_numa(ctx: *mut nhip_ctx, numa_node: *mut c_int, cpus: *mut c_int, cpu_cap: usize,
                            n_cpus: *mut usize) -> c_int;
    pub fn nhip_numa_from_sysfs(sysfs_root: *const c_char, pci_bus_id: *const c_char, numa_node: *mut c_int,
                                cpus: *mut c_int, cpu_cap: usize, n_cpus: *mut usize) -> c_int;
    pub fn nhip_cpulist_parse(list: *const c_char, cpus: *mut c_int, cpu_cap: usize, n_cpus: *mut usize) -> c_int;
    pub fn nhip_host_page_node(ptr: *const c_void) -> c_int;
    pub fn nhip_set_host_threads(ctx: *mut nhip_ctx, threads: c_uint) -> c_int;
    pub fn nhip_host_unregister(p: *mut c_void) -> c_int;
    pub fn nhip_verify_batch(ctx: *mut nhip_ctx, air: *mut nhip_air, params: *const nhip_stark_params,
                             claims: *const nhip_claim, proofs: *const nhip_proof, n: usize,
                             verdicts: *mut u8, stats: *mut nhip_stats) -> c_int;
    pub fn nhip_batch_prepare(ctx: *mut nhip_ctx, air: *mut nhip_air, params: *const nhip_stark_params,
                              claims: *const nhip_claim, proofs: *const nhip_proof, n: usize,
                              out: *mut *mut nhip_batch) -> c_int;
    pub fn nhip_batch_refill(ctx: *mut nhip_ctx, batch: *mut nhip_batch, air: *mut nhip_air,
                             params: *const nhip_stark_params, claims: *const nhip_claim,
                             proofs: *const nhip_proof, n: usize) -> c_int;
    pub fn nhip_batch_run(ctx: *mut nhip_ctx, batch: *mut nhip_batch, verdicts: *mut u8, all_ok: *mut u8) -> c_int;
    pub fn nhip_batch_launch(ctx: *mut nhip_ctx, batch: *mut nhip_batch) -> c_int;
    pub fn nhip_batch_wait(ctx: *mut nhip_ctx, batch: *mut nhip_batch, verdicts: *mut u8, all_ok: *mut u8) -> c_int;
    pub fn nhip_batch_stats(batch: *const nhip_batch, stats: *mut nhip_stats) -> c_int;
    pub fn nhip_batch_transcript(ctx: *mut nhip_ctx, batch: *const nhip_batch, proof: usize,
                                 xfe_out: *mut u64, xfe_cap: usize, idx_out: *mut u32, idx_cap: usize,
                                 fail_bits: *mut u32, n_xfe: *mut usize) -> c_int;
    pub fn nhip_batch_destroy(batch: *mut nhip_batch);
    pub fn nhip_set_fs_form(form: c_int) -> c_int;
    pub fn nhip_set_climb_from_ops(ops: i64) -> c_int;
    pub fn nhip_batch_set_launch_timing(batch: *mut nhip_batch, on: c_int) -> c_int;
    pub fn nhip_batch_set_streams(batch: *mut nhip_batch, streams: c_int) -> c_int;
    pub fn nhip_batch_set_graph(batch: *mut nhip_batch, on: c_int) -> c_int;
    pub fn nhip_queue_create(ctx: *mut nhip_ctx, air: *mut nhip_air, params: *const nhip_stark_params,
                             max_batch: u32, max_wait_us: u32, out: *mut *mut nhip_queue) -> c_int;
    pub fn nhip_queue_verify(queue: *mut nhip_queue, claims: *const nhip_claim, proofs: *const nhip_proof,
                             n: usize, verdicts: *mut u8) -> c_int;
    pub fn nhip_queue_stats(queue: *const nhip_queue, batches: *mut u64, proofs: *mut u64) -> c_int;
    pub fn nhip_queue_profile_read(queue: *const nhip_queue, out: *mut nhip_queue_profile, reset: c_int) -> c_int;
    pub fn nhip_queue_latencies(queue: *const nhip_queue, us_out: *mut f32, cap: usize, n: *mut usize,
                                reset: c_int) -> c_int;
    pub fn nhip_queue_destroy(queue: *mut nhip_queue);
    pub fn nhip_group_create(devices: *const c_int, n_devices: usize, out: *mut *mut nhip_group) -> c_int;
    pub fn nhip_group_init(device_mask: u32, out: *mut *mut nhip_group) -> c_int;
    pub fn nhip_group_destroy(group: *mut nhip_group);
    pub fn nhip_group_size(group: *const nhip_group) -> usize;
    pub fn nhip_group_member(group: *mut nhip_group, i: usize) -> *mut nhip_ctx;
    pub fn nhip_group_shard(proofs: *const nhip_proof, n: usize, n_members: usize, member_of: *mut u32) -> c_int;
    pub fn nhip_group_verify_batch(group: *mut nhip_group, air: *mut nhip_air,
                                   params: *const nhip_stark_params, claims: *const nhip_claim,
                                   proofs: *const nhip_proof, n: usize, verdicts: *mut u8, all_ok: *mut u8) -> c_int;
    pub fn nhip_group_stream_create(group: *mut nhip_group, air: *mut nhip_air, params: *const nhip_stark_params,
                                    out: *mut *mut nhip_group_stream) -> c_int;
    pub fn nhip_group_stream_submit(stream: *mut nhip_group_stream, claims: *const nhip_claim,
                                    proofs: *const nhip_proof, n: usize, verdicts: *mut u8, all_ok: *mut u8) -> c_int;
    pub fn nhip_group_stream_submit_placed(stream: *mut nhip_group_stream, claims: *const nhip_claim,
                                           proofs: *const nhip_proof, member_of: *const u32, n: usize,
                                           verdicts: *mut u8, all_ok: *mut u8) -> c_int;
    pub fn nhip_group_stream_finish(stream: *mut nhip_group_stream) -> c_int;
    pub fn nhip_group_stream_stats(stream: *const nhip_group_stream, batches: *mut u64, proofs: *mut u64,
                                   ms_stage: *mut f64, ms_upload: *mut f64, ms_device: *mut f64) -> c_int;
    pub fn nhip_group_stream_destroy(stream: *mut nhip_group_stream);
    pub fn nhip_proof_from_be_bytes(bytes: *const u8, n_bytes: usize, words: *mut u64, cap: usize,
                                    n_words: *mut usize) -> c_int;
    pub fn nhip_proof_to_be_bytes(words: *const u64, n: usize, out: *mut u8) -> c_int;
    pub fn nhip_claim_hash(ctx: *mut nhip_ctx, claim: *const nhip_claim, digest_out: *mut u64) -> c_int;
    pub fn nhip_blk_scan(bytes: *const u8, n_bytes: usize, pow_tree_height: u32, blocks: *mut nhip_blk_block,
                         cap: usize, n_blocks: *mut usize) -> c_int;
    pub fn nhip_blk_sequences(bytes: *const u8, n_bytes: usize, pow_tree_height: u32,
                              block: *const nhip_blk_block, words: *mut u64, cap: usize, offsets: *mut u64) -> c_int;
    pub fn nhip_blk_claims(bytes: *const u8, n_bytes: usize, block: *const nhip_blk_block, words: *mut u64,
                           claims: *mut nhip_claim) -> c_int;
    pub fn nhip_le_words(bytes: *const u8, n_bytes: usize, offset: u64, n: usize, out: *mut u64) -> c_int;
    pub fn nhip_tx_scan(bytes: *const u8, n_bytes: usize, tx: *mut nhip_tx) -> c_int;
    pub fn nhip_arena_create(group: *mut nhip_group, bytes_per_member: usize, out: *mut *mut nhip_arena) -> c_int;
    pub fn nhip_arena_destroy(arena: *mut nhip_arena);
    pub fn nhip_arena_reset(arena: *mut nhip_arena) -> c_int;
    pub fn nhip_arena_member_info(arena: *const nhip_arena, member: usize, used_words: *mut u64,
                                  cap_words: *mut u64, page_node: *mut c_int) -> c_int;
    pub fn nhip_arena_ingest_spans(arena: *mut nhip_arena, bytes: *const u8, n_bytes: usize, spans: *const u64,
                                   n: usize, proofs: *mut nhip_proof, member_of: *mut u32) -> c_int;
    pub fn nhip_arena_ingest_txs(arena: *mut nhip_arena, bytes: *const u8, n_bytes: usize, max_txs: usize,
                                 proofs: *mut nhip_proof, member_of: *mut u32, proof_cap: usize, n_txs: *mut usize,
                                 n_proofs: *mut usize, consumed: *mut usize) -> c_int;
    pub fn nhip_arena_ingest_blocks(arena: *mut nhip_arena, bytes: *const u8, n_bytes: usize, pow_tree_height: u32,
                                    proofs: *mut nhip_proof, member_of: *mut u32, block_of: *mut u64,
                                    proof_cap: usize, n_proofs: *mut usize, n_blocks: *mut usize) -> c_int;
    pub fn nhip_tx_parts(bytes: *const u8, n_bytes: usize, tx: *const nhip_tx, seq_words: *mut u64,
                         seq_offsets: *mut u64, proof_spans: *mut u64, digests: *mut u64) -> c_int;
    pub fn nhip_pow_mast_commit(ctx: *mut nhip_ctx, mast: *const nhip_pow_mast_paths, out: *mut u64) -> c_int;
    pub fn nhip_pow_preprocess(ctx: *mut nhip_ctx, height: u32, mast: *const nhip_pow_mast_paths,
                               reboot_rules: c_int, prev_block_digest: *const u64,
                               out: *mut *mut nhip_pow_buffer) -> c_int;
    pub fn nhip_pow_buffer_destroy(buffer: *mut nhip_pow_buffer);
    pub fn nhip_pow_buffer_root(ctx: *mut nhip_ctx, buffer: *const nhip_pow_buffer, out: *mut u64) -> c_int;
    pub fn nhip_pow_buffer_leaf(ctx: *mut nhip_ctx, buffer: *const nhip_pow_buffer, index: u64,
                                out: *mut u64) -> c_int;
    pub fn nhip_pow_buffer_path(ctx: *mut nhip_ctx, buffer: *const nhip_pow_buffer, index: u64,
                                out: *mut u64) -> c_int;
    pub fn nhip_pow_guess_batch(ctx: *mut nhip_ctx, buffer: *const nhip_pow_buffer,
                                mast: *const nhip_pow_mast_paths, index_picker_preimage: *const u64,
                                nonces: *const u64, n: usize, target: *const u64, digests_out: *mut u64,
                                indices_out: *mut u64, success_out: *mut u8) -> c_int;
    pub fn nhip_pow_validate_batch(ctx: *mut nhip_ctx, height: u32, roots: *const u64, paths_a: *const u64,
                                   paths_b: *const u64, nonces: *const u64,
                                   masts: *const nhip_pow_mast_paths, targets: *const u64,
                                   parents: *const u64, reboot_rules: *const u8, n: usize, verdicts: *mut u8) -> c_int;
    pub fn nhip_mast_hash_batch(ctx: *mut nhip_ctx, data: *const u64, offsets: *const u64, fields: u32,
                                n: usize, roots_out: *mut u64) -> c_int;
    pub fn nhip_absolute_index_sets(ctx: *mut nhip_ctx, items: *const u64, sender_randomness: *const u64,
                                    receiver_preimages: *const u64, aocl_leaf_indices: *const u64, n: usize,
                                    minimum_out: *mut u64, distances_out: *mut u32) -> c_int;
    pub fn nhip_timing_enable(ctx: *mut nhip_ctx, on: c_int) -> c_int;
    pub fn nhip_timing_read(ctx: *mut nhip_ctx, total_ms: *mut f64, launches: *mut u64, reset: c_int) -> c_int;
}
