/*
 * neptune_hip.h — C ABI of libneptune_hip.so, the MI355X (gfx950) batched verifier
 * library for neptune-core's proof-validation hot path.
 *
 * Conventions (mirroring the reference's Rust types; see INTEGRATION.md for bindings):
 *   - Field elements are passed as canonical u64 (BFieldElement::value()).  Inputs >= p are
 *     reduced mod p, i.e. BFieldElement::new semantics.  The STARK entry points also take them as
 *     they lie in a `Vec<BFieldElement>` (nhip_stark_params.input_form = NHIP_INPUT_MONTGOMERY:
 *     twenty-first's raw word x * 2^64 mod p), so a `Proof` is handed over without a copy.
 *   - A Digest is 5 consecutive u64 (Digest::values()), 40 bytes.
 *   - The caller owns every buffer; buffers are borrowed for the duration of the call.
 *   - Return value: 0 (NHIP_OK) or an infrastructure error code (no device, HIP failure,
 *     out of memory, bad argument).  A verification *failure* is never an error: it is a
 *     verdict byte 0.  Callers must treat a non-zero return as "unknown", never as "accept"
 *     (SURVEY.md §8b).
 *   - Thread safety: a context may be shared by threads; calls on one context are serialized
 *     onto that context's HIP stream.
 *   - Every entry point leaves the calling thread's current HIP device as it found it (a host
 *     with its own HIP user, e.g. torch, is not disturbed).
 *   - One context drives one GPU.  Every GPU of a node is driven from the one neptune-core
 *     process by a group (nhip_group_*: one context per member device, batches LPT-sharded at
 *     proof granularity, verdicts merged on the host; nhip_group_stream_* for batch after batch).
 *     The multi-process form (one rank per GPU, one RCCL verdict all-gather per step) is the
 *     Python host's neptune_hip.shard / bench.py.
 *
 * Reference interfaces replaced (paths relative to /root/reference):
 *   nhip_tip5_hash_pair     <- twenty-first 1.0.0 Tip5::hash_pair, as called by
 *                              neptune-core/src/protocol/consensus/block/pow.rs:112,130,171-175
 *   nhip_tip5_hash_varlen   <- Tip5::hash_varlen, as called by
 *                              neptune-core/src/protocol/proof_abstractions/mast_hash.rs:26,
 *                              neptune-core/src/state/wallet/wallet_entropy.rs:76-82 and the
 *                              STARK row hashing inside triton_vm::verify
 *   nhip_tip5_permutation   <- Tip5::permutation (twenty-first, the sponge core)
 *   nhip_mtree_build        <- MTree::build_inplace, neptune-core/src/protocol/consensus/block/pow.rs:73-119
 *   nhip_mtree_verify       <- MTree::verify,        neptune-core/src/protocol/consensus/block/pow.rs:162-180
 *   nhip_sponge_*           <- Tip5 Sponge (pad_and_absorb_all / squeeze / sample_indices /
 *                              sample_scalars) as driven by triton_vm's ProofStream Fiat-Shamir
 *                              (SURVEY.md §8a a13); single call site of the verifier:
 *                              neptune-core/src/protocol/proof_abstractions/verifier.rs:60-63
 */
#ifndef NEPTUNE_HIP_H
#define NEPTUNE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nhip_ctx nhip_ctx;

enum {
    NHIP_OK = 0,
    NHIP_ERR_NO_DEVICE = 1,
    NHIP_ERR_HIP = 2,
    NHIP_ERR_OOM = 3,
    NHIP_ERR_ARG = 4,
    NHIP_ERR_DECODE = 5  /* malformed bincode input (block files, peer transactions) */
};

/* ---- context --------------------------------------------------------------------------- */
/* Hardware queues per process the verifier's pipeline wants: two batches in flight, each with a
 * hashing and a latency stream, plus the context stream (streams that share a queue serialize; HIP's
 * default is 4).  HIP reads GPU_MAX_HW_QUEUES once, at its initialisation.  The library never
 * changes the environment: the operator, or the host binary's main() before it starts any thread,
 * sets GPU_MAX_HW_QUEUES (e.g. to this value) when it wants more than the default. */
#define NHIP_HW_QUEUES_RECOMMENDED 8
/* Bind to the lowest HIP device whose bit is set in device_mask (0 = device 0). */
int nhip_init(uint32_t device_mask, nhip_ctx **out);
void nhip_destroy(nhip_ctx *ctx);
const char *nhip_strerror(int code);
int nhip_device_ordinal(const nhip_ctx *ctx);
/* ABI version: major * 1000 + minor */
int nhip_abi_version(void);

/* ---- Tip5 primitives (host buffers) ----------------------------------------------------- */
/* states: n x 16 u64, permuted in place. */
int nhip_tip5_permutation(nhip_ctx *ctx, uint64_t *states, size_t n);
/* out[i] = Tip5::hash_pair(left[i], right[i]); left/right/out: n digests. */
int nhip_tip5_hash_pair(nhip_ctx *ctx, const uint64_t *left, const uint64_t *right, size_t n, uint64_t *out);
/* Ragged rows: row i = data[offsets[i] .. offsets[i+1]); offsets has n+1 entries.
 * out[i] = Tip5::hash_varlen(row i). */
int nhip_tip5_hash_varlen(nhip_ctx *ctx, const uint64_t *data, const uint64_t *offsets, size_t n, uint64_t *out);

/* ---- MTree (pow.rs) (host buffers) ------------------------------------------------------ */
/* n_leafs a power of two >= 2.  nodes_out: n_leafs digests; nodes_out[1] is the root,
 * node i = hash_pair(node 2i, node 2i+1), leaf k acts as node n_leafs + k; nodes_out[0] = 0. */
int nhip_mtree_build(nhip_ctx *ctx, const uint64_t *leafs, size_t n_leafs, uint64_t *nodes_out);
/* verdicts[i] = MTree::verify(root_i, indices[i], path_i, leafs[i]).
 * roots: n_roots digests with n_roots == 1 (shared root) or n_roots == n.
 * paths: n x depth digests (sibling of the leaf first).  verdicts: n bytes, 1 = accept. */
int nhip_mtree_verify(nhip_ctx *ctx, const uint64_t *roots, size_t n_roots, const uint64_t *indices,
                      const uint64_t *leafs, const uint64_t *paths, uint32_t depth, size_t n, uint8_t *verdicts);

/* ---- device-resident form (pointers from nhip_dev_alloc; asynchronous on the ctx stream) -- */
int nhip_dev_alloc(nhip_ctx *ctx, size_t bytes, void **dptr);
int nhip_dev_free(nhip_ctx *ctx, void *dptr);
int nhip_memcpy_h2d(nhip_ctx *ctx, void *dst, const void *src, size_t bytes);
int nhip_memcpy_d2h(nhip_ctx *ctx, void *dst, const void *src, size_t bytes);
int nhip_synchronize(nhip_ctx *ctx);
int nhip_tip5_permutation_dev(nhip_ctx *ctx, uint64_t *d_states, size_t n);
int nhip_tip5_hash_pair_dev(nhip_ctx *ctx, const uint64_t *d_left, const uint64_t *d_right, size_t n,
                            uint64_t *d_out);
int nhip_tip5_hash_varlen_dev(nhip_ctx *ctx, const uint64_t *d_data, const uint64_t *d_offsets, size_t n,
                              uint64_t *d_out);
int nhip_mtree_build_dev(nhip_ctx *ctx, const uint64_t *d_leafs, size_t n_leafs, uint64_t *d_nodes);
int nhip_mtree_verify_dev(nhip_ctx *ctx, const uint64_t *d_roots, size_t n_roots, const uint64_t *d_indices,
                          const uint64_t *d_leafs, const uint64_t *d_paths, uint32_t depth, size_t n,
                          uint8_t *d_verdicts);
/* *all_ok = AND of n verdict bytes (device buffer), the per-batch / per-block verdict. */
int nhip_verdicts_all_dev(nhip_ctx *ctx, const uint8_t *d_verdicts, size_t n, uint8_t *all_ok);

/* ---- batched STARK verification ---------------------------------------------------------
 * Replaces triton_vm::verify(Stark::default(), &claim, &proof) -> bool at its single production
 * call site neptune-core/src/protocol/proof_abstractions/verifier.rs:60-63, batched
 * (verify_batch) for the sequential callers proof_collection.rs:342-388, block_program.rs:51-65
 * and state/mod.rs:2226-2272.  Semantics: verdict 1 = accept, 0 = reject (any decode or
 * verification error, incl. empty / short / garbage proofs, as in the reference's reject tests).
 * The AIR is data (nhip_air_create; format in DESIGN.md §9): triton-air's generated constraints
 * are not vendored in the reference, so the AIR is supplied by the caller. */
/* How the field elements of the claims and proofs handed to the STARK entry points are given: */
enum {
    NHIP_INPUT_CANONICAL = 0,  /* canonical values (BFieldElement::value()), any u64 read mod p */
    NHIP_INPUT_MONTGOMERY = 1  /* twenty-first's in-memory words (x * 2^64 mod p, BFieldElement's
                                  repr(transparent) u64): Proof.0.as_ptr(), Digest / input /
                                  output slices as they lie, no conversion; any u64 read mod p */
};
typedef struct {
    uint32_t security_level;          /* Stark::default: 160 */
    uint32_t log2_fri_expansion;      /* 2 (expansion factor 4) */
    uint32_t num_collinearity_checks; /* security_level / log2_fri_expansion = 80; <= 256 */
    uint32_t num_main;                /* main table columns (triton-vm: 379) */
    uint32_t num_aux;                 /* auxiliary table columns (triton-vm: 88) */
    uint32_t num_quotient_segments;   /* 4 */
    uint32_t input_form;              /* NHIP_INPUT_CANONICAL (default) or NHIP_INPUT_MONTGOMERY */
} nhip_stark_params;

/* triton_vm::proof::Claim { program_digest, version, input, output } (field elements in the
 * params' input_form; version is a plain integer) */
typedef struct {
    uint64_t program_digest[5];
    uint32_t version;
    const uint64_t *input;
    size_t input_len;
    const uint64_t *output;
    size_t output_len;
} nhip_claim;

/* triton_vm::proof::Proof(Vec<BFieldElement>) */
typedef struct {
    const uint64_t *words;
    size_t len;
} nhip_proof;

typedef struct {
    uint64_t num_proofs, proof_words;
    uint64_t tip5_perms_static;  /* Fiat-Shamir + row hashing (from the proof shapes) */
    uint64_t tip5_perms_merkle;  /* authentication-structure hash_pairs performed (device-counted) + last-codeword trees */
    double ms_decode, ms_upload;  /* host: layout + staging copy (+ DMA issue), then the wait for the uploads */
    double ms_fiat_shamir, ms_row_hash, ms_merkle, ms_ood_air, ms_fri, ms_deep, ms_device_total; /* device */
    double ms_merkle_hash;          /* the per-level hash_pair launches inside ms_merkle */
    uint64_t merkle_hash_launches;  /* number of those launches (one per tree level) */
    /* the lane-per-op k_mp_hash launches only (HIP events around each launch; the small levels
     * run k_mp_hash_wide): summed kernel time, launch count, permutations they performed */
    double ms_mp_hash_kernel;
    uint64_t mp_hash_kernel_launches, mp_hash_kernel_perms;
    double ms_device_decode;        /* k_decode: the proof-stream walk on the device (every run) */
    /* the same hash launches' own durations (dispatch begin / end timestamps of each launch, as the
     * rocprofv3 kernel trace reports them), summed: ms_mp_hash_kernel minus the gaps between them */
    double ms_mp_hash_exec;
    /* the row-hashing launch's own duration (k_hash_rows: every revealed main / aux / quotient row's
     * hash_varlen; dispatch begin / end timestamps) */
    double ms_row_hash_exec;
} nhip_stats;

typedef struct nhip_air nhip_air;
typedef struct nhip_batch nhip_batch;

void nhip_stark_params_default(nhip_stark_params *out);
int nhip_air_create(const uint64_t *words, size_t n_words, nhip_air **out);
/* The OOD program compiler's options (0 = the default for each): LDS-held value slots (fewer puts the
 * rest in the per-proof global area), instructions per program step, working-slot budget.  Tests of
 * the compiler and of k_ood_air's global-slot path; nhip_air_create(w, n, out) = _ex(w, n, NULL, out). */
typedef struct {
    uint32_t lds_slots;
    uint32_t step_width;   /* 16 .. 65536 */
    uint32_t slot_budget;  /* >= 64 */
} nhip_air_options;
int nhip_air_create_ex(const uint64_t *words, size_t n_words, const nhip_air_options *options, nhip_air **out);
void nhip_air_destroy(nhip_air *air);
int nhip_air_info(const nhip_air *air, uint32_t *num_nodes, uint32_t *num_levels, uint32_t *num_constraints);
/* The OOD evaluator's value slots (liveness-allocated): those in LDS, and those past the LDS budget
 * (~6K XFEs), which live in a per-proof global area (an AIR of triton-air's size class). */
int nhip_air_slots(const nhip_air *air, uint32_t *lds_slots, uint32_t *global_slots);
/* The compiled OOD program (host only, for tools and tests of the compiler): steps + 1 step offsets
 * and 4 u32 per instruction (op, a, b, dst; stark.hpp OodIns).  NULL arrays (or too
 * small capacities) just report the sizes; NHIP_ERR_ARG when a given array is too small. */
int nhip_air_program(const nhip_air *air, uint32_t *step_off, size_t step_cap, uint32_t *ins, size_t ins_cap,
                     size_t *n_steps, size_t *n_ins);
/* Host-only structural decode (no GPU needed): 1 = decodes, 0 = malformed, < 0 = bad argument. */
int nhip_proof_decodes(const nhip_air *air, const nhip_stark_params *params, const nhip_claim *claim,
                       const nhip_proof *proof);
/* Pinned host memory for proofs: proofs whose words lie in a range from nhip_host_alloc or
 * nhip_host_register are DMA'd straight from it (no staging copy); adjacent proofs of one range
 * go as one copy.  Any other host memory works too, through the context's pinned staging. */
int nhip_host_alloc(size_t bytes, void **out);
int nhip_host_free(void *p);
int nhip_host_register(void *p, size_t bytes);
int nhip_host_unregister(void *p);
/* ---- host topology of the feed path (NUMA) -------------------------------------------------
 * The receive path of a node feeding GPU ctx: pinned memory whose pages lie on the NUMA node of
 * ctx's GPU (the socket its PCIe link ends at).  A proof deserialized into it is DMA'd as it lies
 * (no staging copy, no inter-socket traffic); free with nhip_host_free.  Falls back to unplaced
 * pinned memory when the platform reports no node.  Replaces the `Vec<BFieldElement>` a peer
 * message is decoded into (peer_loop.rs:315-323, state/mod.rs:2226-2272). */
int nhip_host_alloc_near(nhip_ctx *ctx, size_t bytes, void **out);
/* The NUMA node of ctx's GPU (-1: none reported) and that node's CPUs this process may use, read
 * from sysfs through the device's PCI bus id.  The context's pinned staging is placed on that node
 * and its staging copy threads are bound to those CPUs (NHIP_NUMA=0 disables both).  cpus may be
 * NULL (count query). */
int nhip_device_numa(nhip_ctx *ctx, int *numa_node, int *cpus, size_t cpu_cap, size_t *n_cpus);
/* The same lookup under another sysfs root (host-only, no GPU: tests use fixture trees) for a PCI
 * bus id "dddd:bb:dd.f": <root>/bus/pci/devices/<id>/numa_node, then
 * <root>/devices/system/node/node<N>/cpulist. */
int nhip_numa_from_sysfs(const char *sysfs_root, const char *pci_bus_id, int *numa_node, int *cpus, size_t cpu_cap,
                         size_t *n_cpus);
/* Parse a kernel cpulist ("0-3,8,10-15:2") into sorted CPU ids (host-only). */
int nhip_cpulist_parse(const char *list, int *cpus, size_t cpu_cap, size_t *n_cpus);
/* The NUMA node holding the page at ptr (-1 if unknown; host-only). */
int nhip_host_page_node(const void *ptr);
/* Staging copy threads per upload for this context (0 = default: up to 16, at most its NUMA
 * node's CPUs).  A group sets each member's share of its node's CPUs. */
int nhip_set_host_threads(nhip_ctx *ctx, unsigned threads);
/* One-shot: upload, decode (on the device), verify, verdicts[n]. */
int nhip_verify_batch(nhip_ctx *ctx, nhip_air *air, const nhip_stark_params *params, const nhip_claim *claims,
                      const nhip_proof *proofs, size_t n, uint8_t *verdicts, nhip_stats *stats);
/* Device-resident form: prepare (stage + one upload of the raw proof words), run (every device
 * phase, starting with the proof-stream decode) any number of times, read stats / the
 * Fiat-Shamir transcript of one proof, destroy. */
int nhip_batch_prepare(nhip_ctx *ctx, nhip_air *air, const nhip_stark_params *params, const nhip_claim *claims,
                       const nhip_proof *proofs, size_t n, nhip_batch **out);
/* Refill an idle batch in place with new proofs (same semantics as prepare; its streams,
 * events and device memory are reused when large enough).  Streaming from host memory:
 * launch(A); refill(B, next); wait(A); launch(B); refill(A, next); ... overlaps each host decode
 * + upload with the other batch's device run.  On failure the batch is left empty (n = 0). */
int nhip_batch_refill(nhip_ctx *ctx, nhip_batch *batch, nhip_air *air, const nhip_stark_params *params,
                      const nhip_claim *claims, const nhip_proof *proofs, size_t n);
int nhip_batch_run(nhip_ctx *ctx, nhip_batch *batch, uint8_t *verdicts, uint8_t *all_ok);
/* Asynchronous form of nhip_batch_run: launch enqueues every phase on the batch's own streams and
 * returns; wait blocks until that batch is done.  Batches launched back to back run concurrently
 * (e.g. two half-batches overlap each other's latency-bound tails). */
int nhip_batch_launch(nhip_ctx *ctx, nhip_batch *batch);
int nhip_batch_wait(nhip_ctx *ctx, nhip_batch *batch, uint8_t *verdicts, uint8_t *all_ok);
int nhip_batch_stats(const nhip_batch *batch, nhip_stats *stats);
/* Per-dispatch begin / end timestamps on the batch's Merkle hash launches and its row-hashing
 * launch, read back as nhip_stats.ms_mp_hash_exec / ms_row_hash_exec (0 when off).  Off by
 * default; a benchmark's kernel timing turns it on.  NHIP_ERR_ARG while the batch is in flight. */
int nhip_batch_set_launch_timing(nhip_batch *batch, int on);
/* 2 (default): the batch's latency-bound chain and its hashing run on two streams and overlap; 1:
 * every phase in order on one stream (one hardware queue), so twice as many batches fit in flight —
 * for many tiny batches at once (e.g. 8-64 proofs each).  NHIP_ERR_ARG while in flight. */
int nhip_batch_set_streams(nhip_batch *batch, int streams);
/* on != 0: every later untimed launch replays the batch's launch sequence from a captured HIP graph
 * (one submission instead of ~25 runtime calls), captured now and again after a refill or a stream
 * change — for resident batches of at most 1,024 proofs relaunched many times (a pipeline enqueueing
 * batches back to back otherwise delays each batch's device start by the host enqueues before it).
 * A replayed launch reports no phase split (nhip_stats phase fields 0; launch timing on = direct).
 * NHIP_ERR_ARG while in flight or past 1,024 proofs. */
int nhip_batch_set_graph(nhip_batch *batch, int on);
/* Fiat-Shamir replay form of later launches, process-wide (tests and A/B runs): -1 = chosen by the
 * batch size (default), 0 = 16-lane row, 1 = two-row pair, 2 = quad.  NHIP_ERR_ARG otherwise. */
int nhip_set_fs_form(int form);
/* Merkle climb-from threshold of later launches, process-wide (tests): -1 = the default (trees of
 * at least 24 hash levels hand their remaining levels to one per-tree climb launch at the first level
 * with at most 4,096 hash ops), 0 = never, k > 0 = at k ops for every depth. */
int nhip_set_climb_from_ops(int64_t ops);
/* Samples squeezed for proof `proof` in squeeze order (challenges, quotient weights, z, linear-
 * combination weights, FRI folding challenges, last-round indeterminate) as canonical XFE
 * triples, the FRI indices, and the proof's failure bits (0 = accepted). */
int nhip_batch_transcript(nhip_ctx *ctx, const nhip_batch *batch, size_t proof, uint64_t *xfe_out, size_t xfe_cap,
                          uint32_t *idx_out, size_t idx_cap, uint32_t *fail_bits, size_t *n_xfe);
void nhip_batch_destroy(nhip_batch *batch);

/* ---- coalescing queue for concurrent single-proof callers ---------------------------------
 * The reference calls triton_vm::verify once per proof from many tokio tasks at once
 * (verifier.rs:60-63; e.g. peer_loop.rs:1342 per peer transaction).  nhip_queue_verify is that
 * call: blocking, thread-safe, nhip_verify_batch semantics for its own proofs; a worker thread
 * gathers the proofs of every caller waiting at the time (up to max_batch proofs, at most
 * max_wait_us after the oldest arrival) into one device batch, with the next batch collected while
 * the current one runs.  Each caller copies its proofs into the queue's pinned arena itself (in
 * parallel with the other callers), so the worker only DMAs them; a request the arena cannot hold
 * at the time goes through the context's staging instead.  max_batch 0 = 4096.
 * Pinned footprint: the arena is min(256 MB, max(16 MB, 4 MB x max_batch)) of pinned host memory
 * per queue; the environment variable NHIP_QUEUE_ARENA_MB (read at create) sets it instead, 0 for
 * none. */
typedef struct nhip_queue nhip_queue;
int nhip_queue_create(nhip_ctx *ctx, nhip_air *air, const nhip_stark_params *params, uint32_t max_batch,
                      uint32_t max_wait_us, nhip_queue **out);
int nhip_queue_verify(nhip_queue *queue, const nhip_claim *claims, const nhip_proof *proofs, size_t n,
                      uint8_t *verdicts);
/* batches launched and proofs verified so far */
int nhip_queue_stats(const nhip_queue *queue, uint64_t *batches, uint64_t *proofs);
/* Where a queue's time goes, summed over its batches since creation (or the last reset). */
typedef struct {
    uint64_t batches, proofs;
    uint64_t size_hist[8];   /* batches of 1, 2-3, 4-7, 8-15, 16-31, 32-63, 64-127, >= 128 proofs */
    double ms_window;        /* oldest request's arrival -> its batch's staging starts (coalescing wait) */
    double ms_stage;         /* host: layout + staging copy + DMA issue of the batch's proofs */
    double ms_upload;        /* host: the wait for those uploads */
    double ms_launch;        /* host: enqueueing the batch's device phases */
    double ms_device;        /* device: first phase start -> verdicts (k_decode to the verdict copy) */
    double ms_wait;          /* worker blocked in nhip_batch_wait on the batch (not overlapped) */
    double ms_turnaround;    /* oldest request's arrival -> its verdicts delivered */
    uint64_t pinned_proofs;  /* proofs their caller's thread copied into the queue's pinned arena (DMA'd
                                from there without a staging copy on the worker) */
} nhip_queue_profile;
int nhip_queue_profile_read(const nhip_queue *queue, nhip_queue_profile *out, int reset);
/* Per-request latency in microseconds (a caller's arrival in nhip_queue_verify -> its verdicts
 * delivered), the last 65,536 requests oldest first: *n = how many are held; up to cap written.
 * reset != 0 forgets them. */
int nhip_queue_latencies(const nhip_queue *queue, float *us_out, size_t cap, size_t *n, int reset);
/* Drains the pending requests, then stops the worker. */
void nhip_queue_destroy(nhip_queue *queue);

/* ---- several GPUs from one process --------------------------------------
 * neptune-core is one process; its batch callers (proof_collection.rs:342-388,
 * state/mod.rs:2226-2272, peer_loop.rs:315-323) end in n calls of triton_vm::verify at
 * verifier.rs:60-63.  A group owns one context per member device (duplicates allowed: several
 * contexts on one GPU).  nhip_group_verify_batch shards the proofs over the members (LPT on the
 * proof length, nhip_group_shard), verifies every shard concurrently on its member (one host
 * thread each, nhip_verify_batch semantics) and writes the verdicts in the caller's order;
 * *all_ok (nullable) = AND of the verdicts.  A non-zero return (any member's infrastructure
 * fault) leaves the verdicts unknown: never "accept". */
typedef struct nhip_group nhip_group;
int nhip_group_create(const int *devices, size_t n_devices, nhip_group **out);
/* One member per set bit of device_mask (0 = every visible device). */
int nhip_group_init(uint32_t device_mask, nhip_group **out);
void nhip_group_destroy(nhip_group *group);
size_t nhip_group_size(const nhip_group *group);
/* Borrowed member context (NULL when i is out of range). */
nhip_ctx *nhip_group_member(nhip_group *group, size_t i);
/* member_of[i] = the member proof i goes to: longest proofs first, each to the least-loaded
 * member (host only, deterministic). */
int nhip_group_shard(const nhip_proof *proofs, size_t n, size_t n_members, uint32_t *member_of);
int nhip_group_verify_batch(nhip_group *group, nhip_air *air, const nhip_stark_params *params,
                            const nhip_claim *claims, const nhip_proof *proofs, size_t n, uint8_t *verdicts,
                            uint8_t *all_ok);
/* Streaming form for callers that verify batch after batch (bootstrap import state/mod.rs:2226-2272,
 * block batches peer_loop.rs:315-323): every member keeps two device batches, so each member's share
 * of the next batch is staged and uploaded while the member's share of the current one still runs.
 * nhip_group_stream_submit shards the batch over the members (nhip_group_shard), refills each
 * member's idle device batch with its share and launches it, then waits for the PREVIOUS submitted
 * batch and writes its verdicts / AND into the buffers given with that batch.  When it returns, the
 * claims / proofs of this batch may be reused (they are on the devices); its `verdicts` (n bytes)
 * and `all_ok` (nullable) stay borrowed until the next submit or nhip_group_stream_finish writes
 * them.  A non-zero return is an infrastructure fault: the batches in flight are drained and their
 * verdicts are unknown (never "accept"); the stream stays usable. */
typedef struct nhip_group_stream nhip_group_stream;
int nhip_group_stream_create(nhip_group *group, nhip_air *air, const nhip_stark_params *params,
                             nhip_group_stream **out);
int nhip_group_stream_submit(nhip_group_stream *stream, const nhip_claim *claims, const nhip_proof *proofs,
                             size_t n, uint8_t *verdicts, uint8_t *all_ok);
/* nhip_group_stream_submit with the caller's placement: proof i goes to member member_of[i] (< the
 * group's size) instead of nhip_group_shard's.  For proofs decoded into a member's arena
 * (nhip_arena_ingest_*, which return that placement): each member's share then lies adjacent in
 * pinned memory on its GPU's node and is DMA'd as it lies. */
int nhip_group_stream_submit_placed(nhip_group_stream *stream, const nhip_claim *claims, const nhip_proof *proofs,
                                    const uint32_t *member_of, size_t n, uint8_t *verdicts, uint8_t *all_ok);
/* Waits for the last submitted batch and writes its verdicts. */
int nhip_group_stream_finish(nhip_group_stream *stream);
/* Host / device milliseconds of the stream's batches so far (summed over members: stage = host
 * staging copy + DMA issue, upload = the wait for it, device = the members' device time). */
int nhip_group_stream_stats(const nhip_group_stream *stream, uint64_t *batches, uint64_t *proofs, double *ms_stage,
                            double *ms_upload, double *ms_device);
void nhip_group_stream_destroy(nhip_group_stream *stream);

/* ---- ingestion formats -------------------------------------------
 * Proof files of neptune-core/src/protocol/proof_abstractions/tasm/program.rs:374-390: 8-byte
 * big-endian chunks, each BFieldElement::new (reduced mod p); n_bytes not a multiple of 8 ->
 * NHIP_ERR_ARG (the reference returns None).  words == NULL: size query (*n_words). */
int nhip_proof_from_be_bytes(const uint8_t *bytes, size_t n_bytes, uint64_t *words, size_t cap, size_t *n_words);
/* Writer side (program.rs:565-572): value().to_be_bytes() per element; out: 8 * n bytes. */
int nhip_proof_to_be_bytes(const uint64_t *words, size_t n, uint8_t *out);
/* Tip5::hash(claim) = hash_varlen(claim.encode()) (program.rs:355-358, proof file name). */
int nhip_claim_hash(nhip_ctx *ctx, const nhip_claim *claim, uint64_t digest_out[5]);

/* ---- block files and peer transactions ----------------------------
 * bincode 1.x as neptune-core writes them; host-only, no GPU.  Field lists, BFieldCodec rules and
 * their pin status: neptune-core_amd/csrc/bincode.cpp and DESIGN.md §8f.
 *
 * Block files replace `blocks_from_file_without_record`
 * (state/archival_state/import_blocks_from_files.rs:100-115): blocks back to back, each
 * `bincode::deserialize::<Block>` then advance by its serialized size; a malformed block fails the
 * whole file (NHIP_ERR_DECODE; *n_blocks = the blocks before it).  pow_tree_height is BlockPow's
 * MERKLE_TREE_HEIGHT (pow.rs:33-37: 29, 10 in the reference's test builds). */
enum { NHIP_BLOCK_PROOF_GENESIS = 0, NHIP_BLOCK_PROOF_INVALID = 1, NHIP_BLOCK_PROOF_SINGLE = 2 };
typedef struct {
    uint64_t offset, size;          /* the block's bytes in the buffer */
    uint64_t height, timestamp;     /* BlockHeader::height, ::timestamp (canonical) */
    uint64_t prev_block_digest[5];
    uint32_t proof_kind;            /* BlockProof variant (block/mod.rs:114-119) */
    uint32_t n_claims;              /* BlockAppendix claims */
    uint64_t proof_offset;          /* SingleProof: byte offset of Proof.0's first word */
    uint64_t proof_len;             /* SingleProof: words */
    uint64_t kernel_offset;         /* byte offset of body.transaction_kernel */
    uint64_t appendix_offset;       /* byte offset of the appendix claims */
    uint64_t claim_words;           /* input + output words of all appendix claims */
    uint64_t seq_words;             /* words of nhip_blk_sequences' output (0 on a count-only scan) */
} nhip_blk_block;
/* blocks == NULL: count only.  Otherwise cap >= the block count. */
int nhip_blk_scan(const uint8_t *bytes, size_t n_bytes, uint32_t pow_tree_height, nhip_blk_block *blocks,
                  size_t cap, size_t *n_blocks);
/* BFieldCodec MAST sequences: the transaction kernel's 8 (transaction_kernel.rs:246-277), then the
 * body's sequences 2-4 (block_body.rs:175-182: mutator set accumulator, lock-free MMR, block MMR;
 * sequence 1 is the kernel's MAST hash).  Sequence i = words[offsets[i] .. offsets[i+1]);
 * words == NULL: offsets only (offsets[11] = total words). */
int nhip_blk_sequences(const uint8_t *bytes, size_t n_bytes, uint32_t pow_tree_height, const nhip_blk_block *block,
                       uint64_t *words, size_t cap, uint64_t offsets[12]);
/* The appendix claims: claims[n_claims] whose input / output point into words[claim_words]. */
int nhip_blk_claims(const uint8_t *bytes, size_t n_bytes, const nhip_blk_block *block, uint64_t *words,
                    nhip_claim *claims);
/* n little-endian u64 words at byte `offset` (any alignment), reduced mod p: proof words straight
 * into a (pinned) staging buffer. */
int nhip_le_words(const uint8_t *bytes, size_t n_bytes, uint64_t offset, size_t n, uint64_t *out);

/* Peer transactions: `TransferTransaction { kernel, proof }` (protocol/peer/transfer_transaction.rs:31-47). */
enum { NHIP_TX_PROOF_COLLECTION = 0, NHIP_TX_SINGLE_PROOF = 1 };
typedef struct {
    uint64_t size;                  /* bytes consumed */
    uint32_t kind;                  /* TransferTransactionProof variant */
    uint32_t n_proofs;              /* 1, or ProofCollection::num_proofs() */
    uint32_t n_lock_scripts, n_type_scripts;    /* lock_scripts_halt / type_scripts_halt lengths */
    uint32_t n_lock_hashes, n_type_hashes, n_merge_path;
    uint32_t n_digests;             /* n_lock_hashes + n_type_hashes + 3 + n_merge_path (ProofCollection) */
    uint64_t seq_words;             /* words of the kernel's 8 MAST sequences */
} nhip_tx;
int nhip_tx_scan(const uint8_t *bytes, size_t n_bytes, nhip_tx *tx);
/* seq_words[tx->seq_words] + seq_offsets[9]: the kernel's MAST sequences; proof_spans[2 * n_proofs]:
 * (byte offset, word count) per proof in ProofCollection field order (removal_records_integrity,
 * collect_lock_scripts, lock_scripts_halt.., kernel_to_outputs, collect_type_scripts,
 * type_scripts_halt..; proof_collection.rs:36-49); digests[5 * n_digests]: lock_script_hashes,
 * type_script_hashes, kernel_mast_hash, salted_inputs_hash, salted_outputs_hash, merge_bit_mast_path. */
int nhip_tx_parts(const uint8_t *bytes, size_t n_bytes, const nhip_tx *tx, uint64_t *seq_words,
                  uint64_t seq_offsets[9], uint64_t *proof_spans, uint64_t *digests);

/* ---- per-member proof arenas: wire bytes decoded straight into pinned memory per GPU (§8f row 2)
 * The receive side of the feed path.  An arena set holds, for every member of a group, bytes_per_member
 * of pinned host memory on that member GPU's NUMA node (nhip_host_alloc_near).  The ingest functions
 * scan bincode bytes (blk files: import_blocks_from_files.rs:100-115; peer TransferTransactions:
 * transfer_transaction.rs:31-47), give each proof to the least-loaded member with room (by words) and
 * decode its words (8-byte little-endian, reduced mod p: nhip_le_words, i.e. canonical values ->
 * nhip_stark_params.input_form NHIP_INPUT_CANONICAL) straight into that member's arena, on copy
 * threads bound to the member's node (NHIP_HOST_THREADS, else the group's share per member).  They
 * return nhip_proof records pointing into the arenas and each proof's member, ready for
 * nhip_group_stream_submit_placed.  The arena's proofs stay valid until nhip_arena_reset; reset only
 * after the submit of the batch holding them has returned (its words are then on the devices).
 * Double-buffer with two arena sets to decode batch k + 1 while batch k uploads. */
typedef struct nhip_arena nhip_arena;
int nhip_arena_create(nhip_group *group, size_t bytes_per_member, nhip_arena **out);
void nhip_arena_destroy(nhip_arena *arena);
int nhip_arena_reset(nhip_arena *arena);
/* words placed since the last reset, capacity in words, and the NUMA node of the member's pages
 * (-1: unknown); each output nullable */
int nhip_arena_member_info(const nhip_arena *arena, size_t member, uint64_t *used_words, uint64_t *cap_words,
                           int *page_node);
/* Proofs given as n (byte offset, word count) pairs `spans` of bytes[n_bytes].  NHIP_ERR_OOM when an
 * arena cannot take a proof (the ones before it are placed and decoded). */
int nhip_arena_ingest_spans(nhip_arena *arena, const uint8_t *bytes, size_t n_bytes, const uint64_t *spans, size_t n,
                            nhip_proof *proofs, uint32_t *member_of);
/* Back-to-back TransferTransactions: up to max_txs of them, every proof (a SingleProof's one, a
 * ProofCollection's in field order) in stream order.  Stops early with NHIP_OK, before the
 * transaction that does not fit, when proof_cap or the arenas are full (*consumed < n_bytes: submit,
 * reset, continue from there); NHIP_ERR_DECODE at a malformed transaction (those before it are placed
 * and counted).  *n_txs, *n_proofs, *consumed nullable. */
int nhip_arena_ingest_txs(nhip_arena *arena, const uint8_t *bytes, size_t n_bytes, size_t max_txs, nhip_proof *proofs,
                          uint32_t *member_of, size_t proof_cap, size_t *n_txs, size_t *n_proofs, size_t *consumed);
/* A blk file's bytes: the SingleProof block proof of every block (block_of[i] = its block's index;
 * nullable).  A malformed block fails the whole file (NHIP_ERR_DECODE, nothing placed); NHIP_ERR_ARG
 * when proof_cap is short of the file's SingleProof blocks, NHIP_ERR_OOM when the arenas are. */
int nhip_arena_ingest_blocks(nhip_arena *arena, const uint8_t *bytes, size_t n_bytes, uint32_t pow_tree_height,
                             nhip_proof *proofs, uint32_t *member_of, uint64_t *block_of, size_t proof_cap,
                             size_t *n_proofs, size_t *n_blocks);

/* ---- proof of work (neptune-core/src/protocol/consensus/block/pow.rs) ---
 * PowMastPaths (pow.rs:202-207): MAST authentication paths of the pow field (BlockHeader, 3),
 * the header (BlockKernel, 2) and the kernel (Block, 1); canonical digests. */
typedef struct {
    uint64_t pow[3][5];
    uint64_t header[2][5];
    uint64_t kernel[1][5];
} nhip_pow_mast_paths;
typedef struct nhip_pow_buffer nhip_pow_buffer;
/* PowMastPaths::commit (pow.rs:209-217) */
int nhip_pow_mast_commit(nhip_ctx *ctx, const nhip_pow_mast_paths *mast, uint64_t out[5]);
/* Pow::preprocess (pow.rs:365-469): the guesser buffer of 2^height leaves (buds, 5 bud layers, the
 * HardforkAlpha bit-reversal swap unless reboot_rules, MTree::build_inplace), resident on the
 * device (2 x 2^height x 40 B).  reboot_rules: ConsensusRuleSet::Reboot (bud prefix = mast
 * commit); else HardforkAlpha (bud prefix = prev_block_digest). */
int nhip_pow_preprocess(nhip_ctx *ctx, uint32_t height, const nhip_pow_mast_paths *mast, int reboot_rules,
                        const uint64_t prev_block_digest[5], nhip_pow_buffer **out);
void nhip_pow_buffer_destroy(nhip_pow_buffer *buffer);
/* MTree::root / leafs[index] / MTree::path (pow.rs:147-160) of the buffer's tree */
int nhip_pow_buffer_root(nhip_ctx *ctx, const nhip_pow_buffer *buffer, uint64_t out[5]);
int nhip_pow_buffer_leaf(nhip_ctx *ctx, const nhip_pow_buffer *buffer, uint64_t index, uint64_t out[5]);
int nhip_pow_buffer_path(nhip_ctx *ctx, const nhip_pow_buffer *buffer, uint64_t index, uint64_t *out /* height x 5 */);
/* Pow::guess (pow.rs:471-507) for n nonces: pow digests (fast_mast_hash), the two opened indices,
 * and success = (digest <= target) under twenty-first's Digest ordering (unpinned: canonical
 * values compared from the last element down).  digests_out / indices_out nullable. */
int nhip_pow_guess_batch(nhip_ctx *ctx, const nhip_pow_buffer *buffer, const nhip_pow_mast_paths *mast,
                         const uint64_t index_picker_preimage[5], const uint64_t *nonces, size_t n,
                         const uint64_t target[5], uint64_t *digests_out, uint64_t *indices_out, uint8_t *success_out);
/* Pow::validate (pow.rs:509-557) for n blocks: verdicts[i] = 1 iff both paths verify against the
 * root and the pow digest meets the target.  paths: n x height x 5; reboot_rules: n bytes. */
int nhip_pow_validate_batch(nhip_ctx *ctx, uint32_t height, const uint64_t *roots, const uint64_t *paths_a,
                            const uint64_t *paths_b, const uint64_t *nonces, const nhip_pow_mast_paths *masts,
                            const uint64_t *targets, const uint64_t *parents, const uint8_t *reboot_rules, size_t n,
                            uint8_t *verdicts);

/* ---- MAST and mutator-set hashing ----------------------------------
 * MastHash::mast_hash (neptune-core/src/protocol/proof_abstractions/mast_hash.rs:22-39) of n
 * objects with `fields` (1..16) field sequences each (TransactionKernel: 8): sequence (i, f) =
 * data[offsets[i*fields+f] .. offsets[i*fields+f+1]); roots_out: n digests. */
int nhip_mast_hash_batch(nhip_ctx *ctx, const uint64_t *data, const uint64_t *offsets, uint32_t fields, size_t n,
                         uint64_t *roots_out);
/* AbsoluteIndexSet::compute (util_types/mutator_set/removal_record/absolute_index_set.rs:86-113)
 * for n removal records: minimum_out n x 2 u64 (u128, little-endian), distances_out n x 45 u32. */
int nhip_absolute_index_sets(nhip_ctx *ctx, const uint64_t *items, const uint64_t *sender_randomness,
                             const uint64_t *receiver_preimages, const uint64_t *aocl_leaf_indices, size_t n,
                             uint64_t *minimum_out, uint32_t *distances_out);

/* ---- kernel timing (HIP events on the ctx stream around every kernel launch) ------------ */
int nhip_timing_enable(nhip_ctx *ctx, int on);
/* Total device time of the kernels launched since the last reset, and their count. */
int nhip_timing_read(nhip_ctx *ctx, double *total_ms, uint64_t *launches, int reset);

#ifdef __cplusplus
}
#endif
#endif /* NEPTUNE_HIP_H */
