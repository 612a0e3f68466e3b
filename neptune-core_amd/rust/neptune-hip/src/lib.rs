//! Drop-in GPU verifier for neptune-core's proof-validation path.
//!
//! Replaces `triton_vm::verify(Stark::default(), &claim, &proof) -> bool` at its single production
//! call site, `neptune-core/src/protocol/proof_abstractions/verifier.rs:60-63`, and adds
//! `verify_batch` for the callers that today verify one proof after another:
//! `ProofCollection::verify` (`proof_collection.rs:342-388`), `BlockProgram::verify`
//! (`block_program.rs:51-65`) and the bootstrap import (`state/mod.rs:2226-2272`).
//!
//! * Semantics are `triton_vm::verify`'s: `true` = accept, `false` = reject (any decode or
//!   verification error).  A [`GpuFault`] is an infrastructure failure (no device, HIP error, out of
//!   memory): the verdict is *unknown*, never "accept"; [`verify_or_cpu`] / [`verify_batch_or_cpu`]
//!   then fall back to the CPU verifier.
//! * The mock-proof gate and the claims cache (`verifier.rs:47-55`) stay in neptune-core, in front
//!   of this crate.
//! * The AIR is data: the descriptor words of triton-air 1.0.0's constraint circuits (format:
//!   DESIGN.md §9 of the neptune-hip repository), exported from the circuits by [`air_export`] and
//!   built once at startup ([`Air::triton`]).
//! * Process-wide use: [`gpu_verifier`] / [`gpu_node`] create the verifier once, on first use,
//!   from the environment (`NEPTUNE_HIP_DEVICE`, `NEPTUNE_HIP_DEVICES`); `None` means "no GPU"
//!   and the callers take the CPU path; why is logged once (`tracing::warn!`) and kept by
//!   [`gpu_verifier_status`] / [`gpu_node_status`].  The library never touches the environment:
//!   call [`provision_hw_queues`] from `main()` before the runtime starts its threads.
//! * Zero copy: proofs and claims are handed to the library as their `BFieldElement` words lie in
//!   memory (Montgomery form, `NHIP_INPUT_MONTGOMERY`); no per-word conversion, no buffer copy.
//!
//! Not compiled in the build container (no Rust toolchain there); the C ABI underneath is
//! exercised by the repository's Python and C99 tests.
use std::ptr;
use std::sync::{Mutex, OnceLock};

pub mod air_export;

use neptune_hip_sys as sys;
use triton_vm::prelude::{BFieldElement, Claim, Digest, Proof, Stark};

/// An infrastructure fault of the GPU path (`NHIP_ERR_*`).  Never means "accept".
#[derive(Debug, Clone, Copy, PartialEq, Eq)]
pub struct GpuFault(pub i32);

impl std::fmt::Display for GpuFault {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        let s = unsafe { std::ffi::CStr::from_ptr(sys::nhip_strerror(self.0)) };
        write!(f, "neptune-hip: {}", s.to_string_lossy())
    }
}
impl std::error::Error for GpuFault {}

fn ok(rc: i32) -> Result<(), GpuFault> {
    if rc == sys::NHIP_OK { Ok(()) } else { Err(GpuFault(rc)) }
}

// twenty-first 1.0.0 holds a BFieldElement as its Montgomery word in a `#[repr(transparent)]`
// u64 newtype, so a `[BFieldElement]` is a `[u64]` of those words: the library reads them as they
// lie (NHIP_INPUT_MONTGOMERY), with no conversion and no copy.
const _: () = assert!(
    std::mem::size_of::<BFieldElement>() == 8 && std::mem::align_of::<BFieldElement>() == std::mem::align_of::<u64>()
);

fn raw_words(v: &[BFieldElement]) -> *const u64 {
    debug_assert!(v.first().map_or(true, |b| unsafe { *(v.as_ptr() as *const u64) } == b.raw_u64()));
    v.as_ptr() as *const u64
}

fn raw_digest(d: &Digest) -> [u64; 5] {
    d.values().map(|b| b.raw_u64())
}

/// `Stark::default()` as the library's parameters (security 160, FRI expansion 4, 80
/// collinearity checks, triton-vm's 379 main / 88 auxiliary columns, 4 quotient segments).
/// Claims and proofs are passed as twenty-first's in-memory words (`input_form` Montgomery).
pub fn default_params() -> sys::nhip_stark_params {
    let mut p = sys::nhip_stark_params::default();
    unsafe { sys::nhip_stark_params_default(&mut p) };
    p.input_form = sys::NHIP_INPUT_MONTGOMERY;
    p
}

/// The AIR descriptor, uploaded lazily to every GPU that uses it.
pub struct Air(*mut sys::nhip_air);
unsafe impl Send for Air {}
unsafe impl Sync for Air {} // read-only after creation; the library guards its device copies

impl Air {
    pub fn from_descriptor(words: &[u64]) -> Result<Self, GpuFault> {
        let mut a = ptr::null_mut();
        ok(unsafe { sys::nhip_air_create(words.as_ptr(), words.len(), &mut a) })?;
        Ok(Air(a))
    }

    /// triton-air 1.0.0's constraints, the AIR `triton_vm::verify` evaluates.  An export failure
    /// is reported as `NHIP_ERR_ARG` (the verifier never runs a partial circuit).
    pub fn triton() -> Result<Self, GpuFault> {
        let words = air_export::triton_air_descriptor().map_err(|_| GpuFault(sys::NHIP_ERR_ARG))?;
        Self::from_descriptor(&words)
    }
}
impl Drop for Air {
    fn drop(&mut self) {
        unsafe { sys::nhip_air_destroy(self.0) }
    }
}

/// The C structs of a batch, pointing straight into the callers' `Claim` / `Proof` memory (no
/// word is converted or copied; the digest's five words are copied into the struct).
struct Marshal<'a> {
    claims: Vec<sys::nhip_claim>,
    proofs: Vec<sys::nhip_proof>,
    _borrow: std::marker::PhantomData<&'a ()>,
}

fn marshal<'a>(items: impl ExactSizeIterator<Item = (&'a Claim, &'a Proof)>) -> Marshal<'a> {
    let mut claims = Vec::with_capacity(items.len());
    let mut proofs = Vec::with_capacity(items.len());
    for (c, p) in items {
        claims.push(sys::nhip_claim {
            program_digest: raw_digest(&c.program_digest),
            version: c.version,
            input: raw_words(&c.input),
            input_len: c.input.len(),
            output: raw_words(&c.output),
            output_len: c.output.len(),
        });
        proofs.push(sys::nhip_proof { words: raw_words(&p.0), len: p.0.len() });
    }
    Marshal { claims, proofs, _borrow: std::marker::PhantomData }
}

/// One GPU: a context, the AIR, and a coalescing queue for single-proof calls.
pub struct Verifier {
    ctx: *mut sys::nhip_ctx,
    air: Air,
    params: sys::nhip_stark_params,
    queue: *mut sys::nhip_queue,
    batch_lock: Mutex<()>,
}
unsafe impl Send for Verifier {}
unsafe impl Sync for Verifier {} // the library serializes calls per context; the queue is thread-safe

impl Verifier {
    /// `device`: HIP ordinal.  `max_wait_us`: how long the queue may hold a single-proof call to
    /// coalesce it with concurrent ones (200 us is a good default: a lone proof takes ~1.7 ms).
    pub fn new(device: u32, air: Air, max_wait_us: u32) -> Result<Self, GpuFault> {
        if device >= 32 {
            return Err(GpuFault(sys::NHIP_ERR_ARG)); // the device mask is 32 bits
        }
        let mut ctx = ptr::null_mut();
        ok(unsafe { sys::nhip_init(1u32 << device, &mut ctx) })?;
        let params = default_params();
        let mut queue = ptr::null_mut();
        if let Err(e) = ok(unsafe { sys::nhip_queue_create(ctx, air.0, &params, 0, max_wait_us, &mut queue) }) {
            unsafe { sys::nhip_destroy(ctx) };
            return Err(e);
        }
        Ok(Verifier { ctx, air, params, queue, batch_lock: Mutex::new(()) })
    }

    /// `triton_vm::verify(Stark::default(), claim, proof)` for one proof, coalesced with the
    /// proofs of concurrent callers (e.g. one tokio blocking task per peer transaction,
    /// `peer_loop.rs:1342`).
    pub fn verify(&self, claim: &Claim, proof: &Proof) -> Result<bool, GpuFault> {
        let m = marshal(std::iter::once((claim, proof)));
        let mut v = [0u8; 1];
        ok(unsafe { sys::nhip_queue_verify(self.queue, m.claims.as_ptr(), m.proofs.as_ptr(), 1, v.as_mut_ptr()) })?;
        Ok(v[0] == 1)
    }

    /// `verify_batch(&[(Claim, Proof)]) -> Vec<bool>`: one device batch.
    pub fn verify_batch(&self, items: &[(Claim, Proof)]) -> Result<Vec<bool>, GpuFault> {
        let m = marshal(items.iter().map(|(c, p)| (c, p)));
        let mut v = vec![0u8; items.len()];
        let _g = self.batch_lock.lock().unwrap_or_else(|e| e.into_inner());
        ok(unsafe {
            sys::nhip_verify_batch(self.ctx, self.air.0, &self.params, m.claims.as_ptr(), m.proofs.as_ptr(),
                                   items.len(), v.as_mut_ptr(), ptr::null_mut())
        })?;
        Ok(v.into_iter().map(|b| b == 1).collect())
    }
}

impl Drop for Verifier {
    fn drop(&mut self) {
        unsafe {
            sys::nhip_queue_destroy(self.queue);
            sys::nhip_destroy(self.ctx);
        }
    }
}

/// Every GPU of the node from the one neptune-core process (`nhip_group`): a batch is split over
/// the GPUs (longest proofs first, each to the least-loaded GPU), the shards are verified
/// concurrently, and the verdicts come back in the caller's order.
pub struct GpuNode {
    group: *mut sys::nhip_group,
    air: Air,
    params: sys::nhip_stark_params,
}
unsafe impl Send for GpuNode {}
unsafe impl Sync for GpuNode {}

impl GpuNode {
    /// One member per set bit of `device_mask` (0 = every visible GPU).
    pub fn init(device_mask: u32, air: Air) -> Result<Self, GpuFault> {
        let mut g = ptr::null_mut();
        ok(unsafe { sys::nhip_group_init(device_mask, &mut g) })?;
        Ok(GpuNode { group: g, air, params: default_params() })
    }

    pub fn gpus(&self) -> usize {
        unsafe { sys::nhip_group_size(self.group) }
    }

    /// (verdicts, AND of the verdicts): the block / ProofCollection verdict is the AND
    /// (`proof_collection.rs:388`).
    pub fn verify_batch(&self, items: &[(Claim, Proof)]) -> Result<(Vec<bool>, bool), GpuFault> {
        let m = marshal(items.iter().map(|(c, p)| (c, p)));
        let mut v = vec![0u8; items.len()];
        let mut all = 0u8;
        ok(unsafe {
            sys::nhip_group_verify_batch(self.group, self.air.0, &self.params, m.claims.as_ptr(), m.proofs.as_ptr(),
                                         items.len(), v.as_mut_ptr(), &mut all)
        })?;
        Ok((v.into_iter().map(|b| b == 1).collect(), all == 1))
    }

    /// Batch after batch (bootstrap import, `state/mod.rs:2226-2272`; block batches,
    /// `peer_loop.rs:315-323`): each GPU's share of the next batch is staged and uploaded while its
    /// share of the current one runs (`nhip_group_stream`).  `on_verdicts(i, verdicts, all_ok)` is
    /// called for batch i once it is verified, in order; the batches are borrowed only until the
    /// next one is submitted.  A fault stops the stream: the batches not yet reported are unknown.
    pub fn verify_stream<'a, I, F>(&self, batches: I, mut on_verdicts: F) -> Result<(), GpuFault>
    where
        I: IntoIterator<Item = &'a [(Claim, Proof)]>,
        F: FnMut(usize, Vec<bool>, bool),
    {
        let mut st = ptr::null_mut();
        ok(unsafe { sys::nhip_group_stream_create(self.group, self.air.0, &self.params, &mut st) })?;
        struct Stream(*mut sys::nhip_group_stream);
        impl Drop for Stream {
            fn drop(&mut self) {
                unsafe { sys::nhip_group_stream_destroy(self.0) }
            }
        }
        let st = Stream(st);
        // verdict buffers of the batch in flight and of the one before it (written one submit later)
        let mut bufs: [(Vec<u8>, u8); 2] = [(Vec::new(), 0), (Vec::new(), 0)];
        let mut k = 0usize;
        for items in batches {
            let m = marshal(items.iter().map(|(c, p)| (c, p)));
            let slot = k & 1;
            bufs[slot].0 = vec![0u8; items.len()];
            let (vp, ap) = (bufs[slot].0.as_mut_ptr(), &mut bufs[slot].1 as *mut u8);
            ok(unsafe { sys::nhip_group_stream_submit(st.0, m.claims.as_ptr(), m.proofs.as_ptr(), items.len(), vp, ap) })?;
            if k > 0 {
                let (v, all) = &bufs[slot ^ 1];
                on_verdicts(k - 1, v.iter().map(|&b| b == 1).collect(), *all == 1);
            }
            k += 1;
        }
        ok(unsafe { sys::nhip_group_stream_finish(st.0) })?;
        if k > 0 {
            let (v, all) = &bufs[(k - 1) & 1];
            on_verdicts(k - 1, v.iter().map(|&b| b == 1).collect(), *all == 1);
        }
        Ok(())
    }
}

impl GpuNode {
    /// (NUMA node, CPUs) of member `i`'s GPU: where its staging lives and its copy threads run.
    pub fn member_numa(&self, i: usize) -> Option<(i32, Vec<i32>)> {
        let ctx = unsafe { sys::nhip_group_member(self.group, i) };
        if ctx.is_null() {
            return None;
        }
        let (mut node, mut n) = (-1i32, 0usize);
        ok(unsafe { sys::nhip_device_numa(ctx, &mut node, ptr::null_mut(), 0, &mut n) }).ok()?;
        let mut cpus = vec![0i32; n];
        let mut got = 0usize;
        ok(unsafe { sys::nhip_device_numa(ctx, &mut node, cpus.as_mut_ptr(), n, &mut got) }).ok()?;
        cpus.truncate(got.min(n));
        Some((node, cpus))
    }

    /// The batch's proofs from a [`ProofArena`] (pinned receive memory): DMA'd as they lie, no
    /// staging copy, split over every GPU (`nhip_group_verify_batch`).  `claims[i]` belongs to
    /// `arena.proof(i)`.
    pub fn verify_arena(&self, claims: &[Claim], arena: &ProofArena) -> Result<(Vec<bool>, bool), GpuFault> {
        let (cs, ps) = arena_marshal(claims, arena)?;
        let mut v = vec![0u8; claims.len()];
        let mut all = 0u8;
        ok(unsafe {
            sys::nhip_group_verify_batch(self.group, self.air.0, &self.params, cs.as_ptr(), ps.as_ptr(), claims.len(),
                                         v.as_mut_ptr(), &mut all)
        })?;
        Ok((v.into_iter().map(|b| b == 1).collect(), all == 1))
    }

    /// One arena per GPU, each on its GPU's NUMA node ([`GpuNode::arenas`]): member `m` verifies the
    /// proofs of `batches[m]` itself (no re-sharding, so no proof crosses the socket link), all
    /// members concurrently.  Returns each member's verdicts and the AND over all of them (the
    /// block / ProofCollection verdict, `proof_collection.rs:388`).
    pub fn verify_arenas(&self, batches: &[(&[Claim], &ProofArena)]) -> Result<(Vec<Vec<bool>>, bool), GpuFault> {
        if batches.len() > self.gpus() {
            return Err(GpuFault(sys::NHIP_ERR_ARG));
        }
        // the C structs hold raw pointers into the arenas and claims, which outlive the scope below
        struct Shard(Vec<sys::nhip_claim>, Vec<sys::nhip_proof>);
        unsafe impl Sync for Shard {}
        let mut marshalled = Vec::with_capacity(batches.len());
        for (claims, arena) in batches {
            let (cs, ps) = arena_marshal(claims, arena)?;
            marshalled.push(Shard(cs, ps));
        }
        let results: Vec<Result<Vec<u8>, GpuFault>> = std::thread::scope(|scope| {
            let handles: Vec<_> = marshalled
                .iter()
                .enumerate()
                .map(|(m, Shard(cs, ps))| {
                    let ctx = unsafe { sys::nhip_group_member(self.group, m) } as usize;
                    let (air, params) = (self.air.0 as usize, &self.params);
                    scope.spawn(move || {
                        let mut v = vec![0u8; cs.len()];
                        ok(unsafe {
                            sys::nhip_verify_batch(ctx as *mut sys::nhip_ctx, air as *mut sys::nhip_air, params, cs.as_ptr(),
                                                   ps.as_ptr(), cs.len(), v.as_mut_ptr(), ptr::null_mut())
                        })
                        .map(|_| v)
                    })
                })
                .collect();
            handles.into_iter().map(|h| h.join().unwrap_or(Err(GpuFault(sys::NHIP_ERR_HIP)))).collect()
        });
        let mut out = Vec::with_capacity(results.len());
        let mut all = true;
        for r in results {
            let v: Vec<bool> = r?.into_iter().map(|b| b == 1).collect();  // any member's fault: unknown
            all &= v.iter().all(|&x| x);
            out.push(v);
        }
        Ok((out, all))
    }

    /// One [`ProofArena`] of `cap_words` words per GPU, each on that GPU's NUMA node.
    pub fn arenas(&self, cap_words: usize) -> Result<Vec<ProofArena>, GpuFault> {
        (0..self.gpus()).map(|m| ProofArena::new(self, m, cap_words)).collect()
    }

    /// Wire bytes to verdicts, batch after batch: each batch is a buffer of back-to-back bincode
    /// `TransferTransaction`s as peers send them (`transfer_transaction.rs:31-47`,
    /// `peer_loop.rs:315-323`).  The library decodes every proof straight into a pinned arena on the
    /// NUMA node of the GPU it places the proof on (`nhip_arena_ingest_txs`) and each GPU DMAs its
    /// share as it lies (`nhip_group_stream_submit_placed`); two arena sets, so batch k + 1 decodes on
    /// a scoped thread while batch k uploads.  `claims(i, bytes)` returns batch i's claims in proof
    /// order (a SingleProof's `single_proof_claim(kernel MAST hash)`, a ProofCollection's member
    /// claims, `proof_collection.rs:286-339`); `on_verdicts(i, verdicts, all_ok)` is called in order.
    /// The arena words are canonical (the wire form), so this stream runs `NHIP_INPUT_CANONICAL`
    /// with canonical claim words.  A malformed transaction is `NHIP_ERR_DECODE` for its batch.
    pub fn verify_wire_batches<'a, I, C, F>(&self, batches: I, bytes_per_gpu: usize, mut claims: C,
                                            mut on_verdicts: F) -> Result<(), GpuFault>
    where
        I: IntoIterator<Item = &'a [u8]>,
        C: FnMut(usize, &[u8]) -> Vec<Claim>,
        F: FnMut(usize, Vec<bool>, bool),
    {
        struct Arena(*mut sys::nhip_arena);
        unsafe impl Send for Arena {}
        impl Drop for Arena {
            fn drop(&mut self) {
                unsafe { sys::nhip_arena_destroy(self.0) }
            }
        }
        struct Stream(*mut sys::nhip_group_stream);
        impl Drop for Stream {
            fn drop(&mut self) {
                unsafe { sys::nhip_group_stream_destroy(self.0) }
            }
        }
        // one decoded batch: proof records into an arena and each proof's GPU
        struct Placed(Vec<sys::nhip_proof>, Vec<u32>);
        unsafe impl Send for Placed {}
        let new_arena = || -> Result<Arena, GpuFault> {
            let mut a = ptr::null_mut();
            ok(unsafe { sys::nhip_arena_create(self.group, bytes_per_gpu, &mut a) })?;
            Ok(Arena(a))
        };
        let arenas = [new_arena()?, new_arena()?];
        let mut params = self.params;
        params.input_form = sys::NHIP_INPUT_CANONICAL;
        let mut st = ptr::null_mut();
        ok(unsafe { sys::nhip_group_stream_create(self.group, self.air.0, &params, &mut st) })?;
        let st = Stream(st);
        let decode = |a: &Arena, bytes: &[u8]| -> Result<Placed, GpuFault> {
            let cap = bytes.len() / 8 + 1;
            let mut p = Placed(vec![sys::nhip_proof { words: ptr::null(), len: 0 }; cap], vec![0u32; cap]);
            let (mut ntx, mut np, mut used) = (0usize, 0usize, 0usize);
            ok(unsafe { sys::nhip_arena_reset(a.0) })?;
            ok(unsafe {
                sys::nhip_arena_ingest_txs(a.0, bytes.as_ptr(), bytes.len(), usize::MAX, p.0.as_mut_ptr(),
                                           p.1.as_mut_ptr(), cap, &mut ntx, &mut np, &mut used)
            })?;
            if used != bytes.len() {
                return Err(GpuFault(sys::NHIP_ERR_OOM));  // the batch does not fit bytes_per_gpu
            }
            p.0.truncate(np);
            p.1.truncate(np);
            Ok(p)
        };
        let batches: Vec<&[u8]> = batches.into_iter().collect();
        let mut bufs: [(Vec<u8>, u8); 2] = [(Vec::new(), 0), (Vec::new(), 0)];
        let mut next = if batches.is_empty() { None } else { Some(decode(&arenas[0], batches[0])?) };
        for k in 0..batches.len() {
            let cur = next.take().expect("decoded batch");
            let cs: Vec<sys::nhip_claim> = canonical_claims(&claims(k, batches[k]));
            if cs.len() != cur.0.len() {
                return Err(GpuFault(sys::NHIP_ERR_ARG));
            }
            let slot = k & 1;
            bufs[slot].0 = vec![0u8; cur.0.len()];
            let (vp, ap) = (bufs[slot].0.as_mut_ptr(), &mut bufs[slot].1 as *mut u8);
            // batch k uploads (and batch k - 1's verdicts come back) while batch k + 1 decodes
            let (submitted, decoded) = std::thread::scope(|scope| {
                let h = (k + 1 < batches.len()).then(|| {
                    let (a, b) = (&arenas[(k + 1) & 1], batches[k + 1]);
                    scope.spawn(move || decode(a, b))
                });
                let rc = unsafe {
                    sys::nhip_group_stream_submit_placed(st.0, cs.as_ptr(), cur.0.as_ptr(), cur.1.as_ptr(), cur.0.len(),
                                                         vp, ap)
                };
                (ok(rc), h.map(|h| h.join().unwrap_or(Err(GpuFault(sys::NHIP_ERR_HIP)))))
            });
            submitted?;
            next = decoded.transpose()?;
            if k > 0 {
                let (v, all) = &bufs[slot ^ 1];
                on_verdicts(k - 1, v.iter().map(|&b| b == 1).collect(), *all == 1);
            }
        }
        ok(unsafe { sys::nhip_group_stream_finish(st.0) })?;
        if let Some(k) = batches.len().checked_sub(1) {
            let (v, all) = &bufs[k & 1];
            on_verdicts(k, v.iter().map(|&b| b == 1).collect(), *all == 1);
        }
        Ok(())
    }
}

/// Claims as canonical words (for the wire-bytes path, whose proof words are canonical): the
/// digest, input and output `value()`s, owned by the returned structs' backing vectors.
fn canonical_claims(claims: &[Claim]) -> Vec<sys::nhip_claim> {
    thread_local! { static WORDS: std::cell::RefCell<Vec<Vec<u64>>> = std::cell::RefCell::new(Vec::new()); }
    WORDS.with(|w| {
        let mut w = w.borrow_mut();
        w.clear();
        claims
            .iter()
            .map(|c| {
                w.push(c.input.iter().map(|b| b.value()).collect());
                w.push(c.output.iter().map(|b| b.value()).collect());
                let (i, o) = (&w[w.len() - 2], &w[w.len() - 1]);
                sys::nhip_claim {
                    program_digest: c.program_digest.values().map(|b| b.value()),
                    version: c.version,
                    input: i.as_ptr(),
                    input_len: i.len(),
                    output: o.as_ptr(),
                    output_len: o.len(),
                }
            })
            .collect()
    })
}

impl Drop for GpuNode {
    fn drop(&mut self) {
        unsafe { sys::nhip_group_destroy(self.group) }
    }
}

fn arena_marshal(claims: &[Claim], arena: &ProofArena) -> Result<(Vec<sys::nhip_claim>, Vec<sys::nhip_proof>), GpuFault> {
    if claims.len() != arena.len() {
        return Err(GpuFault(sys::NHIP_ERR_ARG));
    }
    let mut cs = Vec::with_capacity(claims.len());
    let mut ps = Vec::with_capacity(claims.len());
    for (i, c) in claims.iter().enumerate() {
        cs.push(sys::nhip_claim {
            program_digest: raw_digest(&c.program_digest),
            version: c.version,
            input: raw_words(&c.input),
            input_len: c.input.len(),
            output: raw_words(&c.output),
            output_len: c.output.len(),
        });
        let p = arena.proof(i);
        ps.push(sys::nhip_proof { words: raw_words(p), len: p.len() });
    }
    Ok((cs, ps))
}

/// Pinned receive memory for proofs, on the NUMA node of one GPU (`nhip_host_alloc_near`): the node
/// decodes a peer's proof (`peer_loop.rs:315-323`, `state/mod.rs:2226-2272`) straight into it with
/// [`ProofArena::push_with`] instead of into a `Proof`'s `Vec`, and the verifier DMAs it from there:
/// no staging copy (the pageable path's host copy reads and writes every proof word once more on
/// the host; DESIGN.md §6 budgets both).  Words are `BFieldElement`s as twenty-first keeps them
/// (Montgomery), the form the crate's params declare.
pub struct ProofArena {
    base: *mut BFieldElement,
    cap: usize,
    used: usize,
    spans: Vec<(usize, usize)>,
}
unsafe impl Send for ProofArena {}

impl ProofArena {
    /// `cap_words` words on the NUMA node of `node`'s member `member`.
    pub fn new(node: &GpuNode, member: usize, cap_words: usize) -> Result<Self, GpuFault> {
        let ctx = unsafe { sys::nhip_group_member(node.group, member) };
        if ctx.is_null() {
            return Err(GpuFault(sys::NHIP_ERR_ARG));
        }
        let mut p = ptr::null_mut();
        ok(unsafe { sys::nhip_host_alloc_near(ctx, cap_words.max(1) * 8, &mut p) })?;
        Ok(ProofArena { base: p as *mut BFieldElement, cap: cap_words, used: 0, spans: Vec::new() })
    }

    /// Reserve `len` words for the next proof and let `fill` write them (a deserializer); None when
    /// the arena is full (verify what it holds, then [`ProofArena::clear`]).
    pub fn push_with(&mut self, len: usize, fill: impl FnOnce(&mut [BFieldElement])) -> Option<usize> {
        if self.cap - self.used < len {
            return None;
        }
        // SAFETY: [used, used + len) lies inside the allocation and is not borrowed elsewhere
        let dst = unsafe { std::slice::from_raw_parts_mut(self.base.add(self.used), len) };
        fill(dst);
        self.spans.push((self.used, len));
        self.used += len;
        Some(self.spans.len() - 1)
    }

    /// Copy a decoded proof in (when the decoder cannot write in place).
    pub fn push(&mut self, proof: &Proof) -> Option<usize> {
        self.push_with(proof.0.len(), |d| d.copy_from_slice(&proof.0))
    }

    pub fn proof(&self, i: usize) -> &[BFieldElement] {
        let (at, len) = self.spans[i];
        // SAFETY: a span handed out by push_with, inside the allocation
        unsafe { std::slice::from_raw_parts(self.base.add(at), len) }
    }

    pub fn len(&self) -> usize {
        self.spans.len()
    }

    pub fn is_empty(&self) -> bool {
        self.spans.is_empty()
    }

    pub fn clear(&mut self) {
        self.spans.clear();
        self.used = 0;
    }
}

impl Drop for ProofArena {
    fn drop(&mut self) {
        unsafe {
            sys::nhip_host_free(self.base as *mut std::ffi::c_void);
        }
    }
}

/// Hardware queues the verifier's pipeline uses: two batches in flight, each with a hashing and a
/// latency stream, plus the context stream and one spare (HIP serializes streams that share a
/// queue; its default is 4).
pub const HW_QUEUES: u32 = sys::NHIP_HW_QUEUES_RECOMMENDED;

/// Sets `GPU_MAX_HW_QUEUES` to [`HW_QUEUES`] unless the operator has set it.  HIP reads it once, at
/// its initialisation, and changing the environment races with every thread that reads it: call
/// this from `main()` before the tokio runtime (or anything else) starts a thread.  The library
/// itself never changes the environment.
pub fn provision_hw_queues() {
    if std::env::var_os("GPU_MAX_HW_QUEUES").is_none() {
        std::env::set_var("GPU_MAX_HW_QUEUES", HW_QUEUES.to_string());
    }
}

/// Why the GPU path is not available (kept by the process-wide constructors).
#[derive(Debug, Clone)]
pub enum InitError {
    /// `Air::triton()`: the exporter could not build triton-air's descriptor.
    AirExport(String),
    /// `nhip_*` returned this fault (no device, HIP error, out of memory, bad argument).
    Gpu(GpuFault),
}

impl std::fmt::Display for InitError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        match self {
            InitError::AirExport(e) => write!(f, "neptune-hip: triton-air export failed: {e}"),
            InitError::Gpu(g) => g.fmt(f),
        }
    }
}
impl std::error::Error for InitError {}

fn triton_air() -> Result<Air, InitError> {
    let words = air_export::triton_air_descriptor().map_err(|e| InitError::AirExport(format!("{e:?}")))?;
    Air::from_descriptor(&words).map_err(InitError::Gpu)
}

static GPU_VERIFIER: OnceLock<Result<Verifier, InitError>> = OnceLock::new();
static GPU_NODE: OnceLock<Result<GpuNode, InitError>> = OnceLock::new();

fn logged<T>(what: &str, r: &Result<T, InitError>) {
    if let Err(e) = r {
        tracing::warn!("{what}: GPU verification unavailable, using the CPU verifier: {e}");
    }
}

/// The process's single-GPU verifier, or why there is none (created on first use): device
/// `NEPTUNE_HIP_DEVICE` (default 0), triton-air's AIR, a 200 us coalescing window.
pub fn gpu_verifier_status() -> &'static Result<Verifier, InitError> {
    GPU_VERIFIER.get_or_init(|| {
        let dev = std::env::var("NEPTUNE_HIP_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(0);
        let r = triton_air().and_then(|air| Verifier::new(dev, air, 200).map_err(InitError::Gpu));
        logged("gpu_verifier", &r);
        r
    })
}

/// [`gpu_verifier_status`] as an `Option` (`None`: no usable GPU, the reason was logged).  This is
/// the `GPU_VERIFIER.get()` of INTEGRATION.md.
pub fn gpu_verifier() -> Option<&'static Verifier> {
    gpu_verifier_status().as_ref().ok()
}

/// Every GPU of the node, or why there is none (created on first use): the device mask
/// `NEPTUNE_HIP_DEVICES` (hex or decimal, default 0 = every visible GPU).
pub fn gpu_node_status() -> &'static Result<GpuNode, InitError> {
    GPU_NODE.get_or_init(|| {
        let mask = std::env::var("NEPTUNE_HIP_DEVICES").ok().and_then(|v| {
            v.strip_prefix("0x").map_or_else(|| v.parse().ok(), |h| u32::from_str_radix(h, 16).ok())
        });
        let r = triton_air().and_then(|air| GpuNode::init(mask.unwrap_or(0), air).map_err(InitError::Gpu));
        logged("gpu_node", &r);
        r
    })
}

/// [`gpu_node_status`] as an `Option` (`None`: no usable GPU, the reason was logged).
pub fn gpu_node() -> Option<&'static GpuNode> {
    gpu_node_status().as_ref().ok()
}

/// The drop-in for `verifier.rs:60-63`: the GPU verdict, or on a GPU fault (or without a GPU)
/// the CPU `triton_vm::verify`.  A fault is never turned into "accept".
pub fn verify_or_cpu(gpu: Option<&Verifier>, claim: &Claim, proof: &Proof) -> bool {
    match gpu.map(|v| v.verify(claim, proof)) {
        Some(Ok(verdict)) => verdict,
        _ => triton_vm::verify(Stark::default(), claim, proof),
    }
}

/// Batch form of [`verify_or_cpu`] over every GPU of the node.
pub fn verify_batch_or_cpu(node: Option<&GpuNode>, items: &[(Claim, Proof)]) -> Vec<bool> {
    match node.map(|n| n.verify_batch(items)) {
        Some(Ok((verdicts, _))) => verdicts,
        _ => items.iter().map(|(c, p)| triton_vm::verify(Stark::default(), c, p)).collect(),
    }
}

#[cfg(test)]
mod tests {
    use super::*;

    #[test]
    fn params_are_stark_default() {
        let p = default_params();
        assert_eq!((p.security_level, p.log2_fri_expansion, p.num_collinearity_checks), (160, 2, 80));
        assert_eq!((p.num_main, p.num_aux, p.num_quotient_segments), (379, 88, 4));
    }

    #[test]
    fn device_ordinals_past_the_mask_are_faults() {
        if let Ok(air) = Air::from_descriptor(&[0x41495231, 1, 1, 59, 1, 0, 0, 0, 1, 1, 0, 0, 0, 0]) {
            assert_eq!(Verifier::new(32, air, 200).err(), Some(GpuFault(sys::NHIP_ERR_ARG)));
        }
    }

    #[test]
    fn no_gpu_is_a_fault_never_an_accept() {
        // on a host without a GPU: nhip_init fails, and the fallback is the CPU verifier, which
        // rejects the reference's bogus proofs (verifier.rs:95-118, neptune_proof.rs:118-133)
        let air = Air::from_descriptor(&[0x41495231, 1, 1, 59, 1, 0, 0, 0, 1, 1, 0, 0, 0, 0]);
        if let Ok(air) = air {
            if let Err(fault) = Verifier::new(0, air, 200) {
                assert_ne!(fault.0, sys::NHIP_OK);
            }
        }
        let claim = Claim::new(Digest::default());
        assert!(!verify_or_cpu(None, &claim, &Proof(vec![])));
        assert!(!verify_or_cpu(None, &claim, &Proof(vec![BFieldElement::new(0); 65])));
    }
}
