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
//!   and the callers take the CPU path.
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

fn canon(d: &Digest) -> [u64; 5] {
    d.values().map(|b| b.value())
}

fn words(v: &[BFieldElement]) -> Vec<u64> {
    v.iter().map(|b| b.value()).collect()
}

/// `Stark::default()` as the library's parameters (security 160, FRI expansion 4, 80
/// collinearity checks, triton-vm's 379 main / 88 auxiliary columns, 4 quotient segments).
pub fn default_params() -> sys::nhip_stark_params {
    let mut p = sys::nhip_stark_params::default();
    unsafe { sys::nhip_stark_params_default(&mut p) };
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

/// Canonical-word views of a batch, kept alive while the C structs point into them.
struct Marshal {
    claims: Vec<sys::nhip_claim>,
    proofs: Vec<sys::nhip_proof>,
    _bufs: Vec<Vec<u64>>,
}

fn marshal(items: &[(&Claim, &Proof)]) -> Marshal {
    let mut bufs: Vec<Vec<u64>> = Vec::with_capacity(3 * items.len());
    for (c, p) in items {
        bufs.push(words(&c.input));
        bufs.push(words(&c.output));
        bufs.push(words(&p.0));
    }
    let claims = items
        .iter()
        .enumerate()
        .map(|(i, (c, _))| sys::nhip_claim {
            program_digest: canon(&c.program_digest),
            version: c.version,
            input: bufs[3 * i].as_ptr(),
            input_len: bufs[3 * i].len(),
            output: bufs[3 * i + 1].as_ptr(),
            output_len: bufs[3 * i + 1].len(),
        })
        .collect();
    let proofs = (0..items.len())
        .map(|i| sys::nhip_proof { words: bufs[3 * i + 2].as_ptr(), len: bufs[3 * i + 2].len() })
        .collect();
    Marshal { claims, proofs, _bufs: bufs }
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
        let m = marshal(&[(claim, proof)]);
        let mut v = [0u8; 1];
        ok(unsafe { sys::nhip_queue_verify(self.queue, m.claims.as_ptr(), m.proofs.as_ptr(), 1, v.as_mut_ptr()) })?;
        Ok(v[0] == 1)
    }

    /// `verify_batch(&[(Claim, Proof)]) -> Vec<bool>`: one device batch.
    pub fn verify_batch(&self, items: &[(Claim, Proof)]) -> Result<Vec<bool>, GpuFault> {
        let refs: Vec<(&Claim, &Proof)> = items.iter().map(|(c, p)| (c, p)).collect();
        let m = marshal(&refs);
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
        let refs: Vec<(&Claim, &Proof)> = items.iter().map(|(c, p)| (c, p)).collect();
        let m = marshal(&refs);
        let mut v = vec![0u8; items.len()];
        let mut all = 0u8;
        ok(unsafe {
            sys::nhip_group_verify_batch(self.group, self.air.0, &self.params, m.claims.as_ptr(), m.proofs.as_ptr(),
                                         items.len(), v.as_mut_ptr(), &mut all)
        })?;
        Ok((v.into_iter().map(|b| b == 1).collect(), all == 1))
    }
}

impl Drop for GpuNode {
    fn drop(&mut self) {
        unsafe { sys::nhip_group_destroy(self.group) }
    }
}

/// Hardware queues the verifier's pipeline uses when it is the first HIP user of the process: two
/// batches in flight, each with a hashing and a latency stream, plus the context stream and one
/// spare (HIP serializes streams that share a queue; its default is 4).  Set only if the operator
/// has not set `GPU_MAX_HW_QUEUES`, and only before the first HIP call (later it has no effect).
pub const HW_QUEUES: u32 = 8;

fn provision_hw_queues() {
    if std::env::var_os("GPU_MAX_HW_QUEUES").is_none() {
        std::env::set_var("GPU_MAX_HW_QUEUES", HW_QUEUES.to_string());
    }
}

static GPU_VERIFIER: OnceLock<Option<Verifier>> = OnceLock::new();
static GPU_NODE: OnceLock<Option<GpuNode>> = OnceLock::new();

/// The process's single-GPU verifier (created on first use): device `NEPTUNE_HIP_DEVICE`
/// (default 0), triton-air's AIR, a 200 us coalescing window.  `None` when there is no usable GPU.
/// This is the `GPU_VERIFIER.get()` of INTEGRATION.md.
pub fn gpu_verifier() -> Option<&'static Verifier> {
    GPU_VERIFIER
        .get_or_init(|| {
            provision_hw_queues();
            let dev = std::env::var("NEPTUNE_HIP_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(0);
            Air::triton().and_then(|air| Verifier::new(dev, air, 200)).ok()
        })
        .as_ref()
}

/// Every GPU of the node (created on first use): the device mask `NEPTUNE_HIP_DEVICES` (hex or
/// decimal, default 0 = every visible GPU).  `None` when there is no usable GPU.
pub fn gpu_node() -> Option<&'static GpuNode> {
    GPU_NODE
        .get_or_init(|| {
            provision_hw_queues();
            let mask = std::env::var("NEPTUNE_HIP_DEVICES").ok().and_then(|v| {
                v.strip_prefix("0x").map_or_else(|| v.parse().ok(), |h| u32::from_str_radix(h, 16).ok())
            });
            Air::triton().and_then(|air| GpuNode::init(mask.unwrap_or(0), air)).ok()
        })
        .as_ref()
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
