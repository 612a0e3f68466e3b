// Batched STARK verification: descriptors shared by the host decoder (stark_host.cpp) and the
// phase kernels (stark_kernels.hip).
//
// Restates the structure of `triton_vm::verify(Stark::default(), &claim, &proof)` (triton-vm
// 1.0.0, Cargo.lock:4260; single call site neptune-core/src/protocol/proof_abstractions/
// verifier.rs:60-63).  The verification of one proof is split into phases that run batched over
// all proofs of a call (phase-synchronous design, SURVEY.md §7 "hard parts" 4):
//   k_decode        : BFieldCodec proof stream -> ProofDesc (offsets into the batch word buffer)
//                     and the proof's Fiat-Shamir program, one wave per proof (proof_codec.hpp)
//   k_fs_replay_wide: Fiat-Shamir sponge replay, one 16-lane DPP row (two below 512 proofs) per
//                     proof (challenges, weights, z, FRI folding challenges, indices)
//   k_hash_rows     : Tip5::hash_varlen of every revealed main / aux / quotient row
//   k_mp_plan, k_mp_hash*, k_mp_roots : Merkle authentication structures (main, aux, quotient,
//                     FRI rounds): index-only plan per (proof, tree group), then one launch per
//                     tree level over all trees of all proofs, then the root compares
//   k_ood_air       : AIR circuit at the out-of-domain point, zerofiers, quotient identity; one
//                     workgroup per proof, circuit levels evaluated in LDS
//   k_fri           : collinearity folds, last codeword root / agreement / low degree
//   k_deep          : DEEP recombination at the revealed rows vs the first FRI codeword
// Every check ORs a bit into the proof's fail word; verdict = (fail == 0).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace nhip {

static constexpr int MAX_FRI_ROUNDS = 26;
static constexpr int MAX_CHECKS = 256;        // num_collinearity_checks supported per workgroup
static constexpr uint32_t LOG2_PH_MAX = 28;

enum FailBits : uint32_t {
    FAIL_DECODE = 1u << 0,
    FAIL_OOD = 1u << 1,
    FAIL_MERKLE_MAIN = 1u << 2,
    FAIL_MERKLE_AUX = 1u << 3,
    FAIL_MERKLE_QUOT = 1u << 4,
    FAIL_MERKLE_FRI = 1u << 5,
    FAIL_FRI_LAST_ROOT = 1u << 6,
    FAIL_FRI_LAST_AGREE = 1u << 7,
    FAIL_FRI_DEGREE = 1u << 8,
    FAIL_FRI_EVAL = 1u << 9,
    FAIL_DEEP = 1u << 10,
    FAIL_ZERO_INVERSE = 1u << 11,
};

struct StarkDims {
    uint32_t num_main, num_aux, num_quot_seg, num_checks, num_deep;
    uint32_t log2_expansion, num_trace_randomizers;
    uint32_t num_sampled;       // AIR: sampled challenges
    uint32_t num_constraints;   // AIR: total constraints
};

struct FriResp {
    uint64_t auth_off;    // first digest word (absolute, batch word buffer)
    uint64_t leaves_off;  // first XFE word
    uint32_t auth_n, leaves_n;
};

enum FsOpKind : uint32_t { FS_ABSORB = 0, FS_SQUEEZE_X = 1, FS_SAMPLE_IDX = 2 };
struct FsOp {
    uint32_t kind, n;   // ABSORB: n words; SQUEEZE_X: n XFEs; SAMPLE_IDX: n indices
    uint64_t arg;       // ABSORB: word offset; SAMPLE_IDX: upper bound
};

struct ProofDesc {
    uint32_t log2_ph, log2_T, log2_N, R;
    uint64_t main_root, aux_root, quot_root;  // payload offsets (5 words)
    uint64_t ood_mc, ood_ac, ood_mn, ood_an, ood_qs;
    uint64_t fri_root[MAX_FRI_ROUNDS + 1];
    uint64_t last_cw_off, last_poly_off;
    uint32_t last_cw_n, last_poly_n, last_poly_degree_ok, pad0;
    FriResp fri[MAX_FRI_ROUNDS + 1];          // [0]: round-0 a-values, [1 + r]: round-r b-values
    uint64_t main_rows_off, aux_rows_off, quot_rows_off;
    uint64_t main_auth_off, aux_auth_off, quot_auth_off;
    uint32_t main_auth_n, aux_auth_n, quot_auth_n, rows_n;
    // claim (absolute word offsets of the staged claim fields)
    uint64_t claim_digest_off, claim_in_off, claim_out_off;
    uint32_t claim_in_n, claim_out_n;
    // Fiat-Shamir program
    uint32_t fs_op_off, fs_op_n;
    // scratch: XFE sample area (index of first XFE) and index area
    uint64_t xs_off, idx_off;
    uint32_t n_xs, pad1;
};

// Offsets (in XFEs) of the sampled quantities inside a proof's sample area, in squeeze order.
struct SampleLayout {
    uint32_t chal, quot_w, z, lin_w, alpha, indeterminate, total;
    __host__ __device__ static SampleLayout of(const StarkDims& d, uint32_t R) {
        SampleLayout s;
        s.chal = 0;
        s.quot_w = s.chal + d.num_sampled;
        s.z = s.quot_w + d.num_constraints;
        s.lin_w = s.z + 1;
        s.alpha = s.lin_w + d.num_main + d.num_aux + d.num_quot_seg + d.num_deep;
        s.indeterminate = s.alpha + R;
        s.total = s.indeterminate + 1;
        return s;
    }
};

// AIR circuit node (see oracle/stark_ref.py AirCircuit): op, a, b, c.
enum AirOp : uint32_t { AIR_INPUT = 0, AIR_CONST = 1, AIR_ADD = 2, AIR_SUB = 3, AIR_MUL = 4 };
enum AirInput : uint32_t { IN_MAIN_CURR = 0, IN_AUX_CURR = 1, IN_MAIN_NEXT = 2, IN_AUX_NEXT = 3, IN_CHALLENGE = 4 };
struct AirNode {
    uint32_t op, a, b, pad;
    uint64_t k0, k1, k2;  // AIR_CONST value (raw Montgomery)
};

// The AIR compiled for k_ood_air (nhip_air_create, stark_host.cpp air_compile): steps of independent
// instructions whose results live in reusable slots (liveness-allocated: a slot is reused from the
// step after its value's last use), constants in a global table, OOD-row inputs loaded once into
// slots, and every constraint value copied (ACC) into its own slot among the top C, which the kernel
// weighs into the quotient sum after the last step.
enum OodOp : uint32_t { OOD_ADD = AIR_ADD, OOD_SUB = AIR_SUB, OOD_MUL = AIR_MUL, OOD_LOAD = 5, OOD_ACC = 6 };
// operand reference: [31:30] 0 = LDS slot, 1 = constant table index, 2 = input ([29:27] kind, [26:0] index)
static constexpr uint32_t OOD_REF_SLOT = 0u << 30, OOD_REF_CONST = 1u << 30, OOD_REF_INPUT = 2u << 30;
struct OodIns {
    uint32_t op;   // OodOp
    uint32_t a;    // operand ref (LOAD: input ref, ACC: value ref)
    uint32_t b;    // operand ref (ACC: constraint index)
    uint32_t dst;  // slot written (ACC: the constraint's own slot, slots - C + constraint index)
};
static_assert(sizeof(OodIns) == 16, "k_ood_air loads an instruction as one uint4");

}  // namespace nhip
