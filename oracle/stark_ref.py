"""CPU restatement of the STARK verifier on neptune-core's proof-validation path — TEST ORACLE ONLY.

Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.

What it restates
----------------
`triton_vm::verify(Stark::default(), &claim, &proof) -> bool`, called once per proof at
neptune-core/src/protocol/proof_abstractions/verifier.rs:60-63.  triton-vm 1.0.0 / twenty-first
1.0.0 (Cargo.lock:4260,4297) are NOT vendored and no proof file exists offline,
so everything below past Tip5 follows the public triton-vm 1.0 design and is **parity unpinned**
except where noted:

  * Claim BFieldCodec layout — PINNED by the reference's own TASM `NewClaim`
    (neptune-core/src/protocol/consensus/transaction/validity/tasm/claims/new_claim.rs:38-100,
    tested there against `encode_to_memory(claim)`): fields in reverse order,
    [len(output)+1, len(output), output.., len(input)+1, len(input), input.., version, digest(5)].
  * Stark::default(): security 160, FRI expansion 4, 80 collinearity checks, 86 trace
    randomizers, 4 quotient segments (unpinned).
  * ProofItem order / Fiat-Shamir inclusion, ProofStream codec, FRI (rounds, folding by
    collinearity, last-codeword Merkle root + barycentric/Horner agreement), DEEP with 3 weights,
    multi-leaf Merkle authentication structures (twenty-first `MerkleTreeInclusionProof`):
    restated from the public design (unpinned).
  * The AIR: triton-air's ~600 generated constraints cannot be reproduced offline.  The verifier
    here takes the AIR as *data* (a straight-line XFE circuit, `AirCircuit`); `synth_air()` makes a
    deterministic synthetic AIR with triton-vm's column counts whose traces a synthetic prover
    (`prove()`) can satisfy, so every verifier phase runs on accepting and rejecting proofs.

Tip5 / hashing comes from tip5_ref (pinned by the reference KATs); batch hashing and trees use the
C oracle (coracle) for speed.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

import coracle as CO
import tip5_ref as T
from field_ref import (P, X_ONE, X_ZERO, Domain, GENERATOR, barycentric_evaluate, binv, bpoly_eval, bpoly_mul,
                       coset_evaluate_b, coset_evaluate_x, interpolate_subgroup_x, lift, primitive_root_of_unity,
                       xadd, xbatch_inv, xinv, xmul, xneg, xpoly_degree, xpoly_eval, xpoly_eval_at_b, xpow,
                       xscale, xsub)

EXT = 3
DIGEST_LEN = 5
CURRENT_VERSION = 0  # triton_vm::proof::CURRENT_VERSION (new_claim.rs:97); value unpinned
MAX_FRI_ROUNDS = 26


class VerifyError(Exception):
    pass


# ====================================================================== parameters
class StarkParams:
    """Stark::new(security_level, log2_of_fri_expansion_factor) + table dimensions."""

    def __init__(self, security_level=160, log2_fri_expansion=2, num_main=379, num_aux=88,
                 num_quotient_segments=4, num_collinearity_checks: Optional[int] = None):
        self.security_level = security_level
        self.fri_expansion_factor = 1 << log2_fri_expansion
        self.num_collinearity_checks = (num_collinearity_checks if num_collinearity_checks is not None
                                        else security_level // log2_fri_expansion)
        self.num_out_of_domain_rows = 2
        self.num_trace_randomizers = self.num_collinearity_checks + self.num_out_of_domain_rows * EXT
        self.num_main = num_main
        self.num_aux = num_aux
        self.num_quotient_segments = num_quotient_segments
        self.num_deep = 3

    def randomized_trace_len(self, padded_height: int) -> int:
        return 1 << (padded_height + self.num_trace_randomizers - 1).bit_length()

    def fri_domain(self, padded_height: int) -> Domain:
        return Domain(self.fri_expansion_factor * self.randomized_trace_len(padded_height), GENERATOR)

    def fri_num_rounds(self, fri_len: int) -> int:
        first_round_code_dimension = fri_len // self.fri_expansion_factor
        max_num_rounds = (first_round_code_dimension - 1).bit_length()  # log2 of next pow2
        checking_all = int(math.log2(self.num_collinearity_checks))
        return max(0, max_num_rounds - (checking_all + 1))

    def to_words(self) -> List[int]:
        return [self.security_level, int(math.log2(self.fri_expansion_factor)), self.num_collinearity_checks,
                self.num_main, self.num_aux, self.num_quotient_segments]


# ====================================================================== BFieldCodec
def encode_claim(program_digest: Sequence[int], version: int, inp: Sequence[int], out: Sequence[int]) -> List[int]:
    """PINNED layout (new_claim.rs:38-100)."""
    return ([len(out) + 1, len(out)] + [int(x) % P for x in out] + [len(inp) + 1, len(inp)] +
            [int(x) % P for x in inp] + [version] + [int(x) % P for x in program_digest])


MERKLE_ROOT, OOD_MAIN_ROW, OOD_AUX_ROW, OOD_QUOT_SEGMENTS, AUTH_STRUCTURE, MAIN_ROWS, AUX_ROWS, \
    LOG2_PADDED_HEIGHT, QUOT_SEGMENTS_ELEMENTS, FRI_CODEWORD, FRI_POLYNOMIAL, FRI_RESPONSE = range(12)
ITEM_NAMES = ["MerkleRoot", "OutOfDomainMainRow", "OutOfDomainAuxRow", "OutOfDomainQuotientSegments",
              "AuthenticationStructure", "MasterMainTableRows", "MasterAuxTableRows", "Log2PaddedHeight",
              "QuotientSegmentsElements", "FriCodeword", "FriPolynomial", "FriResponse"]
INCLUDED_IN_FIAT_SHAMIR = {MERKLE_ROOT, OOD_MAIN_ROW, OOD_AUX_ROW, OOD_QUOT_SEGMENTS}


def _xflat(xs):
    return [c for x in xs for c in x]


def encode_item(kind: int, payload, params: StarkParams) -> List[int]:
    """ProofItem encoding: discriminant, then the payload (length-prefixed when dynamically sized)."""
    if kind == MERKLE_ROOT:
        body, dyn = list(payload), False
    elif kind in (OOD_MAIN_ROW, OOD_AUX_ROW, OOD_QUOT_SEGMENTS):
        body, dyn = _xflat(payload), False
    elif kind == LOG2_PADDED_HEIGHT:
        body, dyn = [int(payload)], False
    elif kind == AUTH_STRUCTURE:
        body, dyn = [len(payload)] + [c for d in payload for c in d], True
    elif kind == MAIN_ROWS:
        body, dyn = [len(payload)] + [c for r in payload for c in r], True
    elif kind in (AUX_ROWS, QUOT_SEGMENTS_ELEMENTS):
        body, dyn = [len(payload)] + [c for r in payload for c in _xflat(r)], True
    elif kind == FRI_CODEWORD:
        body, dyn = [len(payload)] + _xflat(payload), True
    elif kind == FRI_POLYNOMIAL:
        deg = xpoly_degree(payload)
        coeffs = list(payload[:deg + 1])
        body, dyn = [len(coeffs)] + _xflat(coeffs), True
    elif kind == FRI_RESPONSE:
        auth, leaves = payload
        rl = [len(leaves)] + _xflat(leaves)
        au = [len(auth)] + [c for d in auth for c in d]
        body, dyn = [len(rl)] + rl + [len(au)] + au, True
    else:
        raise ValueError(kind)
    return [kind] + ([len(body)] + body if dyn else body)


def encode_proof(items: List[Tuple[int, object]], params: StarkParams) -> List[int]:
    """ProofStream { items: Vec<ProofItem> } -> Proof(Vec<BFieldElement>)."""
    enc = [len(items)]
    for kind, payload in items:
        ie = encode_item(kind, payload, params)
        enc += [len(ie)] + ie
    return [len(enc)] + enc


class _Reader:
    def __init__(self, words: Sequence[int], lo: int, hi: int):
        self.w, self.pos, self.hi = words, lo, hi

    def take(self, n: int) -> List[int]:
        if n < 0 or self.pos + n > self.hi:
            raise VerifyError("sequence too short")
        out = list(self.w[self.pos:self.pos + n])
        self.pos += n
        return out

    def one(self) -> int:
        return self.take(1)[0]

    def done(self):
        if self.pos != self.hi:
            raise VerifyError("sequence too long")


def _xs(flat: List[int]) -> List[Tuple[int, int, int]]:
    return [tuple(flat[3 * i:3 * i + 3]) for i in range(len(flat) // 3)]


def decode_item(words: Sequence[int], lo: int, hi: int, params: StarkParams):
    r = _Reader(words, lo, hi)
    kind = r.one()
    if kind >= 12:
        raise VerifyError("invalid discriminant")
    if kind == MERKLE_ROOT:
        payload = r.take(DIGEST_LEN)
    elif kind == OOD_MAIN_ROW:
        payload = _xs(r.take(EXT * params.num_main))
    elif kind == OOD_AUX_ROW:
        payload = _xs(r.take(EXT * params.num_aux))
    elif kind == OOD_QUOT_SEGMENTS:
        payload = _xs(r.take(EXT * params.num_quotient_segments))
    elif kind == LOG2_PADDED_HEIGHT:
        v = r.one()
        if v >= (1 << 32):
            raise VerifyError("u32 out of range")
        payload = v
    else:
        blen = r.one()
        b = _Reader(words, r.pos, r.pos + blen)
        if r.pos + blen > hi:
            raise VerifyError("sequence too short")
        r.pos += blen
        if kind in (AUTH_STRUCTURE, MAIN_ROWS, AUX_ROWS, QUOT_SEGMENTS_ELEMENTS, FRI_CODEWORD, FRI_POLYNOMIAL):
            n = b.one()
            width = {AUTH_STRUCTURE: DIGEST_LEN, MAIN_ROWS: params.num_main, AUX_ROWS: EXT * params.num_aux,
                     QUOT_SEGMENTS_ELEMENTS: EXT * params.num_quotient_segments, FRI_CODEWORD: EXT,
                     FRI_POLYNOMIAL: EXT}[kind]
            if n * width != blen - 1:
                raise VerifyError("length mismatch")
            flat = b.take(n * width)
            if kind == AUTH_STRUCTURE:
                payload = [flat[5 * i:5 * i + 5] for i in range(n)]
            elif kind == MAIN_ROWS:
                payload = [flat[width * i:width * (i + 1)] for i in range(n)]
            elif kind in (AUX_ROWS, QUOT_SEGMENTS_ELEMENTS):
                payload = [_xs(flat[width * i:width * (i + 1)]) for i in range(n)]
            else:
                payload = _xs(flat)
        else:  # FRI_RESPONSE
            lrl = b.one()
            rl = _Reader(words, b.pos, b.pos + lrl)
            b.take(lrl)
            nl = rl.one()
            if 3 * nl != lrl - 1:
                raise VerifyError("length mismatch")
            leaves = _xs(rl.take(3 * nl))
            lau = b.one()
            au = _Reader(words, b.pos, b.pos + lau)
            b.take(lau)
            na = au.one()
            if 5 * na != lau - 1:
                raise VerifyError("length mismatch")
            flat = au.take(5 * na)
            payload = ([flat[5 * i:5 * i + 5] for i in range(na)], leaves)
        b.done()
    r.done()
    return kind, payload


def decode_proof(words: Sequence[int], params: StarkParams) -> List[Tuple[int, object]]:
    words = [int(w) % P for w in words]
    r = _Reader(words, 0, len(words))
    total = r.one()
    if total != len(words) - 1:
        raise VerifyError("proof length mismatch")
    n = r.one()
    items = []
    for _ in range(n):
        ln = r.one()
        lo = r.pos
        r.take(ln)
        items.append(decode_item(words, lo, lo + ln, params))
    r.done()
    return items


# ====================================================================== proof stream (Fiat-Shamir)
class ProofStream:
    def __init__(self, params: StarkParams, items=None):
        self.params = params
        self.items: List[Tuple[int, object]] = list(items or [])
        self.idx = 0
        self.sponge = T.Tip5(fixed_length=False)
        self.transcript: List[Tuple[str, object]] = []  # for intermediate-value parity

    def absorb_words(self, words):
        self.sponge.pad_and_absorb_all(words)

    def enqueue(self, kind, payload):
        if kind in INCLUDED_IN_FIAT_SHAMIR:
            self.absorb_words(encode_item(kind, payload, self.params))
        self.items.append((kind, payload))

    def dequeue(self, expect: int):
        if self.idx >= len(self.items):
            raise VerifyError("proof stream exhausted")
        kind, payload = self.items[self.idx]
        self.idx += 1
        if kind != expect:
            raise VerifyError(f"expected {ITEM_NAMES[expect]}, got {ITEM_NAMES[kind]}")
        if kind in INCLUDED_IN_FIAT_SHAMIR:
            self.absorb_words(encode_item(kind, payload, self.params))
        return payload

    def sample_scalars(self, n: int, tag: str = ""):
        out = [tuple(x) for x in self.sponge.sample_scalars(n)]
        self.transcript.append((tag or "scalars", out))
        return out

    def sample_indices(self, bound: int, n: int, tag: str = "indices"):
        out = self.sponge.sample_indices(bound, n)
        self.transcript.append((tag, out))
        return out


# ====================================================================== Merkle (twenty-first)
def merkle_nodes(leaf_digests: np.ndarray) -> np.ndarray:
    return CO.mtree_build(np.ascontiguousarray(leaf_digests, dtype=np.uint64))


def auth_structure_node_indices(num_leafs: int, leaf_indices: Sequence[int]) -> List[int]:
    needed, computable = set(), set()
    for li in leaf_indices:
        if li >= num_leafs:
            raise VerifyError("leaf index out of range")
        node = li + num_leafs
        while node > 1:
            computable.add(node)
            needed.add(node ^ 1)
            node >>= 1
    return sorted(needed - computable, reverse=True)


def auth_structure(nodes: np.ndarray, leaf_digests: np.ndarray, num_leafs: int, leaf_indices) -> List[List[int]]:
    out = []
    for ni in auth_structure_node_indices(num_leafs, leaf_indices):
        d = leaf_digests[ni - num_leafs] if ni >= num_leafs else nodes[ni]
        out.append([int(x) for x in d])
    return out


def merkle_multiproof_root(tree_height: int, indexed_leafs: Sequence[Tuple[int, Sequence[int]]],
                           auth: Sequence[Sequence[int]]) -> Optional[List[int]]:
    """twenty-first MerkleTreeInclusionProof -> PartialMerkleTree root, or None if malformed."""
    num_leafs = 1 << tree_height
    try:
        idxs = auth_structure_node_indices(num_leafs, [i for i, _ in indexed_leafs])
    except VerifyError:
        return None
    if len(idxs) != len(auth) or not indexed_leafs:
        return None
    nodes: Dict[int, List[int]] = {}
    for ni, d in zip(idxs, auth):
        nodes[ni] = [int(x) % P for x in d]
    for li, d in indexed_leafs:
        ni = li + num_leafs
        d = [int(x) % P for x in d]
        if ni in nodes and nodes[ni] != d:
            return None
        nodes[ni] = d
    level = sorted({li + num_leafs for li, _ in indexed_leafs})
    while level != [1]:
        parents = sorted({n >> 1 for n in level})
        for p in parents:
            l, r = nodes.get(2 * p), nodes.get(2 * p + 1)
            if l is None or r is None:
                return None
            nodes[p] = T.hash_pair(l, r)
        level = parents
    if tree_height == 0:
        return nodes[1]
    return nodes[1]


def merkle_verify(root, tree_height, indexed_leafs, auth) -> bool:
    r = merkle_multiproof_root(tree_height, indexed_leafs, auth)
    return r is not None and list(r) == [int(x) % P for x in root]


def xfe_digest(x) -> List[int]:
    return [x[0], x[1], x[2], 0, 0]


# ====================================================================== AIR as data
INPUT_MAIN_CURR, INPUT_AUX_CURR, INPUT_MAIN_NEXT, INPUT_AUX_NEXT, INPUT_CHALLENGE = range(5)
OP_INPUT, OP_CONST, OP_ADD, OP_SUB, OP_MUL = range(5)
C_INIT, C_CONS, C_TRANS, C_TERM = range(4)


class AirCircuit:
    """Straight-line XFE circuit over OOD row values and challenges.  nodes[i] = (op, a, b, c) with
    OP_INPUT: a = input kind, b = index;  OP_CONST: (a, b, c) = XFE;  ADD/SUB/MUL: node ids a, b.
    constraints: node ids grouped by type in triton order (initial, consistency, transition,
    terminal).  num_sampled challenges are squeezed; 4 more are derived (derive_challenges)."""

    def __init__(self, num_main, num_aux, num_sampled, nodes, constraints_by_type):
        self.num_main, self.num_aux, self.num_sampled = num_main, num_aux, num_sampled
        self.nodes = nodes
        self.constraints = constraints_by_type  # list of 4 lists of node ids

    @property
    def num_constraints(self):
        return sum(len(c) for c in self.constraints)

    @property
    def num_challenges(self):
        return self.num_sampled + NUM_DERIVED_CHALLENGES

    @classmethod
    def from_words(cls, w: Sequence[int]) -> "AirCircuit":
        """Inverse of to_words (the AIR descriptor format)."""
        assert w[0] == 0x41495231, "bad AIR magic"
        num_main, num_aux, num_sampled, n_nodes = w[1], w[2], w[3], w[4]
        counts = w[5:9]
        pos = 9
        nodes = [tuple(w[pos + 4 * i:pos + 4 * i + 4]) for i in range(n_nodes)]
        pos += 4 * n_nodes
        cons = []
        for c in counts:
            cons.append(list(w[pos:pos + c]))
            pos += c
        assert pos == len(w), "trailing AIR words"
        return cls(num_main, num_aux, num_sampled, nodes, cons)

    def to_words(self) -> List[int]:
        w = [0x41495231, self.num_main, self.num_aux, self.num_sampled, len(self.nodes)] + \
            [len(c) for c in self.constraints]
        for op, a, b, c in self.nodes:
            w += [op, a, b, c]
        for cs in self.constraints:
            w += list(cs)
        return w

    def evaluate(self, main_c, aux_c, main_n, aux_n, challenges) -> List[List[Tuple[int, int, int]]]:
        vals = []
        inputs = {INPUT_MAIN_CURR: main_c, INPUT_AUX_CURR: aux_c, INPUT_MAIN_NEXT: main_n,
                  INPUT_AUX_NEXT: aux_n, INPUT_CHALLENGE: challenges}
        for op, a, b, c in self.nodes:
            if op == OP_INPUT:
                v = inputs[a][b]
            elif op == OP_CONST:
                v = (a, b, c)
            elif op == OP_ADD:
                v = xadd(vals[a], vals[b])
            elif op == OP_SUB:
                v = xsub(vals[a], vals[b])
            else:
                v = xmul(vals[a], vals[b])
            vals.append(v)
        return [[vals[i] for i in cs] for cs in self.constraints]


# triton-air 1.0 `ChallengeId` (triton-air 1.0.0, Cargo.lock:4194; the enum in its
# challenge_id.rs, crates.io source not vendored under /root/reference; public design, PARITY
# UNPINNED): the 59 challenges Stark::verify squeezes (Challenges::SAMPLE_COUNT), in declaration
# order, then the 4 that Challenges::new derives, in declaration order.  This list is written out
# independently of include/nhip_challenge_id.h (the table the kernels and the C oracle use);
# tests/test_challenge_ids.py checks that the two agree.
CHALLENGE_IDS = (
    # 0-12: argument indeterminates
    "CompressProgramDigestIndeterminate", "StandardInputIndeterminate", "StandardOutputIndeterminate",
    "InstructionLookupIndeterminate", "HashInputIndeterminate", "HashDigestIndeterminate", "SpongeIndeterminate",
    "OpStackIndeterminate", "RamIndeterminate", "JumpStackIndeterminate", "U32Indeterminate",
    "ClockJumpDifferenceLookupIndeterminate", "RamTableBezoutRelationIndeterminate",
    # 13-15: program table weights
    "ProgramAddressWeight", "ProgramInstructionWeight", "ProgramNextInstructionWeight",
    # 16-19: op stack
    "OpStackClkWeight", "OpStackIb1Weight", "OpStackPointerWeight", "OpStackFirstUnderflowElementWeight",
    # 20-23: RAM
    "RamClkWeight", "RamPointerWeight", "RamValueWeight", "RamInstructionTypeWeight",
    # 24-28: jump stack
    "JumpStackClkWeight", "JumpStackCiWeight", "JumpStackJspWeight", "JumpStackJsoWeight", "JumpStackJsdWeight",
    # 29-31: program attestation, hash table
    "ProgramAttestationPrepareChunkIndeterminate", "ProgramAttestationSendChunkIndeterminate", "HashCIWeight",
    # 32-47: stack weights
    *[f"StackWeight{i}" for i in range(16)],
    # 48-50: hash <-> cascade, 51: cascade <-> lookup, 52-54: lookup table
    "HashCascadeLookupIndeterminate", "HashCascadeLookInWeight", "HashCascadeLookOutWeight",
    "CascadeLookupIndeterminate",
    "LookupTableInputWeight", "LookupTableOutputWeight", "LookupTablePublicIndeterminate",
    # 55-58: U32 table
    "U32LhsWeight", "U32RhsWeight", "U32CiWeight", "U32ResultWeight",
    # 59-62: derived by Challenges::new
    "StandardInputTerminal", "StandardOutputTerminal", "LookupTablePublicTerminal", "CompressedProgramDigest",
)
CHALLENGE_ID = {name: i for i, name in enumerate(CHALLENGE_IDS)}
NUM_DERIVED_CHALLENGES = 4
CHALLENGE_SAMPLE_COUNT = len(CHALLENGE_IDS) - NUM_DERIVED_CHALLENGES  # 59
CH_COMPRESS_PROGRAM_DIGEST_INDETERMINATE = CHALLENGE_ID["CompressProgramDigestIndeterminate"]  # 0
CH_STANDARD_INPUT_INDETERMINATE = CHALLENGE_ID["StandardInputIndeterminate"]  # 1
CH_STANDARD_OUTPUT_INDETERMINATE = CHALLENGE_ID["StandardOutputIndeterminate"]  # 2
CH_LOOKUP_TABLE_PUBLIC_INDETERMINATE = CHALLENGE_ID["LookupTablePublicIndeterminate"]  # 54


def eval_arg_terminal(symbols, challenge, initial=X_ONE):
    """EvalArg::compute_terminal: fold running -> challenge * running + symbol, from
    EvalArg::default_initial() = 1."""
    acc = initial
    for s in symbols:
        acc = xadd(xmul(acc, challenge), lift(int(s) % P))
    return acc


def derive_challenges(sampled, claim) -> List[Tuple[int, int, int]]:
    """Challenges::new(sampled, claim) (triton-vm 1.0 public design, unpinned): sampled ++
    [input terminal, output terminal, lookup-table public terminal, compressed program digest],
    each an evaluation argument folded from 1 with its named indeterminate; the lookup terminal runs
    over twenty-first's tip5::LOOKUP_TABLE."""
    if len(sampled) != CHALLENGE_SAMPLE_COUNT:
        raise VerifyError("Challenges::new takes exactly SAMPLE_COUNT sampled challenges")
    digest, _version, inp, out = claim
    ein = eval_arg_terminal(inp, sampled[CH_STANDARD_INPUT_INDETERMINATE])
    eout = eval_arg_terminal(out, sampled[CH_STANDARD_OUTPUT_INDETERMINATE])
    lut = eval_arg_terminal(T.LOOKUP_TABLE, sampled[CH_LOOKUP_TABLE_PUBLIC_INDETERMINATE])
    comp = eval_arg_terminal(digest, sampled[CH_COMPRESS_PROGRAM_DIGEST_INDETERMINATE])
    return list(sampled) + [ein, eout, lut, comp]


class _SplitMix:
    def __init__(self, seed):
        self.s = seed & 0xFFFFFFFFFFFFFFFF

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        return z ^ (z >> 31)

    def below(self, n):
        return self.next() % n

    def fe(self):
        while True:
            v = self.next()
            if v < P:
                return v


class SynthRecipe:
    """Prover-side construction knowledge for a synthetic AIR (never given to the verifier)."""

    def __init__(self):
        self.free_main: List[int] = []       # free main columns the constraints read
        self.unconstrained_main: List[int] = []  # free main columns no constraint reads (the last one)
        self.targets: List[dict] = []        # definitions in construction order
        self.combos: List[dict] = []         # combination constraints

    @property
    def free_columns(self) -> List[int]:
        """Every main column whose values the prover chooses (the rest are constraint targets)."""
        return self.free_main + self.unconstrained_main


def synth_air(params: StarkParams, num_sampled: int = CHALLENGE_SAMPLE_COUNT, seed: int = 0x5EED, num_constraints: Optional[int] = None):
    """Deterministic synthetic AIR with params' column counts (see module doc)."""
    rng = _SplitMix(seed)
    M, A = params.num_main, params.num_aux
    nodes: List[Tuple[int, int, int, int]] = []
    cache: Dict[tuple, int] = {}

    def node(t):
        if t not in cache:
            cache[t] = len(nodes)
            nodes.append(t)
        return cache[t]

    def inp(kind, idx):
        return node((OP_INPUT, kind, idx, 0))

    def const(v):
        return node((OP_CONST, v[0], v[1], v[2]))

    recipe = SynthRecipe()
    n_free = max(4, (M * 2) // 5)
    recipe.free_main = list(range(n_free))
    # the last main column is free and read by no constraint: the sparse prover
    # (oracle/stark_prover_sparse.py) puts its one non-constant codeword there, in the row's last
    # Tip5 absorption chunk
    recipe.unconstrained_main = [M - 1]
    by_type: List[List[int]] = [[], [], [], []]
    base_by_type: List[List[int]] = [[], [], [], []]  # indices into recipe.targets
    type_weights = [C_CONS] * 10 + [C_TRANS] * 7 + [C_INIT] * 2 + [C_TERM]
    main_targets: List[int] = []

    def pick_type():
        return type_weights[rng.below(len(type_weights))]

    def make_constraint(target_is_aux, tcol, ctype, factors, coef, lin, lin_coef):
        # C = target - (coef * prod(factors) + lin_coef * lin)
        tnode = inp(INPUT_AUX_CURR if target_is_aux else INPUT_MAIN_CURR, tcol)
        prod = const(coef)
        for f in factors:
            prod = node((OP_MUL, prod, inp(*f), 0))
        rhs = prod
        if lin is not None:
            rhs = node((OP_ADD, rhs, node((OP_MUL, const(lin_coef), inp(*lin), 0)), 0))
        return node((OP_SUB, tnode, rhs, 0))

    # main targets: BFE-only products of free columns (+ optional linear earlier target)
    for t in range(n_free, M - 1):
        ctype = pick_type()
        deg = 1 + rng.below(4)
        nxt = ctype == C_TRANS
        factors = []
        for _ in range(deg):
            col = recipe.free_main[rng.below(n_free)]
            kind = INPUT_MAIN_NEXT if (nxt and rng.below(2)) else INPUT_MAIN_CURR
            factors.append((kind, col))
        coef = (1 + rng.below(1 << 20), 0, 0)
        lin = None
        lin_coef = (0, 0, 0)
        if main_targets and rng.below(2):
            lin = (INPUT_MAIN_CURR, main_targets[rng.below(len(main_targets))])
            lin_coef = (1 + rng.below(1 << 16), 0, 0)
        nid = make_constraint(False, t, ctype, factors, coef, lin, lin_coef)
        recipe.targets.append(dict(aux=False, col=t, type=ctype, factors=factors, coef=coef, lin=lin,
                                   lin_coef=lin_coef, node=nid))
        base_by_type[ctype].append(len(recipe.targets) - 1)
        main_targets.append(t)
    # aux targets: challenge-weighted products; the last 4 bind the claim (and the lookup table)
    # through the derived challenges
    aux_targets: List[int] = []
    nd = NUM_DERIVED_CHALLENGES
    for j in range(A):
        if j >= A - nd:
            ctype = C_TERM
            factors = [(INPUT_CHALLENGE, num_sampled + (j - (A - nd)))]
            coef = X_ONE
            lin, lin_coef = None, X_ZERO
        else:
            ctype = pick_type()
            deg = 1 + rng.below(3)
            nxt = ctype == C_TRANS
            factors = [(INPUT_CHALLENGE, rng.below(num_sampled))]
            for _ in range(deg):
                col = recipe.free_main[rng.below(n_free)]
                kind = INPUT_MAIN_NEXT if (nxt and rng.below(2)) else INPUT_MAIN_CURR
                factors.append((kind, col))
            coef = (1 + rng.below(1 << 20), rng.below(1 << 20), 0)
            lin, lin_coef = None, X_ZERO
            if aux_targets and rng.below(2):
                lin = (INPUT_AUX_CURR, aux_targets[rng.below(len(aux_targets))])
                lin_coef = (rng.below(1 << 16), 1 + rng.below(1 << 16), 0)
            elif rng.below(2):
                lin = (INPUT_MAIN_CURR, main_targets[rng.below(len(main_targets))] if main_targets else 0)
                lin_coef = (1 + rng.below(1 << 16), 0, 0)
        nid = make_constraint(True, j, ctype, factors, coef, lin, lin_coef)
        recipe.targets.append(dict(aux=True, col=j, type=ctype, factors=factors, coef=coef, lin=lin,
                                   lin_coef=lin_coef, node=nid))
        base_by_type[ctype].append(len(recipe.targets) - 1)
        aux_targets.append(j)
    for ctype in range(4):
        for ti in base_by_type[ctype]:
            by_type[ctype].append(recipe.targets[ti]["node"])
    # combination constraints C = C_a + lambda * C_b (same zerofier type) up to the requested count
    want = num_constraints if num_constraints is not None else max(len(recipe.targets), int(1.6 * len(recipe.targets)))
    while sum(len(c) for c in by_type) < want:
        ctype = pick_type()
        if len(base_by_type[ctype]) < 2:
            continue
        a = base_by_type[ctype][rng.below(len(base_by_type[ctype]))]
        b = base_by_type[ctype][rng.below(len(base_by_type[ctype]))]
        lam = (1 + rng.below(1 << 24), rng.below(1 << 8), 0)
        nid = node((OP_ADD, recipe.targets[a]["node"], node((OP_MUL, const(lam), recipe.targets[b]["node"], 0)), 0))
        recipe.combos.append(dict(type=ctype, a=a, b=b, lam=lam, node=nid))
        by_type[ctype].append(nid)
    air = AirCircuit(M, A, num_sampled, nodes, by_type)
    return air, recipe


def bloat_air(air: AirCircuit, target_nodes: int, seed: int = 0xB10A7, max_degree: int = 4) -> AirCircuit:
    """The same AIR (every constraint has the same value on every input) as a circuit of about
    `target_nodes` nodes, for tests of the evaluator at triton-air's size class (~600 constraints
    over ~20-30k nodes after degree lowering).  Each constraint C becomes C + sum_t (m_t - m_t'),
    where m_t and m_t' are one random monomial of degree <= max_degree over OOD-row inputs and
    challenges, multiplied in two different orders: identically zero, so the synthetic prover's
    quotients (from the recipe) still satisfy it, but every term is real work for the verifier
    (loads, products, a subtraction, an accumulation)."""
    rng = _SplitMix(seed)
    nodes = list(air.nodes)
    cache = {t: i for i, t in enumerate(nodes)}

    def node(t):
        if t not in cache:
            cache[t] = len(nodes)
            nodes.append(t)
        return cache[t]

    kinds = [(INPUT_MAIN_CURR, air.num_main), (INPUT_AUX_CURR, air.num_aux), (INPUT_MAIN_NEXT, air.num_main),
             (INPUT_AUX_NEXT, air.num_aux), (INPUT_CHALLENGE, air.num_challenges)]

    def rand_input():
        k, n = kinds[rng.below(len(kinds))]
        return node((OP_INPUT, k, rng.below(n), 0))

    def product(fs):
        acc = fs[0]
        for f in fs[1:]:
            acc = node((OP_MUL, acc, f, 0))
        return acc

    n_cons = air.num_constraints
    per = max(1, (target_nodes - len(nodes)) // max(1, 6 * n_cons))
    cons = []
    for cs in air.constraints:
        out = []
        for c in cs:
            acc = c
            for _ in range(per):
                fs = [rand_input() for _ in range(2 + rng.below(max_degree - 1))]
                rev = fs[::-1] if len(fs) > 2 else [fs[1], fs[0]]
                diff = node((OP_SUB, product(fs), product(rev), 0))
                acc = node((OP_ADD, acc, diff, 0))
            out.append(acc)
        cons.append(out)
    return AirCircuit(air.num_main, air.num_aux, air.num_sampled, nodes, cons)


# ====================================================================== verifier
def zerofier_inverses(z, padded_height):
    w = primitive_root_of_unity(padded_height)
    w_inv = binv(w)
    init_inv = xinv(xsub(z, X_ONE))
    cons_inv = xinv(xsub(xpow(z, padded_height), X_ONE))
    except_last = xsub(z, lift(w_inv))
    trans_inv = xmul(except_last, cons_inv)
    term_inv = xinv(except_last)
    return [init_inv, cons_inv, trans_inv, term_inv]


def colinear_y(ax, ay, bx, by, x):
    """y at x of the line through (ax, ay), (bx, by); ax != bx (twenty-first get_colinear_y)."""
    slope = xmul(xsub(by, ay), xinv(xsub(bx, ax)))
    return xadd(ay, xmul(slope, xsub(x, ax)))


def fri_verify(ps: ProofStream, params: StarkParams, domain: Domain):
    R = params.fri_num_rounds(domain.length)
    rounds = []
    d = domain
    for r in range(R + 1):
        root = ps.dequeue(MERKLE_ROOT)
        alpha = ps.sample_scalars(1, f"fri_alpha_{r}")[0] if r < R else None
        rounds.append(dict(domain=d, root=root, alpha=alpha))
        d = d.halve()
    last_codeword = ps.dequeue(FRI_CODEWORD)
    last_poly = ps.dequeue(FRI_POLYNOMIAL)
    n0 = domain.length
    k = params.num_collinearity_checks
    idx = ps.sample_indices(n0, k, "fri_indices")

    def a_idx(r):
        return [i % rounds[r]["domain"].length for i in idx]

    def b_idx(r):
        n = rounds[r]["domain"].length
        return [(i + n // 2) % n for i in idx]

    auth, leaves = ps.dequeue(FRI_RESPONSE)
    if len(leaves) != k:
        raise VerifyError("FRI: wrong number of revealed leaves")
    h0 = int(math.log2(n0))
    if not merkle_verify(rounds[0]["root"], h0, list(zip(a_idx(0), [xfe_digest(x) for x in leaves])), auth):
        raise VerifyError("FRI: bad Merkle authentication (round 0, a)")
    rounds[0]["a"] = leaves
    for r in range(R):
        auth, leaves = ps.dequeue(FRI_RESPONSE)
        if len(leaves) != k:
            raise VerifyError("FRI: wrong number of revealed leaves")
        h = int(math.log2(rounds[r]["domain"].length))
        if not merkle_verify(rounds[r]["root"], h, list(zip(b_idx(r), [xfe_digest(x) for x in leaves])), auth):
            raise VerifyError(f"FRI: bad Merkle authentication (round {r}, b)")
        rounds[r]["b"] = leaves
    for r in range(R):
        dom = rounds[r]["domain"]
        ai, bi = a_idx(r), b_idx(r)
        folded = []
        for j in range(k):
            ax, bx = lift(dom.value(ai[j])), lift(dom.value(bi[j]))
            folded.append(colinear_y(ax, rounds[r]["a"][j], bx, rounds[r]["b"][j], rounds[r]["alpha"]))
        rounds[r + 1]["a"] = folded
    # last round: Merkle root of the codeword, agreement, low degree
    last_len = rounds[R]["domain"].length
    if len(last_codeword) != last_len:
        raise VerifyError("FRI: last codeword length")
    ld = np.array([xfe_digest(x) for x in last_codeword], dtype=np.uint64)
    lroot = [int(x) for x in merkle_nodes(ld)[1]] if last_len > 1 else [int(x) for x in ld[0]]
    if lroot != list(rounds[R]["root"]):
        raise VerifyError("FRI: bad Merkle root for last codeword")
    for j, i in enumerate(a_idx(R)):
        if last_codeword[i] != rounds[R]["a"][j]:
            raise VerifyError("FRI: last codeword mismatch")
    first_max_degree = n0 // params.fri_expansion_factor - 1
    last_max_degree = first_max_degree >> R
    if xpoly_degree(last_poly) > last_max_degree:
        raise VerifyError("FRI: last polynomial degree too high")
    indeterminate = ps.sample_scalars(1, "fri_last_indeterminate")[0]
    if xpoly_eval(last_poly, indeterminate) != barycentric_evaluate(last_codeword, indeterminate):
        raise VerifyError("FRI: last polynomial evaluation mismatch")
    return list(zip(a_idx(0), rounds[0]["a"]))


def verify(params: StarkParams, air: AirCircuit, claim, proof_words: Sequence[int], transcript=None) -> bool:
    """triton_vm::verify semantics: any decode or verification error -> False."""
    try:
        _verify(params, air, claim, proof_words, transcript)
        return True
    except (VerifyError, ZeroDivisionError, ValueError, IndexError, AssertionError):
        return False


def _verify(params, air, claim, proof_words, transcript):
    items = decode_proof(proof_words, params)
    ps = ProofStream(params, items)
    digest, version, inp, out = claim
    ps.absorb_words(encode_claim(digest, version, inp, out))
    log2_ph = ps.dequeue(LOG2_PADDED_HEIGHT)
    if log2_ph > 28:
        raise VerifyError("padded height too large")
    ph = 1 << log2_ph
    fri_dom = params.fri_domain(ph)
    tree_h = int(math.log2(fri_dom.length))
    # sample_indices takes a u32 upper bound; the descriptors hold at most 26 FRI rounds
    if tree_h > 31 or params.fri_num_rounds(fri_dom.length) > MAX_FRI_ROUNDS:
        raise VerifyError("FRI domain too large")
    main_root = ps.dequeue(MERKLE_ROOT)
    sampled = ps.sample_scalars(air.num_sampled, "challenges")
    challenges = derive_challenges(sampled, claim)
    aux_root = ps.dequeue(MERKLE_ROOT)
    quot_w = ps.sample_scalars(air.num_constraints, "quotient_weights")
    quot_root = ps.dequeue(MERKLE_ROOT)
    w_tr = primitive_root_of_unity(ph)
    z = ps.sample_scalars(1, "ood_point")[0]
    z_next = xscale(z, w_tr)
    z_pow = xpow(z, params.num_quotient_segments)
    mc = ps.dequeue(OOD_MAIN_ROW)
    ac = ps.dequeue(OOD_AUX_ROW)
    mn = ps.dequeue(OOD_MAIN_ROW)
    an = ps.dequeue(OOD_AUX_ROW)
    qs = ps.dequeue(OOD_QUOT_SEGMENTS)
    zinv = zerofier_inverses(z, ph)
    by_type = air.evaluate(mc, ac, mn, an, challenges)
    summands = [xmul(v, zinv[t]) for t in range(4) for v in by_type[t]]
    ood_q = X_ZERO
    for w, s in zip(quot_w, summands):
        ood_q = xadd(ood_q, xmul(w, s))
    seg_sum = X_ZERO
    zk = X_ONE
    for s in qs:
        seg_sum = xadd(seg_sum, xmul(zk, s))
        zk = xmul(zk, z)
    if transcript is not None:
        transcript["ood_quotient"] = ood_q
    if ood_q != seg_sum:
        raise VerifyError("out-of-domain quotient value mismatch")
    nw = params.num_main + params.num_aux + params.num_quotient_segments + params.num_deep
    w = ps.sample_scalars(nw, "lincomb_weights")
    w_main = w[:params.num_main]
    w_aux = w[params.num_main:params.num_main + params.num_aux]
    w_quot = w[params.num_main + params.num_aux:params.num_main + params.num_aux + params.num_quotient_segments]
    w_deep = w[-params.num_deep:]

    def lin_main_aux(mrow, arow, main_is_x):
        acc = X_ZERO
        for wi, v in zip(w_main, mrow):
            acc = xadd(acc, xmul(wi, v) if main_is_x else xscale(wi, v))
        for wi, v in zip(w_aux, arow):
            acc = xadd(acc, xmul(wi, v))
        return acc

    ood_curr_mav = lin_main_aux(mc, ac, True)
    ood_next_mav = lin_main_aux(mn, an, True)
    ood_curr_q = X_ZERO
    for wi, v in zip(w_quot, qs):
        ood_curr_q = xadd(ood_curr_q, xmul(wi, v))
    revealed = fri_verify(ps, params, fri_dom)
    indices = [i for i, _ in revealed]
    main_rows = ps.dequeue(MAIN_ROWS)
    main_auth = ps.dequeue(AUTH_STRUCTURE)
    if len(main_rows) != len(indices):
        raise VerifyError("main rows count")
    md = CO.hash_varlen_batch(np.array([c for r in main_rows for c in r] or [0], dtype=np.uint64),
                              np.arange(0, len(main_rows) * params.num_main + 1, params.num_main, dtype=np.uint64))
    if not merkle_verify(main_root, tree_h, list(zip(indices, [list(map(int, d)) for d in md])), main_auth):
        raise VerifyError("main codeword authentication failure")
    aux_rows = ps.dequeue(AUX_ROWS)
    aux_auth = ps.dequeue(AUTH_STRUCTURE)
    if len(aux_rows) != len(indices):
        raise VerifyError("aux rows count")
    wa = EXT * params.num_aux
    ad = CO.hash_varlen_batch(np.array([c for r in aux_rows for c in _xflat(r)] or [0], dtype=np.uint64),
                              np.arange(0, len(aux_rows) * wa + 1, wa, dtype=np.uint64))
    if not merkle_verify(aux_root, tree_h, list(zip(indices, [list(map(int, d)) for d in ad])), aux_auth):
        raise VerifyError("aux codeword authentication failure")
    qrows = ps.dequeue(QUOT_SEGMENTS_ELEMENTS)
    qauth = ps.dequeue(AUTH_STRUCTURE)
    if len(qrows) != len(indices):
        raise VerifyError("quotient rows count")
    wq = EXT * params.num_quotient_segments
    qd = CO.hash_varlen_batch(np.array([c for r in qrows for c in _xflat(r)] or [0], dtype=np.uint64),
                              np.arange(0, len(qrows) * wq + 1, wq, dtype=np.uint64))
    if not merkle_verify(quot_root, tree_h, list(zip(indices, [list(map(int, d)) for d in qd])), qauth):
        raise VerifyError("quotient codeword authentication failure")
    if params.num_collinearity_checks != len(indices):
        raise VerifyError("wrong number of revealed indices")
    for (i, fri_value), mrow, arow, qrow in zip(revealed, main_rows, aux_rows, qrows):
        x = lift(fri_dom.value(i))
        mav = lin_main_aux(mrow, arow, False)
        qv = X_ZERO
        for wi, v in zip(w_quot, qrow):
            qv = xadd(qv, xmul(wi, v))
        t0 = xmul(xsub(mav, ood_curr_mav), xinv(xsub(x, z)))
        t1 = xmul(xsub(mav, ood_next_mav), xinv(xsub(x, z_next)))
        t2 = xmul(xsub(qv, ood_curr_q), xinv(xsub(x, z_pow)))
        deep = xadd(xadd(xmul(t0, w_deep[0]), xmul(t1, w_deep[1])), xmul(t2, w_deep[2]))
        if deep != fri_value:
            raise VerifyError("combination codeword mismatch")
    if ps.idx != len(ps.items):
        raise VerifyError("proof stream has items left")
    if transcript is not None:
        transcript["sponge_samples"] = ps.transcript
        transcript["roots"] = [main_root, aux_root, quot_root]


def expected_kinds(R: int) -> List[int]:
    return ([LOG2_PADDED_HEIGHT, MERKLE_ROOT, MERKLE_ROOT, MERKLE_ROOT, OOD_MAIN_ROW, OOD_AUX_ROW, OOD_MAIN_ROW,
             OOD_AUX_ROW, OOD_QUOT_SEGMENTS] + [MERKLE_ROOT] * (R + 1) + [FRI_CODEWORD, FRI_POLYNOMIAL] +
            [FRI_RESPONSE] * (R + 1) + [MAIN_ROWS, AUTH_STRUCTURE, AUX_ROWS, AUTH_STRUCTURE, QUOT_SEGMENTS_ELEMENTS,
                                        AUTH_STRUCTURE])


def structure_ok(params: StarkParams, proof_words: Sequence[int]) -> bool:
    """Decodes, has the item sequence of Stark::verify and the counts it checks (no arithmetic)."""
    try:
        items = decode_proof(proof_words, params)
    except VerifyError:
        return False
    if not items or items[0][0] != LOG2_PADDED_HEIGHT or items[0][1] > 28:
        return False
    ph = 1 << items[0][1]
    N = params.fri_domain(ph).length
    R = params.fri_num_rounds(N)
    if N > (1 << 31) or R > MAX_FRI_ROUNDS:
        return False
    if [k for k, _ in items] != expected_kinds(R):
        return False
    k = params.num_collinearity_checks
    byk = {}
    for kind, payload in items:
        byk.setdefault(kind, []).append(payload)
    if any(len(leaves) != k for _, leaves in byk[FRI_RESPONSE]):
        return False
    if len(byk[MAIN_ROWS][0]) != k or len(byk[AUX_ROWS][0]) != k or len(byk[QUOT_SEGMENTS_ELEMENTS][0]) != k:
        return False
    return len(byk[FRI_CODEWORD][0]) == N >> R
