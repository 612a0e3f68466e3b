"""Synthetic STARK prover for arbitrarily large padded heights — TEST DATA GENERATOR ONLY.

Same proof structure and Fiat-Shamir order as stark_prover_fast.py (and the verifier
oracle/stark_ref.py), but every committed codeword is *constant*:

  * free main columns are random constants and every AIR target column is its constraint's
    right-hand side evaluated on those constants (curr == next), so every constraint holds
    identically and all quotient segments are zero;
  * the DEEP codeword (f(x) - f(z)) / (x - z) of a constant f is zero, so every FRI codeword is zero,
    the last codeword is zero and the last polynomial is empty;
  * a Merkle tree over 2^h equal leaves has one digest per level, so each root and every
    authentication structure costs O(h) Tip5 permutations instead of O(2^h).

The verifier's work does not depend on the values (same rows hashed, same multiproof shapes, same
FRI rounds), so these proofs are a faithful verification workload for BASELINE config 5 (log2
padded height 23: FRI domain 2^26, 17 rounds) that the full provers cannot reach (their codewords
would need 2^26 x 467 field elements).  tests/test_stark_prover_const.py checks the proofs with the
oracle verifier (accept) and with mutations (reject).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import stark_ref as S
import tip5_ref as T
from field_ref import X_ONE, X_ZERO, lift, xadd, xmul


def _const_tree(leaf: Sequence[int], h: int) -> List[List[int]]:
    """Level digests of a tree of 2^h copies of `leaf`: D[0] = leaf, D[t + 1] = hash_pair(D[t], D[t])."""
    d = [list(map(int, leaf))]
    for _ in range(h):
        d.append([int(x) for x in T.hash_pair(d[-1], d[-1])])
    return d


def _const_auth(levels: List[List[int]], h: int, indices: Sequence[int]) -> List[List[int]]:
    out = []
    for node in S.auth_structure_node_indices(1 << h, list(indices)):
        depth = node.bit_length() - 1
        out.append(levels[h - depth])
    return out


def prove(params: S.StarkParams, air: S.AirCircuit, recipe: S.SynthRecipe, claim, log2_ph: int, seed: int = 1):
    rng = S._SplitMix(seed)
    ph = 1 << log2_ph
    dom = params.fri_domain(ph)
    N = dom.length
    h = N.bit_length() - 1
    M, A, nseg = params.num_main, params.num_aux, params.num_quotient_segments
    ps = S.ProofStream(params)
    digest, version, inp, out = claim
    ps.absorb_words(S.encode_claim(digest, version, inp, out))
    ps.enqueue(S.LOG2_PADDED_HEIGHT, log2_ph)

    target_of = {(t["aux"], t["col"]): i for i, t in enumerate(recipe.targets)}
    free = {c: rng.fe() for c in recipe.free_columns}
    memo: Dict[tuple, tuple] = {}

    def col_value(is_aux: bool, col: int, chal):
        key = (is_aux, col)
        if key in memo:
            return memo[key]
        if not is_aux and col in free:
            v = lift(free[col])
        else:
            t = recipe.targets[target_of[key]]
            acc = t["coef"]
            for kind, idx in t["factors"]:
                if kind == S.INPUT_CHALLENGE:
                    acc = xmul(acc, chal[idx])
                else:
                    acc = xmul(acc, col_value(kind in (S.INPUT_AUX_CURR, S.INPUT_AUX_NEXT), idx, chal))
            if t["lin"] is not None:
                lk, li = t["lin"]
                acc = xadd(acc, xmul(t["lin_coef"], col_value(lk == S.INPUT_AUX_CURR, li, chal)))
            v = acc
        memo[key] = v
        return v

    main_vals = [col_value(False, c, None) for c in range(M)]
    assert all(v[1] == 0 and v[2] == 0 for v in main_vals), "main columns are base-field"
    main_row = [v[0] for v in main_vals]
    main_levels = _const_tree(T.hash_varlen(main_row), h)
    ps.enqueue(S.MERKLE_ROOT, main_levels[h])
    sampled = ps.sample_scalars(air.num_sampled, "challenges")
    chal = S.derive_challenges(sampled, claim)
    aux_vals = [col_value(True, j, chal) for j in range(A)]
    aux_flat = [c for v in aux_vals for c in v]
    aux_levels = _const_tree(T.hash_varlen(aux_flat), h)
    ps.enqueue(S.MERKLE_ROOT, aux_levels[h])
    ps.sample_scalars(air.num_constraints, "quotient_weights")
    q_levels = _const_tree(T.hash_varlen([0] * (3 * nseg)), h)
    ps.enqueue(S.MERKLE_ROOT, q_levels[h])
    ps.sample_scalars(1, "ood_point")
    for kind, payload in ((S.OOD_MAIN_ROW, main_vals), (S.OOD_AUX_ROW, aux_vals), (S.OOD_MAIN_ROW, main_vals),
                          (S.OOD_AUX_ROW, aux_vals), (S.OOD_QUOT_SEGMENTS, [X_ZERO] * nseg)):
        ps.enqueue(kind, payload)
    ps.sample_scalars(M + A + nseg + params.num_deep, "lincomb_weights")
    # FRI over the zero codeword
    R = params.fri_num_rounds(N)
    zero_leaf = [0, 0, 0, 0, 0]
    fri_levels = []
    for r in range(R + 1):
        lv = _const_tree(zero_leaf, h - r)
        fri_levels.append(lv)
        ps.enqueue(S.MERKLE_ROOT, lv[h - r])
        if r < R:
            ps.sample_scalars(1, f"fri_alpha_{r}")
    L = N >> R
    ps.enqueue(S.FRI_CODEWORD, [X_ZERO] * L)
    ps.enqueue(S.FRI_POLYNOMIAL, [])
    k = params.num_collinearity_checks
    idx = ps.sample_indices(N, k, "fri_indices")
    ps.enqueue(S.FRI_RESPONSE, (_const_auth(fri_levels[0], h, idx), [X_ZERO] * k))
    for r in range(R):
        n = N >> r
        ps.enqueue(S.FRI_RESPONSE, (_const_auth(fri_levels[r], h - r, [(i + n // 2) % n for i in idx]), [X_ZERO] * k))
    ps.sample_scalars(1, "fri_last_indeterminate")
    ps.enqueue(S.MAIN_ROWS, [list(main_row)] * k)
    ps.enqueue(S.AUTH_STRUCTURE, _const_auth(main_levels, h, idx))
    ps.enqueue(S.AUX_ROWS, [list(aux_vals)] * k)
    ps.enqueue(S.AUTH_STRUCTURE, _const_auth(aux_levels, h, idx))
    ps.enqueue(S.QUOT_SEGMENTS_ELEMENTS, [[X_ZERO] * nseg] * k)
    ps.enqueue(S.AUTH_STRUCTURE, _const_auth(q_levels, h, idx))
    return S.encode_proof(ps.items, params), ps.transcript
