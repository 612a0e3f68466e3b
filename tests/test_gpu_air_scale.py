"""The OOD AIR evaluator at triton-air's size class (SURVEY §7 hard part 2; triton-air 1.0.0,
Cargo.lock:4194, ~600 constraints, tens of thousands of circuit nodes after degree lowering):
the synthetic AIR with 620 constraints, bloated to ~22k nodes by identically-zero terms
(stark_ref.bloat_air: same constraint values, real evaluation work).  Its compiled program (the
liveness-priority schedule of stark_host.cpp air_compile) keeps every value in LDS; the same circuit
with the LDS part capped (nhip_air_create_ex's lds_slots) runs k_ood_air's global-memory slot
overflow.  An accepting proof and mutated ones give the oracle's verdicts either way, and the
Fiat-Shamir transcript is the oracle's."""
import numpy as np
import pytest

import stark_prover_fast as F
import stark_ref as S
import tip5_ref as T

pytestmark = pytest.mark.gpu


def test_triton_air_sized_circuit_matches_oracle_in_lds_and_with_global_slots(ctx):
    import neptune_hip.stark as NS
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1, num_constraints=620)
    big = S.bloat_air(air, 24000)
    assert big.num_constraints >= 600 and len(big.nodes) >= 20000
    claim = ([3, 1, 4, 1, 5], 0, [9, 2, 6], [5, 3])
    proof, _ = F.prove(params, big, recipe, claim, 10, seed=0xA1)
    gair = NS.Air(big.to_words())
    info = gair.info()
    assert info["global_slots"] == 0 and info["lds_slots"] < 4000, info  # the schedule fits LDS
    gair_g = NS.Air(big.to_words(), lds_slots=600)
    info_g = gair_g.info()
    assert info_g["lds_slots"] == 600 and info_g["global_slots"] > 1000, info_g  # the overflow path
    items = S.decode_proof(proof, params)
    spans, pos = [], 2
    for _ in items:
        spans.append(pos + 1)
        pos += 1 + proof[pos]
    kinds = [k for k, _ in items]
    muts = []
    for k, off in ((S.OOD_MAIN_ROW, 1 + 3 * 200), (S.OOD_AUX_ROW, 1 + 3 * 40 + 2), (S.OOD_QUOT_SEGMENTS, 1 + 4)):
        m = list(proof)
        p = spans[kinds.index(k)] + off
        m[p] = (m[p] + 1) % S.P
        muts.append(m)
    cases = [proof] + muts
    want = [S.verify(params, big, claim, p) for p in cases]
    assert want == [True, False, False, False]
    b = NS.Batch(ctx, gair, NS.Stark.default(), [NS.Claim(*claim)] * len(cases), cases)
    v, _ = b.run()
    assert [bool(x) for x in v] == want
    bg = NS.Batch(ctx, gair_g, NS.Stark.default(), [NS.Claim(*claim)] * len(cases), cases)
    vg, _ = bg.run()
    assert [bool(x) for x in vg] == want
    bg.close()
    tr = {}
    S.verify(params, big, claim, proof, tr)
    samples = [tuple(x) for tag, vals in tr["sponge_samples"] if tag != "fri_indices" for x in vals]
    xs, idx, fail = b.transcript(0)
    assert fail == 0 and xs == samples
    # the same proofs against the un-bloated AIR (all slots in LDS): same verdicts
    small = NS.Air(air.to_words())
    assert small.info()["global_slots"] == 0
    assert NS.verify_batch(ctx, small, NS.Stark.default(), [(NS.Claim(*claim), p) for p in cases]) == want
    # a batch of 256 copies: k_ood_air time at this AIR size (reported)
    many = NS.Batch(ctx, gair, NS.Stark.default(), [NS.Claim(*claim)] * 256, [proof] * 256)
    for _ in range(2):
        v, ok = many.run()
    st = many.stats()
    assert ok
    print(f"k_ood_air, 256 proofs, {len(big.nodes)} nodes / {info['lds_slots']} LDS + "
          f"{info['global_slots']} global slots: {st['ms_ood_air']:.3f} ms")
    many.close()
    # the 256-thread evaluator with global slots (batches past OOD_WIDE_MAX_PROOFS): accepting and
    # OOD-mutated proofs interleaved
    mixed = [proof if i % 2 == 0 else muts[i % 3] for i in range(256)]
    want_m = [i % 2 == 0 for i in range(256)]
    bm = NS.Batch(ctx, gair_g, NS.Stark.default(), [NS.Claim(*claim)] * 256, mixed)
    vm, _ = bm.run()
    assert [bool(x) for x in vm] == want_m
    bm.close()
    b.close()
