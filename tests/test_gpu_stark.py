"""GPU parity of the batched STARK verifier (nhip_verify_batch / nhip_batch_*) with the oracle
(oracle/stark_ref.py): every verdict and every Fiat-Shamir sample (challenges, quotient weights,
OOD point, linear-combination weights, FRI folding challenges, FRI indices, last indeterminate)
identical.  Accepting proofs come from the oracle's synthetic prover; rejecting ones from the
reference's reject cases and from mutations of accepting proofs."""
import json
import os

import numpy as np
import pytest

import stark_prover as SP
import stark_ref as S
import tip5_ref as T

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "stark_tiny.json")


def _ns():
    import neptune_hip.stark as NS
    return NS


@pytest.fixture(scope="module")
def tiny():
    g = json.load(open(GOLD))
    params = S.StarkParams(**g["params"])
    air, _ = S.synth_air(params, num_sampled=g["num_sampled"], seed=g["seed"])
    return g, params, air


def _oracle_samples(params, air, claim, proof):
    tr = {}
    ok = S.verify(params, air, claim, proof, tr)
    if not ok:
        return ok, None, None
    samples = [tuple(x) for tag, vals in tr["sponge_samples"] if tag != "fri_indices" for x in vals]
    indices = [v for tag, vals in tr["sponge_samples"] if tag == "fri_indices" for v in vals]
    return ok, samples, indices


def test_tiny_golden_verdicts_and_transcripts(ctx, tiny):
    NS = _ns()
    g, params, air = tiny
    gair = NS.Air([int(w) for w in g["air"]])
    stark = NS.Stark(num_collinearity_checks=8, num_main=24, num_aux=9)
    claims, proofs = [], []
    for c in g["cases"]:
        cl = c["claim"]
        claims.append(NS.Claim(cl["digest"], cl["version"], cl["input"], cl["output"]))
        proofs.append([int(w) for w in c["proof"]])
    b = NS.Batch(ctx, gair, stark, claims, proofs)
    v, ok = b.run()
    assert list(v) == [1, 1, 1] and ok
    for i, c in enumerate(g["cases"]):
        xs, idx, fail = b.transcript(i)
        assert fail == 0
        assert [[str(x) for x in t] for t in xs] == c["samples"]
        assert idx == c["fri_indices"]


def test_reference_reject_cases_on_gpu(ctx, tiny):
    NS = _ns()
    g, params, air = tiny
    gair = NS.Air([int(w) for w in g["air"]])
    stark = NS.Stark(num_collinearity_checks=8, num_main=24, num_aux=9)
    cl = g["cases"][0]["claim"]
    claim = NS.Claim(cl["digest"], cl["version"], cl["input"], cl["output"])
    bogus = T.hash_varlen(S.encode_claim(cl["digest"], cl["version"], cl["input"], cl["output"]))
    good = [int(w) for w in g["cases"][0]["proof"]]
    pairs = [(claim, p) for p in ([], bogus, [0] * 65, [0], [1], good)]
    assert NS.verify_batch(ctx, gair, stark, pairs) == [False, False, False, False, False, True]
    # the claim is bound: other output / input / digest / version -> reject
    wrong = [NS.Claim(cl["digest"], cl["version"], cl["input"], list(cl["output"]) + [1]),
             NS.Claim(cl["digest"], cl["version"], [5] + list(cl["input"]), cl["output"]),
             NS.Claim([1, 1, 1, 1, 1], cl["version"], cl["input"], cl["output"]),
             NS.Claim(cl["digest"], 1, cl["input"], cl["output"])]
    assert NS.verify_batch(ctx, gair, stark, [(w, good) for w in wrong]) == [False] * 4


def test_tiny_mutations_match_oracle(ctx, tiny):
    NS = _ns()
    g, params, air = tiny
    gair = NS.Air([int(w) for w in g["air"]])
    stark = NS.Stark(num_collinearity_checks=8, num_main=24, num_aux=9)
    c = g["cases"][2]
    cl = c["claim"]
    claim_t = (cl["digest"], cl["version"], cl["input"], cl["output"])
    claim = NS.Claim(*claim_t)
    proof = [int(w) for w in c["proof"]]
    rng = np.random.default_rng(21)
    muts = []
    for pos in sorted(set(rng.integers(0, len(proof), size=70).tolist()) | {0, 1, 2, 3, len(proof) - 1}):
        m = list(proof)
        m[pos] = (m[pos] + 1) % S.P
        muts.append(m)
    got = NS.verify_batch(ctx, gair, stark, [(claim, m) for m in muts])
    ref = [S.verify(params, air, claim_t, m) for m in muts]
    assert got == ref
    assert not any(ref)  # a single-word change always breaks some check


@pytest.fixture(scope="module")
def full():
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    out = []
    for lph, claim in [(4, ([11, 22, 33, 44, 55], 0, [1, 2, 3, 4, 5], [])), (6, ([7, 7, 7, 7, 7], 0, [], [9, 8]))]:
        proof, _ = SP.prove(params, air, recipe, claim, lph, seed=lph)
        out.append((claim, proof))
    return params, air, out


def test_full_size_params_verdicts_and_transcripts(ctx, full):
    NS = _ns()
    params, air, cases = full
    gair = NS.Air(air.to_words())
    stark = NS.Stark.default()
    assert (stark.num_main, stark.num_aux, stark.num_collinearity_checks) == (379, 88, 80)
    claims = [NS.Claim(*c) for c, _ in cases]
    b = NS.Batch(ctx, gair, stark, claims, [p for _, p in cases])
    v, ok = b.run()
    assert list(v) == [1, 1] and ok
    for i, (claim, proof) in enumerate(cases):
        ok_o, samples, indices = _oracle_samples(params, air, claim, proof)
        assert ok_o
        xs, idx, fail = b.transcript(i)
        assert fail == 0 and xs == samples and idx == indices
    st = b.stats()
    assert st["num_proofs"] == 2 and st["tip5_perms_static"] > 0


def test_full_size_targeted_mutations(ctx, full):
    """Corrupt one value inside each verifier phase's input; GPU and oracle both reject."""
    NS = _ns()
    params, air, cases = full
    gair = NS.Air(air.to_words())
    stark = NS.Stark.default()
    claim, proof = cases[1]
    items = S.decode_proof(proof, params)
    # locate item payload starts by re-walking the encoding
    pos, starts = 2, []
    for _ in items:
        ln = proof[pos]
        starts.append(pos + 1)
        pos += 1 + ln
    kinds = [k for k, _ in items]
    targets = {
        "ood_main_row": starts[kinds.index(S.OOD_MAIN_ROW)] + 1 + 3 * 17,
        "ood_quot": starts[kinds.index(S.OOD_QUOT_SEGMENTS)] + 1 + 2,
        "fri_last_codeword": starts[kinds.index(S.FRI_CODEWORD)] + 3 + 5,
        "fri_response_leaf": starts[kinds.index(S.FRI_RESPONSE)] + 4 + 7,
        "main_row_value": starts[kinds.index(S.MAIN_ROWS)] + 3 + 100,
        "aux_row_value": starts[kinds.index(S.AUX_ROWS)] + 3 + 50,
        "quot_row_value": starts[kinds.index(S.QUOT_SEGMENTS_ELEMENTS)] + 3 + 4,
        "main_auth_digest": starts[kinds.index(S.AUTH_STRUCTURE)] + 3 + 2,
        "fri_root": starts[[i for i, k in enumerate(kinds) if k == S.MERKLE_ROOT][3]] + 1,
    }
    muts = []
    for name, p in targets.items():
        m = list(proof)
        m[p] = (m[p] + 12345) % S.P
        muts.append(m)
    got = NS.verify_batch(ctx, gair, stark, [(NS.Claim(*claim), m) for m in muts] + [(NS.Claim(*claim), proof)])
    assert got == [False] * len(muts) + [True], dict(zip(list(targets) + ["clean"], got))
    for m in muts[:3]:
        assert S.verify(params, air, claim, m) is False


def test_bench_pool_heights_9_to_16_match_oracle(ctx):
    """The BASELINE config-3 proof pool (log2 padded heights 9..12 and 16, Stark::default()):
    GPU verdicts and full Fiat-Shamir transcripts equal the oracle's; a flipped MainRows word in
    each rejects on both."""
    import json as _json
    T.use_c_backend()
    NS = _ns()
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_pool.npz"))
    meta = _json.loads(bytes(z["meta"]).decode())
    air_w = [int(w) for w in z["air"]]
    air = S.AirCircuit.from_words(air_w)
    params = S.StarkParams()
    gair = NS.Air(air_w)
    cases, bad = [], []
    for h in meta["heights"]:
        c = meta["claims"][str(h)]
        claim = (c["digest"], c["version"], c["input"], c["output"])
        proof = [int(w) for w in z[f"proof_{h}"]]
        cases.append((claim, proof))
        lo, hi = meta["main_rows"][str(h)]
        m = list(proof)
        m[(lo + hi) // 2] = (m[(lo + hi) // 2] + 1) % S.P
        bad.append((claim, m))
    b = NS.Batch(ctx, gair, NS.Stark.default(), [NS.Claim(*c) for c, _ in cases + bad], [p for _, p in cases + bad])
    v, ok = b.run()
    assert list(v) == [1] * len(cases) + [0] * len(bad) and not ok
    for i, (claim, proof) in enumerate(cases):
        ok_o, samples, indices = _oracle_samples(params, air, claim, proof)
        assert ok_o
        xs, idx, fail = b.transcript(i)
        assert fail == 0 and xs == samples and idx == indices
    for claim, m in bad[:2]:
        assert S.verify(params, air, claim, m) is False
    b.close()


def _pool():
    import json as _json
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_pool.npz"))
    meta = _json.loads(bytes(z["meta"]).decode())
    out = []
    for h in meta["heights"]:
        c = meta["claims"][str(h)]
        out.append(((c["digest"], c["version"], c["input"], c["output"]), z[f"proof_{h}"], meta["main_rows"][str(h)]))
    return z["air"], out


def test_full_size_random_mutations_vs_c_oracle(ctx):
    """Stark::default()-sized proofs (heights 9..16) with one random word changed anywhere in the
    proof (count fields, discriminants, roots, auth structures, FRI data, rows) or the claim
    changed: every GPU verdict equals the C restatement's (oracle/stark_oracle.c)."""
    import coracle as C
    NS = _ns()
    air_w, pool = _pool()
    params = S.StarkParams()
    rng = np.random.default_rng(0xDEE9)
    claims, proofs = [], []
    for claim, proof, _ in pool:
        claims.append(claim)
        proofs.append(proof)
        for _ in range(48):
            m = proof.copy()
            pos = int(rng.integers(0, m.size))
            r = int(rng.integers(0, 3))
            m[pos] = np.uint64((int(m[pos]) + 1) % S.P) if r == 0 else (
                np.uint64(int(rng.integers(0, 1 << 62))) if r == 1 else np.uint64(0))
            claims.append(claim)
            proofs.append(m)
        cl = list(claim)
        cl[2] = list(cl[2]) + [int(rng.integers(0, 1 << 40))]
        claims.append(tuple(cl))
        proofs.append(proof)
    got = NS.verify_batch(ctx, NS.Air([int(w) for w in air_w]), NS.Stark.default(),
                          [(NS.Claim(*c), p) for c, p in zip(claims, proofs)])
    want = [bool(x) for x in C.stark_verify_batch(air_w, params, claims, proofs, threads=16)]
    assert got == want
    assert sum(want) >= len(pool)  # the clean proofs accept (a mutation may hit an unused word)


def test_async_launch_wait_matches_run(ctx):
    """nhip_batch_launch / nhip_batch_wait on two batches in flight at once == nhip_batch_run."""
    NS = _ns()
    air_w, pool = _pool()
    gair = NS.Air([int(w) for w in air_w])
    stark = NS.Stark.default()
    claims = [NS.Claim(*c) for c, _, _ in pool]
    bad = []
    for _, p, (lo, hi) in pool:
        m = p.copy()
        m[(lo + hi) // 2] = np.uint64((int(m[(lo + hi) // 2]) + 7) % S.P)
        bad.append(m)
    b1 = NS.Batch(ctx, gair, stark, claims, [p for _, p, _ in pool])
    b2 = NS.Batch(ctx, gair, stark, claims, bad)
    b1.launch()
    b2.launch()
    v2, ok2 = b2.wait()
    v1, ok1 = b1.wait()
    assert list(v1) == [1] * len(pool) and ok1
    assert list(v2) == [0] * len(pool) and not ok2
    r1, _ = b1.run()
    assert list(r1) == list(v1)
    b1.close()
    b2.close()


def test_launch_timing_switch(ctx):
    """Per-dispatch timestamps are off by default (the product path: exec times read 0) and on after
    nhip_batch_set_launch_timing (the bench's kernel timing); the verdicts are the same either way,
    and the switch is refused while the batch is in flight."""
    NS = _ns()
    air_w, pool = _pool()
    gair = NS.Air([int(w) for w in air_w])
    b = NS.Batch(ctx, gair, NS.Stark.default(), [NS.Claim(*c) for c, _, _ in pool], [p for _, p, _ in pool])
    v0, ok0 = b.run()
    s0 = b.stats()
    assert s0["ms_mp_hash_exec"] == 0.0 and s0["ms_row_hash_exec"] == 0.0
    b.set_launch_timing(True)
    v1, ok1 = b.run()
    s1 = b.stats()
    assert s1["ms_mp_hash_exec"] > 0.0 and s1["ms_row_hash_exec"] > 0.0
    assert list(v0) == list(v1) == [1] * len(pool) and ok0 and ok1
    b.launch()
    with pytest.raises(Exception):
        b.set_launch_timing(False)
    v2, _ = b.wait()
    assert list(v2) == list(v1)
    b.set_launch_timing(False)
    b.run()
    assert b.stats()["ms_mp_hash_exec"] == 0.0
    b.close()


def test_one_stream_batches(ctx):
    """nhip_batch_set_streams: every phase on one stream gives the two-stream verdicts and
    Fiat-Shamir transcripts (mutated proofs included), one-stream batches run concurrently, and the
    switch back to two streams and the refusal while in flight hold."""
    NS = _ns()
    air_w, pool = _pool()
    gair = NS.Air([int(w) for w in air_w])
    stark = NS.Stark.default()
    claims = [NS.Claim(*c) for c, _, _ in pool]
    proofs = [p for _, p, _ in pool]
    bad = []
    for _, p, (lo, hi) in pool:
        m = p.copy()
        m[(lo + hi) // 2] = np.uint64((int(m[(lo + hi) // 2]) + 7) % S.P)
        bad.append(m)
    two = NS.Batch(ctx, gair, stark, claims + claims, proofs + bad)
    v2, _ = two.run()
    ones = [NS.Batch(ctx, gair, stark, claims + claims, proofs + bad).set_streams(1) for _ in range(3)]
    for b in ones:
        b.launch()
    with pytest.raises(Exception):
        ones[0].set_streams(2)
    for b in ones:
        v1, _ = b.wait()
        assert list(v1) == list(v2) == [1] * len(pool) + [0] * len(pool)
    for i in range(len(pool)):
        assert ones[1].transcript(i) == two.transcript(i)
    ones[2].set_streams(2)
    v3, _ = ones[2].run()
    assert list(v3) == list(v2)
    for b in ones + [two]:
        b.close()


def test_empty_and_single_malformed_batches(ctx):
    NS = _ns()
    air_w, pool = _pool()
    gair = NS.Air([int(w) for w in air_w])
    assert NS.verify_batch(ctx, gair, NS.Stark.default(), []) == []
    claim = NS.Claim(*pool[0][0])
    assert NS.verify_batch(ctx, gair, NS.Stark.default(), [(claim, [5, 4, 3])]) == [False]


def test_large_padded_heights_config5_shape(ctx):
    """BASELINE config 5 shape: proofs at log2 padded height 20 and 23 (FRI domain 2^23 / 2^26,
    14 / 17 FRI rounds) from the constant-codeword prover: GPU verdicts and every Fiat-Shamir
    sample equal the oracle's; mutated copies reject on both."""
    import stark_prover_const as K
    T.use_c_backend()
    NS = _ns()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    cases, bad = [], []
    for lph in (20, 23):
        claim = ([lph, 9, 9, 9, 9], 0, [lph], [1, 2])
        proof, _ = K.prove(params, air, recipe, claim, lph, seed=lph)
        cases.append((claim, proof))
        for pos in (len(proof) // 3, len(proof) - 7):
            m = list(proof)
            m[pos] = (m[pos] + 1) % S.P
            bad.append((claim, m))
    b = NS.Batch(ctx, NS.Air(air.to_words()), NS.Stark.default(), [NS.Claim(*c) for c, _ in cases + bad],
                 [p for _, p in cases + bad])
    v, _ = b.run()
    want = [S.verify(params, air, c, p) for c, p in cases + bad]
    assert [bool(x) for x in v] == want and want[:2] == [True, True]
    for i, (claim, proof) in enumerate(cases):
        ok_o, samples, indices = _oracle_samples(params, air, claim, proof)
        xs, idx, fail = b.transcript(i)
        assert ok_o and fail == 0 and xs == samples and idx == indices
    b.close()


def test_config1_singleproof_gpu(ctx):
    """BASELINE config 1 substitute: one SingleProof-shaped proof at log2 padded
    height 21 (tests/golden/config1.npz, the sparse synthetic prover: every one of the 15 FRI
    rounds folds non-zero values, last polynomial of degree 122; claim input = a kernel MAST hash
    reversed, output empty) verified through the GPU path: verdict and every Fiat-Shamir sample
    equal the oracle transcript stored with the fixture; a mutated copy, a mutated last-round FRI
    response and the un-reversed claim reject on the GPU as in the C oracle."""
    import json
    import coracle as C
    T.use_c_backend()
    NS = _ns()
    params = S.StarkParams()
    air, _ = S.synth_air(params, seed=1)
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "config1.npz"))
    m = json.loads(bytes(z["meta"]).decode())
    claim = (m["digest"], m["version"], m["input"], m["output"])
    proof = [int(w) for w in z["proof"]]
    samples = [tuple(int(c) for c in x) for x in z["samples"]]
    indices = [int(i) for i in z["indices"]]
    mutated = list(proof)
    mutated[len(proof) // 2] = (mutated[len(proof) // 2] + 1) % S.P
    late_fri = list(proof)
    late_fri[len(proof) - 1000] = (late_fri[len(proof) - 1000] + 1) % S.P
    unreversed = (m["digest"], m["version"], m["kernel_mast_hash"], m["output"])
    cases = [(claim, proof), (claim, mutated), (claim, late_fri), (unreversed, proof)]
    b = NS.Batch(ctx, NS.Air(air.to_words()), NS.Stark.default(), [NS.Claim(*c) for c, _ in cases],
                 [p for _, p in cases])
    v, _ = b.run()
    want = [bool(x) for x in C.stark_verify_batch(air.to_words(), params, [c for c, _ in cases], [p for _, p in cases],
                                                  threads=4)]
    assert [bool(x) for x in v] == want and want[0] and not any(want[1:])
    xs, idx, fail = b.transcript(0)
    assert fail == 0 and xs == samples and idx == indices
    b.close()


def test_batch_refill_and_streaming(ctx):
    """nhip_batch_refill: an idle batch refilled in place with other proofs (smaller, then larger
    than its device allocation) gives the expected verdicts each time; two batches alternating
    launch / refill / wait (the streaming pattern) too."""
    import bench
    NS = _ns()
    air_words, pool = bench.load_pool()
    gair = NS.Air([int(w) for w in air_words])
    sets = [bench.make_batch(pool, c, 0.25, 100 + c) for c in (2, 1, 6, 3, 4)]
    mk = lambda s: ([NS.Claim(*c) for c in s[0]], s[1])  # noqa: E731
    b = NS.Batch(ctx, gair, NS.Stark.default(), *mk(sets[0]))
    for s in sets:
        b.refill(*mk(s))
        v, ok = b.run()
        assert [bool(x) for x in v] == list(s[2]) and ok == bool(s[2].all())
    a2 = NS.Batch(ctx, gair, NS.Stark.default(), *mk(sets[1]))
    got = []
    b.refill(*mk(sets[0]))
    cur, nxt = b, a2
    cur.launch()
    for s in sets[1:]:
        nxt.refill(*mk(s))
        got.append(cur.wait()[0])
        nxt.launch()
        cur, nxt = nxt, cur
    got.append(cur.wait()[0])
    for v, s in zip(got, sets):
        assert [bool(x) for x in v] == list(s[2])
    b.close()
    a2.close()


def test_fs_row_and_pair_forms_agree(ctx):
    """The Fiat-Shamir replay runs on the two-row pair Tip5 below FS_PAIR_MAX_PROOFS (512) proofs
    and on the one-row form from there on: a 520-proof batch (one-row) and an 8-proof batch (pair)
    of the same pool proofs give the same verdicts and the same transcripts (every sample, every
    FRI index) for every pool height."""
    NS = _ns()
    air_w, pool = _pool()
    gair = NS.Air([int(w) for w in air_w])
    stark = NS.Stark.default()
    claims = [NS.Claim(*c) for c, _, _ in pool]
    proofs = [p for _, p, _ in pool]
    reps = 520 // len(pool) + 1
    big = NS.Batch(ctx, gair, stark, claims * reps, proofs * reps)
    small = NS.Batch(ctx, gair, stark, claims, proofs)
    vb, okb = big.run()
    vs, oks = small.run()
    assert okb and oks and all(vb) and all(vs) and len(vb) >= 520
    for i in range(len(pool)):
        tb = big.transcript(len(pool) * (reps - 1) + i)
        ts = small.transcript(i)
        assert tb == ts and tb[2] == 0
    big.close()
    small.close()


def test_merkle_climb_and_level_paths_agree(ctx):
    """Batches of <= 32 proofs hash their Merkle trees with one workgroup per tree (k_mp_climb, FRI
    beside the plan), larger ones level by level over all trees: the same 32 proofs (pool proofs and
    copies with one word changed in their authentication structures, revealed rows, FRI data or
    last codeword) give the same verdicts and transcripts in a 32-proof batch, inside a 48-proof batch
    (per-level launches, the last small levels in one k_mp_hash_tail launch) and inside a 96-proof
    batch."""
    NS = _ns()
    air_w, pool = _pool()
    gair = NS.Air([int(w) for w in air_w])
    stark = NS.Stark.default()
    rng = np.random.default_rng(0xC11B)
    claims, proofs = [], []
    for claim, proof, _ in pool:
        claims.append(NS.Claim(*claim))
        proofs.append(proof)
    while len(proofs) < 32:
        j = int(rng.integers(0, len(pool)))
        m = pool[j][1].copy()
        pos = int(rng.integers(len(m) // 4, len(m)))  # past the roots and OOD rows
        m[pos] = np.uint64((int(m[pos]) + 1) % S.P)
        claims.append(NS.Claim(*pool[j][0]))
        proofs.append(m)
    small = NS.Batch(ctx, gair, stark, claims, proofs)
    mid = NS.Batch(ctx, gair, stark, claims + claims[:16], proofs + proofs[:16])  # levels + one-launch tail
    big = NS.Batch(ctx, gair, stark, claims * 3, proofs * 3)
    vs, _ = small.run()
    vm, _ = mid.run()
    vb, _ = big.run()
    assert list(vb[64:96]) == list(vs) and list(vb[:32]) == list(vs) and list(vm[:32]) == list(vs)
    assert all(vs[:len(pool)]) and not all(vs)
    for i in range(32):
        assert small.transcript(i) == big.transcript(64 + i) == mid.transcript(i), i
    small.close()
    mid.close()
    big.close()
