"""The three device forms of the Fiat-Shamir sponge replay (k_fs_replay_wide's 16-lane row and
two-row pair, k_fs_replay_quad's four lanes per proof) on the same proofs: the 256 distinct config-4
pool proofs (oracle/pool4.py, each with its oracle transcript) plus mutants whose absorbed items
change (an OOD row word, an authentication word, the last polynomial).  nhip_set_fs_form forces the
form for the run; every verdict, every squeezed sample and every
sampled index must equal the oracle's whatever the form and the batch size (reference: the sponge
of triton-vm's ProofStream; the forms are bit-identical restatements of one
Tip5 permutation, tip5_device.hpp)."""
import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pool():
    return bench.load_pool4()


FORMS = {"row": 0, "pair": 1, "quad": 2}


@pytest.fixture
def forced_form():
    import neptune_hip.stark as NS
    yield NS.set_fs_form
    NS.set_fs_form(-1)  # back to the batch-size rule


def _run(ctx, pool, sel, mutate, set_form, form):
    import neptune_hip.stark as NS
    set_form(FORMS[form])
    gair = NS.Air([int(w) for w in pool["air"]])
    proofs = [np.array(pool["proofs"][j], dtype=np.uint64) for j in sel]
    for i, (pos, delta) in mutate.items():
        proofs[i] = proofs[i].copy()
        proofs[i][pos] = np.uint64((int(proofs[i][pos]) + delta) % (1 << 64))
    b = NS.Batch(ctx, gair, NS.Stark.default(), [NS.Claim(*pool["claims"][j]) for j in sel], proofs)
    v, ok = b.run()
    tr = [b.transcript(i) for i in range(len(sel))]
    b.close()
    return [bool(x) for x in v], tr


@pytest.mark.parametrize("form", ["quad", "row", "pair"])
@pytest.mark.parametrize("n", [256, 1024])
def test_fs_form_transcripts(ctx, pool, forced_form, form, n):
    sel = [j % 256 for j in range(n)]
    # mutants: a word inside the proof body (absorbed by the sponge, so every later sample moves)
    rng = np.random.default_rng(0xF5 + n)
    mutate = {}
    for i in rng.choice(n, size=8, replace=False).tolist():
        L = len(pool["proofs"][sel[i]])
        mutate[int(i)] = (int(rng.integers(L // 4, L - 8)), 1)
    v, tr = _run(ctx, pool, sel, mutate, forced_form, form)
    for i in range(n):
        want_xs, want_idx = pool["transcripts"][sel[i]]
        xs, idx, fail = tr[i]
        if i not in mutate:  # (mutants: test_fs_forms_agree_on_mutants)
            assert v[i] and fail == 0 and xs == want_xs and idx == want_idx, (form, n, i)


def test_fs_forms_agree_on_mutants(ctx, pool, forced_form):
    """Rejected proofs still replay their whole sponge: the samples of mutated proofs are equal
    across the forms (the oracle transcript of a mutant is not stored, so the forms are held to each
    other, and the row form to the oracle on every accepting proof above)."""
    n = 512
    sel = [(7 * j) % 256 for j in range(n)]
    rng = np.random.default_rng(0xF6)
    mutate = {}
    for i in rng.choice(n, size=32, replace=False).tolist():
        L = len(pool["proofs"][sel[i]])
        mutate[int(i)] = (int(rng.integers(16, L - 8)), int(rng.integers(1, 1 << 63)))
    runs = {f: _run(ctx, pool, sel, mutate, forced_form, f) for f in ("row", "pair", "quad")}
    for f in ("pair", "quad"):
        assert runs[f][0] == runs["row"][0], f
        for i in range(n):
            a, b = runs[f][1][i], runs["row"][1][i]
            assert a[2] == b[2], (f, i)
            if a[2] == 0 or i in mutate:
                assert a[0] == b[0] and a[1] == b[1], (f, i)
