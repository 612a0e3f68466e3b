"""The OOD program compiler (stark_host.cpp air_compile, nhip_air_program) on the host, no GPU: the
step schedule is a valid parallel program and computes every constraint.  Within one step the
instructions run concurrently on k_ood_air's threads, so a step may not read a slot another
instruction of the same step writes, nor write a slot twice; values come from earlier steps only.
Interpreting the program step by step under exactly those rules (reads see the state before the
step) on random inputs gives, for every constraint, the value of the oracle's circuit evaluation
(stark_ref.AirCircuit.evaluate), for the synthetic AIR, its triton-air-sized bloat and several step
widths, with every slot in LDS or with the LDS part capped; each constraint ends in its own slot
among the top C, where the kernel weighs it into the quotient sum."""
import numpy as np
import pytest

import bench
import stark_ref as S

OOD_ADD, OOD_SUB, OOD_MUL, OOD_LOAD, OOD_ACC = 2, 3, 4, 5, 6
REF_SLOT, REF_CONST, REF_INPUT = 0, 1, 2


@pytest.fixture(scope="module")
def airs():
    a, _ = bench.load_pool()
    syn = S.AirCircuit.from_words([int(x) for x in a])
    return {"synthetic": syn, "triton-size": S.bloat_air(syn, 24000)}


def _run_program(off, ins, consts, inputs, n_cons, n_slots):
    state, got = {}, {}
    for st in range(len(off) - 1):
        step = ins[off[st]:off[st + 1]]
        reads, writes = set(), set()

        def val(ref):
            t = ref >> 30
            if t == REF_SLOT:
                reads.add(ref)
                return state[ref]
            if t == REF_CONST:
                return consts[ref & 0x3FFFFFFF]
            return inputs[((ref >> 27) & 7, ref & 0x7FFFFFF)]

        out = {}
        for op, a, b, dst in (tuple(int(v) for v in row) for row in step):
            if op == OOD_ACC:  # the constraint's value into its own slot, the top n_cons
                assert b not in got, f"constraint {b} copied twice"
                assert dst == n_slots - n_cons + b, (dst, b)
                got[b] = v = val(a)
            elif op == OOD_LOAD:
                v = val(a)
            else:
                x, y = val(a), val(b)
                v = S.xadd(x, y) if op == OOD_ADD else (S.xsub(x, y) if op == OOD_SUB else S.xmul(x, y))
            assert dst not in writes, f"step {st}: slot {dst} written twice"
            writes.add(dst)
            out[dst] = v
        assert not (reads & writes), f"step {st}: slots read and written in one step: {sorted(reads & writes)[:5]}"
        state.update(out)
    assert sorted(got) == list(range(n_cons))
    # the kernel reads the constraints from their slots after the last step
    assert all(state[n_slots - n_cons + c] == got[c] for c in range(n_cons))
    return [got[c] for c in range(n_cons)]


@pytest.mark.parametrize("name,width,lds_cap,budget", [("synthetic", None, None, None),
                                                        ("triton-size", None, None, None),
                                                        ("triton-size", 256, None, None),
                                                        ("triton-size", 1024, None, None),
                                                        ("triton-size", 512, 600, None),
                                                        ("triton-size", 512, None, 1200)])
def test_compiled_program_is_a_race_free_schedule_of_the_circuit(airs, name, width, lds_cap, budget):
    import neptune_hip.stark as NS
    air = airs[name]
    # budget: a tight working-slot budget (nodes wait unless they retire a value)
    g = NS.Air(air.to_words(), lds_slots=lds_cap or 0, step_width=width or 0, slot_budget=budget or 0)
    info = g.info()
    off, ins = g.program()
    steps = len(off) - 1
    slots = 1 + max(int(r[3]) for r in ins)
    assert slots == info["lds_slots"] + info["global_slots"]
    if lds_cap:
        assert info["lds_slots"] == lds_cap
    else:
        assert info["global_slots"] == 0
    per_step = np.diff(off.astype(np.int64))
    assert per_step.max() <= (width or 512)  # nodes per step + that step's constraint copies
    rng = np.random.default_rng(0x00D)
    rnd = lambda: tuple(int(v) for v in rng.integers(0, S.P, size=3, dtype=np.uint64))
    kinds = {S.INPUT_MAIN_CURR: air.num_main, S.INPUT_AUX_CURR: air.num_aux, S.INPUT_MAIN_NEXT: air.num_main,
             S.INPUT_AUX_NEXT: air.num_aux, S.INPUT_CHALLENGE: air.num_challenges}
    vals = {k: [rnd() for _ in range(n)] for k, n in kinds.items()}
    inputs = {(k, i): v for k, vs in vals.items() for i, v in enumerate(vs)}
    # the constant table in node order (air_compile appends each live constant once, in node order)
    consts = [(a, b, c) for op, a, b, c in air.nodes if op == S.OP_CONST]
    want = [v for cs in air.evaluate(vals[S.INPUT_MAIN_CURR], vals[S.INPUT_AUX_CURR], vals[S.INPUT_MAIN_NEXT],
                                     vals[S.INPUT_AUX_NEXT], vals[S.INPUT_CHALLENGE]) for v in cs]
    live_consts = _live_consts(air)
    got = _run_program(off, ins, [consts[i] for i in live_consts], inputs, air.num_constraints, slots)
    assert got == want
    print(f"{name} width {width or 512}: {steps} steps, {info['lds_slots']} LDS + {info['global_slots']} "
          f"global slots, {len(ins)} instructions")


def _live_consts(air):
    """Indices (among CONST nodes, in node order) of the constants the constraints reach: the
    compiler's table holds exactly those, in node order."""
    reach = set()
    st = [c for cs in air.constraints for c in cs]
    while st:
        i = st.pop()
        if i in reach:
            continue
        reach.add(i)
        op, a, b, _ = air.nodes[i]
        if op in (S.OP_ADD, S.OP_SUB, S.OP_MUL):
            st += [a, b]
    out, k = [], 0
    for i, (op, *_) in enumerate(air.nodes):
        if op == S.OP_CONST:
            if i in reach:
                out.append(k)
            k += 1
    return out
