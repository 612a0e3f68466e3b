"""The triton-air -> AIR-descriptor mapping (rust/neptune-hip/src/air_export.rs, mirrored in
neptune_hip.air_export): hand-built constraint circuits of triton-constraint-circuit's node kinds
(BConst, XConst, Input of both indicator types, Challenge by ChallengeId, Add, Mul; subtraction and
negation as the monad builds them) are exported to descriptor words; the oracle's evaluator
(stark_ref.AirCircuit) on those words gives the same constraint values as evaluating the circuits
directly; shared sub-circuits become one node; the library accepts the descriptor; unknown node
kinds fail the export.  CPU only."""
import numpy as np
import pytest

import stark_ref as S
from field_ref import P, xadd, xmul
from neptune_hip import air_export as E

CH = S.CHALLENGE_ID


def _tables(num_main=12, num_aux=5):
    """A miniature of triton-air's constraint shapes: processor-style initial / consistency /
    transition constraints, running-evaluation and lookup-argument aux columns over named
    challenges, and terminal constraints against the derived challenges of Challenges::new."""
    m = lambda i: E.inp(E.SINGLE_MAIN, i)  # noqa: E731
    a = lambda i: E.inp(E.SINGLE_AUX, i)  # noqa: E731
    cm = lambda i: E.inp(E.DUAL_CURRENT_MAIN, i)  # noqa: E731
    nm = lambda i: E.inp(E.DUAL_NEXT_MAIN, i)  # noqa: E731
    ca = lambda i: E.inp(E.DUAL_CURRENT_AUX, i)  # noqa: E731
    na = lambda i: E.inp(E.DUAL_NEXT_AUX, i)  # noqa: E731
    ch = lambda name: E.challenge(CH[name])  # noqa: E731
    one = E.bconst(1)
    init = [
        m(0),                                                    # clk = 0
        m(1) - 1,                                                # ip = 1 (a BConst operand)
        a(0) - one,                                              # running evaluation starts at 1
        a(1) - (ch("InstructionLookupIndeterminate") - m(2) * ch("ProgramAddressWeight")
                - m(3) * ch("ProgramInstructionWeight")),
    ]
    is_bit = m(4) * (m(4) - 1)                                   # shared below
    cons = [is_bit, is_bit * m(5) + E.xconst((3, 1, 4)) * m(6), -m(7) + m(8) * m(9)]
    step = nm(0) - cm(0) - one
    trans = [
        step,
        step * nm(4),                                            # a sub-circuit reused across constraints
        na(0) - ca(0) * ch("StandardInputIndeterminate") - nm(10),
        na(2) - ca(2) * ch("HashCascadeLookupIndeterminate") + nm(11) * ch("LookupTablePublicIndeterminate"),
        (nm(7) - cm(7)) * (nm(7) - cm(7) - E.xconst((P - 1, 0, 0))),
    ]
    term = [
        a(0) - ch("StandardInputTerminal"),
        a(3) - ch("StandardOutputTerminal"),
        a(4) - ch("LookupTablePublicTerminal") * ch("CompressedProgramDigest"),
    ]
    return num_main, num_aux, init, cons, trans, term


def _rand_rows(rng, num_main, num_aux):
    def x():
        return tuple(int(v) for v in rng.integers(0, P, size=3, dtype=np.uint64))
    return ([x() for _ in range(num_main)], [x() for _ in range(num_aux)], [x() for _ in range(num_main)],
            [x() for _ in range(num_aux)], [x() for _ in range(E.CHALLENGE_COUNT)])


def test_export_round_trip_equals_direct_evaluation():
    M, A, init, cons, trans, term = _tables()
    words = E.export(M, A, init, cons, trans, term)
    air = S.AirCircuit.from_words(words)
    assert (air.num_main, air.num_aux, air.num_sampled) == (M, A, S.CHALLENGE_SAMPLE_COUNT)
    assert [len(g) for g in air.constraints] == [len(init), len(cons), len(trans), len(term)]
    rng = np.random.default_rng(0xA1)
    for _ in range(5):
        mc, ac, mn, an, chal = _rand_rows(rng, M, A)
        got = air.evaluate(mc, ac, mn, an, chal)
        want = [[E.evaluate(c, mc, ac, mn, an, chal, xmul, xadd) for c in g] for g in (init, cons, trans, term)]
        assert got == want


def test_shared_subcircuits_are_one_node_and_every_node_is_distinct():
    M, A, init, cons, trans, term = _tables()
    words = E.export(M, A, init, cons, trans, term)
    n_nodes = words[4]
    seen, stack = {}, [c for g in (init, cons, trans, term) for c in g]
    while stack:  # distinct Circuit objects reachable from the constraints
        c = stack.pop()
        if id(c) in seen:
            continue
        seen[id(c)] = c
        if c.kind == "BinOp":
            stack += [c.arg[1], c.arg[2]]
    assert n_nodes == len(seen)
    nodes = [tuple(words[9 + 4 * i:13 + 4 * i]) for i in range(n_nodes)]
    for i, (op, x, y, _) in enumerate(nodes):  # operands precede their users
        if op in (E.OP_ADD, E.OP_MUL):
            assert x < i and y < i
    # only the descriptor kinds the exporter emits
    assert {op for op, *_ in nodes} <= {E.OP_INPUT, E.OP_CONST, E.OP_ADD, E.OP_MUL}


def test_challenges_keep_their_challenge_id_index():
    M, A, *_ = _tables()
    words = E.export(M, A, [E.challenge(CH["LookupTablePublicIndeterminate"])], [],
                     [], [E.challenge(CH["CompressedProgramDigest"])])
    nodes = [tuple(words[9 + 4 * i:13 + 4 * i]) for i in range(words[4])]
    assert nodes == [(E.OP_INPUT, E.IN_CHALLENGE, 54, 0), (E.OP_INPUT, E.IN_CHALLENGE, 62, 0)]


def test_library_accepts_the_exported_descriptor():
    import neptune_hip.stark as NS
    M, A, init, cons, trans, term = _tables()
    NS.Air(E.export(M, A, init, cons, trans, term))


def test_unknown_nodes_and_bad_indices_fail_the_export():
    M, A, *_ = _tables()
    for bad in (E.Circuit("Neg", E.bconst(1)),                       # not a triton node kind
                E.Circuit("BinOp", ("Sub", E.bconst(1), E.bconst(2))),  # the circuit has no Sub op
                E.inp("PreviousMain", 0),                            # no such indicator
                E.inp(E.SINGLE_MAIN, M), E.inp(E.DUAL_NEXT_AUX, A),  # columns out of range
                E.challenge(63)):                                     # past ChallengeId
        with pytest.raises(E.ExportError):
            E.export(M, A, [bad + 1], [], [], [])
