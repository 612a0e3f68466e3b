"""Python mirror of the triton-air -> AIR-descriptor exporter (rust/neptune-hip/src/air_export.rs).

triton-constraint-circuit 1.0.0 (reference Cargo.lock:4226) represents each AIR constraint as a DAG of
`ConstraintCircuit` nodes whose `expression` is one of BConst, XConst, Input (a main or aux column of
the current or next row), Challenge (a `ChallengeId` index) or BinOp(Add | Mul, lhs, rhs); the
monad's subtraction and negation are built from Add and Mul by -1.  This module models exactly those
node kinds (`Circuit`, with the monad's operators) and maps them to descriptor words the way the Rust
exporter does, so the mapping can be tested here against the oracle's evaluator
(tests/test_air_export.py) — the Rust exporter walks triton-air's real circuits, which are not
available offline.  Any other node kind fails the export.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

P = (1 << 64) - (1 << 32) + 1
AIR_MAGIC = 0x41495231
OP_INPUT, OP_CONST, OP_ADD, OP_SUB, OP_MUL = range(5)
IN_MAIN_CURR, IN_AUX_CURR, IN_MAIN_NEXT, IN_AUX_NEXT, IN_CHALLENGE = range(5)
SAMPLE_COUNT, CHALLENGE_COUNT = 59, 63  # include/nhip_challenge_id.h

# input indicators (triton-constraint-circuit SingleRowIndicator / DualRowIndicator)
SINGLE_MAIN, SINGLE_AUX = "Main", "Aux"
DUAL_CURRENT_MAIN, DUAL_CURRENT_AUX, DUAL_NEXT_MAIN, DUAL_NEXT_AUX = "CurrentMain", "CurrentAux", "NextMain", "NextAux"
_INPUT_KIND = {SINGLE_MAIN: IN_MAIN_CURR, SINGLE_AUX: IN_AUX_CURR, DUAL_CURRENT_MAIN: IN_MAIN_CURR,
               DUAL_CURRENT_AUX: IN_AUX_CURR, DUAL_NEXT_MAIN: IN_MAIN_NEXT, DUAL_NEXT_AUX: IN_AUX_NEXT}


class ExportError(ValueError):
    pass


class Circuit:
    """One ConstraintCircuit node: `kind` in {"BConst", "XConst", "Input", "Challenge", "BinOp"}.
    BConst: value; XConst: (c0, c1, c2); Input: (indicator, column); Challenge: index;
    BinOp: ("Add" | "Mul", lhs, rhs).  Operators build new nodes as the circuit monad does."""

    __slots__ = ("kind", "arg")

    def __init__(self, kind: str, arg):
        self.kind, self.arg = kind, arg

    @staticmethod
    def _lift(x) -> "Circuit":
        return x if isinstance(x, Circuit) else Circuit("BConst", int(x) % P)

    def __add__(self, o):
        return Circuit("BinOp", ("Add", self, Circuit._lift(o)))

    def __radd__(self, o):
        return Circuit("BinOp", ("Add", Circuit._lift(o), self))

    def __mul__(self, o):
        return Circuit("BinOp", ("Mul", self, Circuit._lift(o)))

    def __rmul__(self, o):
        return Circuit("BinOp", ("Mul", Circuit._lift(o), self))

    def __neg__(self):  # the monad: -x = (-1) * x
        return Circuit("BinOp", ("Mul", Circuit("BConst", P - 1), self))

    def __sub__(self, o):  # the monad: a - b = a + (-b)
        return self + (-Circuit._lift(o))

    def __rsub__(self, o):
        return Circuit._lift(o) + (-self)


def bconst(v: int) -> Circuit:
    return Circuit("BConst", int(v) % P)


def xconst(c: Sequence[int]) -> Circuit:
    return Circuit("XConst", tuple(int(x) % P for x in c))


def inp(indicator: str, col: int) -> Circuit:
    return Circuit("Input", (indicator, col))


def challenge(i: int) -> Circuit:
    return Circuit("Challenge", i)


class DescriptorBuilder:
    """One descriptor node per distinct Circuit object (the Rust exporter keys `Rc` addresses),
    operands first (explicit stack: lowered circuits are deep)."""

    def __init__(self, num_main: int, num_aux: int, num_challenges: int = CHALLENGE_COUNT):
        self.num_main, self.num_aux, self.num_challenges = num_main, num_aux, num_challenges
        self.nodes: List[Tuple[int, int, int, int]] = []
        self.memo: Dict[int, int] = {}
        self._keep: List[Circuit] = []  # ids stay unique while the builder lives

    def _leaf(self, c: Circuit) -> Tuple[int, int, int, int]:
        if c.kind == "BConst":
            return (OP_CONST, int(c.arg) % P, 0, 0)
        if c.kind == "XConst":
            return (OP_CONST,) + tuple(int(x) % P for x in c.arg)
        if c.kind == "Input":
            ind, col = c.arg
            if ind not in _INPUT_KIND:
                raise ExportError(f"unknown input indicator {ind!r}")
            kind = _INPUT_KIND[ind]
            lim = self.num_main if kind in (IN_MAIN_CURR, IN_MAIN_NEXT) else self.num_aux
            if not 0 <= col < lim:
                raise ExportError(f"column {col} out of range for {ind}")
            return (OP_INPUT, kind, col, 0)
        if c.kind == "Challenge":
            if not 0 <= c.arg < self.num_challenges:
                raise ExportError(f"challenge index {c.arg}")
            return (OP_INPUT, IN_CHALLENGE, c.arg, 0)
        raise ExportError(f"unknown node kind {c.kind!r}")

    def add(self, root: Circuit) -> int:
        stack = [(root, False)]
        while stack:
            node, expanded = stack.pop()
            if id(node) in self.memo:
                continue
            if node.kind == "BinOp":
                op, a, b = node.arg
                if op not in ("Add", "Mul"):
                    raise ExportError(f"unknown binary operation {op!r}")
                if not expanded:
                    stack += [(node, True), (b, False), (a, False)]
                    continue
                self.nodes.append((OP_ADD if op == "Add" else OP_MUL, self.memo[id(a)], self.memo[id(b)], 0))
            else:
                self.nodes.append(self._leaf(node))
            self.memo[id(node)] = len(self.nodes) - 1
            self._keep.append(node)
        return self.memo[id(root)]

    def finish(self, groups: Sequence[Sequence[int]], num_sampled: int = SAMPLE_COUNT) -> List[int]:
        w = [AIR_MAGIC, self.num_main, self.num_aux, num_sampled, len(self.nodes)] + [len(g) for g in groups]
        for n in self.nodes:
            w += list(n)
        for g in groups:
            w += list(g)
        return w


def export(num_main: int, num_aux: int, init: Sequence[Circuit], cons: Sequence[Circuit],
           trans: Sequence[Circuit], term: Sequence[Circuit]) -> List[int]:
    """Descriptor words of four constraint groups in triton order (initial, consistency,
    transition, terminal), as `air_export::triton_air_descriptor` builds them."""
    b = DescriptorBuilder(num_main, num_aux)
    groups = [[b.add(c) for c in g] for g in (init, cons, trans, term)]
    return b.finish(groups)


def evaluate(c: Circuit, main_curr, aux_curr, main_next, aux_next, challenges, xmul, xadd):
    """Direct evaluation of a circuit (the generated evaluator's semantics), memoised by node."""
    rows = {IN_MAIN_CURR: main_curr, IN_AUX_CURR: aux_curr, IN_MAIN_NEXT: main_next, IN_AUX_NEXT: aux_next}
    memo: Dict[int, tuple] = {}
    stack = [(c, False)]
    while stack:
        n, expanded = stack.pop()
        if id(n) in memo:
            continue
        if n.kind == "BinOp":
            op, a, b = n.arg
            if not expanded:
                stack += [(n, True), (b, False), (a, False)]
                continue
            memo[id(n)] = (xadd if op == "Add" else xmul)(memo[id(a)], memo[id(b)])
        elif n.kind == "BConst":
            memo[id(n)] = (n.arg, 0, 0)
        elif n.kind == "XConst":
            memo[id(n)] = tuple(n.arg)
        elif n.kind == "Input":
            ind, col = n.arg
            memo[id(n)] = rows[_INPUT_KIND[ind]][col]
        else:
            memo[id(n)] = challenges[n.arg]
    return memo[id(c)]
