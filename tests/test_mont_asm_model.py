"""CPU model of the generated gfx950 inline asm in neptune-core_amd/csrc/mont_asm.hpp.

The asm cannot run here, so this test parses the two `asm volatile` statements of every
mont_mulN_asm, executes their instructions on Python integers (per-lane semantics of the gfx9
VOP3 integer ops used) and checks:
  * the result equals twenty-first's montyred(a * b) (the oracle's Montgomery product) for edge
    and random operands;
  * every SGPR carry / mask written by one instruction is read no sooner than 2 instructions
    later (the gfx950 VALU-SGPR-write -> VALU-read wait states that hipcc does not insert inside
    asm), so the string needs no s_nop.
"""
import os
import random
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "neptune-core_amd", "csrc", "mont_asm.hpp")
M32 = (1 << 32) - 1
M64 = (1 << 64) - 1
P = (1 << 64) - (1 << 32) + 1
EPS = M32


def montyred(x):
    """twenty-first BFieldElement::montyred (oracle/tip5_oracle.c mont_reduce)."""
    xl, xh = x & M64, x >> 64
    a = (xl + (xl << 32)) & M64
    e = 1 if a < xl else 0
    b = (a - (a >> 32) - e) & M64
    r = (xh - b) & M64
    return (r - EPS) & M64 if xh < b else r


def _parse():
    src = open(HDR).read()
    fns = {}
    for m in re.finditer(r"void mont_mul(\d+)_asm\(.*?\n}\n", src, re.S):
        n = int(m.group(1))
        stmts = []
        for a in re.finditer(r'asm(?: volatile)?\("(.*?)"\s*:(.*?):(.*?)\);', m.group(0), re.S):
            lines = a.group(1).split("\\n\\t")
            ops = [(c, name, int(i)) for c, name, i in
                   re.findall(r'"([=&+]*[vs])"\((\w+)\[(\d+)\]\)', a.group(2) + "," + a.group(3))]
            stmts.append((lines, ops))
        fns[n] = stmts
    return fns


def _val(tok, regs):
    tok = tok.strip()
    if tok.startswith("%"):
        return regs[int(tok[1:])]
    v = int(tok, 0)
    return v & M32 if v < 0 else v


def _run(lines, regs, width):
    """Execute one statement; regs: operand index -> value; width: operand index -> bits."""
    written = {}
    for pc, line in enumerate(lines):
        op, rest = line.split(None, 1)
        args = [t.strip() for t in rest.split(",")]
        idx = lambda t: int(t[1:])
        # hazard check on SGPR reads (carry-in / mask operands)
        reads = []
        if op in ("v_addc_co_u32_e64", "v_subb_co_u32_e64", "v_cndmask_b32_e64"):
            reads.append(args[-1])
        for t in reads:
            if t.startswith("%") and idx(t) in written:
                assert pc - written[idx(t)] >= 3, f"SGPR {t} read {pc - written[idx(t)]} after write: {line}"
        if op == "v_mad_u64_u32":
            r = _val(args[2], regs) * _val(args[3], regs) + _val(args[4], regs)
            regs[idx(args[0])] = r & M64
            regs[idx(args[1])] = r >> 64
            written[idx(args[1])] = pc
        elif op == "v_cndmask_b32_e64":
            regs[idx(args[0])] = _val(args[2], regs) if regs[idx(args[3])] else _val(args[1], regs)
        elif op in ("v_add_co_u32_e64", "v_addc_co_u32_e64"):
            cin = regs[idx(args[4])] if op == "v_addc_co_u32_e64" else 0
            r = _val(args[2], regs) + _val(args[3], regs) + cin
            regs[idx(args[0])] = r & M32
            regs[idx(args[1])] = r >> 32
            written[idx(args[1])] = pc
        elif op in ("v_sub_co_u32_e64", "v_subb_co_u32_e64"):
            cin = regs[idx(args[4])] if op == "v_subb_co_u32_e64" else 0
            r = _val(args[2], regs) - _val(args[3], regs) - cin
            regs[idx(args[0])] = r & M32
            regs[idx(args[1])] = 1 if r < 0 else 0
            written[idx(args[1])] = pc
        else:
            raise AssertionError(f"unmodelled instruction {op}")
        for k, w in width.items():
            assert regs.get(k, 0) < (1 << w) or k not in regs, (line, k)


def _model(stmts, n, a, b):
    (la, oa), (lb, ob) = stmts
    env = {"a0": [x & M32 for x in a], "a1": [x >> 32 for x in a],
           "b0": [x & M32 for x in b], "b1": [x >> 32 for x in b]}
    wide = {"P", "U", "V", "cy"}
    # stage A
    regs = {k: env[name][i] for k, (_, name, i) in enumerate(oa) if name in env}
    width = {k: (64 if name in wide else 32) for k, (_, name, i) in enumerate(oa)}
    _run(la, regs, width)
    for k, (c, name, i) in enumerate(oa):
        if "=" in c:
            env.setdefault(name, [0] * n)[int(i)] = regs[k]
    env["p0"] = [x & M32 for x in env["P"]]
    env["p1"] = [x >> 32 for x in env["P"]]
    env["u0"] = [x & M32 for x in env["U"]]
    env["u1"] = [x >> 32 for x in env["U"]]
    env["v0"] = [x & M32 for x in env["V"]]
    env["v1"] = [x >> 32 for x in env["V"]]
    # stage B
    regs = {}
    for k, (c, name, i) in enumerate(ob):
        if "+" in c or "=" not in c:
            regs[k] = env[name][int(i)]
    width = {k: (64 if name == "cy" else 32) for k, (_, name, i) in enumerate(ob)}
    _run(lb, regs, width)
    out = {}
    for k, (c, name, i) in enumerate(ob):
        if name in ("rl", "rh"):
            out.setdefault(name, [0] * n)[int(i)] = regs[k]
    return [(h << 32) | l for l, h in zip(out["rl"], out["rh"])]


def test_generated_header_is_current():
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen", os.path.join(ROOT, "tools", "gen_mont_asm.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    assert open(HDR).read() == gen.gen(gen.N_LIST), "re-run tools/gen_mont_asm.py"


@pytest.mark.parametrize("n", [3, 4, 6])
def test_mont_asm_matches_montyred(n):
    fns = _parse()
    assert n in fns and len(fns[n]) == 2
    rng = random.Random(n)
    edge = [0, 1, 2, P - 1, P - 2, M32, 1 << 32, 1 << 63, M64, P, P + 5, EPS << 32]
    pairs = [(x, y) for x in edge for y in edge] + [(rng.getrandbits(64), rng.getrandbits(64)) for _ in range(3000)]
    for k in range(0, len(pairs), n):
        chunk = pairs[k:k + n]
        chunk += [(1, 1)] * (n - len(chunk))
        a = [x for x, _ in chunk]
        b = [y for _, y in chunk]
        got = _model(fns[n], n, a, b)
        assert got == [montyred(x * y) for x, y in chunk], (a, b)
