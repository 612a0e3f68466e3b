#!/usr/bin/env python3
"""Generate neptune-core_amd/csrc/mont_asm.hpp: N-way interleaved Montgomery products in gfx950
inline asm (used by Tip5's x^7 S-box).

Why asm: the 128-bit product a * b needs the carry-out of `v_mad_u64_u32`, which hipcc never
uses; without it every partial product is zero-extended with a `v_mov` (4 per product) and the
carries of interleaved chains are parked in VGPRs with `v_cndmask`.  The asm form is 16 VALU
instructions per product (4 mad + 1 cndmask + 11 add/sub with carry) against ~20.

Two statements per group of N products (hipcc cannot name the halves of a 64-bit asm operand, so
the 64-bit mad results leave stage A as C values whose 32-bit halves feed stage B for free):

  stage A  P = a0*b0;  U = a0*b1;  U = a1*b0 + U -> carry cu;  cuv = cu ? 1 : 0;  V = a1*b1
  stage B  x1 = P1 + U0;  x2 = V0 + U1 + c;  x3 = V1 + cuv + c        (x = a*b, 128 bits)
           twenty-first `montyred(x)`:
           ah = x1 + x0 -> e;  bl = x0 - ah - e;  bh = ah - borrow;
           rl = x2 - bl -> c1;  rh = x3 - bh - c1 -> c;  m = c ? 0xFFFFFFFF : 0;
           rl = rl - m -> c2;  rh = rh - c2

Hazards: a VALU carry-out (SGPR) read by a later VALU as carry-in / mask needs 2 wait states on
gfx950; hipcc does not pad inside asm.  Round-robin interleaving of N >= 3 independent products
puts N - 1 >= 2 instructions between every producer and its consumer, so no s_nop is needed.
The arithmetic is checked instruction-for-instruction by tests/test_mont_asm_model.py.
"""
import sys

N_LIST = (3, 4, 6)


def stage_a(n):
    # operands: outputs P[i] (0..n-1), U[i] (n..2n-1), V[i] (2n..3n-1), cuv[i] (3n..4n-1), C[i] (4n..5n-1)
    # inputs a0[i] (5n..), a1[i] (6n..), b0[i] (7n..), b1[i] (8n..)
    P = lambda i: f"%{i}"
    U = lambda i: f"%{n + i}"
    V = lambda i: f"%{2 * n + i}"
    CU = lambda i: f"%{3 * n + i}"
    C = lambda i: f"%{4 * n + i}"
    A0 = lambda i: f"%{5 * n + i}"
    A1 = lambda i: f"%{6 * n + i}"
    B0 = lambda i: f"%{7 * n + i}"
    B1 = lambda i: f"%{8 * n + i}"
    steps = [
        lambda i: f"v_mad_u64_u32 {P(i)}, {C(i)}, {A0(i)}, {B0(i)}, 0",
        lambda i: f"v_mad_u64_u32 {U(i)}, {C(i)}, {A0(i)}, {B1(i)}, 0",
        lambda i: f"v_mad_u64_u32 {U(i)}, {C(i)}, {A1(i)}, {B0(i)}, {U(i)}",
        lambda i: f"v_cndmask_b32_e64 {CU(i)}, 0, 1, {C(i)}",
        lambda i: f"v_mad_u64_u32 {V(i)}, {C(i)}, {A1(i)}, {B1(i)}, 0",
    ]
    lines = [s(i) for s in steps for i in range(n)]
    outs = [f'"=&v"(P[{i}])' for i in range(n)] + [f'"=&v"(U[{i}])' for i in range(n)] + \
           [f'"=&v"(V[{i}])' for i in range(n)] + [f'"=&v"(cuv[{i}])' for i in range(n)] + \
           [f'"=&s"(cy[{i}])' for i in range(n)]
    ins = [f'"v"(a0[{i}])' for i in range(n)] + [f'"v"(a1[{i}])' for i in range(n)] + \
          [f'"v"(b0[{i}])' for i in range(n)] + [f'"v"(b1[{i}])' for i in range(n)]
    return lines, outs, ins


def stage_b(n):
    # in/out: p0 (0..), p1 (n..), v0 (2n..), v1 (3n..); outputs rl (4n..), rh (5n..), C (6n..)
    # inputs u0 (7n..), u1 (8n..), cuv (9n..)
    p0 = lambda i: f"%{i}"
    p1 = lambda i: f"%{n + i}"
    v0 = lambda i: f"%{2 * n + i}"
    v1 = lambda i: f"%{3 * n + i}"
    rl = lambda i: f"%{4 * n + i}"
    rh = lambda i: f"%{5 * n + i}"
    C = lambda i: f"%{6 * n + i}"
    u0 = lambda i: f"%{7 * n + i}"
    u1 = lambda i: f"%{8 * n + i}"
    cu = lambda i: f"%{9 * n + i}"
    steps = [
        lambda i: f"v_add_co_u32_e64 {p1(i)}, {C(i)}, {p1(i)}, {u0(i)}",            # x1
        lambda i: f"v_addc_co_u32_e64 {v0(i)}, {C(i)}, {v0(i)}, {u1(i)}, {C(i)}",   # x2
        lambda i: f"v_addc_co_u32_e64 {v1(i)}, {C(i)}, {v1(i)}, {cu(i)}, {C(i)}",   # x3
        lambda i: f"v_add_co_u32_e64 {p1(i)}, {C(i)}, {p1(i)}, {p0(i)}",            # ah, e
        lambda i: f"v_subb_co_u32_e64 {p0(i)}, {C(i)}, {p0(i)}, {p1(i)}, {C(i)}",   # bl
        lambda i: f"v_subb_co_u32_e64 {p1(i)}, {C(i)}, {p1(i)}, 0, {C(i)}",         # bh
        lambda i: f"v_sub_co_u32_e64 {rl(i)}, {C(i)}, {v0(i)}, {p0(i)}",            # rl, c1
        lambda i: f"v_subb_co_u32_e64 {rh(i)}, {C(i)}, {v1(i)}, {p1(i)}, {C(i)}",   # rh, c
        lambda i: f"v_cndmask_b32_e64 {p0(i)}, 0, -1, {C(i)}",                      # m
        lambda i: f"v_sub_co_u32_e64 {rl(i)}, {C(i)}, {rl(i)}, {p0(i)}",            # rl - m, c2
        lambda i: f"v_subb_co_u32_e64 {rh(i)}, {C(i)}, {rh(i)}, 0, {C(i)}",         # rh - c2
    ]
    lines = [s(i) for s in steps for i in range(n)]
    outs = [f'"+v"(p0[{i}])' for i in range(n)] + [f'"+v"(p1[{i}])' for i in range(n)] + \
           [f'"+v"(v0[{i}])' for i in range(n)] + [f'"+v"(v1[{i}])' for i in range(n)] + \
           [f'"=&v"(rl[{i}])' for i in range(n)] + [f'"=&v"(rh[{i}])' for i in range(n)] + \
           [f'"=&s"(cy[{i}])' for i in range(n)]
    ins = [f'"v"(u0[{i}])' for i in range(n)] + [f'"v"(u1[{i}])' for i in range(n)] + \
          [f'"v"(cuv[{i}])' for i in range(n)]
    return lines, outs, ins


def asm_stmt(lines, outs, ins, indent="    "):
    body = "\\n\\t".join(lines)
    return (f'{indent}asm("{body}"\n{indent}             : ' + ", ".join(outs) +
            f'\n{indent}             : ' + ", ".join(ins) + ");\n")


def gen_fn(n):
    la, oa, ia = stage_a(n)
    lb, ob, ib = stage_b(n)
    return f"""// out[i] = montyred(a[i] * b[i]) for i < {n}: bit-identical to mont_mul() in goldilocks.hpp.
__device__ __forceinline__ void mont_mul{n}_asm(const uint64_t* a, const uint64_t* b, uint64_t* out) {{
    uint32_t a0[{n}], a1[{n}], b0[{n}], b1[{n}];
#pragma unroll
    for (int i = 0; i < {n}; ++i) {{
        a0[i] = (uint32_t)a[i];
        a1[i] = (uint32_t)(a[i] >> 32);
        b0[i] = (uint32_t)b[i];
        b1[i] = (uint32_t)(b[i] >> 32);
    }}
    uint64_t P[{n}], U[{n}], V[{n}], cy[{n}];
    uint32_t cuv[{n}];
{asm_stmt(la, oa, ia)}    uint32_t p0[{n}], p1[{n}], v0[{n}], v1[{n}], u0[{n}], u1[{n}], rl[{n}], rh[{n}];
#pragma unroll
    for (int i = 0; i < {n}; ++i) {{
        p0[i] = (uint32_t)P[i];
        p1[i] = (uint32_t)(P[i] >> 32);
        u0[i] = (uint32_t)U[i];
        u1[i] = (uint32_t)(U[i] >> 32);
        v0[i] = (uint32_t)V[i];
        v1[i] = (uint32_t)(V[i] >> 32);
    }}
{asm_stmt(lb, ob, ib)}#pragma unroll
    for (int i = 0; i < {n}; ++i) out[i] = ((uint64_t)rh[i] << 32) | rl[i];
}}
"""


def gen(ns):
    fns = "\n".join(gen_fn(n) for n in ns)
    return f"""// GENERATED by tools/gen_mont_asm.py -- do not edit by hand.
// N-way interleaved Montgomery products for gfx950 (see the generator's docstring).
#pragma once
#include <stdint.h>

namespace nhip {{

{fns}
}}  // namespace nhip
"""


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else "neptune-core_amd/csrc/mont_asm.hpp"
    open(out, "w").write(gen(N_LIST))
