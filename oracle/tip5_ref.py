"""Pure-Python CPU restatement of Tip5 / Goldilocks / MTree — TEST ORACLE ONLY.

This module is test infrastructure.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it, and only as the checker.  The
product path (neptune-core_amd/) never imports anything under oracle/.

What it restates (the reference's arithmetic lives in third-party crates that
are NOT vendored under /root/reference; pinned versions from
/root/reference/Cargo.lock):
  * twenty-first 1.0.0 (Cargo.lock:4297): BFieldElement (Goldilocks,
    p = 2^64 - 2^32 + 1, Montgomery form with R = 2^64) and the Tip5
    permutation + sponge (rate 10, capacity 6, 5 rounds, split-and-lookup
    S-box on the raw Montgomery bytes of state[0..4], x^7 on state[4..16],
    16x16 circulant MDS, 80 BLAKE3-derived round constants).
  * neptune-core's own Merkle tree `MTree` semantics,
    neptune-core/src/protocol/consensus/block/pow.rs:60-181
    (build_inplace :73-119, path :148-156, verify :162-180).

Pinning (tests/test_oracle_kat.py):
  * KAT-V: Tip5::hash_varlen, 13 vectors from
    neptune-core/src/state/wallet/mod.rs:1379-1383, input derivation
    neptune-core/src/state/wallet/wallet_entropy.rs:36-44,69-83 with
    GENERATION_FLAG = 79 (state/wallet/address/generation_address.rs:47-48).
  * KAT-F: Tip5::hash_pair + MTree child order, fixture
    neptune-core/test_data/precalculated_pow_solution.json, semantics
    pow.rs:162-180.
  The sponge's squeeze / sample_scalars / sample_indices follow the public
  twenty-first 1.0.0 `Sponge` trait and are NOT pinned by any in-tree vector
  (parity unpinned for those three).

Pure-Python big-int loops: use only for small cases (KATs, a few hundred
permutations).  The C restatement oracle/tip5_oracle.c is the fast oracle.
"""
from __future__ import annotations

from typing import List, Sequence

from blake3_min import blake3_short  # noqa: E402  (oracle dir is put on sys.path by callers)

P = (1 << 64) - (1 << 32) + 1
R = 1 << 64
R_INV = pow(R, -1, P)
STATE_SIZE = 16
RATE = 10
CAPACITY = 6
NUM_ROUNDS = 5
NUM_SPLIT_AND_LOOKUP = 4
DIGEST_LEN = 5
BFE_MAX = P - 1

# twenty-first tip5::LOOKUP_TABLE: L(x) = (x+1)^3 - 1 mod 257 (a permutation of 0..255).
LOOKUP_TABLE = [((x + 1) ** 3 - 1) % 257 for x in range(256)]

# twenty-first tip5::MDS_MATRIX_FIRST_COLUMN. Orientation out[i] = sum_j c[(i-j) mod 16] in[j]
# (the other orientation fails KAT-V).
MDS_FIRST_COLUMN = [61402, 1108, 28750, 33823, 7454, 43244, 53865, 12034,
                    56951, 27521, 41351, 40901, 12021, 59689, 26798, 17845]


def _derive_round_constants() -> List[int]:
    out = []
    for i in range(NUM_ROUNDS * STATE_SIZE):
        raw = int.from_bytes(blake3_short(b"Tip5" + bytes([i]))[:16], "little") % P
        out.append(raw * R_INV % P)  # raw Montgomery value -> canonical value
    return out


# Canonical values of the 80 round constants.
ROUND_CONSTANTS = _derive_round_constants()


# ---------------------------------------------------------------- field helpers
def to_mont(x: int) -> int:
    return x * R % P


def from_mont(r: int) -> int:
    return r * R_INV % P


def split_and_lookup(x: int) -> int:
    """S-box for state[0..4]: bytewise lookup on the raw Montgomery LE bytes."""
    raw = to_mont(x)
    b = raw.to_bytes(8, "little")
    raw2 = int.from_bytes(bytes(LOOKUP_TABLE[c] for c in b), "little")
    return from_mont(raw2)


# ---------------------------------------------------------------- permutation
def permutation(state: Sequence[int]) -> List[int]:
    s = [int(v) % P for v in state]
    assert len(s) == STATE_SIZE
    for r in range(NUM_ROUNDS):
        s = [split_and_lookup(v) for v in s[:NUM_SPLIT_AND_LOOKUP]] + \
            [pow(v, 7, P) for v in s[NUM_SPLIT_AND_LOOKUP:]]
        s = [sum(MDS_FIRST_COLUMN[(i - j) % 16] * s[j] for j in range(16)) % P
             for i in range(16)]
        s = [(s[i] + ROUND_CONSTANTS[r * STATE_SIZE + i]) % P for i in range(16)]
    return s


def use_c_backend():
    """Route every permutation of this module (sponge, hash_pair, hash_varlen) through the C
    restatement oracle/tip5_oracle.c (itself checked against this file and the KATs in
    tests/test_oracle_kat.py); used to time the CPU baseline at realistic speed."""
    global permutation
    import coracle
    permutation = coracle.permutation_list


# ---------------------------------------------------------------- sponge
class Tip5:
    """Sponge with the two domains of twenty-first's Tip5."""

    def __init__(self, fixed_length: bool = False):
        self.state = [0] * STATE_SIZE
        if fixed_length:
            self.state[RATE:] = [1] * CAPACITY

    def permute(self):
        self.state = permutation(self.state)

    def absorb(self, chunk: Sequence[int]):
        assert len(chunk) == RATE
        self.state[:RATE] = [int(v) for v in chunk]
        self.permute()

    def pad_and_absorb_all(self, data: Sequence[int]):
        data = [int(v) for v in data]
        n_full = len(data) // RATE
        for k in range(n_full):
            self.absorb(data[k * RATE:(k + 1) * RATE])
        rem = data[n_full * RATE:]
        last = rem + [1] + [0] * (RATE - len(rem) - 1)
        self.absorb(last)

    def squeeze(self) -> List[int]:
        out = list(self.state[:RATE])
        self.permute()
        return out

    def sample_scalars(self, n: int) -> List[List[int]]:
        """n XFieldElements as [c0, c1, c2] (twenty-first Sponge::sample_scalars)."""
        n_sq = (n * 3 + RATE - 1) // RATE
        flat = []
        for _ in range(n_sq):
            flat += self.squeeze()
        return [flat[3 * k:3 * k + 3] for k in range(n)]

    def sample_indices(self, upper_bound: int, n: int) -> List[int]:
        assert upper_bound & (upper_bound - 1) == 0 and 0 < upper_bound <= (1 << 31)
        out: List[int] = []
        pool: List[int] = []
        while len(out) != n:
            if not pool:
                pool = list(reversed(self.squeeze()))
            e = pool.pop()
            if e != BFE_MAX:
                # `element.value() as u32 % upper_bound` (upper_bound: u32)
                out.append((e & 0xFFFFFFFF) % upper_bound)
        return out


def hash_pair(left: Sequence[int], right: Sequence[int]) -> List[int]:
    s = list(left) + list(right) + [1] * CAPACITY
    return permutation(s)[:DIGEST_LEN]


def hash_varlen(data: Sequence[int]) -> List[int]:
    sp = Tip5(fixed_length=False)
    sp.pad_and_absorb_all(data)
    return sp.state[:DIGEST_LEN]


# ---------------------------------------------------------------- digests
def digest_to_hex(d: Sequence[int]) -> str:
    """Digest LowerHex: each element's canonical value as 8 little-endian bytes."""
    return b"".join(int(v).to_bytes(8, "little") for v in d).hex()


def digest_from_hex(h: str) -> List[int]:
    b = bytes.fromhex(h)
    assert len(b) == 40
    return [int.from_bytes(b[8 * i:8 * i + 8], "little") for i in range(5)]


# ---------------------------------------------------------------- MTree (pow.rs)
def mtree_build(leafs: Sequence[Sequence[int]]) -> List[List[int]]:
    """Internal nodes of pow.rs MTree::build_inplace: node i has children 2i, 2i+1,
    root at index 1, leaf k sits (virtually) at node n + k.  Returns a list of
    length n with [0] unused."""
    n = len(leafs)
    assert n >= 2 and n & (n - 1) == 0
    nodes: List[List[int]] = [[0] * 5 for _ in range(n)]
    for i in range(n // 2, n):
        nodes[i] = hash_pair(leafs[2 * i - n], leafs[2 * i - n + 1])
    for i in range(n // 2 - 1, 0, -1):
        nodes[i] = hash_pair(nodes[2 * i], nodes[2 * i + 1])
    return nodes


def mtree_path(leafs, nodes, index: int) -> List[List[int]]:
    n = len(leafs)
    path = [list(leafs[index ^ 1])]
    running = index + n
    for _ in range(1, n.bit_length() - 1):
        running >>= 1
        path.append(list(nodes[running ^ 1]))
    return path


def mtree_verify(root, index: int, path, element) -> bool:
    """pow.rs:162-180.  Note `index > 1 << path.len()` (strict) and Rust's
    release-mode masking of the shift amount."""
    if index > (1 << (len(path) & 63)):
        return False
    running_index = index
    running = list(element)
    for sib in path:
        if running_index & 1:
            running = hash_pair(sib, running)
        else:
            running = hash_pair(running, sib)
        running_index >>= 1
    return running == list(root)
