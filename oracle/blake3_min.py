"""Minimal BLAKE3 (single-chunk, <= 64-byte input) — TEST INFRASTRUCTURE ONLY.

Part of the oracle (see oracle/README.md): used by tests to re-derive the Tip5
round constants, never by the product path.

Tip5's 80 round constants (twenty-first 1.0.0, `tip5` module, pinned at
/root/reference/Cargo.lock:4297) are derived as
    raw_i = u128::from_le_bytes(BLAKE3(b"Tip5" || [i as u8])[..16]) mod p
and used as the *raw Montgomery* value of the constant.  The derivation is
checked against the reference's own known-answer vectors (KAT-V / KAT-F, see
tests/test_oracle_kat.py): any other derivation fails them.
"""
import struct

_IV = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
       0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
_PERM = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
_M32 = 0xFFFFFFFF
CHUNK_START, CHUNK_END, ROOT = 1, 2, 8


def _rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & _M32


def _g(v, a, b, c, d, mx, my):
    v[a] = (v[a] + v[b] + mx) & _M32
    v[d] = _rotr(v[d] ^ v[a], 16)
    v[c] = (v[c] + v[d]) & _M32
    v[b] = _rotr(v[b] ^ v[c], 12)
    v[a] = (v[a] + v[b] + my) & _M32
    v[d] = _rotr(v[d] ^ v[a], 8)
    v[c] = (v[c] + v[d]) & _M32
    v[b] = _rotr(v[b] ^ v[c], 7)


def _compress(h, m, counter, block_len, flags):
    v = list(h) + _IV[:4] + [counter & _M32, (counter >> 32) & _M32, block_len, flags]
    m = list(m)
    for _ in range(7):
        _g(v, 0, 4, 8, 12, m[0], m[1]); _g(v, 1, 5, 9, 13, m[2], m[3])
        _g(v, 2, 6, 10, 14, m[4], m[5]); _g(v, 3, 7, 11, 15, m[6], m[7])
        _g(v, 0, 5, 10, 15, m[8], m[9]); _g(v, 1, 6, 11, 12, m[10], m[11])
        _g(v, 2, 7, 8, 13, m[12], m[13]); _g(v, 3, 4, 9, 14, m[14], m[15])
        m = [m[_PERM[i]] for i in range(16)]
    return [v[i] ^ v[i + 8] for i in range(8)]


def blake3_short(data: bytes) -> bytes:
    """BLAKE3 hash (32-byte output) of an input of at most 64 bytes."""
    if len(data) > 64:
        raise ValueError("blake3_short handles a single block only")
    block = data + b"\0" * (64 - len(data))
    words = struct.unpack("<16I", block)
    out = _compress(_IV, words, 0, len(data), CHUNK_START | CHUNK_END | ROOT)
    return struct.pack("<8I", *out)
