"""Shared LZ4 test inputs: payloads compressed by liblz4 (pyarrow's "lz4_raw"
codec, the LZ4 block format lz4_flex decodes) and hand-built streams that hit
every branch of the block format (overlapping matches, 255-extension lengths,
malformed sequences)."""
import numpy as np


def lz4_compress(data: bytes) -> bytes:
    import pyarrow as pa
    return pa.Codec("lz4_raw").compress(data, asbytes=True)


def _ext(n):  # length extension bytes for a nibble of 15
    out = []
    while n >= 255:
        out.append(255)
        n -= 255
    out.append(n)
    return bytes(out)


def seq(literals: bytes, offset=None, match_len=0) -> bytes:
    """One LZ4 sequence; offset None = last sequence (literals only)."""
    ll = len(literals)
    tok_l = min(ll, 15)
    if offset is None:
        return bytes([tok_l << 4]) + (_ext(ll - 15) if ll >= 15 else b"") + literals
    ml = match_len - 4
    tok_m = min(ml, 15)
    return (bytes([(tok_l << 4) | tok_m]) + (_ext(ll - 15) if ll >= 15 else b"") + literals +
            offset.to_bytes(2, "little") + (_ext(ml - 15) if ml >= 15 else b""))


def _unaligned_expected(lit300):
    a = bytes(range(7)) + bytes(range(5))  # 7 literals, then 5 bytes from offset 7
    b = a + lit300[:257]                   # a 257-byte literal run starting at output byte 12
    return b + b[len(b) - 200:len(b) - 191] + lit300[:5]


def handmade():
    """(name, stream, expected bytes or None for malformed, uncompressed_length)."""
    r = np.random.default_rng(3)
    lit300 = r.integers(0, 256, 300, dtype=np.uint8).tobytes()
    cases = [
        ("literals_only", seq(b"abc"), b"abc"),
        ("empty_block", seq(b""), b""),
        ("rle_offset1", seq(b"x", 1, 1000) + seq(b"END"), b"x" * 1001 + b"END"),
        ("overlap_offset3", seq(b"abc", 3, 200) + seq(b""), (b"abc" * 80)[:203]),
        ("overlap_offset63", seq(bytes(range(63)), 63, 700) + seq(b"z"),
         (bytes(range(63)) * 20)[:763] + b"z"),
        ("long_literals_ext", seq(lit300) + b"", lit300),
        ("long_lit_then_long_match", seq(lit300, 300, 270 + 255 * 3) + seq(b"q"),
         lit300 + (lit300 * 4)[:270 + 255 * 3] + b"q"),
        ("match_ext_past_window", seq(b"ab", 2, 2000) + seq(b"!"), b"ab" * 1001 + b"!"),
        ("unaligned_literal_runs", seq(bytes(range(7)), 7, 5) + seq(lit300[:257], 200, 9) + seq(lit300[:5]),
         _unaligned_expected(lit300)),
        ("offset0", seq(b"abcd", 0, 8) + seq(b""), None),
        ("offset_beyond", seq(b"abcd", 5, 8) + seq(b""), None),
        ("truncated_offset", seq(b"abcd", 4, 8)[:-1], None),
        ("truncated_literals", seq(b"abcdefgh")[:-3], None),
        ("truncated_ext", bytes([0xF0, 255]), None),
        ("no_input", b"", None),
    ]
    return cases
