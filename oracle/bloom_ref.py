"""bloom_ref -- TEST INFRASTRUCTURE ONLY: a restatement of the bloom filter the
reference's default writer options create, so tests can write and read
segments whose meta block carries a real filter (segment_writer_option.go:20,
segment_writer.go:133-136 and :295-300, segment_reader.go:183-201).

The product never computes a filter: the bytes are an opaque pass-through
(okv_encode_opts.bloom, okv_writer_set_bloom) that a Go caller fills from the
real library.  Restated here from the published algorithms of the pinned
versions (go.sum: github.com/bits-and-blooms/bloom v2.0.3+incompatible,
github.com/spaolacci/murmur3 v1.1.0, github.com/willf/bitset v1.1.11):

  NewWithEstimates(n, p): m = ceil(-n ln p / (ln 2)^2), k = ceil(ln 2 * m / n)
  Add(key): h = baseHashes(key) = murmur3.Sum128(key) ++ Sum128(key ++ [1]);
            for i < k: set bit (h[i % 2] + i * h[2 + ((i + i % 2) % 4) / 2]) mod m
  WriteTo: u64 m, u64 k (big endian), then bitset.WriteTo: u64 length, the
           uint64 words (big endian)

PARITY UNPINNED: no reference test asserts filter bytes (TestRollover only
asserts rows), and the Go module is not vendored here.  The murmur3 vector
below is the canonical MurmurHash3_x64_128 one; nothing on the product path
depends on this file.
"""
from __future__ import annotations

import math
import struct

M64 = (1 << 64) - 1
C1, C2 = 0x87C37B91114253D5, 0x4CF5AD432745937F


def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _fmix(k):
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & M64
    return k ^ (k >> 33)


def murmur3_128(data: bytes, seed: int = 0):
    """MurmurHash3_x64_128 (spaolacci/murmur3 Sum128: (h1, h2))."""
    h1 = h2 = seed & M64
    n = len(data)
    nb = n // 16
    for i in range(nb):
        k1, k2 = struct.unpack_from("<QQ", data, 16 * i)
        k1 = (_rotl((k1 * C1) & M64, 31) * C2) & M64
        h1 ^= k1
        h1 = (_rotl(h1, 27) + h2) & M64
        h1 = (h1 * 5 + 0x52DCE729) & M64
        k2 = (_rotl((k2 * C2) & M64, 33) * C1) & M64
        h2 ^= k2
        h2 = (_rotl(h2, 31) + h1) & M64
        h2 = (h2 * 5 + 0x38495AB5) & M64
    tail = data[16 * nb:]
    k1 = k2 = 0
    for i in range(len(tail) - 1, 7, -1):
        k2 = (k2 << 8) | tail[i]
    if len(tail) > 8:
        k2 = (_rotl((k2 * C2) & M64, 33) * C1) & M64
        h2 ^= k2
    for i in range(min(len(tail), 8) - 1, -1, -1):
        k1 = (k1 << 8) | tail[i]
    if tail:
        k1 = (_rotl((k1 * C1) & M64, 31) * C2) & M64
        h1 ^= k1
    h1 ^= n
    h2 ^= n
    h1 = (h1 + h2) & M64
    h2 = (h2 + h1) & M64
    h1, h2 = _fmix(h1), _fmix(h2)
    h1 = (h1 + h2) & M64
    h2 = (h2 + h1) & M64
    return h1, h2


class BloomFilter:
    """bits-and-blooms/bloom v2.0.3 BloomFilter{m, k, *bitset.BitSet}."""

    def __init__(self, m: int, k: int):
        self.m, self.k = max(1, m), max(1, k)
        self.words = [0] * ((m + 63) >> 6)  # bitset.New(m): wordsNeeded(m)
        self.length = m

    @classmethod
    def with_estimates(cls, n: int, p: float) -> "BloomFilter":
        m = math.ceil(-1 * n * math.log(p) / math.pow(math.log(2), 2))
        k = math.ceil(math.log(2) * m / n)
        return cls(m, k)

    @staticmethod
    def _base(data: bytes):
        v1, v2 = murmur3_128(data)
        v3, v4 = murmur3_128(data + b"\x01")  # hasher.Write([]byte{1}) then Sum128
        return (v1, v2, v3, v4)

    def _locations(self, data: bytes):
        h = self._base(data)
        i = 0
        while i < self.k:
            yield ((h[i % 2] + i * h[2 + ((i + (i % 2)) % 4) // 2]) & M64) % self.m
            i += 1

    def add(self, data: bytes) -> "BloomFilter":
        for loc in self._locations(data):
            self.words[loc >> 6] |= 1 << (loc & 63)
        return self

    def test(self, data: bytes) -> bool:
        """Test (bloom v2.0.3): k probes; bitset.Test reads positions >= the
        bitset's length as false; m == 0 is Go's integer-division panic
        (ZeroDivisionError here)."""
        if self.k == 0:
            return True
        if self.m == 0:
            raise ZeroDivisionError("integer divide by zero")
        for loc in self._locations(data):
            if loc >= self.length or not (self.words[loc >> 6] >> (loc & 63)) & 1:
                return False
        return True

    def to_bytes(self) -> bytes:
        """WriteTo: m, k, bitset length, words -- all big-endian uint64."""
        return struct.pack(f">QQQ{len(self.words)}Q", self.m, self.k, self.length, *self.words)

    @classmethod
    def from_bytes(cls, b: bytes) -> "BloomFilter":
        """ReadFrom (bloom v2.0.3; bitset v1.1.11 ReadFrom): big-endian m, k,
        bitset length, then wordsNeeded(length) words; any short read is an
        error (ValueError), trailing bytes are not read."""
        b = bytes(b or b"")
        if len(b) < 24:
            raise ValueError("bloom ReadFrom: unexpected EOF")
        m, k, length = struct.unpack_from(">QQQ", b)
        words = (M64 >> 6) if length > M64 - 63 else (length + 63) >> 6
        if words > (len(b) - 24) // 8:
            raise ValueError("bloom ReadFrom: unexpected EOF / type mismatch")
        f = cls.__new__(cls)
        f.m, f.k, f.length = m, k, length
        f.words = list(struct.unpack_from(f">{words}Q", b, 24))
        return f


def default_filter() -> BloomFilter:
    """DefaultSegmentWriterOptions: bloom.NewWithEstimates(100_000, 0.000001)
    (segment_writer_option.go:20)."""
    return BloomFilter.with_estimates(100_000, 0.000001)
