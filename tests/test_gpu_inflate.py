"""GPU parity of the decoder: libndfl.so's ndfl_inflate against the reference's known-answer tests
(T/InflaterInputStreamTest.java, fixture tests/golden/inflate_kat.json), its seeded generators,
Python zlib streams, the oracle's own streams (all strategies, stored+fixed mixes) and error
Reasons on corrupted streams (compared with the CPU oracle)."""
import io
import json
import os
import random
import zlib

import pytest

import oracle_lib as O
from test_oracle_inflate import KAT, quasi_log_len, lsb_bits, LSB8, MSB_LIT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import ndfl
    return ndfl.Context(0)


def gpu_inflate(ctx, data):
    reason, out, bits = ctx.inflate(data)
    return (reason.name if reason is not None else None), out, bits


def check_same(ctx, data):
    g = gpu_inflate(ctx, data)
    o = O.inflate(data)
    assert g[0] == o[0], (g[0], o[0])
    assert g[1] == o[1]
    if o[0] is None:
        assert g[2] == o[2]
    return g


@pytest.mark.parametrize("kat", KAT, ids=[k["name"] for k in KAT])
def test_known_answer(ctx, kat):
    rng = random.Random(kat["line"])
    for pad in range(3):
        data = O.bits_to_bytes(kat["bits"], pad, rng)
        reason, out, bits = gpu_inflate(ctx, data)
        if kat["expect_reason"] is None:
            assert reason is None and out == bytes.fromhex(kat["expect_hex"])
            assert (bits + 7) // 8 == len(data)
        else:
            assert reason == kat["expect_reason"]


def test_generators(ctx):
    rng = random.Random(166)
    for _ in range(30):
        nblocks = rng.randrange(30) + 1
        bits, out = "", bytearray()
        for j in range(nblocks):
            bits += "0" if j + 1 < nblocks else "1"
            if rng.random() < 0.5:
                bits += "00"
                while len(bits) % 8:
                    bits += str(rng.randrange(2))
                ln = quasi_log_len(rng, 17)
                bits += lsb_bits(ln | ((~ln) << 16) & 0xFFFFFFFF, 32)
                data = rng.randbytes(ln)
                out += data
                bits += "".join(LSB8[b] for b in data)
            else:
                bits += "10" + "111111111" + "0000000"
                out.append(0xFF)
        reason, got, _ = gpu_inflate(ctx, O.bits_to_bytes(bits, 0, rng))
        assert reason is None and got == bytes(out)


@pytest.mark.parametrize("level", [0, 1, 6, 9])
def test_zlib_streams(ctx, level):
    rng = random.Random(level)
    for n in [0, 1, 100, 5000, 70000, 300000]:
        words = [rng.randbytes(rng.randrange(2, 9)) for _ in range(200)]
        data = b"".join(rng.choice(words) for _ in range(n // 4))[:n]
        co = zlib.compressobj(level, zlib.DEFLATED, -15, 9)
        comp = co.compress(data) + co.flush()
        reason, out, bits = gpu_inflate(ctx, comp + b"\x00\xff")
        assert reason is None and out == data and (bits + 7) // 8 == len(comp)


@pytest.mark.parametrize("strategy", O.STRATEGIES)
def test_oracle_streams_all_strategies(ctx, strategy):
    rng = random.Random(7)
    for n in [0, 1, 1000, 70000, 200000]:
        buf = bytearray()
        while len(buf) < n:
            buf += bytes([rng.randrange(3)]) * rng.randrange(1, 500) if rng.random() < 0.5 else rng.randbytes(50)
        data = bytes(buf[:n])
        if strategy.startswith("FULL") and n > 70000:
            continue
        comp = O.deflate(data, strategy)
        check_same(ctx, comp)


def test_stored_plus_fixed_mix(ctx):
    """Config-2 shape: alternating stored and fixed-Huffman blocks (fixed blocks are invisible to
    the header finder and are reached by chain continuation)."""
    rng = random.Random(2)
    words = [rng.randbytes(rng.randrange(2, 9)) for _ in range(100)]
    data = b"".join(rng.choice(words) + rng.randbytes(rng.randrange(0, 3)) for _ in range(200000))[:1 << 20]
    comp = O.deflate_mixed(data, ["UNCOMPRESSED", "FULL_STATIC", "LITERAL_STATIC", "UNCOMPRESSED", "FULL_STATIC"],
                           chunk_len=40000)
    reason, out, bits = check_same(ctx, comp)
    assert reason is None and out == data


def test_large_roundtrip_gpu_stream(ctx):
    import corpus
    data = corpus.c4_mixed(64 << 20).numpy().tobytes()
    comp = ctx.deflate(data)
    reason, out, bits = gpu_inflate(ctx, comp)
    assert reason is None and out == data and (bits + 7) // 8 == len(comp)


def test_corrupted_streams_match_oracle_reason(ctx):
    """Flip bytes in valid streams: the GPU must report the oracle's Reason and the same prefix."""
    rng = random.Random(9)
    base = []
    for strategy in ["RLE_DYNAMIC", "FULL_STATIC", "UNCOMPRESSED", "LITERAL_DYNAMIC"]:
        data = b"".join(bytes([rng.randrange(4)]) * rng.randrange(1, 50) for _ in range(3000))
        base.append(O.deflate(data, strategy))
    for comp in base:
        for _ in range(40):
            c = bytearray(comp)
            for _ in range(rng.randrange(1, 4)):
                c[rng.randrange(len(c))] ^= 1 << rng.randrange(8)
            if rng.random() < 0.3:
                c = c[:rng.randrange(len(c))]
            check_same(ctx, bytes(c))


def test_corrupted_lz77_streams_prefix_exact(ctx):
    """LZ77-heavy streams (FULL_DYNAMIC, zlib -6) across many blocks, corrupted: every byte the GPU
    reports before the error is produced through deferred copies and the resolve rounds, and must
    equal the oracle's prefix; the Reason and consumed bits must match too."""
    import zlib as Z
    rng = random.Random(19)
    words = [rng.randbytes(rng.randrange(3, 12)) for _ in range(300)]
    data = b"".join(rng.choice(words) for _ in range(120_000))[:1 << 20]
    co = Z.compressobj(6, Z.DEFLATED, -15)
    streams = [O.deflate(data[:300_000], "FULL_DYNAMIC"), co.compress(data) + co.flush()]
    for comp in streams:
        check_same(ctx, comp)
        for _ in range(25):
            c = bytearray(comp)
            for _ in range(rng.randrange(1, 3)):
                c[rng.randrange(len(c) // 4, len(c))] ^= 1 << rng.randrange(8)
            if rng.random() < 0.3:
                c = c[:rng.randrange(len(c) // 2, len(c))]
            check_same(ctx, bytes(c))

