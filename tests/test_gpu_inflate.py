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
from test_oracle_inflate import KAT, quasi_log_len, lsb_bits, LSB8, MSB_LIT, reserved_symbol_streams

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    import ndfl
    c = ndfl.Context(0)
    c.set_stream(torch.cuda.current_stream().cuda_stream)     # ordered with torch's kernels
    return c


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


def test_reserved_symbol_in_the_message(ctx):
    """The reserved symbol reaches the caller as the reference names it: "Reserved run length
    symbol: 287", "Reserved distance symbol: 31" (D/decomp/Open.java:516, 550) -- the four fixed-Huffman
    KATs and two dynamic blocks (287 used by a code, 31 as the padding of a single distance code),
    symbol equal to the oracle's."""
    import ndfl
    for name, data, want, reason, sym in reserved_symbol_streams():
        r, out, _ = ctx.inflate(data)
        assert r is not None and r.name == reason, name
        assert ctx.error_symbol() == sym == (O.inflate(data), O.error_symbol())[1], name
        assert want is None or out == want, name
        e = ctx.data_format_error(r.value + 1)
        prefix = "Reserved run length symbol" if reason == "RESERVED_LENGTH_SYMBOL" else "Reserved distance symbol"
        assert str(e) == f"{prefix}: {sym}", name
        with pytest.raises(ndfl.DataFormatException, match=f": {sym}$"):     # (a read past the good bytes)
            ndfl.InflaterInputStream(io.BytesIO(data), context=ctx).read(bytearray(64), 0, 64)
    assert ctx.inflate(O.deflate(b"abc"))[0] is None and ctx.error_symbol() == -1


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



def test_in_padded_device_input_matches_oracle(ctx):
    """NDFL_IN_PADDED: a device buffer that is 16-byte aligned with IN_PAD_BYTES zeros after the
    stream is decoded in place; results (Reason, bytes, consumed bits) equal the oracle's, for ragged
    lengths, truncated/corrupted streams, and a misaligned pointer (which is staged instead); the
    same through ndfl_inflate_range from a block boundary past bit 0, with and without
    NDFL_DICT_DEFERRED."""
    import torch
    import ndfl
    rng = random.Random(31)
    cases = []
    for strategy in ["RLE_DYNAMIC", "FULL_DYNAMIC", "UNCOMPRESSED", "LITERAL_STATIC"]:
        data = b"".join(bytes([rng.randrange(5)]) * rng.randrange(1, 90) + rng.randbytes(rng.randrange(0, 9))
                        for _ in range(rng.randrange(50, 4000)))
        comp = O.deflate(data, strategy)
        cases.append(comp)
        c = bytearray(comp)
        c[rng.randrange(len(c))] ^= 1 << rng.randrange(8)
        cases.append(bytes(c[:rng.randrange(1, len(c) + 1)]))
    cases.append(b"\x01\x00\x00\xff\xff")                       # empty stored final block
    D = ndfl.IN_DEVICE | ndfl.OUT_DEVICE
    for comp in cases:
        o = O.inflate(comp)
        for shift in (0, 4):                                     # 4: not 16-byte aligned -> staged
            buf = torch.zeros(len(comp) + ndfl.IN_PAD_BYTES + 16, dtype=torch.uint8, device="cuda")
            buf[shift:shift + len(comp)] = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
            out = torch.zeros(max(len(o[1]), 1) + 1024, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            r, olen, bits = ctx.inflate_raw(buf.data_ptr() + shift, len(comp), out.data_ptr(), out.numel(),
                                            D | ndfl.IN_PADDED)
            reason = None if r == 0 else ndfl.Reason(r - 1).name
            assert r >= 0, r
            assert reason == o[0], (reason, o[0])
            assert olen == len(o[1]) and out[:olen].cpu().numpy().tobytes() == o[1]
            if o[0] != "UNEXPECTED_END_OF_STREAM":     # (where the input ran out is not pinned)
                assert bits == o[2], (reason, bits, o[2])
    # range decodes in place: start at the 3rd chunk's block boundary
    data = b"".join(bytes([rng.randrange(4)]) * rng.randrange(1, 200) + rng.randbytes(rng.randrange(0, 30))
                    for _ in range(6000))
    seams = [0] + O.block_bits(data)
    for k in range(1, len(seams)):
        seams[k] += seams[k - 1]
    comp = O.deflate(data)
    a = 2
    pre = a * 65536
    window = data[pre - 32768:pre]
    oref = O.inflate_range(comp, seams[a], None, window)
    buf = torch.zeros(len(comp) + ndfl.IN_PAD_BYTES, dtype=torch.uint8, device="cuda")
    buf[:len(comp)] = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
    for deferred in (False, True):
        out = torch.zeros(32768 + len(oref[1]) + 64, dtype=torch.uint8, device="cuda")
        if not deferred:
            out[:32768] = torch.frombuffer(bytearray(window), dtype=torch.uint8).cuda()
        torch.cuda.synchronize()
        fl = D | ndfl.IN_PADDED | (ndfl.DICT_DEFERRED if deferred else 0)
        r, olen, bits = ctx.inflate_range_raw(buf.data_ptr(), len(comp), seams[a], None, out.data_ptr(), 32768,
                                              out.numel() - 32768, fl)
        if deferred:
            out[:32768] = torch.frombuffer(bytearray(window), dtype=torch.uint8).cuda()
            ctx.inflate_resolve()
        assert (r, olen, bits) == (0, len(oref[1]), oref[2])
        assert out[32768:32768 + olen].cpu().numpy().tobytes() == oref[1] == data[pre:]


class _Pipe(io.RawIOBase):
    """Non-seekable reader handing out at most `step` bytes per read."""

    def __init__(self, data, step):
        self._d, self._p, self._step = data, 0, step

    def readable(self):
        return True

    def read(self, n=-1):
        n = len(self._d) - self._p if n is None or n < 0 else n
        b = self._d[self._p:self._p + min(n, self._step)]
        self._p += len(b)
        return b


@pytest.mark.parametrize("batch", [1 << 10, 40000, 1 << 20])
def test_streaming_inflater_matches_oracle(ctx, batch):
    """InflaterInputStream reads its input incrementally (ndfl_inflate_range with NDFL_IN_PARTIAL):
    fed through a non-seekable pipe in small pieces with small device batches, the output equals the
    oracle's for RLE / FULL / stored / fixed / zlib -6 streams; endExactly leaves a seekable stream
    right after the final block; a corrupted stream yields the oracle's prefix and Reason."""
    import zlib as Z
    import ndfl
    rng = random.Random(batch)
    words = [rng.randbytes(rng.randrange(3, 12)) for _ in range(300)]
    text = b"".join(rng.choice(words) for _ in range(60_000))[:400_000]
    co = Z.compressobj(6, Z.DEFLATED, -15)
    streams = [O.deflate(text), O.deflate(text[:150_000], "FULL_DYNAMIC"), co.compress(text) + co.flush(),
               O.deflate_mixed(text, ["UNCOMPRESSED", "FULL_STATIC", "RLE_DYNAMIC"], chunk_len=30000), O.deflate(b"")]
    old = ndfl.InflaterInputStream.BATCH
    ndfl.InflaterInputStream.BATCH = batch
    try:
        for comp in streams:
            o = O.inflate(comp)
            s = ndfl.InflaterInputStream(_Pipe(comp + b"tail", 777), context=ctx)
            got = bytearray()
            buf = bytearray(5000)
            while (k := s.read(buf, 0, len(buf))) != -1:
                got += buf[:k]
            assert bytes(got) == o[1]
            f = io.BytesIO(b"head" + comp + b"tail")
            f.seek(4)
            s = ndfl.InflaterInputStream(f, True, context=ctx)
            assert s.readall() == o[1]
            assert f.tell() == 4 + (o[2] + 7) // 8 and f.read() == b"tail"
        for pos in range(len(streams[0]) * 2 // 3, len(streams[0])):
            bad = bytearray(streams[0])
            bad[pos] ^= 0x10
            o = O.inflate(bytes(bad))
            if o[0] is not None:
                break
        assert o[0] is not None
        s = ndfl.InflaterInputStream(_Pipe(bytes(bad), 1000), context=ctx)
        got = bytearray()
        with pytest.raises(ndfl.DataFormatException) as ei:
            while (k := s.read(buf, 0, len(buf))) != -1:
                got += buf[:k]
        # the read that reaches the error raises (Open.read, D/decomp/Open.java:83-110): the bytes it
        # had copied before the error are in buf, uncounted
        rest = len(o[1]) - len(got)
        assert ei.value.getReason().name == o[0] and 0 <= rest < len(buf)
        assert bytes(got) + bytes(buf[:rest]) == o[1]
        # one read asking for more than the whole good prefix raises on the first call
        s = ndfl.InflaterInputStream(_Pipe(bytes(bad), 1000), context=ctx)
        big = bytearray(len(o[1]) + 4096)
        with pytest.raises(ndfl.DataFormatException) as ei:
            s.read(big, 0, len(big))
        assert ei.value.getReason().name == o[0] and bytes(big[:len(o[1])]) == o[1]
        # a read ending exactly at the error returns normally, the next one raises
        s = ndfl.InflaterInputStream(_Pipe(bytes(bad), 1000), context=ctx)
        assert s.read(big, 0, len(o[1])) == len(o[1]) and s.read(big, 0, 0) == 0
        with pytest.raises(ndfl.DataFormatException):
            s.read()
    finally:
        ndfl.InflaterInputStream.BATCH = old
