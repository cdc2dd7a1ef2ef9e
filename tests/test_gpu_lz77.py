"""GPU parity of the LZ77 encoder (FULL_* presets and explicit Lz77Huffman parameters).

The reference's longest-match search (D/comp/Lz77Huffman.java:62-130) has no golden vectors of its
own (T/DeflaterOutputStreamTest.java only round-trips), so bytes are checked against the CPU
oracle, whose chain walk is pinned to the reference's literal exhaustive loop in
tests/test_oracle_deflate.py, and every output is also decoded back (GPU inflate + zlib).
"""
import io
import random
import zlib

import pytest

import knobs
import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ndfl():
    import ndfl as N
    return N


@pytest.fixture(scope="module")
def ctx(ndfl):
    return ndfl.Context(0)


def _text(n, seed):
    import corpus
    return corpus.c3_text(n, seed=seed).numpy().tobytes()


def inputs(seed):
    rng = random.Random(seed)
    out = [b"", b"\x00", b"ab", b"aaa", b"abcabcabc", b"\x00" * 1000, b"\x00" * 65537, bytes(range(256)) * 300,
           b"abcdefgh" * 40000]
    for n in [1, 2, 3, 4, 63, 64, 65, 100, 1000, 4097, 65535, 65536, 65537, 131072, 200003]:
        out.append(rng.randbytes(n))
        # repeats of earlier data at random distances (config-5 style)
        buf = bytearray(rng.randbytes(min(n, 50)))
        while len(buf) < n:
            if rng.random() < 0.6 and len(buf) > 3:
                d = rng.randrange(1, min(len(buf), 40000) + 1)
                ln = rng.choice([3, 4, 5, 10, 50, 257, 258, 259, 1000])
                for _ in range(ln):
                    buf.append(buf[-d])
            else:
                buf += rng.randbytes(rng.randrange(1, 20))
        out.append(bytes(buf[:n]))
    return out


def _roundtrip(ctx, comp, data):
    reason, out, _ = ctx.inflate(comp)
    assert reason is None and out == data
    assert zlib.decompress(comp, -15) == data


@pytest.mark.parametrize("strategy", ["FULL_DYNAMIC", "FULL_STATIC"])
def test_full_presets_match_oracle(ctx, strategy):
    for data in inputs(11):
        got = ctx.deflate(data, strategy)
        exp = O.deflate(data, strategy)
        assert got == exp, (strategy, len(data))
        _roundtrip(ctx, got, data)


def test_full_dynamic_text(ctx):
    for n, seed in [(1 << 20, 1), (3 << 20, 2), (123_457, 3)]:
        data = _text(n, seed)
        got = ctx.deflate(data, "FULL_DYNAMIC")
        assert got == O.deflate(data, "FULL_DYNAMIC"), n
        _roundtrip(ctx, got, data)


@pytest.mark.parametrize("params", [(True, 3, 258, 1, 32768), (True, 4, 258, 1, 32768), (True, 3, 100, 1, 32768),
                                    (True, 3, 258, 2, 32768), (True, 3, 258, 1, 300), (False, 5, 20, 3, 4096),
                                    (True, 3, 3, 1, 32768), (True, 258, 258, 1, 32768), (True, 3, 258, 1, 2),
                                    (True, 3, 258, 32768, 32768), (True, 3, 10, 1, 1), (True, 0, 0, 0, 0),
                                    (False, 3, 258, 1, 1)])
def test_lz77_parameters_match_oracle(ndfl, ctx, params):
    strat = ndfl.Lz77Huffman(*params)
    for data in inputs(12)[::2] + [_text(300_000, 4)]:
        got = ctx.deflate(data, strat)
        exp = O.deflate_lz(data, *params)
        assert got == exp, (params, len(data))
        _roundtrip(ctx, got, data)


@pytest.mark.parametrize("chunk_len,hist_limit", [(1000, 32768), (64, 1), (777, 0), (65536, 0), (4096, 100),
                                                  (40000, 32768), (65536, 20000)])
def test_full_chunk_and_history_params(ctx, chunk_len, hist_limit):
    for data in inputs(13)[::3] + [_text(200_000, 5)]:
        got = ctx.deflate(data, "FULL_DYNAMIC", chunk_len=chunk_len, hist_limit=hist_limit)
        assert got == O.deflate(data, "FULL_DYNAMIC", chunk_len, hist_limit), (len(data), chunk_len, hist_limit)


def test_full_crc(ctx):
    for data in inputs(14)[::4]:
        comp, crc = ctx.deflate(data, "FULL_DYNAMIC", with_crc=True)
        assert crc == zlib.crc32(data)
        assert comp == O.deflate(data, "FULL_DYNAMIC")


def test_full_stream_batches(ndfl, ctx):
    """DeflaterOutputStream(FULL_DYNAMIC) with small batches: the history crosses GPU calls."""
    rng = random.Random(15)
    for _ in range(6):
        data = _text(rng.randrange(1, 400_000), rng.randrange(1000))
        bout = io.BytesIO()
        d = ndfl.DeflaterOutputStream(bout, strategy=ndfl.Lz77Huffman.FULL_DYNAMIC, context=ctx,
                                      batch_bytes=rng.choice([1, 65537, 100_000]))
        off = 0
        while off < len(data):
            n = rng.randrange(1, min(90_000, len(data) - off) + 1)
            d.write(data, off, n)
            off += n
        d.finish()
        assert bout.getvalue() == O.deflate(data, "FULL_DYNAMIC")


def test_invalid_parameters(ndfl):
    for bad in [(True, 2, 258, 1, 32768), (True, 3, 259, 1, 32768), (True, 5, 4, 1, 10), (True, 3, 258, 0, 10),
                (True, 3, 258, 1, 32769), (True, 3, 258, 10, 9)]:
        with pytest.raises(ValueError):
            ndfl.Lz77Huffman(*bad)


@pytest.mark.parametrize("env", [{"NDFL_LZ_SEARCH": "chain"}, {"NDFL_LZ_LEAD": "0"}])
def test_search_modes_match_oracle(ndfl, env):
    """The round-3 hash-chain search at every position (NDFL_LZ_SEARCH=chain), and the parse-driven
    search without its tile lead-in (NDFL_LZ_LEAD=0: the parse enters most tiles at positions no
    wave searched, so the encode kernel's fallback search -- lz_match_global -- supplies them):
    both give the oracle's bytes."""
    ctx = knobs.context(**env)
    cases = [(d, "FULL_DYNAMIC", 65536, 32768) for d in inputs(16)[::2]]
    cases += [(_text(3 << 20, 7), "FULL_DYNAMIC", 65536, 32768), (_text(400_000, 8), "FULL_STATIC", 1000, 32768),
              (_text(300_000, 9), "FULL_DYNAMIC", 40000, 20000), (_text(300_000, 10), "FULL_DYNAMIC", 777, 0)]
    for data, strategy, chunk_len, hist_limit in cases:
        got = ctx.deflate(data, strategy, chunk_len=chunk_len, hist_limit=hist_limit)
        assert got == O.deflate(data, strategy, chunk_len, hist_limit), (env, len(data), chunk_len)
    strat = ndfl.Lz77Huffman(False, 5, 20, 3, 4096)
    data = _text(500_000, 11)
    assert ctx.deflate(data, strat) == O.deflate_lz(data, False, 5, 20, 3, 4096)
