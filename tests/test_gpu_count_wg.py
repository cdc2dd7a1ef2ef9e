"""Workgroup rounds of the count pass (inflate_wg.hpp, NDFL_COUNT_W = W waves per chain): the
decode must equal the oracle's -- output, consumed bits, Reason of the first error -- for W = 2, 4
and 8 (rounds of 64W lane segments, waves whose lane 0 verifies from the previous wave's exit;
chains of many blocks on the fixed-Huffman and small-block streams, whose later headers are parsed
in the kernel and whose rounds' records are written per wave and replayed by the emit pass from
SegMeta::rs).  Streams: the config-4 mix (RLE_DYNAMIC: text, binary, random data in
phase-mapped rounds, runs), zlib -6 text (LZ77 distances), zlib Z_FIXED text (phase-locked
fixed-Huffman literals), stored blocks, FULL_DYNAMIC, random bytes alone, the reference's 39
known-answer tests and corrupted streams.  Reference semantics: D/decomp/Open.java:83-618."""
import random
import zlib

import numpy as np
import pytest

import corpus
import knobs
import oracle_lib as O
from test_oracle_inflate import KAT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[2, 4, 8])
def ctx(request):
    c = knobs.context(NDFL_COUNT_W=request.param)
    c.wg = request.param
    return c


def _zraw(data, level, strategy=zlib.Z_DEFAULT_STRATEGY):
    co = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
    return co.compress(data) + co.flush()


STREAMS = {}


def _streams():
    if not STREAMS:
        c4 = corpus.c4_mixed(4 << 20, seed=0x4C).numpy().tobytes()
        text = corpus.c3_text(2 << 20).numpy().tobytes()
        rng = np.random.default_rng(21)
        rnd = rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
        STREAMS.update({
            "rle_c4": O.deflate(c4),
            "zlib6_text": _zraw(text, 6),
            "zlib_fixed_text": _zraw(text, 6, zlib.Z_FIXED),
            "stored_mix": _zraw(rnd[:300_000], 0),
            "full_dynamic": O.deflate(corpus.mixed_bytes(1 << 20, 23), "FULL_DYNAMIC"),
            "random_rle": O.deflate(rnd),
            "small_blocks": O.deflate(c4[:400_000], "RLE_DYNAMIC", chunk_len=4096),
        })
    return STREAMS


def _same(ctx, comp):
    r, out, bits = ctx.inflate(comp)
    oreason, oout, obits = O.inflate(comp)
    assert (None if r is None else r.name) == oreason
    assert out == oout
    if oreason is None:
        assert bits == obits


@pytest.mark.parametrize("name", ["rle_c4", "zlib6_text", "zlib_fixed_text", "stored_mix", "full_dynamic",
                                  "random_rle", "small_blocks"])
def test_workgroup_rounds_match_oracle(ctx, name):
    _same(ctx, _streams()[name])


def test_workgroup_rounds_known_answers(ctx):
    for kat in KAT:
        rng = random.Random(kat["line"])
        for pad in range(3):
            data = O.bits_to_bytes(kat["bits"], pad, rng)
            r, out, bits = ctx.inflate(data)
            if kat["expect_reason"] is None:
                assert r is None and out == bytes.fromhex(kat["expect_hex"]), kat["name"]
                assert (bits + 7) // 8 == len(data)
            else:
                assert r is not None and r.name == kat["expect_reason"], kat["name"]


def test_workgroup_rounds_first_error(ctx):
    comp = _streams()["rle_c4"]
    rng = np.random.default_rng(ctx.wg)
    for _ in range(4):
        bad = bytearray(comp)
        k = int(rng.integers(len(bad) // 8, len(bad)))
        bad[k] ^= 0x5A
        _same(ctx, bytes(bad))
