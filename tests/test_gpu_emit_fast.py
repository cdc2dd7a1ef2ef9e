"""Record-replay fast emit pass (inflate_wave.hpp ndfl_inflate_emit_fast_kernel) and its hand-over
to the full emit kernel: the decode must equal the oracle's -- output, consumed bits, Reason of the
first error -- with the fast pass on (the default), off (NDFL_EMIT_FAST=0: the full kernel alone),
with no table records (NDFL_NO_BT=1: every chain reaching a Huffman block is listed for the full
kernel, which runs it from its start again -- stored blocks the fast pass already wrote before the
hand-over are rewritten identically), and with every stored-header alias counted on its own
(NDFL_NO_ALIAS=1; by default the count pass counts one of the candidates that share a stored
block's LEN position and BFINAL bit and copies its result and records to the others).  Streams: the config-4 mix (RLE_DYNAMIC), zlib -6 text (LZ77
distances, deferred copies across lanes and chains), zlib Z_FIXED text, the config-2 layout (stored
and fixed-Huffman pieces alternating), stored blocks alone, the reference's 39 known-answer tests and
corrupted streams.  Reference semantics: D/decomp/Open.java:83-618."""
import os
import random
import zlib

import numpy as np
import pytest

import corpus
import oracle_lib as O
from test_oracle_inflate import KAT

pytestmark = pytest.mark.gpu




def _env(name, value):
    old = os.environ.get(name)
    if value is None:
        os.environ.pop(name, None)
    else:
        os.environ[name] = str(value)
    return old


MODES = {"fast": {}, "full_only": {"NDFL_EMIT_FAST": "0"}, "hand_over": {"NDFL_NO_BT": "1"},
         "no_alias": {"NDFL_NO_ALIAS": "1"}}


@pytest.fixture(scope="module", params=list(MODES))
def ctx(request):
    """A context per mode: the library reads its switches when a context is created."""
    import ndfl
    olds = {k: _env(k, v) for k, v in MODES[request.param].items()}
    try:
        c = ndfl.Context(0)
    finally:
        for k, v in olds.items():
            _env(k, v)
    c.mode = request.param
    return c


def _zraw(data, level, strategy=zlib.Z_DEFAULT_STRATEGY):
    co = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
    return co.compress(data) + co.flush()


STREAMS = {}


def _streams():
    if not STREAMS:
        c4 = corpus.c4_mixed(4 << 20, seed=0x4F).numpy().tobytes()
        text = corpus.c3_text(2 << 20).numpy().tobytes()
        rng = np.random.default_rng(22)
        rnd = rng.integers(0, 256, 300_000, dtype=np.uint8).tobytes()
        _, c2raw, _ = corpus.c2_gzip(3 << 20, seed=0xC7)
        STREAMS.update({
            "rle_c4": O.deflate(c4),
            "zlib6_text": _zraw(text, 6),
            "zlib_fixed_text": _zraw(text, 6, zlib.Z_FIXED),
            "c2_layout": c2raw,
            "stored": _zraw(rnd, 0),
        })
    return STREAMS


def _same(ctx, comp):
    r, out, bits = ctx.inflate(comp)
    oreason, oout, obits = O.inflate(comp)
    assert (None if r is None else r.name) == oreason
    assert out == oout
    if oreason is None:
        assert bits == obits


@pytest.mark.parametrize("name", ["rle_c4", "zlib6_text", "zlib_fixed_text", "c2_layout", "stored"])
def test_emit_modes_match_oracle(ctx, name):
    _same(ctx, _streams()[name])


def test_emit_modes_known_answers(ctx):
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


@pytest.mark.parametrize("name", ["rle_c4", "c2_layout"])
def test_emit_modes_first_error(ctx, name):
    comp = _streams()[name]
    rng = np.random.default_rng(len(ctx.mode))
    for _ in range(4):
        bad = bytearray(comp)
        k = int(rng.integers(len(bad) // 8, len(bad)))
        bad[k] ^= 0x5A
        _same(ctx, bytes(bad))


@pytest.mark.parametrize("emit_fast", ["1", "0"])
def test_count_record_check_fails_loudly(emit_fast):
    """both emit kernels check every lane's segment against the count pass's record
    (the replay lands on the next segment's start having produced exactly the counted bytes).  With
    one record's byte count perturbed (NDFL_TEST_SEGFLIP) the decode must fail with NDFL_E_INTERNAL,
    not return wrong bytes or a data-format Reason."""
    import ndfl
    from ndfl import _lib
    olds = {k: _env(k, v) for k, v in {"NDFL_TEST_SEGFLIP": "1", "NDFL_EMIT_FAST": emit_fast}.items()}
    try:
        c = ndfl.Context(0)
    finally:
        for k, v in olds.items():
            _env(k, v)
    with pytest.raises(_lib.NdflError) as ei:
        c.inflate(_streams()["rle_c4"])
    assert ei.value.code == _lib.E_INTERNAL
