"""The partitioned header finder (inflate_kernels.hip: ndfl_inflate_find_sparse_kernel): on long
streams the range is cut into partitions and each is scanned only up to its first accepted block
header.  NDFL_FIND_PART_BITS forces partitions of that many bits on small streams here, so every
path of the decoder sees chains that span many blocks, and partitions with no header at all.

Each decode is compared with the oracle (output, consumed bits, Reason of the first error):
RLE_DYNAMIC streams of the config-4 mix, zlib streams (fixed, dynamic and stored blocks of any
length), an LZ77 (FULL_DYNAMIC) stream, a corrupted stream, range decodes with a window, and the
streaming inflater's partial-input batches.  Reference semantics: D/decomp/Open.java:83-435.
"""
import io
import os
import zlib

import numpy as np
import pytest

import corpus
import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ndfl():
    import ndfl as M
    return M


@pytest.fixture(scope="module")
def ctx(ndfl):
    return ndfl.Context(0)


@pytest.fixture(params=[262144, 524288, 2097152])
def parts(request):
    old = os.environ.get("NDFL_FIND_PART_BITS")
    os.environ["NDFL_FIND_PART_BITS"] = str(request.param)
    yield request.param
    if old is None:
        del os.environ["NDFL_FIND_PART_BITS"]
    else:
        os.environ["NDFL_FIND_PART_BITS"] = old


def _zraw(data, level, strategy=zlib.Z_DEFAULT_STRATEGY):
    co = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
    return co.compress(data) + co.flush()


def _streams():
    c4 = corpus.c4_mixed(6 << 20).numpy().tobytes()
    text = corpus.c3_text(3 << 20).numpy().tobytes()
    rng = np.random.default_rng(9)
    mixed = corpus.mixed_bytes(3 << 20, 17)
    return {
        "rle_c4": O.deflate(c4),
        "zlib6_text": _zraw(text, 6),
        "zlib1_c4": _zraw(c4, 1),
        "zlib_fixed_text": _zraw(text, 6, zlib.Z_FIXED),
        "stored_mix": _zraw(rng.integers(0, 256, 2 << 20, dtype=np.uint8).tobytes(), 0),
        "full_dynamic": O.deflate(mixed[:1 << 20], "FULL_DYNAMIC"),
    }


STREAMS = None


def _get():
    global STREAMS
    if STREAMS is None:
        STREAMS = _streams()
    return STREAMS


@pytest.mark.parametrize("name", ["rle_c4", "zlib6_text", "zlib1_c4", "zlib_fixed_text", "stored_mix", "full_dynamic"])
def test_partitioned_finder_matches_oracle(ctx, parts, name):
    comp = _get()[name]
    r, out, bits = ctx.inflate(comp)
    oreason, oout, obits = O.inflate(comp)
    assert oreason is None
    assert r is None and bits == obits and out == oout


def test_partitioned_finder_first_error(ctx, parts):
    comp = bytearray(_get()["rle_c4"])
    rng = np.random.default_rng(parts)
    for _ in range(3):
        bad = bytearray(comp)
        k = int(rng.integers(len(bad) // 4, len(bad)))
        bad[k] ^= 0x5A
        r, out, bits = ctx.inflate(bytes(bad))
        oreason, oout, obits = O.inflate(bytes(bad))
        assert (None if r is None else r.name) == oreason
        assert out == oout
        if oreason is not None:
            assert bits == obits


def test_partitioned_finder_range_with_window(ctx, ndfl, parts):
    comp = _get()["zlib6_text"]
    r0, full, bits = ctx.inflate(comp)
    assert r0 is None
    # a block boundary well inside the stream: decode [b, end) with the 32 KiB before it as window
    bnd = ctx.inflate_sync_raw(*_host(ndfl, comp), len(comp) * 4, 8 << 20, 0)
    assert bnd is not None
    oreason, head, _ = O.inflate_range(comp, 0, bnd)
    assert oreason is None
    win = head[-32768:]
    reason, tail, tbits = O.inflate_range(comp, bnd, None, win)
    import ctypes
    src = ctypes.create_string_buffer(comp, len(comp))
    cap = len(full) + 65536
    out = ctypes.create_string_buffer(win, len(win) + cap)
    rc, olen, cbits = ctx.inflate_range_raw(ctypes.addressof(src), len(comp), bnd, None, ctypes.addressof(out),
                                            len(win), cap, 0)
    assert rc == 0 and cbits == tbits and out.raw[len(win):len(win) + olen] == tail == full[len(head):]


def _host(ndfl, comp):
    import ctypes
    buf = ctypes.create_string_buffer(comp, len(comp))
    _host.keep = buf
    return ctypes.addressof(buf), len(comp)


def test_partitioned_finder_streaming_batches(ndfl, ctx, parts):
    comp = _get()["rle_c4"]
    s = ndfl.InflaterInputStream(io.BytesIO(comp), context=ctx)
    s._batch = 1 << 20                        # partial-input batches of 1 MiB
    assert s.readall() == O.inflate(comp)[1]
