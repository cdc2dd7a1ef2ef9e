"""The decoder's header finder + strict stage against the oracle, header by header.

The GPU decoder starts its decode chains at the block headers that its finder (every bit position,
cheap masks + the code-length code's Kraft test) and strict stage (the reference's own header checks,
D/decomp/Open.java:232-241 / :336-431) accept.  A header lost there costs parallelism, not output
bytes (the chain before it decodes through it), so the output tests cannot see it; this test
compares the accepted set itself (ndfl_inflate_headers) with the oracle's scan of every bit
position (or_scan_headers, the same checks restated on the CPU).  Exact equality, except in 64 KiB
segments holding more than SEG_CAP (256) accepted headers, where the decoder keeps 256 of them.

Streams: the config-4 mix (its run segments hold ~17 headers per 64 KiB segment, where round 4's
3- and 5-wave strict builds lost headers), a stored-block stream whose data repeats a 32-bit
pattern that passes the finder's filters every 32 bits (more than the finder's 1,024-entry LDS
list per workgroup, and more than its default survivor list), tiny blocks (chunk_len 64: segments
over SEG_CAP), zlib level 6 (LZ77 + dynamic blocks), and the config-2 mix of stored and fixed
blocks.
"""
import zlib

import numpy as np
import pytest

import corpus
import oracle_lib as O

pytestmark = pytest.mark.gpu

SEG_BITS = 65536 * 8
SEG_CAP = 256


@pytest.fixture(scope="module")
def ctx():
    import ndfl
    return ndfl.Context(0)


def check_headers(ctx, comp, min_true=None):
    exp = O.scan_headers(comp)
    got, stats = ctx.inflate_headers(comp)
    assert got == sorted(got)
    segs_e, segs_g = {}, {}
    for p in exp:
        segs_e.setdefault(p // SEG_BITS, []).append(p)
    for p in got:
        segs_g.setdefault(p // SEG_BITS, []).append(p)
    over = 0
    for k in sorted(set(segs_e) | set(segs_g)):
        e, g = segs_e.get(k, []), segs_g.get(k, [])
        if len(e) <= SEG_CAP:
            if e != g:
                lost, extra = sorted(set(e) - set(g)), sorted(set(g) - set(e))
                raise AssertionError(f"segment {k}: {len(lost)} headers lost (first {lost[:8]}), "
                                     f"{len(extra)} extra (first {extra[:8]})")
        else:
            over += 1
            assert len(g) == SEG_CAP and set(g) <= set(e), f"segment {k}: capped list not a subset"
    assert stats[1] == len(exp), (stats, len(exp))     # accepted before the cap
    assert stats[2] == over
    assert stats[3] == 0                               # no survivor dropped
    if min_true is not None:
        assert set(min_true) <= set(exp)
    return exp, got, stats


def block_starts(data, strategy="RLE_DYNAMIC", chunk_len=65536):
    bb = O.block_bits(data, strategy, chunk_len)
    starts = np.concatenate([[0], np.cumsum(np.array(bb, dtype=np.uint64))[:-1]]).astype(np.uint64)
    return [int(x) for x in starts[1:-1]]          # interior headers (the first is bit 0, the last final)


def test_c4_mix_headers(ctx):
    data = corpus.c4_mixed(24 << 20).numpy().tobytes()
    comp = ctx.deflate(data)
    exp, got, stats = check_headers(ctx, comp, min_true=block_starts(data))
    dense = max(np.bincount(np.array(exp, dtype=np.uint64) // SEG_BITS))
    assert dense >= 17                                  # the run segments are in the sample
    assert len(exp) >= len(data) // 65536 - 2


def test_periodic_stored_data_overflows_the_finder_lists(ctx):
    # 0xe9240004 LSB first: BFINAL 0, BTYPE 2, HLIT 0, HDIST 0, HCLEN 0, four 2-bit code-length
    # code lengths (complete): a finder survivor every 32 bits of the stored data
    pat = bytes.fromhex("040024e9")
    data = pat * ((3 << 20) // 4)
    comp = O.deflate(data, "UNCOMPRESSED")
    exp, got, stats = check_headers(ctx, comp)
    assert stats[0] > 16 * (len(comp) * 8 // 131072)   # past 1,024 per finder workgroup on average
    assert stats[0] > len(comp) * 8 // 256 + 65536       # past the default survivor list
    assert len(exp) >= len(data) // 65535 - 2           # the stored headers themselves
    r, out, bits = ctx.inflate(comp)
    assert r is None and out == data


def test_tiny_blocks_over_the_segment_cap(ctx):
    rng = np.random.default_rng(5)
    data = (rng.integers(0, 4, 1 << 20, dtype=np.uint8) * 7).tobytes()
    comp = O.deflate(data, "RLE_DYNAMIC", chunk_len=64)
    exp, got, stats = check_headers(ctx, comp)
    assert stats[2] > 0


def test_zlib_and_config2_headers(ctx):
    text = corpus.c3_text(4 << 20).numpy().tobytes()
    raw = zlib.compress(text, 6)[2:-4]
    check_headers(ctx, raw)
    gz, raw2, _ = corpus.c2_gzip(8 << 20)
    check_headers(ctx, raw2)
