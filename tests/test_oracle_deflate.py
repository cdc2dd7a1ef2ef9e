"""Pins the CPU oracle's encoder.  The reference's own tests only round-trip the encoder
(T/DeflaterOutputStreamTest.java:109-115), so encoder bytes are pinned here by:
  (1) N-version agreement with tests/pyref_deflate.py (independent restatement, different algorithms),
  (2) the hand-derived known-answer tests of SURVEY.md App. A.8,
  (3) round-trip validity through Python zlib and through the oracle's own decoder,
  (4) equivalence of the exhaustive distance loop and the exact-prefix chain walk (FULL_*).
"""
import random
import zlib

import pytest

import oracle_lib as O
import pyref_deflate as P


def samples(seed):
    rng = random.Random(seed)
    out = [b"", b"\x00", b"ab", b"aaa", b"\x00" * 5000, bytes(range(256)) * 3]
    for n in [7, 100, 1000, 3000]:
        out.append(bytes(rng.randrange(256) for _ in range(n)))
        out.append(bytes(rng.choice(b"ab") for _ in range(n)))
        buf = bytearray()
        while len(buf) < n:
            buf += bytes([rng.randrange(4)]) * rng.randrange(1, 300)
        out.append(bytes(buf[:n]))
        words = [b"the ", b"of ", b"deflate ", b"gpu ", b"xgmi ", b"\n"]
        out.append(b"".join(rng.choice(words) for _ in range(n // 4))[:n])
    return out


@pytest.mark.parametrize("strategy", list(P.PRESETS))
def test_nversion_presets(strategy):
    for i, data in enumerate(samples(1)):
        for chunk_len, hist in [(65536, 32768), (1000, 32768), (97, 1), (500, 0), (256, 100)]:
            if strategy.startswith("FULL") and len(data) > 1200:
                continue
            a = O.deflate(data, strategy, chunk_len, hist)
            b = P.deflate(data, strategy, chunk_len, hist)
            assert a == b, (strategy, i, chunk_len, hist)


def test_nversion_custom_lz_params():
    rng = random.Random(5)
    for _ in range(20):
        data = bytes(rng.choice(b"abc") for _ in range(rng.randrange(0, 900)))
        min_run = rng.randrange(3, 10)
        max_run = rng.randrange(min_run, 259)
        min_dist = rng.randrange(1, 20)
        max_dist = rng.randrange(min_dist, 400)
        dyn = rng.random() < 0.5
        a = O.deflate_lz(data, dyn, min_run, max_run, min_dist, max_dist, 300, 32768)
        b = P.deflate(data, chunk_len=300, params=(dyn, min_run, max_run, min_dist, max_dist))
        assert a == b


@pytest.mark.parametrize("strategy", O.STRATEGIES)
def test_roundtrip_zlib_and_oracle(strategy):
    rng = random.Random(11)
    for data in samples(2) + [bytes(rng.randrange(256) for _ in range(150000)), b"\x07" * 200000]:
        if strategy.startswith("FULL") and len(data) > 20000:
            data = data[:20000]
        comp = O.deflate(data, strategy)
        assert zlib.decompress(comp, -15) == data
        reason, out, bits = O.inflate(comp)
        assert reason is None and out == data and (bits + 7) // 8 == len(comp)


def test_full_brute_equals_chain_walk():
    rng = random.Random(7)
    words = [bytes(rng.randrange(97, 101) for _ in range(rng.randrange(2, 6))) for _ in range(30)]
    for n in [0, 5, 300, 4000, 20000]:
        data = b" ".join(rng.choice(words) for _ in range(n // 3))[:n]
        for chunk_len, hist in [(65536, 32768), (3000, 32768), (1500, 700)]:
            for strat in ["FULL_DYNAMIC", "FULL_STATIC"]:
                assert O.deflate(data, strat, chunk_len, hist, brute=True) == O.deflate(data, strat, chunk_len, hist)


def test_package_merge_tie_order_kat():
    """chunk 0 of 1 MiB zeros has litHist {0:1, 256:1, 257:1, 285:254} and the
    reference's tie order gives 285->1, 257->2, 0->3, 256->3 (not 0->2)."""
    h = [0] * 286
    h[0], h[256], h[257], h[285] = 1, 1, 1, 254
    L = P.package_merge(h, 15)
    assert (L[285], L[257], L[0], L[256]) == (1, 2, 3, 3)
    h = [0] * 286
    h[256], h[258], h[285] = 1, 1, 254
    L = P.package_merge(h, 15)
    assert (L[285], L[256], L[258]) == (1, 2, 2)


def test_zeros_1mib_structure():
    data = b"\x00" * (1 << 20)
    comp = O.deflate(data)
    assert comp == P.deflate(data)
    bits = O.block_bits(data)
    assert len(bits) == 16
    assert len(set(bits[1:])) == 1          # chunks 1..15 identical blocks (different from chunk 0)
    assert bits[0] != bits[1]
    assert zlib.decompress(comp, -15) == data
    # bfinal only on the last block: first 3 bits of the stream = bfinal 0, btype 2
    assert comp[0] & 7 == 0b100


def test_empty_input():
    comp = O.deflate(b"")
    assert comp == P.deflate(b"")
    assert zlib.decompress(comp, -15) == b""
    assert comp[0] & 7 == 0b101            # bfinal=1, btype=2 (dynamic)


def test_gzip_config1_fixture():
    """Config 1: gzip of 1 MiB zeros named zeros_1MiB.bin, mtime 1700000000."""
    data = b"\x00" * (1 << 20)
    gz = O.gzip_compress(data, name=b"zeros_1MiB.bin", mtime=1700000000, os_=3, header_crc=True)
    hdr = bytes.fromhex("1f8b080a00f15365000" + "3" + "7a65726f735f314d69422e62696e00")
    assert gz[:len(hdr)] == hdr
    assert gz[len(hdr):len(hdr) + 2] == (zlib.crc32(hdr) & 0xFFFF).to_bytes(2, "little")
    assert gz[-8:] == bytes.fromhex("1cea38a700001000")
    assert zlib.decompress(gz, 31) == data
    reason, out, hd, end = O.gunzip(gz + b"trailing")
    assert reason is None and out == data and end == len(gz)
    assert hd["mtime"] == 1700000000 and hd["os"] == 3 and hd["has_header_crc"]


MULTI_SETS = [
    ["UNCOMPRESSED"],
    [P.PRESETS["RLE_DYNAMIC"], "UNCOMPRESSED"],
    ["UNCOMPRESSED", P.PRESETS["LITERAL_STATIC"]],
    [P.PRESETS["LITERAL_DYNAMIC"], P.PRESETS["RLE_STATIC"], "UNCOMPRESSED", P.PRESETS["FULL_DYNAMIC"]],
    [P.PRESETS["FULL_STATIC"], P.PRESETS["FULL_DYNAMIC"]],
]


@pytest.mark.parametrize("k", range(len(MULTI_SETS)))
def test_nversion_multistrategy(k):
    """MultiStrategy / Uncompressed: the oracle (closed-form Uncompressed lengths, D/comp/
    Uncompressed.java:22-26) against pyref (lengths measured by writing) and round trips."""
    subs = MULTI_SETS[k]
    rng = random.Random(40 + k)
    for data in samples(3)[:12] + [bytes(rng.randrange(256) for _ in range(70000)), b"\x05" * 70000]:
        for chunk_len, hist in [(65536, 32768), (700, 32768), (97, 1), (65535, 0)]:
            if any(s != "UNCOMPRESSED" and s[4] > 1 for s in subs) and len(data) > 5000:
                continue
            a = O.deflate_multi(data, subs, chunk_len, hist)
            b = P.deflate_multi(data, subs, chunk_len, hist)
            assert a == b, (k, len(data), chunk_len, hist)
            assert zlib.decompress(a, -15) == data


def test_uncompressed_preset_equals_single_multistrategy():
    for data in samples(4)[:10]:
        assert O.deflate(data, "UNCOMPRESSED") == O.deflate_multi(data, ["UNCOMPRESSED"])
        assert O.deflate(data, "RLE_DYNAMIC") == O.deflate_multi(data, [P.PRESETS["RLE_DYNAMIC"]])


@pytest.mark.parametrize("sub", [P.PRESETS["RLE_DYNAMIC"], P.PRESETS["FULL_STATIC"], P.PRESETS["LITERAL_DYNAMIC"],
                                 "UNCOMPRESSED"])
def test_nversion_binarysplit(sub):
    """BinarySplit: oracle against pyref (lengths measured by writing, the reference's position-0
    accumulation kept in both) and round trips."""
    rng = random.Random(60)
    datas = samples(5)[:14] + [bytes(rng.randrange(256) for _ in range(3000)) + b"\x00" * 3000]
    for data in datas:
        for chunk_len, hist, m in [(65536, 32768, 64), (700, 32768, 50), (1024, 0, 100), (300, 10, 1)]:
            if sub != "UNCOMPRESSED" and sub[4] > 1 and len(data) > 2000:
                continue
            a = O.deflate_binsplit(data, sub, m, chunk_len, hist)
            b = P.deflate_binsplit(data, sub, m, chunk_len, hist)
            assert a == b, (sub, len(data), chunk_len, hist, m)
            assert zlib.decompress(a, -15) == data


def test_strategy_ref_pinned_by_oracle():
    """tests/strategy_ref.py (the checker of the GPU plugin tests) agrees with the oracle's own
    MultiStrategy / BinarySplit drivers wherever both apply."""
    import random
    import strategy_ref as R
    rng = random.Random(3)
    data = b"".join(bytes([rng.randrange(3)]) * rng.randrange(1, 400) + rng.randbytes(rng.randrange(0, 300))
                    for _ in range(600))[:150_000]
    assert R.stream(data, R.LzLeaf("RLE_DYNAMIC")) == O.deflate(data, "RLE_DYNAMIC")
    assert R.stream(data, R.Multi(R.LzLeaf("RLE_DYNAMIC"), R.UncLeaf())) == \
        O.deflate_multi(data, [(1, 3, 258, 1, 1), "UNCOMPRESSED"])
    assert R.stream(data, R.Split(R.UncLeaf(), 1000)) == O.deflate_binsplit(data, "UNCOMPRESSED", 1000)
    assert R.stream(data, R.Split(R.LzLeaf("RLE_DYNAMIC"), 2000)) == O.deflate_binsplit(data, (1, 3, 258, 1, 1), 2000)
