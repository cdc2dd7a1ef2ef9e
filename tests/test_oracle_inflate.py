"""Pins the CPU oracle's decoder to the reference's own known-answer tests.

Mirrors T/InflaterInputStreamTest.java: the 39 deterministic tests (fixture generated from that
file by tests/golden/make_inflate_kat.py), its three randomized generators restated with a seeded
RNG (:131-163, :166-208, :306-338), and Python zlib as an independent decoder/encoder for valid
streams.
"""
import json
import os
import random
import zlib

import pytest

import oracle_lib as O

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "inflate_kat.json")))["tests"]


def check(bits, expect_hex, expect_reason, rng):
    """The reference harness test()/testFail() (T/InflaterInputStreamTest.java:519-593)."""
    for pad_mode in range(3):
        data = O.bits_to_bytes(bits, pad_mode, rng)
        reason, out, consumed = O.inflate(data)
        if expect_reason is None:
            assert reason is None, reason
            assert out == bytes.fromhex(expect_hex)
            # endExactly: the underlying stream is exactly at EOF afterwards (:557-558)
            assert (consumed + 7) // 8 == len(data)
        else:
            assert reason == expect_reason


@pytest.mark.parametrize("kat", KAT, ids=[k["name"] for k in KAT])
def test_known_answer(kat):
    check(kat["bits"], kat["expect_hex"], kat["expect_reason"], random.Random(kat["line"]))


def quasi_log_len(rng, n):
    """`int len = rand.nextInt(n); if (len > 0) { len = 1 << (len-1); len |= rand.nextInt(len); }`"""
    ln = rng.randrange(n)
    if ln > 0:
        ln = 1 << (ln - 1)
        ln |= rng.randrange(ln)
    return ln


def lsb_bits(v, n):
    return "".join(str((v >> k) & 1) for k in range(n))


LSB8 = [lsb_bits(b, 8) for b in range(256)]
MSB_LIT = [format(b + 48, "08b") if b < 144 else format(b - 144 + 400, "09b") for b in range(256)]


def test_uncompressed_random():
    rng = random.Random(131)
    for _ in range(100):
        nblocks = rng.randrange(30) + 1
        bits, out = [], bytearray()
        for j in range(nblocks):
            bits.append("0" if j + 1 < nblocks else "1")
            bits.append("00")
            bits.append("".join(str(rng.randrange(2)) for _ in range(5)))
            ln = quasi_log_len(rng, 17)
            bits.append(lsb_bits(ln | ((~ln) << 16) & 0xFFFFFFFF, 32))
            data = rng.randbytes(ln)
            out += data
            bits.append("".join(LSB8[b] for b in data))
        check("".join(bits), out.hex(), None, rng)


def test_uncompressed_random_and_short_fixed_huffman():
    rng = random.Random(166)
    for _ in range(100):
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
                bits += "10" + "111111111" + "0000000"   # literal 0xFF, end of block (19 bits)
                out.append(0xFF)
        check(bits, out.hex(), None, rng)


def test_fixed_huffman_literals_random():
    rng = random.Random(306)
    for _ in range(100):
        nblocks = rng.randrange(100) + 1
        bits, out = [], bytearray()
        for j in range(nblocks):
            bits.append("0" if j + 1 < nblocks else "1")
            bits.append("10")
            ln = quasi_log_len(rng, 16)
            for _ in range(ln):
                b = rng.randrange(256)
                bits.append(MSB_LIT[b])
                out.append(b)
            bits.append("0000000")
        check("".join(bits), out.hex(), None, rng)


def corpus(rng, n):
    words = [bytes(rng.randrange(97, 123) for _ in range(rng.randrange(2, 9))) for _ in range(300)]
    out = bytearray()
    while len(out) < n:
        r = rng.random()
        if r < 0.6:
            out += rng.choice(words) + b" "
        elif r < 0.7:
            out += bytes([rng.randrange(256)]) * rng.randrange(1, 600)
        else:
            out += bytes(rng.randrange(256) for _ in range(rng.randrange(1, 40)))
    return bytes(out[:n])


@pytest.mark.parametrize("level", [0, 1, 6, 9])
def test_zlib_streams_decode(level):
    """Python zlib 1.2.11 as an independent encoder: the oracle must reproduce its input and
    stop exactly at the end of the raw DEFLATE stream."""
    rng = random.Random(level)
    for n in [0, 1, 2, 100, 5000, 70000, 200000]:
        data = corpus(rng, n)
        co = zlib.compressobj(level, zlib.DEFLATED, -15, 9)
        comp = co.compress(data) + co.flush()
        reason, out, bits = O.inflate(comp + b"\xAB\xCD")   # trailing bytes must be ignored
        assert reason is None
        assert out == data
        assert (bits + 7) // 8 == len(comp)


def test_reserved_symbols_and_quirks():
    # B.3.4: a single distance code of length 1 at index 31 cannot be padded -> under-full.
    # Dynamic header: HLIT=0 (257), HDIST=31 (32 codes), code-length code {1:1, 0:1} complete.
    # Build via a bit string: clc lengths in order 16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1 -> give 0 and 1 length 1
    clc = [0] * 19
    clc[3] = 1     # symbol 0
    clc[17] = 1    # symbol 1
    hdr = "1" + "01" + lsb_bits(0, 5) + lsb_bits(31, 5) + lsb_bits(14, 4) + "".join(lsb_bits(x, 3) for x in clc[:18])
    # codes: symbol 0 -> '0', symbol 1 -> '1'
    lens = [0] * 257 + [0] * 32
    lens[0] = 1
    lens[256] = 1
    lens[257 + 31] = 1
    body = "".join("1" if x == 1 else "0" for x in lens)
    reason, _, _ = O.inflate(O.bits_to_bytes(hdr + body + "0" * 16))
    assert reason == "HUFFMAN_CODE_UNDER_FULL"
    # 286/287 accepted in the header (HLIT up to 31): a code using them is legal until used.
    lens = [0] * 288 + [0]
    lens[0] = 1
    lens[287] = 1
    hdr2 = "1" + "01" + lsb_bits(31, 5) + lsb_bits(0, 5) + lsb_bits(14, 4) + "".join(lsb_bits(x, 3) for x in clc[:18])
    # lens[256] == 0 -> END_OF_BLOCK_CODE_ZERO_LENGTH
    body = "".join("1" if x == 1 else "0" for x in lens)
    reason, _, _ = O.inflate(O.bits_to_bytes(hdr2 + body + "0" * 16))
    assert reason == "END_OF_BLOCK_CODE_ZERO_LENGTH"


def reserved_symbol_streams():
    """(name, stream, expected output or None, Reason, symbol) for each reserved symbol the reference names
    in its message ("Reserved run length symbol: " + sym, "Reserved distance symbol: " + sym,
    D/decomp/Open.java:516, 550, 659, 674): the four fixed-Huffman KATs of T/InflaterInputStreamTest.java
    (the symbol is in their names) and two dynamic blocks -- a code that uses length symbol 287, and a
    single one-bit distance code, which the reference pads with symbol 31 (:398-425) and a 1 bit then
    decodes (lit code {65: 1, 256: 2, 287 or 257: 2}; code-length code {0: 1, 1: 2, 2: 2})."""
    out = []
    for k in KAT:
        if k["expect_reason"] in ("RESERVED_LENGTH_SYMBOL", "RESERVED_DISTANCE_SYMBOL"):
            sym = int(k["name"].rsplit("Code", 1)[1])
            out.append((k["name"], O.bits_to_bytes(k["bits"], 0, random.Random(0)), None, k["expect_reason"], sym))
    clc = [0] * 19
    clc[3], clc[17], clc[15] = 1, 2, 2            # code-length symbols 0, 1, 2 (positions in CLO)
    enc = {0: "0", 1: "10", 2: "11"}
    for name, hlit, lsym, dist_len, data_bits, reason, sym in [
            ("dynamicLengthSymbol287", 31, 287, 0, "0" + "11", "RESERVED_LENGTH_SYMBOL", 287),
            ("dynamicPaddedDistanceSymbol31", 1, 257, 1, "0" + "11" + "1", "RESERVED_DISTANCE_SYMBOL", 31)]:
        nlit = hlit + 257
        lens = [0] * nlit + [dist_len]
        lens[65], lens[256], lens[lsym] = 1, 2, 2
        bits = ("1" + "01" + lsb_bits(hlit, 5) + lsb_bits(0, 5) + lsb_bits(14, 4)
                + "".join(lsb_bits(x, 3) for x in clc[:18]) + "".join(enc[x] for x in lens) + data_bits)
        out.append((name, O.bits_to_bytes(bits + "0" * 16), b"A", reason, sym))
    return out


def test_oracle_reports_the_reserved_symbol():
    streams = reserved_symbol_streams()
    assert len(streams) == 6
    for name, data, want, reason, sym in streams:
        r, out, _ = O.inflate(data)
        assert (r, O.error_symbol()) == (reason, sym), name
        assert want is None or out == want, name
    assert O.inflate(O.deflate(b"abc"))[0] is None and O.error_symbol() == -1


@pytest.mark.parametrize("strategy,chunk_len", [("RLE_DYNAMIC", 65536), ("FULL_DYNAMIC", 4096),
                                                ("UNCOMPRESSED", 65536), ("RLE_DYNAMIC", 300)])
def test_scan_headers_finds_every_chain_start(strategy, chunk_len):
    # or_scan_headers (the GPU header finder's expected accepted set, tests/test_gpu_headers.py):
    # every interior block boundary of an encoder's stream (but the final block's) is found, in
    # ascending order, and a decode started at a found position reads past its header
    rng = random.Random(7)
    data = b"".join(bytes([rng.randrange(4)]) * rng.randrange(1, 400) + rng.randbytes(rng.randrange(0, 90))
                    for _ in range(1500))
    comp = O.deflate(data, strategy, chunk_len=chunk_len)
    bb = O.block_bits(data, strategy, chunk_len)
    starts, acc = [], 0
    for b in bb[:-1]:
        acc += b
        starts.append(acc)
    found = O.scan_headers(comp)
    assert found == sorted(found)
    assert set(starts[:-1]) <= set(found)
    for p in found[:40]:
        r, out, bits = O.inflate_range(comp, start_bit=p, out_cap=4 * len(data) + 65536)
        assert bits > p + 3
