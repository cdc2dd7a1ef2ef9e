"""GPU decode of dynamic blocks whose codes are much longer than the decoder's primary tables
(10-bit literal/length, 8-bit distance, csrc/hip/inflate_wave.hpp).  Codes longer than the primary
go to per-prefix second-level tables when they fit the extension area (320 / 64 words), otherwise
to the canonical slow path; both must decode exactly as the oracle does (D/decomp/Open.java:446-618).

The blocks are written here from chosen code lengths (every length sent as a plain code-length
symbol under a 4-bit code-length code), with random symbol sequences that use every code.
"""
import random

import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

CL_ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
LEN_BASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
            227, 258]
LEN_EXTRA = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DIST_BASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
             4097, 6145, 8193, 12289, 16385, 24577]
DIST_EXTRA = [0, 0, 0, 0] + [k // 2 for k in range(2, 28)]


def canonical(lens):
    """Canonical codes (MSB-first values) of a list of code lengths."""
    codes, code = [0] * len(lens), 0
    for ln in range(1, 16):
        for s, l in enumerate(lens):
            if l == ln:
                codes[s] = code
                code += 1
        code <<= 1
    return codes


class Bits:
    def __init__(self):
        self.v, self.n = 0, 0

    def put(self, val, n):              # LSB first
        self.v |= val << self.n
        self.n += n

    def huff(self, code, n):            # Huffman codes go MSB first
        self.put(int(format(code, f"0{n}b")[::-1], 2), n)

    def bytes(self):
        return self.v.to_bytes((self.n + 7) // 8, "little")


def dynamic_block(lit_lens, dist_lens, rng, ntok=6000):
    assert len(lit_lens) == 286 and len(dist_lens) == 30 and lit_lens[256]
    w = Bits()
    w.put(1, 1)                         # final
    w.put(2, 2)                         # dynamic
    w.put(286 - 257, 5)
    w.put(30 - 1, 5)
    w.put(19 - 4, 4)
    cl_lens = [4 if s < 16 else 0 for s in range(19)]
    for s in CL_ORDER:
        w.put(cl_lens[s], 3)
    cl_codes = canonical(cl_lens)
    for l in lit_lens + dist_lens:
        w.huff(cl_codes[l], 4)
    lc, dc = canonical(lit_lens), canonical(dist_lens)
    lits = [s for s in range(256) if lit_lens[s]]
    runs = [s for s in range(257, 286) if lit_lens[s]]
    dists = [s for s in range(30) if dist_lens[s]]
    out = 0
    # every code at least once, then a random mix (literals first so copies have a source)
    seq = [("L", s) for s in lits] + [("R", s) for s in runs] + [("D", s) for s in dists]
    seq += [(rng.choice("LLLRD"), None) for _ in range(ntok)]
    for kind, s in seq:
        if kind == "L" or out < 300:
            s = s if kind == "L" and s is not None else rng.choice(lits)
            w.huff(lc[s], lit_lens[s])
            out += 1
            continue
        r = s if kind == "R" and s is not None else rng.choice(runs)
        d = s if kind == "D" and s is not None else rng.choice(dists)
        while DIST_BASE[d] > out:
            d = rng.choice(dists)
        w.huff(lc[r], lit_lens[r])
        re = rng.randrange(1 << LEN_EXTRA[r - 257]) if LEN_EXTRA[r - 257] else 0
        w.put(re, LEN_EXTRA[r - 257])
        w.huff(dc[d], dist_lens[d])
        de = rng.randrange(min(1 << DIST_EXTRA[d], out - DIST_BASE[d] + 1)) if DIST_EXTRA[d] else 0
        w.put(de, DIST_EXTRA[d])
        out += LEN_BASE[r - 257] + re
    w.huff(lc[256], lit_lens[256])
    return w.bytes()


def long_lit_lens():
    """3 short codes (1, 2, 3 bits) and 283 long ones filling the last eighth of the code space:
    254 of 11 bits, 3 of 14, 26 of 15 (16*254 + 2*3 + 26 = 4096 units of 2^-15).  Second-level
    entries: 127 prefixes x 2 + one prefix x 32 = 286 of the 320-word extension area."""
    lens = [1, 2, 3] + [11] * 254 + [14] * 3 + [15] * 26
    # the short ones are the literals 'A' 'B' 'C'; end of block gets a 15-bit code
    order = [65, 66, 67] + [s for s in range(286) if s not in (65, 66, 67, 256)] + [256]
    out = [0] * 286
    for s, l in zip(order, lens):
        out[s] = l
    return out


def kraft(lens):
    return sum(2.0 ** -l for l in lens if l)


@pytest.fixture(scope="module")
def ctx():
    import torch
    import ndfl
    c = ndfl.Context(0)
    c.set_stream(torch.cuda.current_stream().cuda_stream)
    return c


@pytest.mark.parametrize("dist_kind", ["fallback_15bit", "two_level_12bit"])
def test_long_codes_decode_like_oracle(ctx, dist_kind):
    lit = long_lit_lens()
    assert abs(kraft(lit) - 1.0) < 1e-12
    if dist_kind == "fallback_15bit":
        # 1..14, 15, 15: the prefix holding the two 15-bit codes needs a 128-entry table (> 64)
        dist = list(range(1, 15)) + [15, 15] + [0] * 14
    else:
        dist = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 12] + [0] * 17
    assert abs(kraft(dist) - 1.0) < 1e-12
    rng = random.Random(7 if dist_kind == "fallback_15bit" else 11)
    for rep in range(3):
        comp = dynamic_block(lit, dist, rng)
        oreason, oout, obits = O.inflate(comp)
        assert oreason is None, oreason
        r, out, bits = ctx.inflate(comp)
        assert r is None and out == oout and bits == obits
        # and as one of many blocks: a stored prefix moves it off bit 0 (other lanes/phases)
        pre = b"\x00\x05\x00\xfa\xffhello"
        r, out, bits = ctx.inflate(pre + comp)
        oreason, oout, obits = O.inflate(pre + comp)
        assert oreason is None and r is None and out == oout and bits == obits
