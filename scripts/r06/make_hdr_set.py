"""Block headers of a real stream for the table-build microbenchmark (scripts/r06/build_bench.hip):
the oracle's RLE_DYNAMIC encoding of N bytes of the config-4 corpus, every block's header parsed here
(RFC 1951 3.2.7 / D/decomp/Open.java:336-431) into the decoder's S.lens layout -- literal/length
lengths at [0, 288), distance lengths at [288, 320) -- plus (btype, numlit, numdist).
Usage: python scripts/r06/make_hdr_set.py OUT.bin [MiB]   (measurement tooling, not product code)"""
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402
import corpus  # noqa: E402

CLO = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class Bits:
    def __init__(self, b, pos):
        self.v = int.from_bytes(b, "little")
        self.p = pos

    def get(self, n):
        x = (self.v >> self.p) & ((1 << n) - 1)
        self.p += n
        return x


def canon(lens):
    """code (MSB-first int) -> (symbol, length) of a canonical code."""
    bl = [0] * 16
    for l in lens:
        if l:
            bl[l] += 1
    code, nxt = 0, [0] * 16
    for l in range(1, 16):
        code = (code + bl[l - 1]) << 1 if l > 1 else 0
        nxt[l] = code
    out = {}
    for s, l in enumerate(lens):
        if l:
            out[(nxt[l], l)] = s
            nxt[l] += 1
    return out


def read_sym(r, table):
    c, l = 0, 0
    while True:
        c = (c << 1) | r.get(1)
        l += 1
        if (c, l) in table:
            return table[(c, l)]


def parse(stream, pos):
    r = Bits(stream, pos)
    r.get(1)
    bt = r.get(2)
    if bt != 2:
        return None
    nl, nd, nc = r.get(5) + 257, r.get(5) + 1, r.get(4) + 4
    cl = [0] * 19
    for i in range(nc):
        cl[CLO[i]] = r.get(3)
    t = canon(cl)
    vals = []
    while len(vals) < nl + nd:
        s = read_sym(r, t)
        if s < 16:
            vals.append(s)
        elif s == 16:
            vals += [vals[-1]] * (r.get(2) + 3)
        elif s == 17:
            vals += [0] * (r.get(3) + 3)
        else:
            vals += [0] * (r.get(7) + 11)
    lens = vals[:nl] + [0] * (288 - nl) + vals[nl:nl + nd] + [0] * (32 - nd)
    return bt, nl, nd, bytes(lens)


def main():
    out = sys.argv[1]
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    data = corpus.c4_mixed(mib << 20, seed=0xC4).numpy().tobytes()
    stream = O.deflate(data, "RLE_DYNAMIC")
    seams, acc = [], 0
    for v in O.block_bits(data, "RLE_DYNAMIC"):
        seams.append(acc)
        acc += v
    recs = []
    for p in seams:
        h = parse(stream[p // 8:p // 8 + 2048], p % 8)
        if h:
            recs.append(struct.pack("<4I", h[0], h[1], h[2], 0) + h[3])
    open(out, "wb").write(b"".join(recs))
    print(f"{len(recs)} dynamic headers of {len(seams)} blocks -> {out}")


if __name__ == "__main__":
    main()
