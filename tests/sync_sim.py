"""Diagnostic (not a test): how far a speculative decode from an arbitrary bit position runs before
it meets a true token boundary, per data type -- the count pass's verify succeeds when that happens
within a lane segment.  Encodes one 64 KiB block with the oracle (RLE_DYNAMIC), decodes its tokens
in Python from the data start (true boundaries), then from 400 random bit positions.

    python tests/sync_sim.py            # text, LE-int32 and byte-soup blocks of the c4 generators
"""
import os
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import corpus  # noqa: E402
import oracle_lib as O  # noqa: E402

ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


def canon(lens):
    d, code = {}, 0
    for L in range(1, 16):
        for s, l in enumerate(lens):
            if l == L:
                d[(L, code)] = s
                code += 1
        code <<= 1
    return d


def header(bits):
    pos = [0]

    def get(n):
        v = sum(bits[pos[0] + i] << i for i in range(n))
        pos[0] += n
        return v
    get(1)
    assert get(2) == 2
    hlit, hdist, hclen = get(5) + 257, get(5) + 1, get(4) + 4
    cl = [0] * 19
    for i in range(hclen):
        cl[ORDER[i]] = get(3)
    t = canon(cl)
    lens = []
    while len(lens) < hlit + hdist:
        c = L = 0
        while (L, c) not in t:
            c = (c << 1) | get(1)
            L += 1
        s = t[(L, c)]
        if s < 16:
            lens.append(s)
        elif s == 16:
            lens += [lens[-1]] * (get(2) + 3)
        elif s == 17:
            lens += [0] * (get(3) + 3)
        else:
            lens += [0] * (get(7) + 11)
    return lens[:hlit], lens[hlit:], pos[0]


def sync_distances(block, samples=400, seed=1):
    c = O.deflate(block)
    bits = [(c[p >> 3] >> (p & 7)) & 1 for p in range(len(c) * 8)]
    nb = len(bits)
    lit, dist, start = header(bits)
    LT, DT = canon(lit), canon(dist)

    def sym(p, T):
        cd = L = 0
        while (L, cd) not in T:
            if p + L >= nb or L > 15:
                return None, p
            cd = (cd << 1) | bits[p + L]
            L += 1
        return T[(L, cd)], p + L

    def tok(p):
        s, p = sym(p, LT)
        if s is None or s == 256 or s > 285:
            return None
        if s < 256:
            return p
        k = s - 257
        p += 0 if k < 8 or k == 28 else (k >> 2) - 1
        d, p = sym(p, DT)
        if d is None or d >= 30:
            return None
        return p + (0 if d < 4 else (d >> 1) - 1)
    B, p = set(), start
    while p is not None:
        B.add(p)
        end, p = p, tok(p)
    rng = random.Random(seed)
    out = []
    for _ in range(samples):
        s = p = rng.randrange(start, end - 2000)
        d = None
        while p is not None and p - s < 2000:
            if p in B:
                d = p - s
                break
            p = tok(p)
        out.append(d if d is not None else 1 << 30)
    return sorted(out)


if __name__ == "__main__":
    g = torch.Generator().manual_seed(3)
    b = corpus._binary(g, 256 << 20, "cpu").numpy().tobytes()
    blocks = {"text": corpus._text(torch.Generator().manual_seed(7), 65536, "cpu").numpy().tobytes()}
    for off in (0, 60 << 20, 120 << 20):
        blocks[f"int32@{off >> 20}M"] = b[off:off + 65536]
    blocks["soup"] = b[200 << 20:(200 << 20) + 65536]
    for name, blk in blocks.items():
        d = sync_distances(blk)
        n = len(d)
        print(f"{name:12s} median {d[n // 2]:>6} bits  p90 {d[int(n * .9)]:>10}  >128 bits {sum(x > 128 for x in d) / n:.3f}"
              f"  >448 bits {sum(x > 448 for x in d) / n:.3f}", flush=True)
