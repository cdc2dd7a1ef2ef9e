"""Seeded synthetic corpora of SURVEY.md §8d, generated with torch on any device.

    c4_mixed(n, seed=0xC4)   Silesia-style mix in 1 MiB segments: ~40 % text/XML-ish, ~35 % binary
                             tables (LE int32 with small deltas, skewed byte soup), ~10 % random,
                             ~15 % byte runs.
    c3_text(n, seed=0xC3)    enwik-style text: Zipf(1.07) words over a 65,536-word vocabulary,
                             punctuation/newlines, [[link]] and <tag> markup.

Deterministic per (seed, device type).  Test/bench infrastructure, not product code.
"""
import math

import torch

SEG = 1 << 20


def _vocab(g, nwords, device, maxlen=12):
    lens = torch.randint(2, maxlen + 1, (nwords,), generator=g, device=device)
    letters = torch.randint(97, 123, (nwords, maxlen + 1), generator=g, device=device, dtype=torch.int64)
    letters[:, -1] = 32
    idx = torch.arange(maxlen + 1, device=device)
    words = torch.where(idx[None, :] < lens[:, None], letters, torch.full_like(letters, 32))
    # word bytes followed by one space; length = lens + 1
    return words.to(torch.uint8), lens + 1


def _zipf_ids(g, count, nwords, s, device):
    ranks = torch.arange(1, nwords + 1, device=device, dtype=torch.float64)
    p = ranks.pow(-s)
    cdf = torch.cumsum(p, 0)
    cdf = cdf / cdf[-1]
    u = torch.rand(count, generator=g, device=device, dtype=torch.float64)
    return torch.searchsorted(cdf, u).clamp_(max=nwords - 1)


def _text(g, n, device, nwords=4096, s=1.07, markup=True):
    words, wl = _vocab(g, nwords, device)
    avg = float(wl.float().mean())
    count = int(n / avg * 1.1) + 64
    ids = _zipf_ids(g, count, nwords, s, device)
    if markup:
        # every ~40 words: newline word, "[[" link, "<tag>" -- emulate by special vocab entries
        special = torch.tensor([list(b"\n" + b" " * 12), list(b"[[link]] " + b" " * 4), list(b"<tag> " + b" " * 7)],
                               dtype=torch.uint8, device=device)
        slen = torch.tensor([1, 9, 6], device=device)
        words = torch.cat([words, special])
        wl = torch.cat([wl, slen])
        mark = torch.rand(count, generator=g, device=device) < (1.0 / 40)
        kind = torch.randint(0, 3, (count,), generator=g, device=device)
        ids = torch.where(mark, nwords + kind, ids)
    L = wl[ids]
    total = int(L.sum())
    while total < n:   # rare
        extra = _zipf_ids(g, count // 4 + 16, nwords, s, device)
        ids = torch.cat([ids, extra])
        L = wl[ids]
        total = int(L.sum())
    starts = torch.cumsum(L, 0) - L
    rep = torch.repeat_interleave(torch.arange(ids.numel(), device=device), L)[:n]
    off = torch.arange(n, device=device) - starts[rep]
    return words[ids[rep], off]


def _runs(g, n, device):
    # run lengths ~ geometric (mean ~ 300), values from a small alphabet with some random bytes
    count = n // 150 + 64
    u = torch.rand(count, generator=g, device=device)
    lens = (torch.log1p(-u) / math.log1p(-1 / 300.0)).long() + 1
    vals = torch.randint(0, 256, (count,), generator=g, device=device)
    small = torch.rand(count, generator=g, device=device) < 0.7
    vals = torch.where(small, vals % 4, vals).to(torch.uint8)
    while int(lens.sum()) < n:
        lens = torch.cat([lens, lens])
        vals = torch.cat([vals, vals.flip(0)])
    return torch.repeat_interleave(vals, lens)[:n]


def _binary(g, n, device):
    half = n // 2
    # LE int32 with small deltas
    k = (half + 3) // 4
    d = torch.randint(-3, 4, (k,), generator=g, device=device, dtype=torch.int32)
    base = torch.randint(0, 1 << 20, (1,), generator=g, device=device, dtype=torch.int32)
    v = torch.cumsum(d, 0, dtype=torch.int32) + base
    tab = v.view(torch.uint8)[:half]
    # skewed byte soup: geometric-ish byte values
    m = n - half
    u = torch.rand(m, generator=g, device=device)
    soup = (torch.log1p(-u) / math.log1p(-0.15)).clamp_(max=255).to(torch.uint8)
    return torch.cat([tab, soup])


def c4_mixed(n, seed=0xC4, device="cpu"):
    g = torch.Generator(device=device).manual_seed(seed)
    nseg = max(1, -(-n // SEG))
    probs = torch.tensor([0.40, 0.35, 0.10, 0.15], device=device)
    types = torch.multinomial(probs, nseg, replacement=True, generator=g).tolist()
    out = torch.empty(nseg * SEG, dtype=torch.uint8, device=device)
    for t in range(4):
        segs = [i for i, x in enumerate(types) if x == t]
        # generate in batches of <= 256 segments to bound temporaries
        for b0 in range(0, len(segs), 256):
            sl = segs[b0:b0 + 256]
            m = len(sl) * SEG
            if t == 0:
                blob = _text(g, m, device)
            elif t == 1:
                blob = _binary(g, m, device)
            elif t == 2:
                blob = torch.randint(0, 256, (m,), generator=g, device=device, dtype=torch.uint8)
            else:
                blob = _runs(g, m, device)
            blob = blob.view(len(sl), SEG)
            idx = torch.tensor(sl, device=device)
            out.view(nseg, SEG)[idx] = blob
    return out[:n]


def c3_text(n, seed=0xC3, device="cpu"):
    g = torch.Generator(device=device).manual_seed(seed)
    return _text(g, n, device, nwords=65536)


def mixed_bytes(n_total, seed):
    """Small host-side mix (random spans, byte runs, 7-letter text) for the multi-rank and range
    tests: bytes, seeded numpy generator."""
    import numpy as np
    rng = np.random.default_rng(seed)
    parts, size = [], 0
    while size < n_total:
        kind = rng.integers(0, 3)
        ln = int(rng.integers(1000, 60000))
        if kind == 0:
            parts.append(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
        elif kind == 1:
            parts.append(bytes([int(rng.integers(0, 256))]) * ln)
        else:
            parts.append(bytes(rng.choice(list(b"abcde \n"), ln).astype(np.uint8)))
        size += ln
    return b"".join(parts)[:n_total]


def c2_gzip(target_comp=64 << 20, seed=0xC2):
    """Config 2: one gzip member whose DEFLATE stream alternates stored blocks (random
    bytes, random lengths 1..65535, plus the empty stored blocks of each sync flush) and fixed-Huffman
    blocks (about 64 KiB of enwik-style text, greedily LZ77-coded with dist 1..32768, len 3..258 by
    zlib's Z_FIXED strategy), until the compressed size reaches `target_comp`.  Pieces are
    byte-aligned by Z_SYNC_FLUSH, so their concatenation is one valid stream.
    Returns (gz_bytes, raw_deflate_bytes, data).  Deterministic (numpy PCG64 + zlib 1.2.11)."""
    import zlib
    import numpy as np
    rng = np.random.default_rng(seed)
    text = c3_text(8 << 20, seed=seed).numpy().tobytes()
    parts, datas, size = [], [], 0
    while size < target_comp:
        if rng.random() < 0.5:
            ln = int(rng.integers(1, 65536))
            d = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            co = zlib.compressobj(0, zlib.DEFLATED, -15)
        else:
            ln = int(rng.integers(32768, 98304))
            o = int(rng.integers(0, len(text) - ln))
            d = text[o:o + ln]
            co = zlib.compressobj(6, zlib.DEFLATED, -15, 9, zlib.Z_FIXED)
        p = co.compress(d) + co.flush(zlib.Z_SYNC_FLUSH)
        parts.append(p)
        datas.append(d)
        size += len(p)
    raw = b"".join(parts) + b"\x03\x00"          # final fixed block holding only EOB
    data = b"".join(datas)
    hdr = bytes([0x1F, 0x8B, 8, 0, 0, 0, 0, 0, 0, 3])
    trailer = (zlib.crc32(data) & 0xFFFFFFFF).to_bytes(4, "little") + (len(data) & 0xFFFFFFFF).to_bytes(4, "little")
    return hdr + raw + trailer, raw, data


def c5_random_repeat(n, seed=0xC5):
    """Config 5: 50 % random-byte spans and 50 % "repeat" spans -- copies of earlier
    data at dist U[1, 32768] with lengths 3 + geometric (capped at 258), and byte runs up to 4 KiB.
    numpy PCG64, deterministic; returns a uint8 numpy array of n bytes."""
    import numpy as np
    rng = np.random.default_rng(seed)
    a = np.empty(n + 4096 + 258 * 16, dtype=np.uint8)
    p = 0
    while p < n:
        u = rng.random()
        if u < 0.5 or p < 64:                         # random span
            ln = int(rng.integers(64, 4096))
            a[p:p + ln] = rng.integers(0, 256, ln, dtype=np.uint8)
        elif u < 0.6:                                 # byte run up to 4 KiB
            ln = int(rng.integers(3, 4097))
            a[p:p + ln] = int(rng.integers(0, 256))
        else:                                         # a few copies from earlier data
            ln = 0
            for _ in range(int(rng.integers(1, 16))):
                q = p + ln
                d = int(rng.integers(1, min(32768, q) + 1))
                ll = min(258, 3 + int(rng.geometric(1 / 20)))
                if d >= ll:
                    a[q:q + ll] = a[q - d:q - d + ll]
                else:
                    a[q:q + ll] = np.resize(a[q - d:q], ll)
                ln += ll
        p += ln
    return a[:n]


def c5_device(n, seed=0xC5, device="cuda", batch=256 << 20):
    """Config 5 at its defined size (16 GiB), generated on the device: the same span mix as
    c5_random_repeat -- 50 % random-byte spans (64..4095 B), ~10 % byte runs (3..4096 B), ~40 %
    copies of earlier data (dist U[1, 32768], length 3 + geometric(1/20), capped at 258; overlapping
    copies repeat their period) -- drawn per 256 MiB batch with a torch generator (seed + batch
    index).  A copy's source is resolved by pointer jumping over the batch (copies of copies), and a
    copy never reaches before its batch.  Deterministic per (seed, device type); not tiled."""
    out = torch.empty(n, dtype=torch.uint8, device=device)
    for b0 in range(0, n, batch):
        m = min(batch, n - b0)
        g = torch.Generator(device=device).manual_seed(seed * 1000003 + b0 // batch)
        k = m // 300 + 1024                              # spans (mean length ~ 700 B, with slack)
        while True:
            u = torch.rand(k, generator=g, device=device)
            kind = torch.where(u < 0.5, 0, torch.where(u < 0.6, 1, 2))          # random / run / copy
            lr = torch.randint(64, 4096, (k,), generator=g, device=device)
            lrun = torch.randint(3, 4097, (k,), generator=g, device=device)
            gu = torch.rand(k, generator=g, device=device).clamp_(min=1e-12)
            lcopy = (3 + torch.floor(torch.log(gu) / math.log(1 - 1 / 20.0)).long()).clamp_(max=258)
            ln = torch.where(kind == 0, lr, torch.where(kind == 1, lrun, lcopy))
            if int(ln.sum()) >= m:
                break
            k *= 2
        starts = torch.cumsum(ln, 0) - ln
        span = torch.repeat_interleave(torch.arange(k, device=device), ln)[:m]
        pos = torch.arange(m, device=device)
        sk = kind[span]
        rnd = torch.randint(0, 256, (m,), generator=g, device=device, dtype=torch.uint8)
        runv = torch.randint(0, 256, (k,), generator=g, device=device, dtype=torch.uint8)
        val = torch.where(sk == 1, runv[span], rnd)
        # copies: distance per span, U[1, min(32768, span start)]; the first 64 bytes are random
        dmax = starts.clamp(min=1, max=32768)
        d = (torch.rand(k, generator=g, device=device) * dmax).long() + 1
        d = torch.minimum(d, dmax)
        is_copy = (sk == 2) & (pos >= 64)
        src = torch.where(is_copy, pos - d[span], pos)
        del span, sk, rnd, runv
        for _ in range(40):                              # pointer jumping: sources of sources
            nxt = src[src]
            if torch.equal(nxt, src):
                break
            src = nxt
        out[b0:b0 + m] = val[src]
        del src, val, pos, is_copy
    return out
