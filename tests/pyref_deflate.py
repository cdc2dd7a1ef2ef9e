"""Independent pure-Python restatement of the reference encoder (N-version check).

Written from SURVEY.md App. A (not from oracle/ndfl_oracle.c) with DIFFERENT algorithms where
the reference's behaviour allows it, so that agreement with the C oracle is evidence for both:
  * RLE presets: closed-form run-piece parse (App. A.2) instead of a per-position search;
  * package-merge: explicit merge of (packages, sorted leaves) with ties to packages, then a
    level-by-level prefix backtrack (the formulation the GPU kernel uses) instead of node trees;
  * code-length RLE: per-maximal-run decomposition instead of the greedy index loop.
Test infrastructure only.  Slow; use for inputs up to a few hundred KiB.
"""

CLC_ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class BitWriter:
    def __init__(self):
        self.acc = 0
        self.n = 0

    def bits(self, v, nb):
        assert 0 <= nb <= 31 and v >> nb == 0
        self.acc |= v << self.n
        self.n += nb

    def getbytes(self):
        nbytes = (self.n + 7) // 8
        return self.acc.to_bytes(nbytes, "little") if nbytes else b""


def len_sym(run):
    """Length symbol, extra-bit count, extra value (App. A.4)."""
    if run < 11:
        return run + 254, 0, 0
    if run == 258:
        return 285, 0, 0
    x = run - 3
    ne = x.bit_length() - 3
    return (ne << 2) + (x >> ne) + 257, ne, x & ((1 << ne) - 1)


def dist_sym(d):
    if d < 5:
        return d - 1, 0, 0
    x = d - 1
    ne = x.bit_length() - 2
    return (ne << 1) + (x >> ne), ne, x & ((1 << ne) - 1)


def package_merge(freqs, max_len):
    """Code lengths with the reference's tie order (packages before leaves on equal frequency,
    leaves in ascending (freq, symbol))."""
    n = len(freqs)
    leaves = sorted([(f, s) for s, f in enumerate(freqs) if f > 0])
    nl = len(leaves)
    lens = [0] * n
    if nl < 2:
        return lens
    lf = [f for f, _ in leaves]
    pk = []                 # package frequencies of the previous level
    is_pkg_levels = []
    for _ in range(max_len):
        merged = []
        i = j = 0
        while i < len(pk) or j < nl:
            if j >= nl or (i < len(pk) and pk[i] <= lf[j]):
                merged.append((pk[i], True)); i += 1
            else:
                merged.append((lf[j], False)); j += 1
        is_pkg_levels.append([p for _, p in merged])
        pk = [merged[2 * k][0] + merged[2 * k + 1][0] for k in range(len(merged) // 2)]
    m = 2 * (nl - 1)
    for flags in reversed(is_pkg_levels):
        k = sum(flags[:m])
        nleaf = m - k
        for r in range(nleaf):
            lens[leaves[r][1]] += 1
        m = 2 * k
    return lens


def canonical(lens, max_len):
    codes = [None] * len(lens)
    nxt = 0
    for cl in range(1, max_len + 1):
        nxt <<= 1
        for s, l in enumerate(lens):
            if l == cl:
                assert nxt >> cl == 0, "over-full"
                codes[s] = (int(format(nxt, f"0{cl}b")[::-1], 2), cl)
                nxt += 1
    assert nxt == 1 << max_len, "under-full"
    return codes


def cl_rle(seq):
    """Greedy code-length RLE (App. A.5 step 5) by maximal-run decomposition."""
    out = []
    i, n = 0, len(seq)
    while i < n:
        v = seq[i]
        j = i
        while j < n and seq[j] == v:
            j += 1
        L = j - i
        if v == 0:
            while L > 0:
                r = min(L, 138)
                if r < 3:
                    out.extend([(0, None)] * r); L -= r
                elif r < 11:
                    out.append((17, r - 3)); L -= r
                else:
                    out.append((18, r - 11)); L -= r
        else:
            out.append((v, None))
            L -= 1
            while L >= 3:
                r = min(L, 6)
                out.append((16, r - 3)); L -= r
            out.extend([(v, None)] * L)
        i = j
    return out


STATIC_LIT_LENS = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8


def parse_tokens(buf, hist_len, data_len, min_run, max_run, min_dist, max_dist):
    """Greedy parse of buf[hist_len : hist_len+data_len] -> list of ('L', byte) / ('M', run, dist)."""
    start, end = hist_len, hist_len + data_len
    toks = []
    if max_dist == 0:
        return [("L", buf[i]) for i in range(start, end)]
    if min_dist == 1 and max_dist == 1:
        # closed-form run pieces (App. A.2)
        i = start
        while i < end:
            v = buf[i]
            j = i
            while j < end and buf[j] == v:
                j += 1
            lead = not (i > 0 and buf[i - 1] == v)
            R = (j - i) - (1 if lead else 0)
            if lead:
                toks.append(("L", v))
            big = max_run
            for _ in range(R // big):
                toks.append(("M", big, 1))
            m = R % big
            if m >= min_run:
                toks.append(("M", m, 1))
            else:
                toks.extend([("L", v)] * m)
            i = j
        return toks
    i = start
    while i < end:
        best, bestd = 0, 0
        for d in range(min_dist, min(max_dist, i) + 1):
            r = 0
            while r < max_run and i + r < end and buf[i + r] == buf[i + r - d]:
                r += 1
            if r > best:
                best, bestd = r, d
                if best >= max_run:
                    break
        if best < min_run or best == 0:
            toks.append(("L", buf[i])); i += 1
        else:
            toks.append(("M", best, bestd)); i += best
    return toks


def compress_block(w, buf, hist_len, data_len, params, final):
    dynamic, min_run, max_run, min_dist, max_dist = params
    toks = parse_tokens(buf, hist_len, data_len, min_run, max_run, min_dist, max_dist)
    lit = [0] * 286
    dist = [0] * 30
    for t in toks:
        if t[0] == "L":
            lit[t[1]] += 1
        else:
            lit[len_sym(t[1])[0]] += 1
            dist[dist_sym(t[2])[0]] += 1
    lit[256] += 1
    w.bits(1 if final else 0, 1)
    w.bits(2 if dynamic else 1, 2)
    if not dynamic:
        lcodes = canonical(STATIC_LIT_LENS, 9)
        dcodes = canonical([5] * 32, 5)
    else:
        if data_len == 0:
            lit[0] += 1
        ln = 286
        while ln > 257 and lit[ln - 1] == 0:
            ln -= 1
        lit = lit[:ln]
        llens = package_merge(lit, 15)
        used = [i for i, c in enumerate(dist) if c]
        if len(used) == 1:
            u = used[0]
            dist[u + 1 if u < 29 else u - 1] = 1
        dn = 30
        while dn > 1 and dist[dn - 1] == 0:
            dn -= 1
        dist = dist[:dn]
        empty = dn == 1 and dist[0] == 0
        dlens = [0] if empty else package_merge(dist, 15)
        seq = cl_rle(llens + dlens)
        clh = [0] * 19
        for s, _ in seq:
            clh[s] += 1
        cllens = package_merge(clh, 7)
        reo = [cllens[CLC_ORDER[i]] for i in range(19)]
        ncl = 19
        while ncl > 4 and reo[ncl - 1] == 0:
            ncl -= 1
        w.bits(ln - 257, 5)
        w.bits(dn - 1, 5)
        w.bits(ncl - 4, 4)
        for i in range(ncl):
            w.bits(reo[i], 3)
        clcodes = canonical(cllens, 7)
        for s, e in seq:
            c, l = clcodes[s]
            w.bits(c, l)
            if s >= 16:
                w.bits(e, {16: 2, 17: 3, 18: 7}[s])
        lcodes = canonical(llens, 15)
        dcodes = None if empty else canonical(dlens, 15)
    for t in toks:
        if t[0] == "L":
            c, l = lcodes[t[1]]
            w.bits(c, l)
        else:
            s, ne, ex = len_sym(t[1])
            c, l = lcodes[s]
            w.bits(c, l)
            w.bits(ex, ne)
            s, ne, ex = dist_sym(t[2])
            c, l = dcodes[s]
            w.bits(c, l)
            w.bits(ex, ne)
    c, l = lcodes[256]
    w.bits(c, l)


PRESETS = {
    "LITERAL_STATIC": (False, 0, 0, 0, 0), "LITERAL_DYNAMIC": (True, 0, 0, 0, 0),
    "RLE_STATIC": (False, 3, 258, 1, 1), "RLE_DYNAMIC": (True, 3, 258, 1, 1),
    "FULL_STATIC": (False, 3, 258, 1, 32768), "FULL_DYNAMIC": (True, 3, 258, 1, 32768),
}


def deflate(data, strategy="RLE_DYNAMIC", chunk_len=65536, hist_limit=32768, params=None):
    params = params or PRESETS[strategy]
    w = BitWriter()
    pos = 0
    n = len(data)
    while True:
        dlen = min(n - pos, chunk_len)
        final = pos + dlen >= n
        hlen = min(pos, hist_limit)
        compress_block(w, data[pos - hlen: pos + dlen], hlen, dlen, params, final)
        pos += dlen
        if final:
            break
    return w.getbytes()


def stored_blocks(w, data, final):
    """Uncompressed (D/comp/Uncompressed.java:33-46), restated from RFC 1951 §3.2.4: blocks of at
    most 65535 bytes, each byte-aligned after its 3 header bits."""
    i = 0
    while True:
        n = min(len(data) - i, 65535)
        w.bits(1 if final and i + n == len(data) else 0, 1)
        w.bits(0, 2)
        w.bits(0, (8 - w.n % 8) % 8)
        w.bits(n, 16)
        w.bits(n ^ 0xFFFF, 16)
        for b in data[i:i + n]:
            w.bits(b, 8)
        i += n
        if i >= len(data):
            break


def deflate_multi(data, subs, chunk_len=65536, hist_limit=32768):
    """MultiStrategy(subs...) (D/comp/MultiStrategy.java): per chunk, the first substrategy giving the
    fewest bits from the writer's current bit position.  Lengths are measured by writing each
    candidate into a scratch writer at that position (no closed form)."""
    w = BitWriter()
    pos = 0
    n = len(data)
    while True:
        dlen = min(n - pos, chunk_len)
        final = pos + dlen >= n
        hlen = min(pos, hist_limit)
        buf = data[pos - hlen: pos + dlen]
        best = None
        for st in subs:
            t = BitWriter()
            t.n = w.n % 8
            if st == "UNCOMPRESSED":
                stored_blocks(t, buf[hlen:], False)
            else:
                compress_block(t, buf, hlen, dlen, tuple(st), False)
            if best is None or t.n < best[0]:
                best = (t.n, st)
        if best[1] == "UNCOMPRESSED":
            stored_blocks(w, buf[hlen:], final)
        else:
            compress_block(w, buf, hlen, dlen, tuple(best[1]), final)
        pos += dlen
        if final:
            break
    return w.getbytes()


class _Leaf:
    """The substrategy's own decision over buf[hl, hl + dl); lengths measured by writing."""

    def __init__(self, buf, hl, dl, sub):
        self.buf, self.hl, self.dl, self.sub = buf, hl, dl, sub
        self.bits = []
        for pos in range(8):
            t = BitWriter()
            t.n = pos
            self.emit(t, False)
            self.bits.append(t.n - pos)

    def emit(self, w, final):
        if self.sub == "UNCOMPRESSED":
            stored_blocks(w, self.buf[self.hl:self.hl + self.dl], final)
        else:
            compress_block(w, self.buf[:self.hl + self.dl], self.hl, self.dl, tuple(self.sub), final)


class _Split:
    def __init__(self, bits, picks):
        self.bits, self.picks = bits, picks

    def emit(self, w, final):
        decs = self.picks[w.n % 8]
        for j, d in enumerate(decs):
            d.emit(w, final and j == len(decs) - 1)


def _bs_decide(buf, hl, dl, sub, m, cur):
    """BinarySplit.decide (D/comp/BinarySplit.java:33-66) restated; the split length is accumulated
    from position 0 for every starting position, as the reference's loops do."""
    bits = list(cur.bits)
    picks = [[cur] for _ in range(8)]
    first = (dl + 1) // 2
    second = dl - first
    if min(first, second) > m:
        sp = [_Leaf(buf, hl, first, sub), _Leaf(buf, hl + first, second, sub)]

        def total(decs):
            bl = 0
            for d in decs:
                bl += d.bits[bl % 8]
            return bl
        improved = any(total(sp) < bits[i] for i in range(8))
        if improved:
            sp = [_bs_decide(buf, hl, first, sub, m, sp[0]), _bs_decide(buf, hl + first, second, sub, m, sp[1])]
        t = total(sp)
        for i in range(8):
            if t < bits[i]:
                bits[i] = t
                picks[i] = sp
    return _Split(bits, picks)


def deflate_binsplit(data, sub, min_block_len, chunk_len=65536, hist_limit=32768):
    w = BitWriter()
    pos = 0
    n = len(data)
    while True:
        dlen = min(n - pos, chunk_len)
        final = pos + dlen >= n
        hlen = min(pos, hist_limit)
        buf = data[pos - hlen: pos + dlen]
        _bs_decide(buf, hlen, dlen, sub, min_block_len, _Leaf(buf, hlen, dlen, sub)).emit(w, final)
        pos += dlen
        if final:
            break
    return w.getbytes()
