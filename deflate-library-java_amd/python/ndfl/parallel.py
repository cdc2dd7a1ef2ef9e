"""Multi-GPU DEFLATE of ONE stream: one process per GPU, shard by 64 KiB chunk.

The reference is single-threaded; its stream is a sequence of chunk blocks whose bits depend only
on raw input (D/DeflaterOutputStream.java:119-137).  So rank r compresses chunks
[r*K, (r+1)*K) by itself.  The exchange steps are the only places where ranks talk to each other:

  compress    (1) the raw bytes preceding the shard (the encoder's history, <= 32 KiB) go from
                  rank r-1 to rank r, point to point (one all_gather of every rank's last 32 KiB when
                  shards are shorter than that, so a history spans several earlier shards);
              (2) all_gather of every shard's bit count and byte count: the seam index;
              (3) each rank moves its bits to its global bit offset mod 8 (ndfl_bits_shift), so
                  the global stream is the concatenation of the shards with the shared boundary
                  bytes ORed (BitOut's packing, D/DeflaterOutputStream.java:147-156);
              (4) gather_stream: the root receives every part at its byte offset (point to point)
                  and ORs the shared bytes on device -- one global stream on one GPU.
  decompress  (seam index, from deflate_shard) inflate_shard, below; (foreign stream, no index)
              inflate_split: each rank probes for a confirmed block boundary near its share of the
              bits (ndfl_inflate_sync), the seams are proven by the range decodes themselves.
  decompress  each rank decodes its seam-delimited bit range with a deferred window
              (ndfl_inflate_range + NDFL_DICT_DEFERRED), all ranks in parallel; then one
              all_gather of every rank's last 32 KiB as a map of its window
              (ndfl_inflate_tail_map) gives each rank its window (the reference's dictionary ring,
              D/decomp/Open.java:592-603, carried across all earlier shards) by composing the
              maps before it, and each rank re-emits only the blocks that read it
              (ndfl_inflate_resolve).

The protocol is codec-agnostic: `DeviceCodec` runs it on the GPU through the C ABI; the CPU tests
drive the same functions with a checker codec over gloo.
"""
from dataclasses import dataclass, field

WINDOW = 32768


@dataclass
class Part:
    """One rank's piece of the global stream."""
    buf: object                 # uint8 tensor: the shard's bits start at bit `shift` of buf[0]
    nbits: int                  # bits of this shard
    shift: int                  # global bit offset mod 8
    bit_offsets: list = field(default_factory=list)    # seam index: global bit offset per rank (+ total)
    byte_offsets: list = field(default_factory=list)   # uncompressed byte offset per rank (+ total)
    hist: object = None         # the raw bytes before the shard the encoder used as history

    @property
    def nbytes(self):
        return (self.shift + self.nbits + 7) // 8


class DeviceCodec:
    """The GPU codec (libndfl.so through ndfl.Context) on torch device tensors."""

    def __init__(self, ctx, torch):
        self.ctx = ctx
        self.torch = torch
        self.device = torch.device("cuda", ctx.device)
        ctx.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def empty(self, n):
        return self.torch.empty(max(1, n), dtype=self.torch.uint8, device=self.device)

    def bound(self, n, chunk_len):
        from . import _lib
        return _lib.load().ndfl_deflate_bound(n, chunk_len) + 64

    def deflate_chunks(self, hist, data, final, out, strategy, chunk_len, hist_limit):
        from . import IN_DEVICE, OUT_DEVICE, _strategy_id
        hl = 0 if hist is None else hist.numel()
        endbits, _ = self.ctx.deflate_chunks_raw(hist.data_ptr() if hl else None, hl, hist_limit, data.data_ptr(),
                                                 data.numel(), chunk_len, _strategy_id(strategy), final, 0,
                                                 out.data_ptr(), out.numel(), IN_DEVICE | OUT_DEVICE)
        return endbits

    def bits_shift(self, src, nbits, shift, dst):
        self.ctx.bits_shift_raw(src.data_ptr(), nbits, shift, dst.data_ptr(), dst.numel())

    def inflate_range(self, src, in_len, start_bit, end_bit, out, dict_len, deferred):
        from . import IN_DEVICE, OUT_DEVICE, DICT_DEFERRED
        flags = IN_DEVICE | OUT_DEVICE | (DICT_DEFERRED if deferred else 0)
        return self.ctx.inflate_range_raw(src.data_ptr(), in_len, start_bit, end_bit, out.data_ptr(), dict_len,
                                          out.numel() - dict_len, flags)

    def resolve(self):
        return self.ctx.inflate_resolve()

    def tail(self, n):
        """The last n output bytes of the pending deferred decode (its window written), before the
        resolve; None if a reference chain is too long to follow (resolve first)."""
        t = self.empty(n)
        return t[:n] if self.ctx.inflate_tail_raw(n, t.data_ptr()) else None

    def tail_map(self, n, dst):
        """The last n output bytes of the pending deferred decode as a map of its window, into the
        int32 tensor dst[:n] (ndfl_inflate_tail_map); False if a reference chain is too long."""
        return self.ctx.inflate_tail_map_raw(n, dst.data_ptr())

    def sync(self, src, in_len, from_bit, window_bits):
        from . import IN_DEVICE
        return self.ctx.inflate_sync_raw(src.data_ptr(), in_len, from_bit, window_bits, IN_DEVICE)


def init_process_group(dist, backend, device=None, timeout_s=120.0):
    """One process per GPU: the process group every exchange below runs on, with a finite timeout,
    so a rank that stalls (or an exchange issued out of order) ends the run with an error instead of
    a hang.  `backend` "nccl" is RCCL over xGMI (`device`: this rank's GPU, bound at init); "gloo"
    only for the CPU tests and one-GPU rehearsals."""
    import datetime
    import os
    # RCCL: a timed-out operation aborts the communicator and raises on the host (the watchdog's
    # default handling tears the process down), the gloo backend raises from the call itself
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "3")
    kw = dict(timeout=datetime.timedelta(seconds=timeout_s))
    if device is not None:
        kw["device_id"] = device
    dist.init_process_group(backend, **kw)


def _staged(dist, t):
    """gloo moves host tensors only: stage device tensors through the host (tests / rehearsals on a
    single GPU); RCCL moves device tensors directly over xGMI."""
    return t.is_cuda and dist.get_backend() == "gloo"


def _send(dist, t, dst):
    dist.send(t.cpu() if _staged(dist, t) else t, dst)


def _recv(dist, t, src):
    if _staged(dist, t):
        tmp = t.cpu()
        dist.recv(tmp, src)
        t.copy_(tmp)
    else:
        dist.recv(t, src)


def _gather_ints(dist, torch, value, world, device):
    """all_gather of one int64 per rank."""
    dev = "cpu" if dist.get_backend() == "gloo" else device
    t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
    lst = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(lst, t)
    return [int(x.item()) for x in lst]


def _exchange_prev(dist, torch, send_t, recv_t, rank, world):
    """send_t -> rank+1, recv_t <- rank-1 (point to point, all pairs at once)."""
    if _staged(dist, send_t) or _staged(dist, recv_t):
        # host staging: even ranks send first, odd ranks receive first (no deadlock on blocking p2p)
        for phase in (0, 1):
            if (rank + phase) % 2 == 0:
                if rank + 1 < world:
                    _send(dist, send_t, rank + 1)
            elif rank > 0:
                _recv(dist, recv_t, rank - 1)
        return
    ops = []
    if rank + 1 < world:
        ops.append(dist.P2POp(dist.isend, send_t, rank + 1))
    if rank > 0:
        ops.append(dist.P2POp(dist.irecv, recv_t, rank - 1))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()


def deflate_shard(codec, dist, torch, shard, rank, world, *, strategy="RLE_DYNAMIC", chunk_len=65536,
                  hist_limit=WINDOW, work=None, out=None):
    """Compress this rank's shard as chunks [r*K, (r+1)*K) of one stream.  Every shard but the
    last must hold whole chunks.  `work`/`out`: optional preallocated buffers (bound bytes)."""
    n = shard.numel()
    if rank + 1 < world and (n == 0 or n % chunk_len):
        raise ValueError("every shard but the last must be a positive multiple of chunk_len")
    # (1) history: the last min(hist_limit, bytes before the shard) raw bytes of the stream
    hlen = min(hist_limit, n)
    sizes = _gather_ints(dist, torch, n, world, codec.device)
    want_h = min(hist_limit, sum(sizes[:rank]))
    if all(v >= hist_limit for v in sizes[:-1]):
        # every shard holds a whole window: the previous rank's last bytes, point to point
        prev_h = min(hist_limit, sizes[rank - 1]) if rank > 0 else 0
        hist = codec.empty(prev_h)[:prev_h]
        _exchange_prev(dist, torch, shard[n - hlen:].contiguous() if hlen else codec.empty(0)[:0], hist, rank,
                       world)
    else:
        # shards shorter than the window (small inputs over many ranks): the history spans several
        # earlier shards -- one all_gather of every rank's last <= hist_limit bytes (padded to one size)
        tail = codec.empty(hist_limit)[:hist_limit] if hist_limit else codec.empty(1)[:1]
        if hlen:
            tail[hist_limit - hlen:] = shard[n - hlen:]
        tails = _all_gather_tensor(dist, torch, tail, world)
        pieces = [tails[k][hist_limit - min(hist_limit, sizes[k]):hist_limit] for k in range(rank)]
        hist = torch.cat(pieces)[-want_h:] if want_h else codec.empty(0)[:0]
        prev_h = want_h
    if prev_h < want_h:
        raise ValueError("a shard shorter than the history window precedes this one")
    # local compress at bit 0
    cap = codec.bound(n, chunk_len)
    work = work if work is not None else codec.empty(cap)
    nbits = codec.deflate_chunks(hist if prev_h else None, shard, rank == world - 1, work, strategy, chunk_len,
                                 hist_limit)
    # (2) seam index
    nb = _gather_ints(dist, torch, nbits, world, codec.device)
    bit_offsets = [0]
    for v in nb:
        bit_offsets.append(bit_offsets[-1] + v)
    byte_offsets = [0]
    for v in sizes:
        byte_offsets.append(byte_offsets[-1] + v)
    # (3) realign to the global bit offset
    shift = bit_offsets[rank] % 8
    out = out if out is not None else codec.empty(cap + 1)
    codec.bits_shift(work, nbits, shift, out)
    return Part(out, nbits, shift, bit_offsets, byte_offsets, hist if prev_h else None)


TAIL_LITERAL = -(1 << 31)      # NDFL_TAIL_LITERAL as an int32 map entry: a byte value, not a window index


def _all_gather_tensor(dist, torch, t, world):
    """all_gather of one equal-size tensor per rank (gloo: staged through the host)."""
    staged = _staged(dist, t)
    src = t.cpu() if staged else t
    lst = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(lst, src)
    return [x.to(t.device) for x in lst] if staged else lst


def window_from_maps(torch, maps, lens, rank):
    """Rank `rank`'s window from the tail maps of ranks 0..rank-1 (ndfl_inflate_tail_map): rank k's
    last lens[k] output bytes as a function of its own window, composed from rank 0 on."""
    w = None
    for k in range(rank):
        m = maps[k][:lens[k]].long()
        lit = m < 0
        vals = m & 0xFF
        if w is not None:
            vals = torch.where(lit, vals, w[torch.where(lit, torch.zeros_like(m), m)])
        w = vals
    return w.to(torch.uint8)


def inflate_shard(codec, dist, torch, part, out, rank, world):
    """Decode this rank's range of the stream into out[dict_len:], out[:dict_len] = the window.
    Returns (code, out_len, dict_len): code 0 or the Reason+1 of the FIRST error in stream order
    over all ranks (every rank returns the same code).

    All ranks decode at once with a deferred window.  The window chain -- rank r's window is the
    last 32 KiB of rank r-1's output, which depends on rank r-1's own window -- is then one
    all_gather: each rank describes its last 32 KiB as a map of its window (ndfl_inflate_tail_map:
    per byte a window index or a value), and rank r composes the maps of ranks 0..r-1 into its
    window itself, so no rank waits for the one before it.  Only if some rank cannot describe its
    tail (a back-reference chain longer than the map kernel follows) does the chain run rank by
    rank (_window_chain)."""
    dict_len = min(WINDOW, part.byte_offsets[rank])
    deferred = rank > 0 and dict_len > 0
    code, olen, _ = codec.inflate_range(part.buf, part.nbytes, part.shift, part.shift + part.nbits, out, dict_len,
                                        deferred)
    if code < 0:
        raise RuntimeError(f"inflate_range failed: {code}")
    nxt = min(WINDOW, part.byte_offsets[rank + 1]) if rank + 1 < world else 0
    end = dict_len + olen
    m = torch.full((WINDOW,), TAIL_LITERAL, dtype=torch.int32, device=codec.device)
    ok = 1
    if nxt and code == 0 and end >= nxt:
        if deferred:
            ok = int(bool(codec.tail_map(nxt, m)))
        else:
            m[:nxt] = out[end - nxt:end].int() | TAIL_LITERAL
    # (an error ends the stream here: the next rank gets a window of zeros, as the chain would)
    flags = _gather_ints(dist, torch, code * 2 + ok, world, codec.device)
    codes = [f >> 1 for f in flags]
    if all(f & 1 for f in flags):
        maps = _all_gather_tensor(dist, torch, m, world)
        if deferred:
            lens = [min(WINDOW, part.byte_offsets[k + 1]) for k in range(world - 1)]
            out[:dict_len] = window_from_maps(torch, maps, lens, rank)
            if code == 0:
                codec.resolve()
    else:
        _window_chain(codec, dist, torch, out, rank, world, code, dict_len, end, nxt)
    first = next((c for c in codes if c != 0), 0)
    return first, olen, dict_len


def _window_chain(codec, dist, torch, out, rank, world, code, dict_len, end, nxt):
    """The window chain rank by rank: rank r-1's last 32 KiB of output -> rank r.  Rank r passes its
    own last 32 KiB on as soon as its window is in (ndfl_inflate_tail follows those bytes'
    references), and resolves the rest of its range after that."""
    sent = False
    if rank > 0 and dict_len:
        _recv(dist, out[:dict_len], rank - 1)
        if code == 0 and nxt and end >= nxt:
            tail = codec.tail(nxt)
            if tail is not None:
                _send(dist, tail, rank + 1)
                sent = True
        if code == 0:
            codec.resolve()
    if rank + 1 < world and not sent:
        if code == 0 and end >= nxt:
            _send(dist, out[end - nxt:end].contiguous(), rank + 1)
        else:                                    # an error ends the stream here: keep the chain moving
            _send(dist, torch.zeros(nxt, dtype=torch.uint8, device=codec.device), rank + 1)


SYNC_WINDOW = 8 << 20          # bits a sync probe looks ahead (1 MiB of stream)
_lib_E_ARG = -1                # NDFL_E_ARG: the range end is no block boundary


def inflate_split(codec, dist, torch, stream, in_len, out, rank, world):
    """Decode ONE stream that carries no seam index (a foreign .gz member, a single-GPU encoding)
    across the ranks (SURVEY §8e decompress).  Every rank holds the stream.

      (1) rank r > 0 probes for the first confirmed block boundary at or past r * C / N
          (ndfl_inflate_sync: a header the reference's checks accept whose chain of blocks decodes
          exactly to the next one) -- all ranks at once; all_gather of the seams;
      (2) rank r decodes [seam_r, seam_{r+1}) with ndfl_inflate_range and a deferred window.  The
          range decode's exact-boundary check proves each seam inductively from bit 0: rank r-1,
          started at a proven boundary, must stop exactly at seam_r;
      (3) the window chain and the first-error reduction as in inflate_shard.
    If a seam is not proven (a false candidate, a corrupt stream) or a rank's output is shorter than
    the 32 KiB window, rank 0 decodes the whole stream alone (the single-GPU result, exact by
    construction).  out[:32768] is the window slot, the rank's bytes follow.
    Returns (code, out_len, dict_len, byte_offset) -- code 0 or the Reason+1 of the first error in
    stream order (the same on every rank); byte_offset = where this rank's bytes start in the output."""
    nbits = in_len * 8
    seam = 0
    if rank > 0:
        s = codec.sync(stream, in_len, nbits * rank // world, SYNC_WINDOW)
        seam = nbits if s is None else s
    seams = _gather_ints(dist, torch, seam, world, codec.device)
    for r in range(1, world):                   # monotonic: a rank without a seam gets nothing
        seams[r] = max(seams[r], seams[r - 1])
    end = seams[rank + 1] if rank + 1 < world and seams[rank + 1] < nbits else None
    dict_len = WINDOW if rank > 0 else 0
    empty = seams[rank] >= nbits or (end is not None and end <= seams[rank])
    if empty:
        code, olen = 0, 0
    else:
        code, olen, consumed = codec.inflate_range(stream, in_len, seams[rank], end, out, dict_len, rank > 0)
        if code == 0 and end is not None and consumed != end:
            code = _lib_E_ARG                    # the final block came before the next seam
    codes = _gather_ints(dist, torch, code, world, codec.device)
    olens = _gather_ints(dist, torch, olen, world, codec.device)
    offs = [0]
    for v in olens:
        offs.append(offs[-1] + v)
    # seams proven and windows available: every rank but the last ended exactly at its seam with no
    # error, and the output before each rank > 0 holds a full window within its predecessor
    ok = all(c == 0 for c in codes[:-1]) and codes[-1] >= 0 and \
        all(olens[r - 1] >= WINDOW for r in range(1, world) if seams[r] < nbits)
    if not ok:
        # single-GPU fallback: rank 0 decodes everything
        if rank == 0:
            code, olen, _ = codec.inflate_range(stream, in_len, 0, None, out, 0, False)
        else:
            code, olen = 0, 0
        code = _gather_ints(dist, torch, code, world, codec.device)[0]
        if code < 0:
            raise RuntimeError(f"inflate_range failed: {code}")
        return code, olen, 0, 0
    # window chain: rank r-1's last 32 KiB of output -> rank r (ranks with output only)
    if rank > 0 and not empty:
        _recv(dist, out[:dict_len], rank - 1)
        codec.resolve()
    if rank + 1 < world and seams[rank + 1] < nbits:
        e = dict_len + olen
        _send(dist, out[e - WINDOW:e].contiguous(), rank + 1)
    first = next((c for c in codes if c != 0), 0)
    return first, olen, dict_len, offs[rank]


class Pending:
    """An asynchronous gather_stream: wait() completes the transfers (and, on the root, ORs the shared
    first bytes in) and returns what gather_stream returns."""

    def __init__(self, reqs, finish):
        self._reqs, self._finish, self._done, self._value = reqs, finish, False, None

    def wait(self):
        if not self._done:
            for r in self._reqs:
                r.wait()
            self._value = self._finish()
            self._done = True
        return self._value


def gather_stream(codec, dist, torch, part, rank, world, root=0, out=None, async_op=False):
    """Reassemble the global stream on `root` (SURVEY §8e compress step 4): every rank sends its
    realigned part -- the first byte (shared with the previous shard when the global bit offset is
    not byte-aligned) and the body -- and the root receives each body straight into its byte offset
    of the output buffer (point to point over RCCL/xGMI; ncclGather needs equal counts), then ORs the
    first bytes in: BitOut's byte packing (D/DeflaterOutputStream.java:147-156) across GPUs, on
    device.  Returns the stream tensor (bytes ceil(total bits / 8)) on the root, None elsewhere.
    `out`: an optional preallocated root buffer of at least that many bytes (its old contents do not
    matter: only the bytes every part's first byte is ORed into are cleared).
    async_op: return a Pending at once (RCCL moves the parts on its own stream while the caller goes
    on, e.g. decoding its shard); host-staged (gloo) transfers complete before it returns."""
    offs = part.bit_offsets
    B = [o // 8 for o in offs[:-1]]
    nb = [(offs[r] % 8 + offs[r + 1] - offs[r] + 7) // 8 for r in range(world)]
    total = (offs[-1] + 7) // 8
    staged = _staged(dist, part.buf)
    if rank == root:
        if out is None or out.numel() < max(1, total):
            out = torch.empty(max(1, total), dtype=torch.uint8, device=codec.device)
        # every byte is either inside some part's body or a part's first byte: only the first bytes
        # need a defined value before the OR (a part's last byte, shared with the next part's first,
        # arrives with the body)
        firsts_at = [B[r] for r in range(world) if nb[r]]
        if firsts_at:
            out[torch.tensor(firsts_at, dtype=torch.int64, device=codec.device)] = 0
        firsts = torch.zeros(world, dtype=torch.uint8, device=codec.device)
        ops = []
        for r in range(world):
            if nb[r] == 0:
                continue
            if r == rank:
                out[B[r] + 1:B[r] + nb[r]] = part.buf[1:nb[r]]
                firsts[r:r + 1] = part.buf[0:1]
                continue
            if staged:
                if nb[r] > 1:
                    _recv(dist, out[B[r] + 1:B[r] + nb[r]], r)
                _recv(dist, firsts[r:r + 1], r)
            else:
                if nb[r] > 1:
                    ops.append(dist.P2POp(dist.irecv, out[B[r] + 1:B[r] + nb[r]], r))
                ops.append(dist.P2POp(dist.irecv, firsts[r:r + 1], r))
        reqs = dist.batch_isend_irecv(ops) if ops else []

        def finish():
            for r in range(world):
                if nb[r]:
                    out[B[r]:B[r] + 1].bitwise_or_(firsts[r:r + 1])
            return out[:total]
        pend = Pending(reqs, finish)
        return pend if async_op else pend.wait()
    reqs = []
    if nb[rank]:
        if staged:
            if nb[rank] > 1:
                _send(dist, part.buf[1:nb[rank]], root)
            _send(dist, part.buf[0:1], root)
        else:
            ops = [dist.P2POp(dist.isend, part.buf[0:1].contiguous(), root)]
            if nb[rank] > 1:
                ops.insert(0, dist.P2POp(dist.isend, part.buf[1:nb[rank]], root))
            reqs = dist.batch_isend_irecv(ops)
    pend = Pending(reqs, lambda: None)
    return pend if async_op else pend.wait()


def assemble(parts):
    """Join the parts (host bytes objects with their shift/nbits) into the global stream, ORing the
    byte each pair of neighbours shares.  Used by the tests and by a writer that gathers to one rank."""
    out = bytearray()
    for buf, shift, nbits in parts:
        nbytes = (shift + nbits + 7) // 8
        b = bytes(buf[:nbytes])
        if shift and out:
            out[-1] |= b[0]
            out += b[1:]
        else:
            out += b
    return bytes(out)
