"""Host logic of the streaming InflaterInputStream mirror (ndfl/streams.py), on the CPU.

The codec behind it is a checker stand-in for the C ABI's ndfl_inflate_range(NDFL_IN_PARTIAL)
built on the oracle (test infrastructure: the oracle decodes, block boundaries come from the
oracle's own per-block bit counts).  It enforces the ABI's buffer contract -- out[0, dict_len) is
the window and at most out_cap bytes follow it -- against the size of the buffer the stream
actually allocated, so a batch whose output lands between out_cap and out_cap + window (the
round-2 heap overflow: the whole buffer size was passed as out_cap) fails here, on any machine.

Also covered: a bounded output per batch (MAX_BATCH_OUT: the input is cut shorter instead of
allocating the whole expansion), and short reads from a pipe-like source decoded as they arrive
(Open decodes whatever its fill returned, D/decomp/Open.java:181-192).
Reference semantics: D/InflaterInputStream.java:96-164, D/decomp/Open.java:83-124.
"""
import ctypes
import io
import itertools

import numpy as np
import pytest

import oracle_lib as O

ndfl = pytest.importorskip("ndfl")
from ndfl import _lib, streams  # noqa: E402


class _Allocs:
    """Records the size of every ctypes buffer streams.py allocates, by address."""

    def __init__(self):
        self.size = {}
        self._real = ctypes.create_string_buffer

    def create_string_buffer(self, init, size=None):
        b = self._real(init, size) if size is not None else self._real(init)
        self.size[ctypes.addressof(b)] = ctypes.sizeof(b)
        return b

    def __getattr__(self, name):
        return getattr(ctypes, name)


class OracleRangeCtx:
    """ndfl_inflate_range(IN_PARTIAL) semantics over a stream with known block boundaries."""

    def __init__(self, stream, boundaries, allocs):
        self.stream = stream
        self.bounds = boundaries          # absolute bit positions of every block end
        self.allocs = allocs
        self.base = 0                     # absolute byte of the caller's input buffer start
        self.calls = []

    def inflate_range_raw(self, in_addr, n, start_bit, end_bit, out_addr, dict_len, out_cap, flags):
        assert end_bit is None
        room = self.allocs.size[out_addr]
        assert dict_len + out_cap <= room, f"out_cap {out_cap} + window {dict_len} > buffer {room}"
        src = ctypes.string_at(in_addr, n)
        assert src == self.stream[self.base:self.base + n]
        window = ctypes.string_at(out_addr, dict_len)
        a0 = self.base * 8 + start_bit
        lim = (self.base + n) * 8
        done = [b for b in self.bounds if a0 < b <= lim]
        final = self.bounds[-1] <= lim
        self.calls.append((self.base, n, flags))
        if not final and not (flags & _lib.IN_PARTIAL):
            return 1, 0, 0                # UNEXPECTED_END_OF_STREAM (not exercised here)
        stop = self.bounds[-1] if final else (done[-1] if done else a0)
        if stop == a0:
            return _lib.NEED_INPUT, 0, start_bit
        reason, out, bits = O.inflate_range(self.stream, a0, None if final else stop, window)
        assert reason is None
        if len(out) > out_cap:
            return _lib.E_CAPACITY, len(out), 0
        ctypes.memmove(out_addr + dict_len, out, len(out))
        rel = bits - self.base * 8
        if final:
            return 0, len(out), rel
        self.base += rel // 8
        return _lib.NEED_INPUT, len(out), rel


class ShortReads(io.RawIOBase):
    """A pipe: every read returns at most `piece` bytes.  `ready`: what available() reports (0: a
    slow producer, nothing more has arrived after each piece; > 0: a fast producer with data
    waiting; None: a source that cannot tell)."""

    def __init__(self, data, piece, ready=0):
        self._b = io.BytesIO(data)
        self._piece = piece
        self._ready = ready

    def readable(self):
        return True

    def available(self):
        return self._ready

    def read1(self, n=-1):
        return self._b.read(min(n, self._piece) if n >= 0 else self._piece)

    def read(self, n=-1):
        return self.read1(n)


def _stream(data, chunk_len):
    comp = O.deflate(data, "RLE_DYNAMIC", chunk_len=chunk_len)
    bounds = list(itertools.accumulate(O.block_bits(data, "RLE_DYNAMIC", chunk_len=chunk_len)))
    return comp, bounds


def _run(monkeypatch, comp, bounds, reader, batch, max_out=None):
    allocs = _Allocs()
    monkeypatch.setattr(streams, "ctypes", allocs)
    ctx = OracleRangeCtx(comp, bounds, allocs)
    s = streams.InflaterInputStream(reader, context=ctx)
    s._batch = batch
    if max_out is not None:
        s.MAX_BATCH_OUT = max_out
    return s.readall(), ctx


def test_window_plus_output_never_exceeds_the_buffer(monkeypatch):
    """Batches of 1..4 KiB of a stream that expands ~10x: with the 32 KiB window present, many
    batches need more than 4n + 65536 - window bytes -- the band where the old out_cap overflowed."""
    rng = np.random.default_rng(1)
    data = b"".join(bytes([int(v)]) * int(r) + rng.integers(0, 256, int(k), dtype=np.uint8).tobytes()
                    for v, r, k in zip(rng.integers(0, 4, 4000), rng.integers(20, 400, 4000),
                                       rng.integers(0, 8, 4000)))
    comp, bounds = _stream(data, 4096)
    for batch in (1024, 2048, 4096):
        got, ctx = _run(monkeypatch, comp, bounds, io.BytesIO(comp), batch)
        assert got == data
        assert any(c[1] < len(comp) for c in ctx.calls)


def test_batch_output_is_bounded(monkeypatch):
    """1 MiB of zeros compresses ~1000x: with MAX_BATCH_OUT = 64 KiB the stream decodes the input
    in shorter prefixes instead of allocating the whole expansion at once."""
    data = bytes(1 << 20)
    comp, bounds = _stream(data, 8192)
    got, ctx = _run(monkeypatch, comp, bounds, io.BytesIO(comp), 1 << 20, max_out=64 << 10)
    assert got == data
    assert len(ctx.calls) > 8                         # many bounded batches, not one


def test_short_reads_decode_as_they_arrive(monkeypatch):
    """A slow pipe (700-byte pieces, nothing more ready after each): decoding starts before the
    whole batch has arrived."""
    rng = np.random.default_rng(2)
    data = rng.integers(0, 3, 300_000, dtype=np.uint8).tobytes()
    comp, bounds = _stream(data, 16384)
    got, ctx = _run(monkeypatch, comp, bounds, ShortReads(comp, 700), 1 << 20)
    assert got == data
    assert max(c[1] for c in ctx.calls) < len(comp)   # never waited for the whole stream


def test_fast_pipe_is_read_ahead_to_the_batch(monkeypatch):
    """A pipe with data waiting (available() > 0) returning 700-byte pieces is read on up to the
    batch: one decode for the whole stream, not one per pipe read."""
    rng = np.random.default_rng(2)
    data = rng.integers(0, 3, 300_000, dtype=np.uint8).tobytes()
    comp, bounds = _stream(data, 16384)
    got, ctx = _run(monkeypatch, comp, bounds, ShortReads(comp, 700, ready=1 << 16), 1 << 20)
    assert got == data
    assert len(ctx.calls) == 1


def test_unknown_readiness_reads_a_minimum_before_decoding(monkeypatch):
    """A source that cannot say whether more input is ready: short reads end the read-ahead only
    after MIN_UNKNOWN_READY new bytes, so decodes come in bounded numbers."""
    rng = np.random.default_rng(3)
    data = rng.integers(0, 3, 300_000, dtype=np.uint8).tobytes()
    comp, bounds = _stream(data, 16384)
    monkeypatch.setattr(streams.InflaterInputStream, "MIN_UNKNOWN_READY", 20_000)
    got, ctx = _run(monkeypatch, comp, bounds, ShortReads(comp, 700, ready=None), 1 << 20)
    assert got == data
    assert 2 <= len(ctx.calls) <= len(comp) // 20_000 + 2


class ErrorCtx:
    """The decode of a corrupted stream as the ABI reports it: the bytes before the error, then
    the Reason (+1), all from the oracle."""

    def __init__(self, stream):
        self.reason, self.out, self.bits = O.inflate(stream)

    def inflate_range_raw(self, in_addr, n, start_bit, end_bit, out_addr, dict_len, out_cap, flags):
        if len(self.out) > out_cap:
            return _lib.E_CAPACITY, len(self.out), 0
        ctypes.memmove(out_addr + dict_len, self.out, len(self.out))
        return O.REASONS.index(self.reason) + 1, len(self.out), self.bits

    def data_format_error(self, code):
        return ndfl.DataFormatException(ndfl.Reason(code - 1))


def _corrupt_stream():
    rng = np.random.default_rng(4)
    data = rng.integers(0, 3, 200_000, dtype=np.uint8).tobytes()
    comp = bytearray(O.deflate(data, "RLE_DYNAMIC", chunk_len=16384))
    for k in range(len(comp) * 3 // 4, len(comp)):
        bad = bytearray(comp)
        bad[k] ^= 0xFF
        reason, out, _ = O.inflate(bytes(bad))
        if reason is not None and len(out) > 50_000:
            return bytes(bad), out, reason
    raise AssertionError("no corruption found")


def test_error_raised_by_the_read_that_reaches_it():
    """Open.read throws from the call that reaches the error (D/decomp/Open.java:83-110): a read
    asking past the last good byte raises at once (its bytes land in b uncounted); a read ending
    exactly at the error returns normally and the next one raises; every later read that needs
    data raises again, an empty read returns 0 (DataFormatException is unchecked, so the stream does
    not enter its sticky state, D/InflaterInputStream.java:151-159)."""
    bad, good, reason = _corrupt_stream()
    s = streams.InflaterInputStream(io.BytesIO(bad), context=ErrorCtx(bad))
    b = bytearray(len(good) + 1000)
    with pytest.raises(ndfl.DataFormatException) as ei:
        s.read(b, 0, len(b))
    assert ei.value.reason.name == reason
    assert bytes(b[:len(good)]) == good
    assert s.read(b, 0, 0) == 0
    with pytest.raises(ndfl.DataFormatException):
        s.read(b, 0, 1)
    s = streams.InflaterInputStream(io.BytesIO(bad), context=ErrorCtx(bad))
    assert s.read(b, 0, len(good)) == len(good)      # up to the error: no exception yet
    with pytest.raises(ndfl.DataFormatException):
        s.read()
    with pytest.raises(ndfl.DataFormatException):
        s.read(b, 0, 10)
