"""Stream classes mirroring io.nayuki.deflate's public API on top of libndfl.so.

Java exception mapping: IllegalArgumentException -> ValueError, IllegalStateException ->
RuntimeError, IOException -> OSError, DataFormatException -> ndfl.DataFormatException.
"""
import ctypes
import enum
import dataclasses
import os
from typing import Optional

from . import _lib
from ._lib import check, load

INT_MAX = 2**31 - 1


def _ctx(context):
    from . import default_context
    return context if context is not None else default_context()


class DeflaterOutputStream:
    """D/DeflaterOutputStream.java:30-173.  Chunks of `dataLookaheadLimit` bytes from stream start
    become one block each; a chunk is flushed only once more data arrives (so the final block holds
    1..limit bytes, or 0 for empty input).  Many chunks are batched into one GPU call."""

    def __init__(self, out, dataLookaheadLimit=64 * 1024, historyLookbehindLimit=32 * 1024, strategy=None,
                 context=None, batch_bytes=64 << 20):
        from . import Strategy, _strategy_id, _batchable
        if out is None:
            raise TypeError("out")
        if (dataLookaheadLimit < 1 or historyLookbehindLimit < 0 or historyLookbehindLimit > 32 * 1024
                or dataLookaheadLimit + historyLookbehindLimit > INT_MAX):
            raise ValueError("Invalid capacities")
        self._out = out
        self._chunk = dataLookaheadLimit
        self._hist_limit = historyLookbehindLimit
        strategy = strategy if strategy is not None else Strategy.RLE_DYNAMIC
        # the batched GPU calls take the library's strategies whole; any other Strategy (a user
        # object with decide(), or trees the batched calls do not cover) runs chunk by chunk
        # through the plugin API, as Strategy.decide / Decision.compressTo (D/DeflaterOutputStream.java:119-137)
        self._plugin = None if _batchable(strategy) else strategy
        self._strategy = _strategy_id(strategy) if self._plugin is None else None
        self._strategy_obj = strategy
        self._ctx = _ctx(context)
        self._batch = max(batch_bytes, dataLookaheadLimit + 1)
        self._pending = bytearray()
        self._hist = b""
        self._bitbuf = 0          # pending partial byte
        self._bitlen = 0          # 0..7
        self._ended = False
        self._crc = None          # GzipOutputStream asks for a CRC pass fused into the encoder
        self._adler = None        # ZlibOutputStream: Adler-32 over each batch, on the GPU

    def getUnderlyingStream(self):
        if self._out is None:
            raise RuntimeError("Stream already closed")
        return self._out

    def write(self, b, off=0, length=None):
        if self._ended:
            raise RuntimeError("Stream already ended")
        if isinstance(b, int):
            self._pending.append(b & 0xFF)
        else:
            mv = memoryview(bytes(b))
            if length is None:
                length = len(mv) - off
            if off < 0 or length < 0 or off + length > len(mv):
                raise IndexError("Range out of bounds")
            self._pending += mv[off:off + length]
        if len(self._pending) > self._batch:
            self._flush(False)

    def _flush(self, final):
        n = len(self._pending)
        if final:
            take = n
        else:
            k = (n - 1) // self._chunk
            take = k * self._chunk
            if take == 0:
                return
        data = bytes(self._pending[:take])
        if self._plugin is not None:
            self._flush_plugin(data, final)
            del self._pending[:take]
            return
        L = load()
        cap = L.ndfl_deflate_bound(take, self._chunk) + 16
        out = ctypes.create_string_buffer(cap)
        src = ctypes.create_string_buffer(data, max(1, len(data)))
        hist = ctypes.create_string_buffer(self._hist, max(1, len(self._hist)))
        try:
            endbits, crc = self._ctx.deflate_chunks_raw(
                ctypes.addressof(hist) if self._hist else None, len(self._hist), self._hist_limit,
                ctypes.addressof(src), take, self._chunk, self._strategy, final, self._bitlen,
                ctypes.addressof(out), cap, 0, crc=self._crc)
        except _lib.NdflError as e:
            if e.code != _lib.E_UNSUPPORTED:
                raise
            # a configuration the batched call does not take (e.g. BinarySplit halvings of odd
            # lengths): the plugin path from here on
            self._plugin = self._strategy_obj
            self._flush_plugin(data, final)
            del self._pending[:take]
            return
        if self._crc is not None:
            self._crc = crc
        if self._adler is not None and data:
            self._adler = self._ctx.adler32(data, self._adler)
        nbytes = (endbits + 7) // 8
        raw = bytearray(out.raw[:nbytes])
        if raw:
            raw[0] |= self._bitbuf
        whole = endbits // 8
        self._out.write(bytes(raw[:whole]))
        self._bitlen = endbits % 8
        self._bitbuf = raw[whole] if self._bitlen else 0
        del self._pending[:take]
        if self._hist_limit:
            self._hist = (self._hist + data)[-self._hist_limit:]

    def _flush_plugin(self, data, final):
        """Chunk by chunk: Strategy.decide(combined, 0, historyLen, dataLen) then
        Decision.compressTo(bitOut, isFinal) (D/DeflaterOutputStream.java:119-137)."""
        from .plugin import BitBuffer, decide_any
        bo = BitBuffer(self._bitlen, self._bitbuf)
        n = len(data)
        pos = 0
        while True:
            k = min(self._chunk, n - pos)
            last = final and pos + k == n
            combined = self._hist + data[pos:pos + k]
            dec = decide_any(self._plugin, combined, 0, len(self._hist), k, self._ctx)
            dec.compressTo(bo, last)
            if self._hist_limit:
                self._hist = combined[-self._hist_limit:]
            pos += k
            if pos >= n:
                break
        if self._crc is not None and data:
            self._crc = self._ctx.crc32(data, self._crc)
        if self._adler is not None and data:
            self._adler = self._ctx.adler32(data, self._adler)
        self._out.write(bo.take_bytes())
        self._bitlen = bo.nbits & 7
        self._bitbuf = bo.partial

    def finish(self):
        if self._ended:
            raise RuntimeError("Stream already ended")
        self._flush(True)
        if self._bitlen:
            self._out.write(bytes([self._bitbuf]))   # BitOut.finish zero-pads (:164-169)
            self._bitbuf = 0
            self._bitlen = 0
        self._ended = True

    def close(self):
        if not self._ended:
            self.finish()
        if self._out is not None:
            self._out.close()
            self._out = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class _Pushback:
    """Mark support for a non-seekable underlying stream: the bytes the inflater read past the end of
    the DEFLATE data are pushed back and served first -- the BufferedInputStream that
    GzipInputStream / ZlibInputStream wrap around a non-markable stream (D/GzipInputStream.java:41-42,
    D/ZlibInputStream.java:39-40)."""

    def __init__(self, raw):
        self._raw = raw
        self._back = b""

    def unread(self, b):
        self._back = bytes(b) + self._back

    def read(self, n=-1):
        if n is None or n < 0:
            rest = self._raw.read()
            out, self._back = self._back + (rest or b""), b""
            return out
        out = self._back[:n]
        self._back = self._back[n:]
        while len(out) < n:
            b = self._raw.read(n - len(out))
            if not b:
                break
            out += b
        return out

    def read1(self, n=-1):
        """At most one read of the underlying stream (the pushed-back bytes first)."""
        if self._back:
            k = len(self._back) if n is None or n < 0 else n
            out, self._back = self._back[:k], self._back[k:]
            return out
        rd = getattr(self._raw, "read1", None) or self._raw.read
        return rd(n)

    def available(self):
        if self._back:
            return len(self._back)
        r = _input_ready(self._raw)
        return None if r is None else int(r)       # (None: the raw stream cannot tell)

    def close(self):
        self._raw.close()


def _markable(f):
    return hasattr(f, "unread") or (hasattr(f, "seek") and hasattr(f, "tell") and _seekable(f))


class InflaterInputStream:
    """D/InflaterInputStream.java:26-181 over Open (D/decomp/Open.java).  The underlying stream is
    read incrementally: batches of at least `inBufLen` (and by default 64 MiB) compressed bytes are
    decoded on the GPU with ndfl_inflate_range(NDFL_IN_PARTIAL), which stops at the last block
    boundary the batch completes; the decode continues from that bit with more input and the last
    32 KiB of output as the window.  Memory stays bounded by the batch, whatever the stream length,
    and pipes / sockets work.  read(b, off, len) returns -1..len and 0 only when len == 0; -1 at end
    of stream.  A DataFormatException is raised by the read call that reaches the error, as
    Open.read throws from inside the call (D/decomp/Open.java:83-110): a read that asks for more
    bytes than remain before the error copies those bytes into `b` uncounted and raises; a read that
    ends at or before the error returns normally; every later read that needs data raises it again.
    An OSError from the underlying stream is sticky (StickyException,
    D/InflaterInputStream.java:151-159)."""

    BATCH = 64 << 20
    WINDOW = 32768

    def __init__(self, inp, endExactly=False, inBufLen=16 * 1024, context=None):
        if inp is None:
            raise TypeError("in")
        if inBufLen <= 0:
            raise ValueError("Non-positive input buffer size")
        if endExactly and not _markable(inp):
            raise ValueError("Input stream not markable, cannot support detachment")
        self._in = inp
        self._end_exactly = endExactly
        self._ctx = _ctx(context)
        self._state = "open"
        self._batch = max(inBufLen, self.BATCH)
        self._ibuf = bytearray()      # unconsumed input; its first byte holds bit self._bit of the stream
        self._bit = 0
        self._eof = False             # the underlying stream is exhausted
        self._final = False           # the final block has been decoded
        self._window = b""            # last <= 32 KiB of output (the dictionary of the next batch)
        self._buf = b""               # decoded bytes not yet served
        self._pos = 0
        self._error = None
        self._sticky = None
        self._on_batch = None         # container hook: called with every decoded batch (CRC / Adler)

    MIN_UNKNOWN_READY = 1 << 20   # a short read from a source that cannot say whether more input
    # is ready ends the read-ahead only after this many new bytes

    def _read_more(self, want):
        """Read until `want` bytes are buffered or the stream ends.  A read that returns fewer bytes
        than asked for ends the read-ahead early only when the source has no more input ready
        (available() == 0, or nothing to select on its descriptor): then what is buffered is decoded
        first, as Open decodes from whatever its fill returned (D/decomp/Open.java:181-192), so a
        peer that waits for our output is not deadlocked -- while a pipe with data waiting is read on
        up to the batch size, so a fast producer still gets one GPU decode per batch, not one per
        pipe read."""
        rd = getattr(self._in, "read1", None) or self._in.read
        start = len(self._ibuf)
        try:
            while len(self._ibuf) < want and not self._eof:
                ask = want - len(self._ibuf)
                b = rd(ask)
                if not b:
                    self._eof = True
                else:
                    self._ibuf += b
                    if len(b) < ask:
                        ready = _input_ready(self._in)
                        if ready is False or (ready is None and len(self._ibuf) - start >= self.MIN_UNKNOWN_READY):
                            break
        except OSError as e:
            self._sticky = e
            raise

    MAX_BATCH_OUT = 1 << 30       # output bytes per decoded batch before the input is cut shorter

    def _fill(self):
        """Decode the next batch into self._buf (empty only at end of stream or on an error)."""
        from . import DataFormatException, Reason
        want = self._batch
        while True:
            self._read_more(want)
            n_all = len(self._ibuf)
            n = n_all
            wl = len(self._window)
            while True:
                # a prefix of the buffered input (the whole of it unless its output would exceed
                # MAX_BATCH_OUT): IN_PARTIAL unless it is all of a finished stream
                flags = 0 if (self._eof and n == n_all) else _lib.IN_PARTIAL
                src = ctypes.create_string_buffer(bytes(self._ibuf[:n]), max(1, n))
                room = 4 * n + 65536                      # bytes after the window (out_cap)
                while True:
                    out = ctypes.create_string_buffer(self._window, max(1, wl + room))
                    r, olen, bits = self._ctx.inflate_range_raw(ctypes.addressof(src), n, self._bit, None,
                                                                ctypes.addressof(out), wl, room, flags)
                    if r == _lib.E_CAPACITY and (olen <= self.MAX_BATCH_OUT or n <= 1):
                        room = olen + 16
                        continue
                    break
                if r == _lib.E_CAPACITY:
                    n = max(1, n // 2)                    # too much output for one batch: less input
                    continue
                if r == _lib.NEED_INPUT and olen == 0 and bits == self._bit and n < n_all:
                    # the shorter prefix completes no block: take the whole output of the full input
                    n = n_all
                    flags = 0 if self._eof else _lib.IN_PARTIAL
                    src = ctypes.create_string_buffer(bytes(self._ibuf), max(1, n))
                    room = 4 * n + 65536
                    while True:
                        out = ctypes.create_string_buffer(self._window, max(1, wl + room))
                        r, olen, bits = self._ctx.inflate_range_raw(ctypes.addressof(src), n, self._bit, None,
                                                                    ctypes.addressof(out), wl, room, flags)
                        if r == _lib.E_CAPACITY:
                            room = olen + 16
                            continue
                        break
                break
            if r == _lib.NEED_INPUT and olen == 0 and bits == self._bit:
                if self._eof:
                    check(_lib.E_INTERNAL, "ndfl_inflate_range")   # unreachable: no IN_PARTIAL at EOF
                # no block completed: read more.  The next attempt re-decodes the incomplete block
                # from its start (the ABI resumes at block boundaries only), so it waits for at least
                # as much new input again -- or for the source to run dry, see _read_more
                want = len(self._ibuf) + max(self._batch, len(self._ibuf))
                continue
            if r < 0 or (r > len(_lib.REASONS) and r != _lib.NEED_INPUT):
                check(r, "ndfl_inflate_range")
            data = out.raw[wl:wl + olen]
            self._window = (self._window + data)[-self.WINDOW:]
            self._buf, self._pos = data, 0
            if data and self._on_batch is not None:
                self._on_batch(data)
            if r == _lib.NEED_INPUT:
                del self._ibuf[:bits // 8]
                self._bit = bits % 8
                return
            if r == 0:
                self._final = True
                used = (bits + 7) // 8          # a byte with some bits consumed counts as consumed
                rest = bytes(self._ibuf[used:])
                self._ibuf = bytearray()
                if self._end_exactly and rest:   # Open.finish (D/decomp/Open.java:113-124)
                    if hasattr(self._in, "unread"):
                        self._in.unread(rest)
                    else:
                        self._in.seek(-len(rest), os.SEEK_CUR)
                return
            self._error = self._ctx.data_format_error(r)
            return

    def _ensure(self):
        # (a batch may end at a boundary after blocks with no output, e.g. empty stored blocks)
        while self._pos == len(self._buf) and not self._final and self._error is None:
            self._fill()

    def _raise_error(self):
        # DataFormatException is unchecked in the reference (a RuntimeException,
        # D/DataFormatException.java:15): InflaterInputStream does not turn it into its sticky state,
        # so an empty read still returns 0; a later read that needs data raises it again here (the
        # reference's decoder would go on from the bits after the bad symbol)
        raise self._error

    def read(self, b=None, off=0, length=None):
        """read() -> int byte or -1;  read(bytearray, off, len) -> count or -1."""
        if self._state == "closed":
            raise RuntimeError("Stream already closed")
        if self._sticky is not None:
            raise self._sticky
        if b is None:
            self._ensure()
            if self._pos < len(self._buf):
                v = self._buf[self._pos]
                self._pos += 1
                return v
            if self._error is not None:
                self._raise_error()
            return -1
        if length is None:
            length = len(b) - off
        if off < 0 or length < 0 or off + length > len(b):
            raise IndexError("Range out of bounds")
        total = 0
        while total < length:
            self._ensure()
            avail = len(self._buf) - self._pos
            if avail == 0:
                break
            k = min(avail, length - total)
            b[off + total:off + total + k] = self._buf[self._pos:self._pos + k]
            self._pos += k
            total += k
        if total < length and self._error is not None:
            self._raise_error()          # the bytes before the error are in b, uncounted
        if total == 0 and length > 0:
            return -1
        if total == 0 and self._final and self._pos == len(self._buf):
            return -1          # len == 0 at end of stream (D/decomp/Open.java:109)
        return total

    def readall(self):
        if self._sticky is not None:
            raise self._sticky
        if self._error is not None and self._pos == len(self._buf):
            self._raise_error()
        parts = []
        while True:
            self._ensure()
            if self._pos < len(self._buf):
                parts.append(self._buf[self._pos:])
                self._pos = len(self._buf)
                continue
            break
        if self._error is not None:
            self._raise_error()
        return b"".join(parts)

    def close(self):
        if self._state != "closed" and self._in is not None:
            self._in.close()
        self._state = "closed"


def _input_ready(f):
    """Whether the source has input ready without blocking: its available() (a Java-style stream),
    else a zero-timeout select on its descriptor (pipes, sockets; regular files are always ready),
    else None (unknown)."""
    av = getattr(f, "available", None)
    if callable(av):
        try:
            n = av()
        except Exception:
            return None
        return None if n is None else n > 0
    try:
        fd = f.fileno()
    except Exception:
        return None
    try:
        import select
        return bool(select.select([fd], [], [], 0)[0])
    except Exception:
        return None


def _seekable(f):
    try:
        return f.seekable()
    except Exception:
        return False


# ---- gzip container (RFC 1952) --------------------------------------------------------------

OS_NAMES = ["FAT_FILESYSTEM", "AMIGA", "VMS", "UNIX", "VM_CMS", "ATARI_TOS", "HPFS_FILESYSTEM", "MACINTOSH",
            "Z_SYSTEM", "CPM", "TOPS_20", "NTFS_FILESYSTEM", "QDOS", "ACORN_RISCOS", "UNKNOWN"]


@dataclasses.dataclass
class GzipMetadata:
    """D/GzipMetadata.java:30-242 (record components in the same order)."""
    compressionMethod: str = "DEFLATE"
    isFileText: bool = False
    modificationTimeUnixS: Optional[int] = None
    extraFlags: int = 0
    operatingSystem: str = "UNIX"
    extraField: Optional[bytes] = None
    fileName: Optional[str] = None
    comment: Optional[str] = None
    hasHeaderCrc: bool = False

    def __post_init__(self):
        if self.modificationTimeUnixS == 0:
            raise ValueError("Modification timestamp is zero")
        if self.extraFlags >> 8 != 0:
            raise ValueError("Invalid extra flags value")
        if self.extraField is not None and len(self.extraField) > 0xFFFF:
            raise ValueError("Extra field too long")
        if self.operatingSystem not in OS_NAMES:
            raise ValueError("operatingSystem")

    def header_bytes(self):
        flags = ((1 if self.isFileText else 0) | (2 if self.hasHeaderCrc else 0) |
                 (4 if self.extraField is not None else 0) | (8 if self.fileName is not None else 0) |
                 (16 if self.comment is not None else 0))
        mt = self.modificationTimeUnixS or 0
        osb = 0xFF if self.operatingSystem == "UNKNOWN" else OS_NAMES.index(self.operatingSystem)
        h = bytearray([0x1F, 0x8B, 8, flags]) + (mt & 0xFFFFFFFF).to_bytes(4, "little") + bytes([self.extraFlags, osb])
        if self.extraField is not None:
            h += len(self.extraField).to_bytes(2, "little") + self.extraField
        if self.fileName is not None:
            h += self.fileName.encode("latin-1") + b"\0"
        if self.comment is not None:
            h += self.comment.encode("latin-1") + b"\0"
        return h

    def write(self, out, context=None):
        h = self.header_bytes()
        if self.hasHeaderCrc:
            crc = _ctx(context).crc32(bytes(h)) & 0xFFFF
            h += crc.to_bytes(2, "little")
        out.write(bytes(h))

    @staticmethod
    def read(inp, context=None):
        """GzipMetadata.read (D/GzipMetadata.java:73-146); raises DataFormatException(reason)."""
        from . import DataFormatException, Reason
        got = bytearray()

        def rd(n):
            b = inp.read(n)
            if b is None or len(b) < n:
                raise DataFormatException(Reason.UNEXPECTED_END_OF_STREAM)
            got.extend(b)
            return b

        if rd(2) != b"\x1f\x8b":
            raise DataFormatException(Reason.GZIP_INVALID_MAGIC_NUMBER, "Invalid GZIP magic number")
        cm = rd(1)[0]
        if cm != 8:
            raise DataFormatException(Reason.UNSUPPORTED_COMPRESSION_METHOD, f"Unsupported compression method: {cm}")
        flags = rd(1)[0]
        if flags & 0xE0:
            raise DataFormatException(Reason.GZIP_RESERVED_FLAGS_SET, "Reserved flags are set")
        mt = int.from_bytes(rd(4), "little")
        xfl = rd(1)[0]
        osv = rd(1)[0]
        if osv < 14:
            osname = OS_NAMES[osv]
        elif osv == 0xFF:
            osname = "UNKNOWN"
        else:
            raise DataFormatException(Reason.GZIP_UNSUPPORTED_OPERATING_SYSTEM, "Unsupported operating system value")
        extra = None
        if flags & 4:
            ln = int.from_bytes(rd(2), "little")
            extra = bytes(rd(ln))
        name = comment = None
        if flags & 8:
            s = bytearray()
            while (c := rd(1)[0]) != 0:
                s.append(c)
            name = s.decode("latin-1")
        if flags & 16:
            s = bytearray()
            while (c := rd(1)[0]) != 0:
                s.append(c)
            comment = s.decode("latin-1")
        hcrc = bool(flags & 2)
        if hcrc:
            expect = _ctx(context).crc32(bytes(got)) & 0xFFFF
            actual = int.from_bytes(rd(2), "little")
            if actual != expect:
                raise DataFormatException(Reason.HEADER_CHECKSUM_MISMATCH, "Header CRC-16 mismatch")
        return GzipMetadata("DEFLATE", bool(flags & 1), mt if mt != 0 else None, xfl, osname, extra, name, comment,
                            hcrc)


class GzipOutputStream:
    """D/GzipOutputStream.java:19-80.  The CRC-32 pass is fused into the GPU encoder kernel."""

    def __init__(self, out, meta, context=None):
        dout = out if isinstance(out, DeflaterOutputStream) else DeflaterOutputStream(out, context=context)
        if meta is None:
            raise TypeError("meta")
        meta.write(dout.getUnderlyingStream(), context=dout._ctx)
        self._d = dout
        self._d._crc = 0
        self._len = 0
        self._ended = False

    def write(self, b, off=0, length=None):
        if self._ended:
            raise RuntimeError("Stream already ended")
        if isinstance(b, int):
            b = bytes([b & 0xFF])
        mv = memoryview(bytes(b))
        if length is None:
            length = len(mv) - off
        self._d.write(mv, off, length)
        self._len += length

    def finish(self):
        if self._ended:
            raise RuntimeError("Stream already ended")
        self._d.finish()
        crc = self._d._crc
        out = self._d.getUnderlyingStream()
        out.write(crc.to_bytes(4, "little"))
        out.write((self._len & 0xFFFFFFFF).to_bytes(4, "little"))
        self._ended = True

    def close(self):
        if not self._ended:
            self.finish()
        self._d.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class GzipInputStream:
    """D/GzipInputStream.java:22-100.  Single member; trailing bytes ignored.  The CRC-32 and length
    are updated on the GPU over every batch the inflater decodes."""

    def __init__(self, inp, context=None):
        if inp is None:
            raise TypeError("in")
        self._ctx = _ctx(context)
        self.metadata = GzipMetadata.read(inp, self._ctx)
        if not _markable(inp):
            inp = _Pushback(inp)
        self._raw = inp
        self._inf = InflaterInputStream(inp, True, context=self._ctx)
        self._inf._on_batch = self._update
        self._done = False
        self._crc = 0
        self._len = 0

    def _update(self, data):
        self._crc = self._ctx.crc32(data, self._crc)
        self._len += len(data)

    def getMetadata(self):
        return self.metadata

    def _trailer(self):
        from . import DataFormatException, Reason
        t = self._raw.read(8)
        if t is None or len(t) < 8:
            raise DataFormatException(Reason.UNEXPECTED_END_OF_STREAM)
        if int.from_bytes(t[:4], "little") != self._crc:
            raise DataFormatException(Reason.DECOMPRESSED_CHECKSUM_MISMATCH, "Decompression CRC-32 mismatch")
        if int.from_bytes(t[4:], "little") != (self._len & 0xFFFFFFFF):
            raise DataFormatException(Reason.DECOMPRESSED_SIZE_MISMATCH, "Decompressed size mismatch")

    def readall(self):
        if self._done:
            return b""
        out = self._inf.readall()
        self._done = True
        self._trailer()
        return out

    def read(self, b=None, off=0, length=None):
        if self._done:
            return -1
        r = self._inf.read(b, off, length)
        if r == -1:
            self._done = True
            self._trailer()
        return r

    def close(self):
        self._raw.close()


class ZlibMetadata:
    """D/ZlibMetadata.java:19-127 (record of compressionMethod, compressionInfo, presetDictionary,
    compressionLevel).  presetDictionary is None or the 32-bit DICTID."""

    class CompressionMethod(enum.Enum):
        DEFLATE = 0
        RESERVED = 1

    class CompressionLevel(enum.Enum):
        FASTEST = 0
        FAST = 1
        DEFAULT = 2
        MAXIMUM = 3

    CHECKSUM_MODULUS = 31

    def __init__(self, compressionMethod, compressionInfo, presetDictionary, compressionLevel):
        if compressionMethod is None or compressionLevel is None:
            raise TypeError("null")
        if compressionInfo >> 4 != 0 or (compressionMethod == ZlibMetadata.CompressionMethod.DEFLATE
                                         and compressionInfo > 7):
            raise ValueError("Invalid compression info value")           # (:37-38)
        self.compressionMethod = compressionMethod
        self.compressionInfo = compressionInfo
        self.presetDictionary = presetDictionary
        self.compressionLevel = compressionLevel

    def __eq__(self, o):
        return isinstance(o, ZlibMetadata) and (self.compressionMethod, self.compressionInfo, self.presetDictionary,
                                                  self.compressionLevel) == (o.compressionMethod, o.compressionInfo,
                                                                             o.presetDictionary, o.compressionLevel)

    @staticmethod
    def read(inp):
        """(:52-83): header checksum, method, DICTID (big-endian), level."""
        from . import DataFormatException, Reason
        hb = inp.read(2)
        if hb is None or len(hb) < 2:
            raise DataFormatException(Reason.UNEXPECTED_END_OF_STREAM)
        cmf, flg = hb[0], hb[1]
        if (cmf << 8 | flg) % ZlibMetadata.CHECKSUM_MODULUS != 0:
            raise DataFormatException(Reason.HEADER_CHECKSUM_MISMATCH, "Header checksum mismatch")
        cm = cmf & 0xF
        if cm == 8:
            method = ZlibMetadata.CompressionMethod.DEFLATE
        elif cm == 15:
            method = ZlibMetadata.CompressionMethod.RESERVED
        else:
            raise DataFormatException(Reason.UNSUPPORTED_COMPRESSION_METHOD, f"Unsupported compression method: {cm}")
        dictid = None
        if (flg >> 5) & 1:
            d = inp.read(4)
            if d is None or len(d) < 4:
                raise DataFormatException(Reason.UNEXPECTED_END_OF_STREAM)
            dictid = int.from_bytes(d, "big")
        return ZlibMetadata(method, cmf >> 4, dictid, ZlibMetadata.CompressionLevel(flg >> 6))

    def header_bytes(self):
        """(:90-108)."""
        cm = 8 if self.compressionMethod == ZlibMetadata.CompressionMethod.DEFLATE else 15
        cmf = cm | self.compressionInfo << 4
        flg = (1 if self.presetDictionary is not None else 0) << 5 | self.compressionLevel.value << 6
        flg |= (31 - (cmf << 8 | flg) % 31) % 31
        out = bytes([cmf, flg])
        if self.presetDictionary is not None:
            out += (self.presetDictionary & 0xFFFFFFFF).to_bytes(4, "big")
        return out

    def write(self, out):
        out.write(self.header_bytes())


ZlibMetadata.DEFAULT = ZlibMetadata(ZlibMetadata.CompressionMethod.DEFLATE, 7, None,
                                    ZlibMetadata.CompressionLevel.DEFAULT)


class ZlibOutputStream:
    """D/ZlibOutputStream.java:19-91.  Adler-32 on the GPU over each batch the encoder takes."""

    def __init__(self, out, meta, context=None):
        dout = out if isinstance(out, DeflaterOutputStream) else DeflaterOutputStream(out, context=context)
        if meta is None:
            raise TypeError("meta")
        meta.write(dout.getUnderlyingStream())
        self._d = dout
        self._d._adler = 1
        self._ended = False

    def write(self, b, off=0, length=None):
        if self._ended:
            raise RuntimeError("Stream already ended")
        if isinstance(b, int):
            b = bytes([b & 0xFF])
        mv = memoryview(bytes(b))
        if length is None:
            length = len(mv) - off
        self._d.write(mv, off, length)

    def finish(self):
        if self._ended:
            raise RuntimeError("Stream already ended")
        self._d.finish()
        self._d.getUnderlyingStream().write(self._d._adler.to_bytes(4, "big"))     # (:70-71)
        self._ended = True

    def close(self):
        if not self._ended:
            self.finish()
        self._d.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class ZlibInputStream:
    """D/ZlibInputStream.java:22-100: header, inflate with exact end, big-endian Adler-32 trailer
    (EOF -> UNEXPECTED_END_OF_STREAM, mismatch -> DECOMPRESSED_CHECKSUM_MISMATCH).  A preset
    dictionary is recorded but not applied, as in the reference.  Adler-32 on the GPU per batch."""

    def __init__(self, inp, context=None):
        if inp is None:
            raise TypeError("in")
        self._ctx = _ctx(context)
        self.metadata = ZlibMetadata.read(inp)
        if not _markable(inp):
            inp = _Pushback(inp)
        self._raw = inp
        self._inf = InflaterInputStream(inp, True, context=self._ctx)
        self._inf._on_batch = self._update
        self._done = False
        self._adler = 1

    def _update(self, data):
        self._adler = self._ctx.adler32(data, self._adler)

    def getMetadata(self):
        return self.metadata

    def _trailer(self):
        from . import DataFormatException, Reason
        t = self._raw.read(4)
        if t is None or len(t) < 4:
            raise DataFormatException(Reason.UNEXPECTED_END_OF_STREAM)
        if int.from_bytes(t, "big") != self._adler:
            raise DataFormatException(Reason.DECOMPRESSED_CHECKSUM_MISMATCH, "Decompression Adler-32 mismatch")

    def readall(self):
        if self._done:
            return b""
        out = self._inf.readall()
        self._done = True
        self._trailer()
        return out

    def read(self, b=None, off=0, length=None):
        if self._done:
            return -1
        r = self._inf.read(b, off, length)
        if r == -1:
            self._done = True
            self._trailer()
        return r

    def close(self):
        self._raw.close()
