"""The reference's command-line apps over the GPU codec: `python -m ndfl.gzip In Out.gz` is
S/gzip.java and `python -m ndfl.gunzip In.gz Out` is S/gunzip.java -- same arguments, stderr lines
and exit status 1 on a reported error.  As in the reference, a DataFormatException (unchecked in
Java) is not caught by gunzip: it ends the program with a stack trace and status 1."""
import datetime
import os
import sys
import time

from .streams import GzipInputStream, GzipMetadata, GzipOutputStream

_READ = 64 << 20


def _path_errors(args, usage):
    if len(args) != 2:
        return usage
    inp, out = args
    if not os.path.exists(inp):
        return f"Input path does not exist: {inp}"
    if os.path.isdir(inp):
        return f"Input path is a directory: {inp}"
    if os.path.isdir(out):
        return f"Output path is a directory: {out}"
    return None


def _speeds(inp, out, elapsed_ns):
    sys.stderr.write(f"Input  speed: {os.path.getsize(inp) / 1e6 / elapsed_ns * 1.0e9:.2f} MB/s\n")
    sys.stderr.write(f"Output speed: {os.path.getsize(out) / 1e6 / elapsed_ns * 1.0e9:.2f} MB/s\n")


def gzip_submain(args):
    """S/gzip.java:37-77.  Returns None or the error message."""
    msg = _path_errors(args, "Usage: java gzip InputFile OutputFile.gz")
    if msg:
        return msg
    inp, out = args
    mod = (os.stat(inp).st_mtime_ns // 1_000_000) // 1000          # File.lastModified() / 1000
    mod = (mod + 2**31) % 2**32 - 2**31                             # (int) cast
    meta = GzipMetadata("DEFLATE", False, mod if mod != 0 else None, 0, "UNIX", None, os.path.basename(inp),
                        None, True)
    t0 = time.perf_counter_ns()
    try:
        with open(inp, "rb") as fi, open(out, "wb") as fo:
            g = GzipOutputStream(fo, meta)
            while True:
                b = fi.read(_READ)
                if not b:
                    break
                g.write(b)
            g.finish()
    except OSError as e:
        return f"I/O exception: {e.strerror or e}"
    _speeds(inp, out, time.perf_counter_ns() - t0)
    return None


_OS_TEXT = {"FAT_FILESYSTEM": "FAT filesystem", "AMIGA": "Amiga", "VMS": "VMS", "UNIX": "Unix", "VM_CMS": "VM/CMS",
            "ATARI_TOS": "Atari TOS", "HPFS_FILESYSTEM": "HPFS filesystem", "MACINTOSH": "Macintosh",
            "Z_SYSTEM": "Z-System", "CPM": "CP/M", "TOPS_20": "TOPS-20", "NTFS_FILESYSTEM": "NTFS filesystem",
            "QDOS": "QDOS", "ACORN_RISCOS": "Acorn RISCOS", "UNKNOWN": "Unknown"}


def _instant(t):
    """java.time.Instant.EPOCH.plusSeconds(t).toString() for a whole-second instant."""
    t = (t + 2**31) % 2**32 - 2**31                                 # the record holds a Java int
    d = datetime.datetime(1970, 1, 1) + datetime.timedelta(seconds=t)
    return d.strftime("%Y-%m-%dT%H:%M:%SZ")


def gunzip_submain(args):
    """S/gunzip.java:37-109.  Returns None or the error message."""
    msg = _path_errors(args, "Usage: java gunzip InputFile.gz OutputFile")
    if msg:
        return msg
    inp, out = args
    try:
        with open(inp, "rb") as fi:
            g = GzipInputStream(fi)
            meta = g.getMetadata()
            err = sys.stderr
            mt = meta.modificationTimeUnixS
            err.write(f"Last modified: {_instant(mt) if mt is not None else 'N/A'}\n")
            xf = meta.extraFlags
            err.write("Extra flags: " + {2: "Maximum compression", 4: "Fastest compression"}.get(xf, f"Unknown ({xf})")
                      + "\n")
            err.write(f"Operating system: {_OS_TEXT[meta.operatingSystem]}\n")
            err.write(f"File mode: {'Text' if meta.isFileText else 'Binary'}\n")
            if meta.extraField is not None:
                err.write(f"Extra field: {len(meta.extraField)} bytes\n")
            if meta.fileName is not None:
                err.write(f"File name: {meta.fileName}\n")
            if meta.comment is not None:
                err.write(f"Comment: {meta.comment}\n")
            t0 = time.perf_counter_ns()
            with open(out, "wb") as fo:
                fo.write(g.readall())
            _speeds(inp, out, time.perf_counter_ns() - t0)
    except OSError as e:
        return f"I/O exception: {e.strerror or e}"
    return None


def _main(sub):
    msg = sub(sys.argv[1:])
    if msg is not None:
        sys.stderr.write(msg + "\n")
        sys.exit(1)
