"""Headline benchmark: DEFLATE round trip (compress + decompress) on MI355X.

metric  "input MiB/s (compress+decompress)" (BASELINE.json): bytes fed to the two operations
        (N uncompressed into the encoder + C compressed into the decoder) per second of the step,
        MiB = 2^20, whole job over all ranks.
step    one round trip over one batch: the rank's share of the 4 GiB config-4 corpus
        (Silesia-style mix, seed 0xC4; all of it at N = 1) is compressed with the gzip default encoder
        (RLE_DYNAMIC, 64 KiB blocks, bit-exact with the reference) into one DEFLATE stream, and that
        stream is decompressed again.  Inputs and outputs are resident in HBM (device pointers
        through the C ABI); no host copies inside the timed region.
N > 1   rank r owns chunks [r*K, (r+1)*K) of ONE global stream.  Ranks exchange the bytes before
        their shard (history) and their compressed bit totals (RCCL all_gather over xGMI), shift
        their bits to the global bit offset on device, and decode their own bit range with the
        previous rank's last 32 KiB of output as the dictionary (RCCL point-to-point).
        --scaling strong (default): config 4 as BASELINE.json defines it, 4 GiB in total split over
        the ranks, so every N shares the N = 1 workload; --scaling weak: 4 GiB per rank (seed
        0xC4 + rank).  The step also gathers the global stream onto rank 0 (RCCL point-to-point into
        its byte offsets, shared bytes ORed on device).
Run: python bench.py [--gpus N --steps K --warmup W].  With --gpus N > 1 and no WORLD_SIZE in the
environment, bench.py starts N ranks itself (torch.distributed.run on 127.0.0.1, before anything
touches the GPU) and exits with their status; under torch.distributed.run it is one rank.
N > 1 gathers the global stream onto rank 0 in every step by default (north_star: "RCCL gather over
xGMI to reassemble the output stream"; --no-gather leaves it out).
bit_exact: every rank compares its WHOLE shard's stream with the oracle's (chunk-parallel on the
host, outside the timed region), and the flag is the AND over ranks; with N > 1 and strong scaling
rank 0 also compares the stream the gather assembled with the oracle's encoding of the whole corpus.
Every collective has a timeout (--dist-timeout, 120 s): a rank that stalls ends the run with an error
instead of a hang.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "deflate-library-java_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK = 8.0e12          # MI355X HBM3E spec, bytes/s (MI355X_MICROARCH.md)
# the encoder is a 4-kernel pipeline (deflate_split.hip); its HIP-event time spans all four
DEFLATE_KERNELS = "ndfl_deflate_hist_kernel+ndfl_deflate_codes_kernel+ndfl_deflate_offsets_kernel+ndfl_deflate_emit_kernel"
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=4 << 30, help="corpus bytes (in total; per rank with --scaling weak)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 30, help="bytes for the CPU baseline leg (about 20 s of oracle work)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL over xGMI); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="strong (default): --size bytes in total (config 4); weak: --size bytes per rank")
    ap.add_argument("--dist-timeout", type=float, default=120.0,
                    help="seconds any collective / point-to-point exchange may wait before the run fails")
    ap.add_argument("--gather", action="store_true", help="(default for N > 1) gather the global stream onto rank 0")
    ap.add_argument("--no-gather", action="store_true", help="N > 1: leave the gather to rank 0 out of the step")
    ap.add_argument("--verify-threads", type=int, default=0, help="host threads of the full-stream oracle check "
                    "(0: min(16, cpus / ranks))")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    import torch
    import ndfl
    import corpus

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        from ndfl import parallel as P
        P.init_process_group(dist, args.backend, torch.device("cuda", local) if args.backend == "nccl" else None,
                             args.dist_timeout)

    gather = world > 1 and not args.no_gather
    if args.scaling == "strong" and world > 1:
        # one global corpus, rank r takes its 64 KiB-aligned share (the last rank the remainder)
        per = (args.size // world) // 65536 * 65536
        off = rank * per
        n = per if rank + 1 < world else args.size - off
        # rank 0 generates the corpus once and sends every rank its share (point to point; the
        # ranks of a one-GPU rehearsal would otherwise all generate 4 GiB on the same card)
        from ndfl import parallel as P
        shares = [((args.size // world) // 65536 * 65536) * r for r in range(world)] + [args.size]
        if rank == 0:
            full = corpus.c4_mixed(args.size, seed=0xC4, device="cuda")
            data = full[off:off + n].clone()
            for r in range(1, world):
                P._send(dist, full[shares[r]:shares[r + 1]].contiguous(), r)
            if not gather:
                del full              # (rank 0 keeps it to check the gathered stream)
        else:
            data = torch.empty(n, dtype=torch.uint8, device="cuda")
            P._recv(dist, data, 0)
    else:
        n = args.size
        data = corpus.c4_mixed(n, seed=0xC4 + rank, device="cuda")
    torch.cuda.synchronize()
    progress(rank, f"corpus ready ({n / 2**30:g} GiB on cuda:{local})")
    ctx = ndfl.Context(local)
    L = ndfl._lib.load()
    cap = L.ndfl_deflate_bound(n, 65536) + 64
    # IN_PAD_BYTES of slack after the stream: the decode reads the encoder's output in place
    comp = torch.empty(cap + ndfl.IN_PAD_BYTES, dtype=torch.uint8, device="cuda")
    RLE_DYNAMIC = 3
    DEV = ndfl.IN_DEVICE | ndfl.OUT_DEVICE
    state = {"dict_len": 0}
    if world > 1:
        from ndfl import parallel as P
        codec = P.DeviceCodec(ctx, torch)
        shifted = torch.empty(cap + 1, dtype=torch.uint8, device="cuda")
        dec = torch.empty(P.WINDOW + n + 64, dtype=torch.uint8, device="cuda")
    else:
        dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")

    def step():
        if world == 1:
            endbits, _ = ctx.deflate_chunks_raw(None, 0, 32768, data.data_ptr(), n, 65536, RLE_DYNAMIC, True, 0,
                                                comp.data_ptr(), cap, DEV)
            t_c = ctx.timings()["deflate"]
            cbytes = (endbits + 7) // 8
            # the NDFL_IN_PADDED contract: zero bytes after the stream (the encoder's last word is
            # already zero-filled past its end bit; the slack is not written by it)
            comp[cbytes:cbytes + ndfl.IN_PAD_BYTES].zero_()
            torch.cuda.current_stream().synchronize()
            r, olen, bits = ctx.inflate_raw(comp.data_ptr(), cbytes, dec.data_ptr(), dec.numel(),
                                            DEV | ndfl.IN_PADDED)
            ndfl.check(r, "inflate")
        else:
            # one global stream: history halo + seam index + realignment, then range decode with the
            # window chain (ndfl/parallel.py)
            part = P.deflate_shard(codec, dist, torch, data, rank, world, work=comp, out=shifted)
            state["hist"] = part.hist
            t_c = ctx.timings()["deflate"]
            endbits = part.nbits
            cbytes = (endbits + 7) // 8
            # the gather runs on RCCL's stream while this rank decodes its own range (the parts it
            # moves are final once deflate_shard returns); the step ends when both are done
            pend = P.gather_stream(codec, dist, torch, part, rank, world, out=state.get("stream"),
                                   async_op=True) if gather else None
            r, olen, dl = P.inflate_shard(codec, dist, torch, part, dec, rank, world)
            if pend is not None:
                state["stream"] = pend.wait()
            state["dict_len"] = dl
            state["total_bits"] = part.bit_offsets[-1]
        if r != 0:
            raise RuntimeError(f"decode error {r}")
        tm = ctx.timings()
        state.update(endbits=endbits, cbytes=cbytes, olen=olen, t_deflate=t_c, t_emit=tm["inflate_emit"],
                     t_find=tm["inflate_find"], t_count=tm["inflate_count"], t_inflate_span=tm["inflate_span"],
                     chains=tm["inflate_chains"], repairs=tm["inflate_repairs"], cands=tm["inflate_candidates"])
        return cbytes

    for _ in range(args.warmup):
        step()
    progress(rank, f"{args.warmup} warmup steps done")
    if not args.no_verify:
        assert state["olen"] == n, (state["olen"], n)
        dl = state["dict_len"]
        assert torch.equal(dec[dl:dl + n], data), "round trip mismatch"

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    t1 = time.perf_counter()
    per = (t1 - t0) / args.steps
    progress(rank, f"{args.steps} timed steps: {per * 1e3:.3f} ms per step")
    c_total = state["cbytes"]
    if dist is not None:
        cdev = "cpu" if args.backend == "gloo" else "cuda"
        t = torch.tensor([per], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        per = float(t.item())
        cb = torch.tensor([state["cbytes"]], dtype=torch.int64, device=cdev)
        dist.all_reduce(cb)
        c_total = int(cb.item())

    total_n = n
    if dist is not None:
        tn = torch.tensor([n], dtype=torch.int64, device="cpu" if args.backend == "gloo" else "cuda")
        dist.all_reduce(tn)
        total_n = int(tn.item())
    total_in = total_n + c_total         # bytes fed to compress + bytes fed to decompress
    value = total_in / per / MIB

    # roofline of the dominant kernel (longest average launch): algorithmic bytes per launch are
    # N + C for the encoder and the decoder's write pass, C for the decoder's read-only passes
    # (header finder + strict stage, count pass) -- SURVEY §8d
    kd, ke = state["t_deflate"], state["t_emit"]
    cands = [(DEFLATE_KERNELS, kd, n + state["cbytes"]),
             ("ndfl_inflate_count_wave_kernel", state["t_count"], state["cbytes"]),
             ("ndfl_inflate_find_compact_kernel+ndfl_inflate_strict_kernel", state["t_find"], state["cbytes"]),
             ("ndfl_inflate_emit_fast_kernel+ndfl_inflate_emit_wave_kernel", ke, n + state["cbytes"])]
    dom, kms, alg = max(cands, key=lambda x: x[1])
    achieved = alg / (kms / 1e3)
    traffic, traffic_src = pmc_traffic(dom, n)

    # bit-exactness of the whole shard: `comp` holds this rank's stream at bit 0 (the single-GPU
    # stream, or the shard before its realignment), compared with the oracle's encoding of the same
    # chunks with the same history and final flag
    exact = None
    if not args.no_cpu:
        threads = args.verify_threads or max(1, min(16, (os.cpu_count() or 1) // world))
        hist = state.get("hist")
        progress(rank, "whole-shard oracle check")
        exact = verify_stream(data, None if hist is None else hist.cpu().numpy().tobytes(), rank == world - 1,
                              comp, state["endbits"], threads)
        progress(rank, f"whole-shard oracle check: bit_exact {exact['bit_exact']}")
        if dist is not None:
            f = torch.tensor([1 if exact["bit_exact"] else 0], dtype=torch.int64,
                             device="cpu" if args.backend == "gloo" else "cuda")
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            exact["all_ranks"] = bool(f.item())
        if rank == 0 and gather and args.scaling == "strong":
            # the stream rank 0 actually holds after the last step's gather (parts received into a
            # reused buffer while the shards decoded) against the oracle's single-stream encoding
            # of the whole corpus: the one-GPU stream of the same bytes, bit for bit
            progress(rank, "gathered-stream oracle check")
            g = verify_stream(full, None, True, state["stream"], state["total_bits"],
                              args.verify_threads or max(1, min(16, os.cpu_count() or 1)))
            exact["gathered"] = {k: g[k] for k in ("bit_exact", "bits_compared", "sha256", "total_s")}
            del full
    cpu = None
    if rank == 0 and not args.no_cpu:
        progress(rank, "CPU baseline (oracle, 1 thread)")
        cpu = cpu_baseline(data, args.cpu_sample)
        cpu["bit_exact"] = (exact["all_ranks"] and exact.get("gathered", {"bit_exact": True})["bit_exact"]) \
            if world > 1 else exact["bit_exact"]
        cpu["verify"] = exact

    if rank == 0:
        line = {
            "metric": "input MiB/s (compress+decompress)",
            "value": round(value, 1),
            "unit": "MiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(per * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (config-4 Silesia-style mix, generated on device, " +
                    ("seed 0xC4, one corpus split over the ranks)" if args.scaling == "strong" and world > 1
                     else "seed 0xC4+rank)"),
            "config": {"workload": "config4: gzip-default (RLE_DYNAMIC, 64 KiB blocks) compress + decompress of a "
                                   + (f"{args.size / 2**30:g} GiB mixed corpus in total" if args.scaling == "strong" and world > 1
                                      else f"{n / 2**30:g} GiB mixed corpus per GPU") + ", bit-exact",
                       "bytes_per_gpu": n, "bytes_total": total_n, "compressed_bytes": c_total,
                       "ratio": round(c_total / total_n, 4), "parallelism": f"shard-by-block x{world}",
                       "gather_to_rank0": gather},
            "phases_ms": {"deflate_kernel": round(kd, 3), "inflate_find": round(state["t_find"], 3),
                          "inflate_count": round(state["t_count"], 3), "inflate_emit": round(ke, 3),
                          "inflate_device_span": round(state["t_inflate_span"], 3),
                          "inflate_chains": int(state["chains"]), "inflate_repairs": int(state["repairs"]),
                          "inflate_candidates": int(state["cands"])},
            # per direction, against the 8 TB/s peak: the encoder reads N and writes C; the decoder reads
            # C and writes N.  north_star's decompress bar is quoted on the read side (C / span); at
            # N >= C a decoder moving C + N bytes cannot read faster than peak * C / (C + N), so the
            # (C + N) fraction is the one a decoder can approach ("The decompress bar")
            "directions": directions(n, state["cbytes"], kd, state["t_inflate_span"]),
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved / 1e9, 2), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": alg, "avg_kernel_ms": round(kms, 3)},
            "cpu_baseline": cpu,
            "bit_exact": None if cpu is None else cpu.get("bit_exact"),
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


_T_START = time.perf_counter()


def progress(rank, msg):
    """One progress line on stderr (the JSON result stays the only stdout line)."""
    print(f"[bench rank {rank} +{time.perf_counter() - _T_START:.1f}s] {msg}", file=sys.stderr, flush=True)


def launch_ranks(n):
    """bench.py --gpus N without a launcher: run N ranks under torch.distributed.run (one process
    per GPU, rendezvous on 127.0.0.1) as a child process and return its exit status.  Nothing here
    touches the GPU, so the ranks are the only processes that do."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def directions(n, c, deflate_ms, inflate_span_ms):
    """Achieved bytes per second of each direction on one rank (algorithmic bytes / device span) and
    their fractions of the HBM peak: compress moves N + C, decompress C + N, and the decompress read
    side alone is C / span (north_star's bar)."""
    def rate(b, ms):
        return b / (ms / 1e3) if ms > 0 else 0.0
    comp = rate(n + c, deflate_ms)
    dec = rate(c + n, inflate_span_ms)
    rd = rate(c, inflate_span_ms)
    return {"compress": {"bytes": n + c, "ms": round(deflate_ms, 3), "GBps": round(comp / 1e9, 1),
                         "frac_of_peak": round(comp / HBM_PEAK, 4)},
            "decompress": {"bytes": c + n, "ms": round(inflate_span_ms, 3), "GBps": round(dec / 1e9, 1),
                           "frac_of_peak": round(dec / HBM_PEAK, 4), "read_GBps": round(rd / 1e9, 1),
                           "read_frac_of_peak": round(rd / HBM_PEAK, 4),
                           "read_frac_ceiling": round(c / (c + n), 4) if c + n else None}}


def pmc_traffic(kernel, n):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 --pmc summary of this same
    bench command (profiles/rNN_traffic.json, made by scripts/profile_bench.sh + scripts/traffic_summary.py
    from a FETCH_SIZE and a WRITE_SIZE pass).  FETCH_SIZE is corrected per kernel by the factor the
    JSON records for it (`fetch_correction`, calibrated on known byte counts in the kernel's own load
    shapes by scripts/r06/fetch_calib.hip; the guide's x2 for 16-B/lane and LDS-DMA loads); WRITE_SIZE
    is taken as reported.  Counters cannot be read from inside the timed run, so the value is the
    profiled one, quoted only for the default 4 GiB workload."""
    import glob
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_traffic.json")))
    path = found[-1] if found else os.path.join(ROOT, "profiles", "r01_traffic.json")
    if n != 4 << 30 or not os.path.exists(path):
        return None, None
    tab = json.load(open(path))
    recs = [tab.get(k) for k in kernel.split("+")]      # a '+' name is a pipeline: bytes summed
    if any(r is None for r in recs):
        return None, None
    fb, wb = sum(r["fetch_bytes"] for r in recs), sum(r["write_bytes"] for r in recs)
    return fb + wb, f"profiles/{os.path.basename(path)} (fetch {fb} B + write {wb} B per launch)"


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _append_final_empty_block(comp, nbits):
    """A non-final stream of nbits bits + a final fixed-Huffman block holding only end-of-block
    (bits 1, 01, 0000000): a valid stream with the same decode work."""
    b = bytearray(comp[:(nbits + 7) // 8]) + b"\0\0"
    v = 0b011 << (nbits % 8)
    i = nbits // 8
    b[i] |= v & 0xFF
    b[i + 1] |= (v >> 8) & 0xFF
    return bytes(b[:(nbits + 10 + 7) // 8])


def verify_stream(data_dev, hist, final, comp_dev, nbits, threads, strategy="RLE_DYNAMIC"):
    """Whole-stream bit-exactness: the oracle (C restatement of the reference encoder) compresses
    the shard chunk-parallel -- `threads` pieces of whole 64 KiB chunks, each with its own 32 KiB of
    raw history, as the reference's blocks depend only on raw input -- and every
    piece's bits are compared with the GPU stream at that piece's bit offset.  The GPU stream's
    SHA-256 and bit count are reported beside the flag."""
    import hashlib
    import numpy as np
    import oracle_lib as O
    from concurrent.futures import ThreadPoolExecutor
    t0 = time.perf_counter()
    n = data_dev.numel()
    host = data_dev.cpu().numpy().tobytes()
    nb = (nbits + 7) // 8
    g = np.frombuffer(comp_dev[:nb + 1].cpu().numpy().tobytes(), dtype=np.uint8)
    nch = max(1, -(-n // 65536))
    per = -(-nch // threads)
    pieces = []
    for k in range(0, nch, per):
        a, b = k * 65536, min(n, (k + per) * 65536)
        h = (hist or b"")[-32768:] if a == 0 else host[max(0, a - 32768):a]
        pieces.append((h, a, b, final and b == n))
    with ThreadPoolExecutor(threads) as ex:
        outs = list(ex.map(lambda p: O.deflate_chunks(p[0], host[p[1]:p[2]], final=p[3], strategy=strategy), pieces))
    t1 = time.perf_counter()
    ok = sum(o[1] for o in outs) == nbits
    off = 0
    for pb, pbits in outs:
        if not ok:
            break
        s, q = off % 8, off // 8
        m = (pbits + 7) // 8
        seg = g[q:q + m + 1].astype(np.uint16)
        if len(seg) < m + 1:
            seg = np.concatenate([seg, np.zeros(m + 1 - len(seg), np.uint16)])
        x = ((seg[:-1] >> s) | (seg[1:] << (8 - s))).astype(np.uint8)
        if pbits % 8:
            x[-1] &= (1 << (pbits % 8)) - 1
        ok = x.tobytes() == pb[:m]
        off += pbits
    sha = hashlib.sha256(g[:nb].tobytes()).hexdigest()
    return {"bit_exact": bool(ok), "bits_compared": int(nbits), "bytes_in": n, "pieces": len(pieces), "strategy": strategy,
            "threads": threads, "oracle_s": round(t1 - t0, 2), "total_s": round(time.perf_counter() - t0, 2),
            "sha256": sha}


def cpu_baseline(data_dev, sample_bytes):
    """The oracle (C restatement of the reference algorithm) on a bounded sample of the same
    workload: compress the first `sample_bytes` of the corpus as the first chunks of the stream
    (non-final, exactly what the GPU wrote for them), decompress that (closed by an empty final
    block); same metric.  1 thread; beside it the compress leg chunk-parallel on 16 host threads
    (threads over 64 KiB-aligned pieces, each with its 32 KiB history)."""
    import oracle_lib as O
    from concurrent.futures import ThreadPoolExecutor
    m = min(sample_bytes, data_dev.numel())
    m -= m % 65536
    host = data_dev[:m].cpu().numpy().tobytes()
    t0 = time.perf_counter()
    comp, nbits = O.deflate_chunks(b"", host, final=False)
    t1 = time.perf_counter()
    stream = _append_final_empty_block(comp, nbits)
    reason, out, bits = O.inflate(stream, out_cap=m + 64)
    t2 = time.perf_counter()
    assert reason is None and out == host and bits == nbits + 10
    cores = max(1, min(16, os.cpu_count() or 1))          # the GPU box's CPU share is 16
    step = max(65536, (m // cores) // 65536 * 65536)
    pieces = [(max(0, o - 32768), o, min(m, o + step)) for o in range(0, m, step)]
    tp0 = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:
        list(ex.map(lambda p: O.deflate_chunks(host[p[0]:p[1]], host[p[1]:p[2]], final=False), pieces))
    tp1 = time.perf_counter()
    return {"value": round((m + len(comp)) / (t2 - t0) / MIB, 2), "unit": "MiB/s", "cores": 1, "kind": "port",
            "sample": f"first {m >> 20} MiB of rank 0's shard, as the first {m // 65536} chunks of the stream: "
                      f"oracle compress {t1 - t0:.2f}s + decompress {t2 - t1:.2f}s (1 thread)",
            "compress_MiBps": round(m / (t1 - t0) / MIB, 2),
            "decompress_input_MiBps": round(len(comp) / (t2 - t1) / MIB, 2),
            "all_cores": {"cores": cores, "compress_MiBps": round(m / (tp1 - tp0) / MIB, 2),
                          "note": "chunk-parallel oracle compress (threads over 64 KiB-aligned pieces with their "
                                  "32 KiB history); a single DEFLATE stream decodes serially on the CPU"},
            "host": {"nproc": os.cpu_count(), "cpu_model": _cpu_model()}}


if __name__ == "__main__":
    main()
