"""Multi-process (gloo, CPU) checks of the sharded one-stream protocol in ndfl.parallel
(SURVEY §8e): world sizes 2, 3 and 8 (the driver's node), seams inside byte runs, a short last
shard, the window maps composed across all 8 ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_workers(world, cfg):
    env = dict(os.environ, NDFL_PAR_CFG=json.dumps(cfg), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "parallel_worker.py")]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


@pytest.mark.parametrize("world,cfg", [
    (2, dict(chunk_len=65536, chunks_per_rank=3, last_bytes=100000, seed=1, strategy="RLE_DYNAMIC", seam_run=True)),
    (3, dict(chunk_len=65536, chunks_per_rank=2, last_bytes=7, seed=2, strategy="RLE_DYNAMIC", seam_run=True)),
    (2, dict(chunk_len=32768, chunks_per_rank=4, last_bytes=32768, seed=3, strategy="RLE_STATIC", seam_run=False)),
    (2, dict(chunk_len=65536, chunks_per_rank=2, last_bytes=65536, seed=4, strategy="FULL_DYNAMIC", seam_run=True)),
    (3, dict(chunk_len=65536, chunks_per_rank=2, last_bytes=40000, seed=6, strategy="RLE_DYNAMIC", seam_run=True,
             async_gather=True)),
    # the driver's 8-GPU node: 7 seams, the window composed through 7 maps, an 8-part gather
    (8, dict(chunk_len=65536, chunks_per_rank=2, last_bytes=90001, seed=21, strategy="RLE_DYNAMIC", seam_run=True,
             async_gather=True)),
    (8, dict(chunk_len=32768, chunks_per_rank=1, last_bytes=5, seed=22, strategy="FULL_DYNAMIC", seam_run=True)),
    # shards far shorter than the window: a rank's encoder history spans several earlier shards, and
    # its decode window is composed through the maps of up to 7 earlier ranks, each of whose tail maps
    # points back into that rank's own window (its output alone is shorter than 32 KiB)
    (8, dict(chunk_len=4096, chunks_per_rank=1, last_bytes=3001, seed=23, strategy="FULL_DYNAMIC", seam_run=False)),
    (8, dict(chunk_len=4096, chunks_per_rank=2, last_bytes=100, seed=24, strategy="RLE_DYNAMIC", seam_run=False)),
])
def test_sharded_stream_roundtrip(world, cfg):
    res = run_workers(world, cfg)
    assert res[0]["stream_equal"], "assembled shards differ from the single-stream encoding"
    assert all(r["gathered_equal"] for r in res), "the root's gathered stream differs from the oracle's"
    for r in res:
        assert r["code"] == 0
        assert r["decoded_equal"]
    assert all(r["resolved"] == 1 for r in res[1:])
    # the ranks between the first and the last describe their window's effect on their tail
    # (ndfl_inflate_tail_map); the window chain is one all_gather, not a hop per rank
    assert all(r["tail_maps"] == 1 for r in res[1:-1])
    assert all(r["tails"] == 0 for r in res)


def test_stalled_rank_times_out():
    """bench.py's process group has a finite timeout: with one rank stalled before the protocol's
    first exchange, the other rank fails within the timeout (non-zero exit, a timeout message)
    instead of hanging until an outside limit."""
    import time
    t0 = time.time()
    env = dict(os.environ, OMP_NUM_THREADS="1",
               NDFL_PAR_CFG=json.dumps(dict(mode="stall", stall_rank=1, stall_s=60, timeout_s=4)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "parallel_worker.py")]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    took = time.time() - t0
    assert p.returncode != 0
    assert "RESULT" not in p.stdout
    assert took < 50, took                      # well before the stalled rank would have woken
    assert "timed out" in (p.stdout + p.stderr).lower() or "timeout" in (p.stdout + p.stderr).lower()


@pytest.mark.parametrize("world,lie", [(2, False), (3, False), (2, True), (8, False), (8, True)])
def test_split_decode_without_seam_index(world, lie):
    """inflate_split: one oracle stream decoded across ranks from probed seams (the checker's probe
    knows the true block boundaries; `lie` moves one seam off a boundary, which the range decodes
    must catch and answer with the single-rank fallback)."""
    n = 600_000 if world < 8 else 2_400_000       # (every rank's range must hold a 32 KiB window)
    res = run_workers(world, dict(mode="split", n=n, seed=5, stream="RLE_DYNAMIC", lie=lie))
    assert res[0]["equal"]
    assert all(r["code"] == 0 for r in res)
    assert res[0]["split"] == (not lie)
