"""Escape-prefix literal blocks counted one lane per block (inflate_wave.hpp count_flat_group):
incompressible data, whose blocks' literal/length code is 255 (254, 252) literals of 8 bits with the
longer codes under the remaining all-ones prefix.  The decode must equal the oracle's -- output,
consumed bits, Reason of the first error -- with the flat groups on (the default) and off
(NDFL_FLAT=0: every block in wave form), one wave per chain (NDFL_COUNT_W=1), and the flat
groups must actually have counted chains.
Streams: random bytes; random bytes with sparse byte runs (length codes under the escape prefix,
decoded through the global table record); with dense runs (more than NDFL_FLAT_OTHER_MAX such
tokens per block: the chain goes back to the wave decode); random blocks between text blocks;
truncated and corrupted random streams (errors inside a flat block go back to the wave decode,
which reports them).  Every decode also passes the emit passes' check of each count-pass segment
record (NDFL_E_INTERNAL otherwise).  Reference semantics: D/decomp/Open.java:83-618."""
import os

import numpy as np
import pytest

import corpus
import oracle_lib as O

pytestmark = pytest.mark.gpu


def _ctx(flat):
    """A context with the flat groups on or off and one wave per chain (NDFL_COUNT_W=1: streams this
    small would otherwise be counted four waves per chain, a kernel without flat groups), flat groups
    at any stream size (NDFL_FLAT_MIN=0)."""
    import ndfl
    env = {"NDFL_FLAT": str(flat), "NDFL_COUNT_W": "1", "NDFL_FLAT_MIN": "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return ndfl.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def ctxs():
    return {1: _ctx(1), 0: _ctx(0)}


def _runs(data, every, ln, rng):
    b = bytearray(data)
    for p in range(int(rng.integers(0, every)), len(b) - ln, every):
        b[p:p + ln] = bytes([b[p]]) * ln
    return bytes(b)


STREAMS = {}


def _streams():
    if not STREAMS:
        rng = np.random.default_rng(61)
        rnd = rng.integers(0, 256, 3 << 20, dtype=np.uint8).tobytes()
        text = corpus.c3_text(1 << 20).numpy().tobytes()
        mixed = b"".join(rnd[i:i + 65536] + text[i // 3:i // 3 + 65536] for i in range(0, 1 << 20, 65536))
        STREAMS.update({
            "random": O.deflate(rnd),
            "random_sparse_runs": O.deflate(_runs(rnd, 2500, 7, rng)),
            "random_dense_runs": O.deflate(_runs(rnd, 400, 5, rng)),
            "random_text": O.deflate(mixed),
            "random_dynamic_stream": O.deflate(rnd[:1 << 20], "FULL_DYNAMIC"),
        })
    return STREAMS


def _same(ctx, comp):
    r, out, bits = ctx.inflate(comp)
    oreason, oout, obits = O.inflate(comp)
    assert (None if r is None else r.name) == oreason
    assert out == oout
    if oreason is None:
        assert bits == obits
    return ctx.timings()["inflate_flat_chains"]


@pytest.mark.parametrize("name", ["random", "random_sparse_runs", "random_dense_runs", "random_text",
                                  "random_dynamic_stream"])
def test_flat_groups_match_oracle(ctxs, name):
    comp = _streams()[name]
    nflat = _same(ctxs[1], comp)
    assert _same(ctxs[0], comp) == 0
    if name in ("random", "random_text"):
        assert nflat > 0                        # (the path under test ran)


def test_flat_truncated_and_corrupted(ctxs):
    comp = _streams()["random"]
    rng = np.random.default_rng(5)
    cases = [comp[:len(comp) // 2], comp[:len(comp) // 3 + 17]]
    for _ in range(4):
        bad = bytearray(comp)
        k = int(rng.integers(len(bad) // 8, len(bad)))
        bad[k] ^= 0x5A
        cases.append(bytes(bad))
    for c in cases:
        _same(ctxs[1], c)
