"""GPU parity of the compressor plugin API: Strategy.decide /
Decision.getBitLengths / Decision.compressTo through ndfl_decide / ndfl_compress_to, any strategy
tree (BinarySplit over Uncompressed / MultiStrategy / BinarySplit, MultiStrategy over BinarySplit),
and user-written strategies mixed with the library's, against the test-side restatement
(tests/strategy_ref.py, leaves from the C oracle)."""
import io
import random
import zlib

import pytest

import oracle_lib as O
import strategy_ref as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def N():
    import ndfl
    return ndfl


def sample(seed, n):
    rng = random.Random(seed)
    buf = bytearray()
    while len(buf) < n:
        r = rng.random()
        if r < 0.3:
            buf += rng.randbytes(rng.randrange(1, 3000))
        elif r < 0.6:
            buf += bytes([rng.randrange(4)]) * rng.randrange(1, 700)
        else:
            buf += bytes(rng.choice(b"abcdefgh \n") for _ in range(rng.randrange(1, 2000)))
    return bytes(buf[:n])


def trees(N):
    L, U = N.Lz77Huffman, N.Uncompressed.SINGLETON
    return [
        ("binsplit(unc)", N.BinarySplit(U, 1000), R.Split(R.UncLeaf(), 1000)),
        ("binsplit(multi(rle,unc))", N.BinarySplit(N.MultiStrategy(L.RLE_DYNAMIC, U), 2000),
         R.Split(R.Multi(R.LzLeaf("RLE_DYNAMIC"), R.UncLeaf()), 2000)),
        ("multi(binsplit(rle),unc)", N.MultiStrategy(N.BinarySplit(L.RLE_DYNAMIC, 4000), U),
         R.Multi(R.Split(R.LzLeaf("RLE_DYNAMIC"), 4000), R.UncLeaf())),
        ("binsplit(binsplit(lit_static))", N.BinarySplit(N.BinarySplit(L.LITERAL_STATIC, 3000), 5000),
         R.Split(R.Split(R.LzLeaf("LITERAL_STATIC"), 3000), 5000)),
        ("multi(full_static,rle_static,unc)", N.MultiStrategy(L.FULL_STATIC, L.RLE_STATIC, U),
         R.Multi(R.LzLeaf("FULL_STATIC"), R.LzLeaf("RLE_STATIC"), R.UncLeaf())),
    ]


def test_decide_bit_lengths(N):
    data = sample(1, 70000)
    for name in ["RLE_DYNAMIC", "LITERAL_STATIC", "FULL_DYNAMIC"]:
        st = getattr(N.Lz77Huffman, name)
        for hl in (0, 1, 5000):
            d = st.decide(data, 100, hl, 40000)
            e = R.LzLeaf(name).decide(data, 100, hl, 40000)
            assert d.getBitLengths() == e.getBitLengths(), (name, hl)
    d = N.Uncompressed.SINGLETON.decide(data, 0, 0, 65536)
    assert d.getBitLengths() == R.UncLeaf().decide(data, 0, 0, 65536).getBitLengths()


@pytest.mark.parametrize("idx", range(5))
def test_strategy_trees_match_reference(N, idx):
    name, st, ref = trees(N)[idx]
    for n, chunk in [(0, 65536), (1, 65536), (150_001, 65536), (90_000, 30000)]:
        data = sample(idx * 10 + n % 7, n)
        exp = R.stream(data, ref, chunk)
        b = io.BytesIO()
        d = N.DeflaterOutputStream(b, chunk, 32768, st)
        d.write(data[:n // 3])
        d.write(data[n // 3:])
        d.finish()
        assert b.getvalue() == exp, (name, n, chunk)
        assert zlib.decompress(exp, -15) == data


def test_user_strategy_mixes_with_library(N):
    """A user Strategy (stored blocks for chunks that look incompressible, the library's
    RLE_DYNAMIC otherwise, and a BinarySplit over itself) plugged into DeflaterOutputStream."""
    class Picky:
        def __init__(self, a, b):
            self.a, self.b = a, b

        def decide(self, b, off, hl, dl):
            chunk = bytes(b[off + hl:off + hl + dl])
            return (self.a if len(set(chunk[:256])) > 64 else self.b).decide(b, off, hl, dl)

    data = sample(7, 200_000)
    lib_st = Picky(N.Uncompressed.SINGLETON, N.Lz77Huffman.RLE_DYNAMIC)
    ref_st = Picky(R.UncLeaf(), R.LzLeaf("RLE_DYNAMIC"))
    for st, ref in [(lib_st, ref_st), (N.BinarySplit(lib_st, 5000), R.Split(ref_st, 5000)),
                    (N.MultiStrategy(lib_st, N.Lz77Huffman.LITERAL_DYNAMIC),
                     R.Multi(ref_st, R.LzLeaf("LITERAL_DYNAMIC")))]:
        b = io.BytesIO()
        d = N.DeflaterOutputStream(b, 65536, 32768, st)
        d.write(data)
        d.finish()
        exp = R.stream(data, ref)
        assert b.getvalue() == exp
        r, out, _ = O.inflate(exp)
        assert r is None and out == data


def test_plugin_validation(N):
    with pytest.raises(ValueError):
        N.BinarySplit(N.Uncompressed.SINGLETON, 0)
    with pytest.raises(ValueError):
        N.MultiStrategy()
    with pytest.raises(TypeError):
        N.MultiStrategy(object())
