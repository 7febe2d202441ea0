"""Parity of the HIP path (through the C ABI) with the reference's outputs and the CPU oracle.
Bit-exact on every record and hash. Needs an MI355X: `pytest -m gpu`."""
from __future__ import annotations

import errno
import hashlib
import os
import random
import sys

import numpy as np
import pytest

from conftest import REPO, golden_cases, load_case, load_digests

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def _bits(words, n):
    return [int((int(words[k >> 6]) >> (k & 63)) & 1) for k in range(n)]


def _assert_same(gpu, cpu, what=""):
    (gr, gh, gn), (cr, ch, cn) = gpu, cpu
    assert gn == cn, f"{what}: line count {gn} != {cn}"
    if not np.array_equal(gr, cr):
        bad = np.nonzero(gr != cr)[0]
        i = int(bad[0])
        raise AssertionError(f"{what}: {len(bad)} records differ; first at {i}: gpu={gr[i]} cpu={cr[i]}")
    if gh is not None and not np.array_equal(gh, ch):
        bad = np.nonzero(gh != ch)[0]
        raise AssertionError(f"{what}: {len(bad)} hashes differ; first at {int(bad[0])}")


@pytest.fixture(scope="module")
def router_factory(pkg):
    made = []

    def make(n, max_batch=64 << 20, alive=None):
        r = pkg.Router(n, max_batch)
        if alive is not None:
            r.set_alive(alive)
        made.append(r)
        return r

    yield make
    for r in made:
        r.close()


@pytest.mark.parametrize("name", golden_cases())
def test_golden_fixture(pkg, router_factory, name):
    c = load_case(name)
    framed = pkg.frame_datagrams(c["dgrams"])
    r = router_factory(c["n"], alive=c["alive"] if c["n"] else None)
    recs, hs, n = r.route(framed, want_hashes=True)
    assert n == len(c["records"])
    _assert_same((recs, hs, n), (c["records"], c["hashes"], len(c["records"])), name)


def test_full_config_digests(pkg, router_factory):
    for key, d in sorted(load_digests().items()):
        s = pkg.gen_stream(d["nbytes"], d["line_lens"], seed=d["seed"], p_invalid=d["p_invalid"])
        words = np.array([int(x, 16) for x in d["alive"]], dtype=np.uint64)
        r = router_factory(d["n_downstreams"], alive=words)
        recs, hs, n = r.route(s.data, want_hashes=True)
        assert n == d["n_lines"], key
        assert hashlib.sha256(recs.tobytes()).hexdigest() == d["sha256_records"], key
        assert hashlib.sha256(hs.tobytes()).hexdigest() == d["sha256_hashes"], key


def _hostile_stream(seed, approx_bytes):
    import make_golden as G

    rng = random.Random(seed)
    parts, size = [], 0
    while size < approx_bytes:
        d = G.rnd_datagrams(rng, 1)[0]
        parts.append(d)
        size += len(d) + 1
    return parts


@pytest.mark.parametrize("seed", range(12))
def test_random_hostile_streams(pkg, oracle, router_factory, seed):
    rng = random.Random(100 + seed)
    n = rng.choice([1, 2, 3, 4, 16, 64, 100])
    alive = [1 if rng.random() > 0.3 else 0 for _ in range(n)]
    framed = pkg.frame_datagrams(_hostile_stream(seed, rng.choice([1000, 40_000, 300_000, 1_500_000])))
    r = router_factory(n, alive=alive)
    _assert_same(r.route(framed, want_hashes=True), oracle.route(framed, n, alive), f"seed {seed}")


def _lines_stream(lengths, seed=0, colon=True):
    rng = np.random.default_rng(seed)
    out = bytearray()
    for L in lengths:
        if L == 1:
            out += b"\n"
            continue
        body = bytearray(rng.integers(97, 123, L - 1, dtype=np.uint8).tobytes())
        if colon and L >= 3:
            body[int(rng.integers(0, L - 1))] = ord(":")
        out += body + b"\n"
    return bytes(out)


@pytest.mark.parametrize("case", [
    "tile_straddle_1449", "long_lines_over_tile", "dense_newlines", "one_byte_tail", "sizes_not_aligned",
    "colon_first_and_last", "straddle_colon_before_tile", "mixed_lengths_1_to_1600",
])
def test_tile_boundary_shapes(pkg, oracle, router_factory, case):
    T = 16384
    if case == "tile_straddle_1449":
        data = _lines_stream([1449] * 200, seed=1)
    elif case == "long_lines_over_tile":
        data = _lines_stream([100, 40_000, 7, 16_384, 16_385, 33_000, 64, 1449], seed=2, colon=True)
    elif case == "dense_newlines":            # > kWindow lines per tile, many windows
        data = b"\n" * (3 * T + 5) + _lines_stream([6] * 9000, seed=3) + b"\n" * 100
    elif case == "one_byte_tail":
        data = _lines_stream([64] * 256, seed=4) + b"a:b|c\n" + b"\n"
    elif case == "sizes_not_aligned":
        data = _lines_stream([7, 13, 61, 255, 1021, 3, 1], seed=5) * 97
    elif case == "colon_first_and_last":
        data = b"".join([b":" + b"x" * (L - 3) + b"y\n" for L in (6, 100, 1449)] +
                        [b"x" * (L - 2) + b":\n" for L in (6, 100, 1449)]) * 300
    elif case == "straddle_colon_before_tile":
        # lines whose ':' sits just before a tile boundary and whose '\n' is just after it
        pre = _lines_stream([T - 30], seed=6, colon=False)
        data = pre + b"n" * 10 + b":" + b"v" * 40 + b"\n" + _lines_stream([1000] * 40, seed=7)
    else:
        rng = np.random.default_rng(8)
        data = _lines_stream(rng.integers(1, 1600, 3000).tolist(), seed=9)
    for n, alive in ((4, None), (4, [1, 0, 1, 1]), (64, [int(i % 3 != 0) for i in range(64)])):
        r = router_factory(n, alive=alive)
        _assert_same(r.route(data, want_hashes=True), oracle.route(data, n, alive), f"{case} N={n}")


def test_repeated_launches_keep_lookback_consistent(pkg, oracle, router_factory):
    """The per-context ticket/epoch state must survive many back-to-back launches of
    different sizes (tile counts shrink and grow)."""
    r = router_factory(16)
    rng = np.random.default_rng(11)
    for it in range(60):
        nbytes = int(rng.choice([100, 16384, 16385, 50_000, 1 << 20, 3 << 20]))
        s = pkg.gen_stream(nbytes, [64, 256, 1024], seed=1000 + it, p_invalid=0.1)
        _assert_same(r.route(s.data, want_hashes=True), oracle.route(s.data, 16), f"iter {it}")


def test_alive_toggles_between_batches(pkg, oracle, router_factory):
    n = 7
    r = router_factory(n)
    s = pkg.gen_stream(2 << 20, [64, 256], seed=5)
    rng = random.Random(6)
    for _ in range(12):
        alive = [rng.randrange(2) for _ in range(n)]
        r.set_alive(alive)
        _assert_same(r.route(s.data, want_hashes=True), oracle.route(s.data, n, alive), str(alive))


@pytest.mark.parametrize("n,dead", [(64, 17), (1000, 600), (1000, 999), (65533, 65000), (200, 200)])
def test_many_dead_downstreams_wide_probe(pkg, oracle, router_factory, n, dead):
    rng = random.Random(n + dead)
    alive = [1] * n
    for k in rng.sample(range(n), dead):
        alive[k] = 0
    s = pkg.gen_stream(1 << 20, [64, 256], seed=n, p_invalid=0.05)
    r = router_factory(n, max_batch=2 << 20, alive=alive)
    _assert_same(r.route(s.data, want_hashes=True), oracle.route(s.data, n, alive), f"N={n} dead={dead}")


def test_record_capacity_overflow(pkg, oracle, router_factory):
    s = pkg.gen_stream(1 << 20, [64], seed=3)
    r = router_factory(4)
    recs, hs, n = r.route(s.data, max_records=1000, want_hashes=True)
    cr, ch, cn = oracle.route(s.data, 4)
    assert n == cn and len(recs) == 1000
    assert np.array_equal(recs, cr[:1000]) and np.array_equal(hs, ch[:1000])


def test_empty_and_unterminated_batches(pkg, router_factory):
    r = router_factory(4)
    recs, _, n = r.route(b"")
    assert n == 0 and len(recs) == 0
    with pytest.raises(OSError) as ei:
        r.route(b"abc:1|c")
    assert ei.value.errno == errno.EINVAL


def test_device_resident_path(pkg, oracle, torch_stream):
    import torch

    s = pkg.gen_stream(16 << 20, [64], seed=0x5EED0002)
    with pkg.Router(4, 16 << 20) as r:
        d_in = torch.from_numpy(s.data).to("cuda")
        d_out = torch.empty(s.n_lines * 8, dtype=torch.uint8, device="cuda")
        d_h = torch.empty(s.n_lines, dtype=torch.int64, device="cuda")
        d_n = torch.zeros(1, dtype=torch.int64, device="cuda")
        r.set_stream(torch_stream.cuda_stream)
        for _ in range(3):
            r.route_device(d_in.data_ptr(), s.data.size, d_out.data_ptr(), s.n_lines, d_h.data_ptr(), d_n.data_ptr())
        torch.cuda.synchronize()
        recs = d_out.cpu().numpy().view(pkg.RECORD_DTYPE)
        hs = d_h.cpu().numpy().view(np.uint64)
        _assert_same((recs, hs, int(d_n.item())), oracle.route(s.data, 4), "device path")


@pytest.mark.parametrize("dead", [0, 1, 20])
def test_device_many_batches_one_launch(pkg, oracle, dead, torch_stream):
    """sr_route_device_many: batches of different shapes (incl. empty and tiny ones) routed in one
    launch, each exactly as the oracle routes it alone; 20 dead of 40 takes the wide probe path
    (one launch per batch)."""
    import torch

    n = 40
    alive = [0 if k < dead else 1 for k in range(n)]
    parts = [
        pkg.gen_stream(3 << 20, [64], seed=11).data,
        np.frombuffer(b"", dtype=np.uint8),
        np.frombuffer(pkg.frame_datagrams(_hostile_stream(5, 200_000)), dtype=np.uint8),
        np.frombuffer(b"a:1|c\n", dtype=np.uint8),
        pkg.gen_stream(1 << 20, [256], seed=12, p_invalid=0.1).data,
        np.frombuffer(_lines_stream([1449, 7, 1, 1600, 64] * 300, seed=3), dtype=np.uint8),
    ] + [pkg.gen_stream(70_000 + 9_999 * i, [64, 256, 1024], seed=20 + i).data for i in range(14)]
    with pkg.Router(n, 4 << 20) as r:
        r.set_alive(alive)
        r.set_stream(torch_stream.cuda_stream)
        d_in, d_out, d_h, descs = [], [], [], []
        d_n = torch.full((len(parts),), -1, dtype=torch.int64, device="cuda")
        for i, p in enumerate(parts):
            cap = max(int(p.size), 1)
            d_in.append(torch.from_numpy(p.copy() if p.size else np.zeros(1, np.uint8)).to("cuda"))
            d_out.append(torch.empty(cap * 8, dtype=torch.uint8, device="cuda"))
            d_h.append(torch.empty(cap, dtype=torch.int64, device="cuda"))
            descs.append((d_in[-1].data_ptr(), int(p.size), d_out[-1].data_ptr(), cap, d_h[-1].data_ptr(),
                          d_n.data_ptr() + 8 * i))
        for _ in range(2):
            r.route_device_many(descs)
        torch.cuda.synchronize()
        counts = d_n.cpu().numpy()
        for i, p in enumerate(parts):
            k = int(counts[i])
            recs = d_out[i].cpu().numpy().view(pkg.RECORD_DTYPE)[:k]
            hs = d_h[i].cpu().numpy().view(np.uint64)[:k]
            _assert_same((recs, hs, k), oracle.route(p, n, alive), f"batch {i}")


def test_device_many_splits_past_launch_limit(pkg, oracle, torch_stream):
    """More batches than one launch takes (SR_MAX_BATCHES_PER_LAUNCH): split into launches."""
    import torch

    n = pkg.SR_MAX_BATCHES_PER_LAUNCH + 9
    parts = [pkg.gen_stream(20_000 + 3_001 * i, [64, 256], seed=400 + i, p_invalid=0.05).data for i in range(n)]
    with pkg.Router(7, 1 << 20) as r:
        r.set_stream(torch_stream.cuda_stream)
        d_in = [torch.from_numpy(p.copy()).to("cuda") for p in parts]
        d_out = [torch.empty(int(p.size) * 8, dtype=torch.uint8, device="cuda") for p in parts]
        d_n = torch.full((n,), -1, dtype=torch.int64, device="cuda")
        r.route_device_many([(d_in[i].data_ptr(), int(p.size), d_out[i].data_ptr(), int(p.size), None,
                              d_n.data_ptr() + 8 * i) for i, p in enumerate(parts)])
        torch.cuda.synchronize()
        counts = d_n.cpu().numpy()
        for i, p in enumerate(parts):
            k = int(counts[i])
            recs = d_out[i].cpu().numpy().view(pkg.RECORD_DTYPE)[:k]
            exp, _, en = oracle.route(p, 7)
            assert k == en and np.array_equal(recs, exp), f"batch {i}"


# ---- the records-only path (no hashes requested), over many tiles and repeated launches ----------

def test_full_config_digests_records_only(pkg, router_factory):
    for key, d in sorted(load_digests().items()):
        s = pkg.gen_stream(d["nbytes"], d["line_lens"], seed=d["seed"], p_invalid=d["p_invalid"])
        words = np.array([int(x, 16) for x in d["alive"]], dtype=np.uint64)
        r = router_factory(d["n_downstreams"], alive=words)
        for _ in range(2):   # twice: the granules then hold the previous launch's epoch
            recs, hs, n = r.route(s.data)
            assert hs is None and n == d["n_lines"], key
            assert hashlib.sha256(recs.tobytes()).hexdigest() == d["sha256_records"], key


@pytest.mark.parametrize("seed", range(3))
def test_hostile_stream_records_only(pkg, oracle, router_factory, seed):
    """Hostile datagrams over ~550 tiles (records only)."""
    rng = random.Random(700 + seed)
    n = rng.choice([1, 4, 64])
    alive = [1 if rng.random() > 0.2 else 0 for _ in range(n)]
    framed = pkg.frame_datagrams(_hostile_stream(900 + seed, 9_000_000))
    r = router_factory(n, max_batch=16 << 20, alive=alive)
    cr, _, cn = oracle.route(framed, n, alive)
    for _ in range(2):
        recs, _, k = r.route(framed)
        assert k == cn
        assert np.array_equal(recs, cr), f"seed {seed}"


def test_device_many_records_only(pkg, oracle, torch_stream):
    """16 batches of 4 MiB in one launch (two batches per XCD class), records only, and short-line
    tiles with several windows."""
    import torch

    parts = [pkg.gen_stream(4 << 20, [[64], [256], [64, 256, 1024], [16, 24]][i % 4], seed=800 + i,
                            p_invalid=0.05 * (i % 3)).data for i in range(16)]
    with pkg.Router(16, 4 << 20) as r:
        r.set_stream(torch_stream.cuda_stream)
        d_in = [torch.from_numpy(p.copy()).to("cuda") for p in parts]
        d_out = [torch.empty(int(p.size) * 8, dtype=torch.uint8, device="cuda") for p in parts]
        d_n = torch.full((16,), -1, dtype=torch.int64, device="cuda")
        descs = [(d_in[i].data_ptr(), int(p.size), d_out[i].data_ptr(), int(p.size), None, d_n.data_ptr() + 8 * i)
                 for i, p in enumerate(parts)]
        for _ in range(3):
            r.route_device_many(descs)
        torch.cuda.synchronize()
        counts = d_n.cpu().numpy()
        for i, p in enumerate(parts):
            k = int(counts[i])
            recs = d_out[i].cpu().numpy().view(pkg.RECORD_DTYPE)[:k]
            exp, _, en = oracle.route(p, 16)
            assert k == en and np.array_equal(recs, exp), f"batch {i}"


@pytest.mark.gpu
@pytest.mark.parametrize("nb", [1, 2, 5, 7, 8, 9, 15, 16, 31, 32])
def test_device_many_class_tables(pkg, oracle, nb, torch_stream):
    """Batch lookup table (cls_tab) shapes: 1-7 batches share one class (no XCD-local dealing; every
    row of the block-indexed table holds every batch), 8 and more are dealt to the 8 XCD classes (row r
    = block residue r, its class (r - nb) mod 8, so nb mod 8 shifts the rows); sizes differ a lot so
    classes are unbalanced and padding blocks appear."""
    import torch

    rng = random.Random(1000 + nb)
    parts = [pkg.gen_stream(rng.choice([900, 40_000, 300_000, 2_000_000]), rng.choice([[64], [256], [64, 1024]]),
                            seed=1100 + nb * 40 + i, p_invalid=0.05).data for i in range(nb)]
    with pkg.Router(9, 2 << 20) as r:
        r.set_stream(torch_stream.cuda_stream)
        d_in = [torch.from_numpy(p.copy()).to("cuda") for p in parts]
        d_out = [torch.empty(int(p.size) * 8, dtype=torch.uint8, device="cuda") for p in parts]
        d_n = torch.full((nb,), -1, dtype=torch.int64, device="cuda")
        descs = [(d_in[i].data_ptr(), int(p.size), d_out[i].data_ptr(), int(p.size), None, d_n.data_ptr() + 8 * i)
                 for i, p in enumerate(parts)]
        for _ in range(2):
            r.route_device_many(descs)
        torch.cuda.synchronize()
        counts = d_n.cpu().numpy()
        for i, p in enumerate(parts):
            k = int(counts[i])
            recs = d_out[i].cpu().numpy().view(pkg.RECORD_DTYPE)[:k]
            exp, _, en = oracle.route(p, 9)
            assert k == en and np.array_equal(recs, exp), f"{nb} batches: batch {i}"


@pytest.mark.parametrize("n,dead_k", [(2, 0), (2, 1), (3, 2), (100, 99), (100, 0), (1025, 512), (65533, 65532),
                                      (65533, 7)])
def test_exactly_one_dead_any_size(pkg, oracle, router_factory, n, dead_k):
    """Exactly one dead downstream (KV_DEAD1's closed-form two picks, its second reciprocal a kernel
    argument) from N = 2 to 65533, the dead one first, last or inside: records, hashes and the
    probed-dead bitmap (sr-main.c:106) against the restatement."""
    alive = [1] * n
    alive[dead_k] = 0
    s = pkg.gen_stream(1 << 20, [64, 256, 1024], seed=n + dead_k, p_invalid=0.05)
    r = router_factory(n, max_batch=2 << 20, alive=alive)
    _assert_same(r.route(s.data, want_hashes=True), oracle.route(s.data, n, alive), f"N={n} dead={dead_k}")
    assert r.last_probed_dead().tolist() == oracle.probed_dead(s.data, n, alive).tolist()
