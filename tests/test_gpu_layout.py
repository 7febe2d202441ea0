"""The route kernel's lane layouts (sr_set_layout): KV_UNIFORM (one lane group per line, sized by
the tile's mean line length), KV_SEGMENTS (one lane per 64-byte name segment in tiles of mixed
lengths) and KV_CHUNKS (route_chunk_kernel: every lane hashes the 64 bytes it loaded, lines joined by
a block scan and, across tiles, by the tail look-back) must give the same records and hashes bit for
bit, all equal to the oracle; AUTO follows the segment statistics the kernel publishes. Needs an
MI355X: `pytest -m gpu`."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import load_digests
from test_gpu_parity import _assert_same, _hostile_stream, _lines_stream

pytestmark = pytest.mark.gpu

UNIFORM, SEGMENTS, CHUNKS = 1, 2, 3
LAYOUTS = (UNIFORM, SEGMENTS, CHUNKS)


def _streams(pkg):
    rng = np.random.default_rng(5)
    yield "c5_mixed_1MiB", pkg.gen_stream(1 << 20, [64, 256, 1024], seed=0x5EED0005).data
    yield "c2_64B_1MiB", pkg.gen_stream(1 << 20, [64], seed=0x5EED0002).data
    yield "c3_invalid", pkg.gen_stream(1 << 20, [256], seed=3, p_invalid=0.1).data
    yield "lengths_1_to_1600", _lines_stream(rng.integers(1, 1600, 3000).tolist(), seed=9)
    yield "short_and_1449", _lines_stream([6, 1449, 7, 64, 1449, 1449, 9, 200] * 400, seed=10)
    yield "empty_names", b"".join([b":1|c\n", b"x" * 900 + b":v\n", b"ab:\n", b":\n"] * 500)
    # mean under 64 B (G = 1) with long lines among the short: two-segment units over two rounds
    yield "tiny_and_1449_two_rounds", _lines_stream(([6] * 15 + [1449]) * 300, seed=11)
    yield "dense_newlines", b"\n" * 40_000 + _lines_stream([6] * 9000, seed=3) + b"\n" * 100
    yield "hostile", pkg.frame_datagrams(_hostile_stream(7, 300_000))


@pytest.mark.parametrize("n,dead", [(4, 0), (64, 0), (64, 20)])
def test_layouts_match_oracle(pkg, oracle, n, dead):
    alive = [0 if i < dead else 1 for i in range(n)]
    for layout in LAYOUTS:
        r = pkg.Router(n, 4 << 20)
        try:
            r.set_alive(alive)
            r.set_layout(layout)
            for name, data in _streams(pkg):
                _assert_same(r.route(data, want_hashes=True), oracle.route(data, n, alive),
                             f"{name} layout={layout} N={n} dead={dead}")
                assert r.last_layout() == layout
        finally:
            r.close()


def test_layouts_full_size_digests(pkg):
    """The 16 MiB configuration digests (C2..C5) under each forced layout."""
    for layout in LAYOUTS:
        for key, d in sorted(load_digests().items()):
            s = pkg.gen_stream(d["nbytes"], d["line_lens"], seed=d["seed"], p_invalid=d["p_invalid"])
            words = np.array([int(x, 16) for x in d["alive"]], dtype=np.uint64)
            r = pkg.Router(d["n_downstreams"], d["nbytes"])
            try:
                r.set_alive(words)
                r.set_layout(layout)
                recs, hs, n = r.route(s.data, want_hashes=True)
                assert n == d["n_lines"], (key, layout)
                assert hashlib.sha256(recs.tobytes()).hexdigest() == d["sha256_records"], (key, layout)
                assert hashlib.sha256(hs.tobytes()).hexdigest() == d["sha256_hashes"], (key, layout)
            finally:
                r.close()


def test_auto_follows_the_traffic(pkg, oracle):
    """AUTO: the first launch probes the traffic with the segment layout; mixed-length traffic
    switches to the chunk layout, uniform traffic drops back to the uniform layout; every 32nd
    launch probes again."""
    mixed = pkg.gen_stream(4 << 20, [64, 256, 1024], seed=0x5EED0005).data
    uniform = pkg.gen_stream(4 << 20, [1024], seed=0x5EED0004).data
    r = pkg.Router(64, 4 << 20)
    try:
        seen = []
        for data in [mixed, mixed, mixed, uniform, uniform, uniform]:
            _assert_same(r.route(data, want_hashes=True), oracle.route(data, 64), "auto")
            seen.append(r.last_layout())
        assert seen == [SEGMENTS] + [CHUNKS] * 5   # chunk launches publish no statistics
        for _ in range(32 - len(seen)):       # launches 6..31 stay on the chunk layout
            r.route(uniform)
            assert r.last_layout() == CHUNKS
        _assert_same(r.route(uniform, want_hashes=True), oracle.route(uniform, 64), "probe")
        assert r.last_layout() == SEGMENTS    # launch 32: a probe, weighing uniform traffic
        for _ in range(3):
            r.route(uniform)
            assert r.last_layout() == UNIFORM
        r.route(mixed)                        # decided before this batch's statistics
        assert r.last_layout() == UNIFORM
    finally:
        r.close()


def test_set_layout_rejects_unknown(pkg):
    r = pkg.Router(4, 1 << 20)
    try:
        with pytest.raises(pkg.SrError):
            r.set_layout(4)
        assert r.last_layout() == 0
    finally:
        r.close()


def _tile_straddles(rng):
    """Lines placed so that 16 KiB tile boundaries fall before, on and after their first ':' and
    their '\\n', plus lines longer than a tile (a tile with no '\\n' at all) and one-byte names."""
    out = bytearray()
    T = 16384
    for k in range(40):
        boundary = (len(out) // T + 1) * T
        gap = boundary - len(out)
        pre = int(rng.integers(0, 1500))
        if gap > pre + 8:   # pad up to `pre` bytes before the boundary with short lines
            fill = gap - pre
            while fill > 0:
                L = int(min(fill, rng.integers(6, 300)))
                out += (b"p" * (L - 1) + b"\n") if L < 4 else (b"f" * (L - 4) + b":1|\n")[:L - 1] + b"\n"
                fill -= L
        kind = k % 5
        L = int(rng.integers(8, 1449))
        if kind == 4:
            L = int(rng.integers(T + 10, 2 * T + 500))   # no '\n' in a whole tile
        c = int(rng.integers(0, L - 1))
        body = bytearray(rng.integers(97, 123, L - 1, dtype=np.uint8).tobytes())
        if kind != 3:
            body[c] = ord(":")
        out += bytes(body) + b"\n"
    out += b"x:1|c\n" * 10
    return bytes(out)


@pytest.mark.parametrize("spin", [None, 0])
def test_chunks_tile_straddles_and_lookback(pkg, oracle, spin):
    """KV_CHUNKS across tile boundaries: the straddling line from its predecessor's tail granules,
    and (SR_KNOB_LB_SPIN 0) from the global-memory fallback that runs when a predecessor never published."""
    rng = np.random.default_rng(12)
    for n, dead in [(4, 0), (64, 20), (7, 1)]:
        alive = [0 if i < dead else 1 for i in range(n)]
        r = pkg.Router(n, 4 << 20)
        try:
            if spin is not None:
                r.set_knob(pkg.SR_KNOB_LB_SPIN, spin)
            r.set_alive(alive)
            r.set_layout(CHUNKS)
            for name, data in list(_streams(pkg)) + [("straddles", _tile_straddles(rng))]:
                _assert_same(r.route(data, want_hashes=True), oracle.route(data, n, alive),
                             f"{name} chunks N={n} dead={dead} spin={spin}")
        finally:
            r.close()
