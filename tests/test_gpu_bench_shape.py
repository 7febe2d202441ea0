"""GPU: route + MTU packing at exactly the configuration bench.py times.

bench.py's route_pack leg routes 32 distinct 16 MiB batches in one sr_route_device_many launch and
packs all of them in one sr_pack_packets_many. With eight batches or more the packing deals each
batch's chunks to one XCD (sr_route.hip, mtu_chunk_slot, padded grid slots) and a full-size C2
batch has about 65,536 lines per shard: 15 chained 4608-line chunks that mtu_emit's walk follows
lane by lane. These tests run that launch shape (8, 9 and 32 batches; the bench's own seeds, so
batch b is bench.py's batch b of rank 0) and compare EVERY batch with the oracle: routed records,
sorted records, packet descriptors, counts and pending bytes out, from random pending bytes in
(sr-main.c:49-83, push_to_downstream / ds_schedule_flush; the dead-downstream drop of :106).
The chunk lane layout (route_chunk_kernel) is also forced on a 32-batch launch of C5 batches, the
shape bench.py captures for C5. Needs an MI355X: `pytest -m gpu`."""
from __future__ import annotations

import numpy as np
import pytest

import bench
from conftest import load_digests

pytestmark = pytest.mark.gpu

_STREAMS: dict = {}
_ORACLE: dict = {}


def _cfg(cfg):
    desc, batch_bytes, lens, p_inv, shards, seed0, dkey = bench.CONFIGS[cfg]
    return batch_bytes, lens, p_inv, shards, seed0, dkey


def _streams(pkg, cfg, nb):
    """bench.py's batches 0 .. nb-1 of rank 0 (same generator, same seeds)."""
    batch_bytes, lens, p_inv, _, seed0, _ = _cfg(cfg)
    have = _STREAMS.setdefault(cfg, [])
    while len(have) < nb:
        b = len(have)
        have.append(pkg.gen_stream(batch_bytes, lens, seed=seed0 + 65_537 * b, p_invalid=p_inv))
    return have[:nb]


def _alive(cfg, dead):
    """All alive, or the dead25 mask of tests/golden/digests.json (what bench.py --dead 0.25 uses)."""
    _, _, _, shards, _, dkey = _cfg(cfg)
    if not dead:
        return [1] * shards
    words = [int(w, 16) for w in load_digests()[f"{dkey}/dead25"]["alive"]]
    return [(words[k >> 6] >> (k & 63)) & 1 for k in range(shards)]


def _oracle_route(oracle, cfg, dead, b, stream, n, alive):
    key = (cfg, dead, b)
    if key not in _ORACLE:
        recs, _, cnt = oracle.route(stream.data, n, alive)
        _ORACLE[key] = (recs, cnt, oracle.probed_dead(stream.data, n, alive))
    return _ORACLE[key]


def _route_pack_many(pkg, streams, n, alive, fills, layout=None, knobs=(), fused=False):
    """One sr_route_device_many launch over every batch (probed-dead bitmaps asked for, as the router
    and bench.py do), then ONE sr_pack_packets_many over all of them, each from its own fills."""
    import torch

    nb = len(streams)
    size = max(int(s.data.size) for s in streams)
    cap = max(s.n_lines for s in streams)
    mp = pkg.max_packets(size, n)
    d_in = torch.zeros((nb, size), dtype=torch.uint8, device="cuda")
    for b, s in enumerate(streams):
        d_in[b, : s.data.size].copy_(torch.from_numpy(s.data))
    d_rec = torch.zeros((nb, cap), dtype=torch.int64, device="cuda")
    d_cnt = torch.zeros(nb, dtype=torch.int64, device="cuda")
    d_pd = torch.zeros((nb, max((n + 63) // 64, 1)), dtype=torch.int64, device="cuda")
    d_srt = torch.zeros((nb, cap), dtype=torch.int64, device="cuda")
    d_pk = torch.zeros((nb, mp * 2), dtype=torch.int64, device="cuda")
    d_counts = torch.zeros((nb, 3), dtype=torch.int64, device="cuda")
    d_fin = torch.from_numpy(np.ascontiguousarray(fills, dtype=np.uint16).view(np.int16)).cuda()
    d_fout = torch.full((nb, n), -1, dtype=torch.int16, device="cuda")
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream), pkg.Router(n, size) as r:
        r.set_alive(alive)
        r.set_stream(stream.cuda_stream)
        if layout is not None:
            r.set_layout(layout)
        for k, v in knobs:
            r.set_knob(k, v)
        if fused:   # sr_route_pack_many: the route kernel's tile histograms feed the packing's sort
            r.route_pack_many([(d_in[b].data_ptr(), int(s.data.size), d_rec[b].data_ptr(), cap, None,
                                d_cnt[b].data_ptr(), d_pd[b].data_ptr(), d_fin[b].data_ptr(), d_srt[b].data_ptr(),
                                d_pk[b].data_ptr(), mp, d_counts[b].data_ptr(), d_fout[b].data_ptr())
                               for b, s in enumerate(streams)])
            used_layout = r.last_layout()
        else:
            r.route_device_many([(d_in[b].data_ptr(), int(s.data.size), d_rec[b].data_ptr(), cap, None,
                                  d_cnt[b].data_ptr(), d_pd[b].data_ptr()) for b, s in enumerate(streams)])
            used_layout = r.last_layout()
            r.pack_packets_many([(d_rec[b].data_ptr(), d_cnt[b].data_ptr(), cap, d_fin[b].data_ptr(), d_pd[b].data_ptr(),
                                  d_srt[b].data_ptr(), d_pk[b].data_ptr(), mp, d_counts[b].data_ptr(),
                                  d_fout[b].data_ptr()) for b in range(nb)])
        stream.synchronize()
    out = []
    counts = d_counts.cpu().numpy()
    for b in range(nb):
        n_lines = int(d_cnt[b].item())
        np_, nv, nl = (int(x) for x in counts[b])
        out.append({
            "n_lines": n_lines,
            "recs": np.frombuffer(d_rec[b].cpu().numpy().tobytes(), dtype=pkg.RECORD_DTYPE)[:n_lines],
            "probed": pkg.bitmap_shards(np.frombuffer(d_pd[b].cpu().numpy().tobytes(), dtype=np.uint64), n),
            "counts": (np_, nv, nl),
            "sorted": np.frombuffer(d_srt[b].cpu().numpy().tobytes(), dtype=pkg.RECORD_DTYPE)[:nl],
            "packets": np.frombuffer(d_pk[b].cpu().numpy().tobytes(), dtype=pkg.PACKET_DTYPE)[:np_],
            "fill_out": d_fout[b].cpu().numpy().view(np.uint16).copy(),
        })
    return out, used_layout


CASES = [
    # (config, a quarter of the shards dead, batches in the launch, pending bytes in[, fused])
    ("c2", False, 32, "zero", True),   # bench.py's route_pack leg: sr_route_pack_many (tile histograms)
    ("c2", False, 9, "random", True),
    ("c3", False, 32, "random", True),
    ("c4", False, 32, "random", True),
    ("c5", False, 32, "random", True),   # 64 shards: the counting pass (no histograms)
    ("c2", True, 32, "random", True),    # dead shards: the counting pass
    ("c5", True, 32, "random", True),    # 16 of 64 dead (deferred probes)
    ("c2", False, 8, "random"),
    ("c2", False, 9, "random"),
    ("c2", False, 32, "random"),
    ("c2", False, 32, "zero"),      # bench.py's route_pack leg exactly
    ("c2", True, 32, "random"),
    ("c3", True, 32, "random"),
    ("c4", True, 32, "random"),
    ("c5", False, 32, "random"),
    ("c5", True, 8, "random"),
    ("c5", True, 9, "random"),
    ("c5", True, 32, "random"),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(map(str, c)))
def test_route_pack_many_full_size(pkg, oracle, case):
    cfg, dead, nb, fill = case[:4]
    fused = len(case) > 4 and case[4]
    _, _, _, n, _, _ = _cfg(cfg)
    alive = _alive(cfg, dead)
    streams = _streams(pkg, cfg, nb)
    rng = np.random.default_rng(1000 * nb + n + (7 if dead else 0))
    fills = rng.integers(0, 1451, (nb, n)) if fill == "random" else np.zeros((nb, n), dtype=np.int64)
    got, _ = _route_pack_many(pkg, streams, n, alive, fills, fused=fused)
    for b, s in enumerate(streams):
        recs, cnt, probed = _oracle_route(oracle, cfg, dead, b, s, n, alive)
        g = got[b]
        assert g["n_lines"] == cnt == s.n_lines, b
        assert np.array_equal(g["recs"], recs), f"batch {b}: routed records differ"
        assert g["probed"].tolist() == probed.tolist(), f"batch {b}: probed-dead shards differ"
        srt_o, pk_o, fo_o, nv_o = oracle.pack_packets(recs, n, fills[b], probed)
        assert g["counts"] == (len(pk_o), nv_o, cnt), (b, g["counts"], (len(pk_o), nv_o, cnt))
        assert np.array_equal(g["sorted"], srt_o), f"batch {b}: sorted records differ"
        assert np.array_equal(g["packets"].view(np.uint8), pk_o.view(np.uint8)), f"batch {b}: descriptors differ"
        assert g["fill_out"].tolist() == fo_o.tolist(), f"batch {b}: pending bytes out differ"


@pytest.mark.parametrize("dead", [False, True])
def test_chunk_layout_32_batch_launch_c5(pkg, oracle, dead):
    """SR_LAYOUT_CHUNKS forced on one 32-batch launch of full-size C5 batches (bench.py's C5 shape:
    XCD-local classes, the tail look-back across tiles), every batch against the oracle, then
    packed in the same sr_pack_packets_many call shape."""
    n = 64
    alive = _alive("c5", dead)
    streams = _streams(pkg, "c5", 32)
    fills = np.random.default_rng(55 + dead).integers(0, 1451, (32, n))
    got, layout = _route_pack_many(pkg, streams, n, alive, fills, layout=3)
    assert layout == 3
    for b, s in enumerate(streams):
        recs, cnt, probed = _oracle_route(oracle, "c5", dead, b, s, n, alive)
        assert got[b]["n_lines"] == cnt, b
        assert np.array_equal(got[b]["recs"], recs), f"batch {b}: chunk-layout records differ"
        srt_o, pk_o, fo_o, _ = oracle.pack_packets(recs, n, fills[b], probed)
        assert np.array_equal(got[b]["packets"].view(np.uint8), pk_o.view(np.uint8)), b
        assert got[b]["fill_out"].tolist() == fo_o.tolist(), b


def test_route_pack_many_shapes(pkg, oracle):
    """sr_route_pack_many on shapes its tile-histogram sort must get right: tiles of 2,700 six-byte
    lines (several 1024-record rounds per group of tiles), empty and one-line batches, 16 shards (the
    largest with histograms) and 17 (the counting pass), both layouts of the route kernel."""
    rng = np.random.default_rng(404)
    shapes = [([6, 7], 3, 1 << 20), ([64, 256, 1024], 16, 1 << 20), ([40, 70, 100, 130], 17, 1 << 20),
              ([1449, 6], 2, 1 << 19)]
    for lens, n, size in shapes:
        streams = [pkg.gen_stream(size - 7919 * b, lens, seed=4040 + b, p_invalid=0.05) for b in range(9)]
        streams[3] = pkg.Stream(np.zeros(0, np.uint8), np.zeros(0, np.uint32), 0)
        streams[5] = pkg.gen_stream(40, [13], seed=5)
        fills = rng.integers(0, 1451, (len(streams), n))
        for layout in (1, 2):
            got, _ = _route_pack_many(pkg, streams, n, [1] * n, fills, layout=layout, fused=True)
            for b, s in enumerate(streams):
                recs, _, cnt = oracle.route(s.data, n, None) if s.data.size else (np.zeros(0, pkg.RECORD_DTYPE), None, 0)
                srt_o, pk_o, fo_o, nv_o = oracle.pack_packets(recs, n, fills[b], [])
                g = got[b]
                assert g["n_lines"] == cnt, (lens, n, b)
                assert g["counts"] == (len(pk_o), nv_o, cnt), (lens, n, b, layout)
                assert np.array_equal(g["sorted"], srt_o), (lens, n, b, layout)
                assert np.array_equal(g["packets"].view(np.uint8), pk_o.view(np.uint8)), (lens, n, b, layout)
                assert g["fill_out"].tolist() == fo_o.tolist(), (lens, n, b, layout)


def test_route_pack_many_counting_pass_knob(pkg, oracle):
    """SR_KNOB_HIST 0: sr_route_pack_many with the packing's own counting pass gives the same outputs."""
    streams = _streams(pkg, "c2", 9)
    fills = np.random.default_rng(9).integers(0, 1451, (9, 4))
    a, _ = _route_pack_many(pkg, streams, 4, [1] * 4, fills, fused=True)
    b, _ = _route_pack_many(pkg, streams, 4, [1] * 4, fills, fused=True, knobs=[(pkg.SR_KNOB_HIST, 0)])
    for x, y in zip(a, b):
        assert x["counts"] == y["counts"]
        assert np.array_equal(x["sorted"], y["sorted"]) and np.array_equal(x["packets"], y["packets"])
        assert x["fill_out"].tolist() == y["fill_out"].tolist()


def test_route_pack_many_rejects_mismatched_batches(pkg):
    """sr_route_pack_many packs what it routes: a pack batch reading other records is refused."""
    import torch

    with pkg.Router(4, 1 << 16) as r:
        a = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
        rec = torch.zeros(1 << 13, dtype=torch.int64, device="cuda")
        other = torch.zeros(1 << 13, dtype=torch.int64, device="cuda")
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        out = torch.zeros(1 << 14, dtype=torch.int64, device="cuda")
        fill = torch.zeros(8, dtype=torch.int16, device="cuda")
        ok = (a.data_ptr(), 100, rec.data_ptr(), 1 << 13, None, cnt.data_ptr(), None, fill.data_ptr(),
              out.data_ptr(), out.data_ptr() + 8 * 8192, 100, cnt.data_ptr() + 8, fill.data_ptr() + 8)
        bad = list(ok)
        bad[2] = other.data_ptr()
        import ctypes
        n = 1
        ra, pa = (pkg.SrBatch * n)(), (pkg.SrPackBatch * n)()
        ra[0] = pkg.SrBatch(ok[0], ok[1], ok[2], ok[3], None, ok[5], None)
        pa[0] = pkg.SrPackBatch(bad[2], ok[5], ok[3], ok[7], None, ok[8], ok[9], ok[10], ok[11], ok[12])
        assert pkg.lib().sr_route_pack_many(r.handle, ra, pa, 1) == -22


@pytest.mark.parametrize("cfg,layout,dead,pf", [("c2", 3, False, 0), ("c5", 3, False, 0), ("c5", 3, True, 224),
                                                ("c4", 3, False, 224), ("c2", 1, True, 224)])
def test_prefetch_knob_same_records(pkg, oracle, cfg, layout, dead, pf):
    """SR_KNOB_PREFETCH (the chunk kernel's touches of tiles ahead of its own loads; default 64) changes no
    output at other values: a 9-batch route + pack launch against the oracle, all alive and a quarter dead."""
    _, _, _, n, _, _ = _cfg(cfg)
    alive = _alive(cfg, dead)
    streams = _streams(pkg, cfg, 9)
    fills = np.random.default_rng(88).integers(0, 1451, (9, n))
    got, used = _route_pack_many(pkg, streams, n, alive, fills, layout=layout, fused=True,
                                 knobs=[(pkg.SR_KNOB_PREFETCH, pf)])
    for b, s in enumerate(streams):
        recs, cnt, probed = _oracle_route(oracle, cfg, dead, b, s, n, alive)
        assert got[b]["n_lines"] == cnt, b
        assert np.array_equal(got[b]["recs"], recs), f"batch {b}: records differ with prefetch"
        srt_o, pk_o, fo_o, _ = oracle.pack_packets(recs, n, fills[b], probed)
        assert np.array_equal(got[b]["packets"].view(np.uint8), pk_o.view(np.uint8)), b
        assert got[b]["fill_out"].tolist() == fo_o.tolist(), b


@pytest.mark.parametrize("cfg,layout,dead_k", [("c5", 3, 0), ("c5", 3, 63), ("c5", 3, 17), ("c2", 1, 3), ("c2", 1, 0),
                                               ("c4", 2, 15), ("c2", 3, 2)])
def test_exactly_one_dead_shard(pkg, oracle, cfg, layout, dead_k):
    """Exactly one dead shard (KV_DEAD1: find_downstream's two picks in closed form), the last shard, the
    first and one inside, in each lane layout: a 9-batch route + pack launch against the oracle, records,
    probed-dead bitmaps, packets and pending bytes."""
    _, _, _, n, _, _ = _cfg(cfg)
    alive = [0 if k == dead_k else 1 for k in range(n)]
    streams = _streams(pkg, cfg, 9)
    fills = np.random.default_rng(300 + dead_k).integers(0, 1451, (9, n))
    got, used = _route_pack_many(pkg, streams, n, alive, fills, layout=layout, fused=True)
    assert used == layout
    for b, s in enumerate(streams):
        recs, _, cnt = oracle.route(s.data, n, alive)
        probed = oracle.probed_dead(s.data, n, alive)
        assert got[b]["n_lines"] == cnt, b
        assert np.array_equal(got[b]["recs"], recs), f"batch {b}: records differ"
        assert got[b]["probed"].tolist() == probed.tolist(), b
        srt_o, pk_o, fo_o, _ = oracle.pack_packets(recs, n, fills[b], probed)
        assert np.array_equal(got[b]["packets"].view(np.uint8), pk_o.view(np.uint8)), b
        assert got[b]["fill_out"].tolist() == fo_o.tolist(), b


@pytest.mark.parametrize("cfg,n_dead,fuse", [("c4", 7, 1), ("c5", 16, 1), ("c5", 17, 1), ("c3", 2, 1), ("c5", 16, 0),
                                             ("c5", 3, 1)])
def test_fused_deferral(pkg, oracle, cfg, n_dead, fuse):
    """Route + pack with two or more dead shards: the packing's counting pass runs the route launch's
    deferred probes (SR_KNOB_FUSE_DEFER 1, up to 16 dead; 17 falls back to probe_defer_kernel and the
    wide probe), against the oracle: records (routes written back), probed-dead bitmaps, packets."""
    _, _, _, n, _, _ = _cfg(cfg)
    rng = np.random.default_rng(500 + n_dead)
    dead = set(rng.choice(n, n_dead, replace=False).tolist())
    alive = [0 if k in dead else 1 for k in range(n)]
    streams = _streams(pkg, cfg, 9)
    fills = rng.integers(0, 1451, (9, n))
    got, _ = _route_pack_many(pkg, streams, n, alive, fills, fused=True, knobs=[(pkg.SR_KNOB_FUSE_DEFER, fuse)])
    for b, s in enumerate(streams):
        recs, _, cnt = oracle.route(s.data, n, alive)
        probed = oracle.probed_dead(s.data, n, alive)
        assert got[b]["n_lines"] == cnt, b
        assert np.array_equal(got[b]["recs"], recs), f"batch {b}: records differ"
        assert got[b]["probed"].tolist() == probed.tolist(), b
        srt_o, pk_o, fo_o, nv_o = oracle.pack_packets(recs, n, fills[b], probed)
        assert got[b]["counts"] == (len(pk_o), nv_o, cnt), b
        assert np.array_equal(got[b]["sorted"], srt_o), b
        assert np.array_equal(got[b]["packets"].view(np.uint8), pk_o.view(np.uint8)), b
        assert got[b]["fill_out"].tolist() == fo_o.tolist(), b
