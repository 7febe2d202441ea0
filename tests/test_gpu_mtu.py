"""GPU: the dead-downstream side effect (sr-main.c:106) and the on-device per-downstream MTU packing
(push_to_downstream + ds_schedule_flush, sr-main.c:49-83) through the C ABI, bit for bit against the
oracle's restatements (which tests/test_oracle_router.py pins to the compiled reference)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import load_case

pytestmark = pytest.mark.gpu


def _dead(n, frac, seed):
    rng = np.random.default_rng(seed)
    alive = np.ones(n, dtype=int)
    k = int(round(frac * n))
    if k:
        alive[rng.choice(n, k, replace=False)] = 0
    return alive.tolist()


STREAMS = [
    # (line lengths, n_downstreams, dead fraction, p_invalid, bytes, seed)
    ([64], 4, 0.0, 0.0, 1 << 20, 1),
    ([64], 4, 0.25, 0.0, 1 << 20, 2),
    ([256], 4, 0.25, 0.1, 1 << 20, 3),
    ([1024], 16, 0.25, 0.0, 1 << 20, 4),
    ([64, 256, 1024], 64, 0.25, 0.05, 1 << 20, 5),
    ([64, 256, 1024], 64, 0.5, 0.0, 1 << 19, 6),   # > 16 dead: the wide probe kernel
    ([6, 7, 13], 3, 0.0, 0.0, 1 << 19, 7),         # tiny lines: 241-line packets, multi-chunk shards
    ([1449, 700, 6], 5, 0.2, 0.0, 1 << 19, 8),     # lines up to the 1449-byte limit
    ([64], 1, 0.0, 0.0, 1 << 18, 9),
    ([64, 256], 300, 0.3, 0.1, 1 << 19, 10),
    ([64], 4, 1.0, 0.0, 1 << 16, 11),              # every downstream dead
    ([6, 7], 1, 0.0, 0.0, 1 << 20, 12),            # one shard, > 131 k line capacity: 4096-line chunks
    ([6, 7], 2, 0.5, 0.0, 1 << 20, 13),            # the same through the probe, one shard alive
    # narrow length ranges: the table kernel's next() search runs only over [cap / max, cap / min]
    ([145, 146], 3, 0.0, 0.0, 1 << 19, 14),        # 9 or 10 lines a packet: a 2-wide search
    ([483, 484, 725, 726], 4, 0.0, 0.0, 1 << 19, 15),
    ([1449], 2, 0.0, 0.0, 1 << 18, 16),            # one line a packet: no search
    ([725], 3, 0.0, 0.1, 1 << 18, 17),             # exactly two lines a packet
]


@pytest.mark.parametrize("lens,n,dead,p_inv,nbytes,seed", STREAMS)
def test_probed_dead_matches_oracle(pkg, oracle, lens, n, dead, p_inv, nbytes, seed):
    s = pkg.gen_stream(nbytes, lens, seed=0xD00D + seed, p_invalid=p_inv)
    alive = _dead(n, dead, seed)
    with pkg.Router(n, nbytes) as r:
        r.set_alive(alive)
        recs, _, cnt = r.route(s.data)
        got = r.last_probed_dead()
    want = oracle.probed_dead(s.data, n, alive)
    assert cnt == s.n_lines
    assert got.tolist() == want.tolist()
    assert all(alive[k] == 0 for k in got)


@pytest.mark.parametrize("name", ["random_n4_s1", "random_n7_s8", "random_n64_s3", "random_n1000_s6",
                                  "edge_n3_mid_dead", "edge_n4_all_dead"])
def test_probed_dead_golden(pkg, oracle, name):
    """Against the compiled reference's own drop (tests/golden/probed_dead.json via the harness)."""
    import json
    import os

    from conftest import GOLDEN

    case = load_case(name)
    want = json.load(open(os.path.join(GOLDEN, "probed_dead.json")))[name]
    data = pkg.frame_datagrams(case["dgrams"])
    with pkg.Router(case["n"], max(len(data), 1)) as r:
        r.set_alive(case["alive"].astype(np.uint64))
        r.route(data)
        got = r.last_probed_dead()
    assert got.tolist() == want


def _check_pack(pkg, oracle, data, n, alive, fill, r):
    srt, pk, fo, nv, pr = r.route_pack(data, fill)
    recs, _, _ = oracle.route(data, n, alive)
    probed = oracle.probed_dead(data, n, alive)
    srt_o, pk_o, fo_o, nv_o = oracle.pack_packets(recs, n, fill, probed)
    assert pr.tolist() == probed.tolist()
    assert nv == nv_o
    assert np.array_equal(srt, srt_o), "sorted records differ"
    assert len(pk) == len(pk_o), (len(pk), len(pk_o))
    assert np.array_equal(pk.view(np.uint8), pk_o.view(np.uint8)), "packet descriptors differ"
    assert np.array_equal(fo, fo_o), "pending bytes after the batch differ"
    return srt, pk, fo


@pytest.mark.parametrize("lens,n,dead,p_inv,nbytes,seed", STREAMS)
def test_route_pack_matches_oracle(pkg, oracle, lens, n, dead, p_inv, nbytes, seed):
    s = pkg.gen_stream(nbytes, lens, seed=0xFACE + seed, p_invalid=p_inv)
    alive = _dead(n, dead, seed)
    rng = np.random.default_rng(seed)
    with pkg.Router(n, nbytes) as r:
        r.set_alive(alive)
        for fill in (None, rng.integers(0, 1451, n).tolist(), [1450] * n, [1] * n):
            _check_pack(pkg, oracle, s.data, n, alive, fill, r)


def test_route_pack_chained_batches(pkg, oracle):
    """Pending bytes carried across batches, alive toggles in between; materialised packet bytes
    equal the oracle's."""
    n = 6
    rng = np.random.default_rng(3)
    fill_g = [0] * n
    fill_o = [0] * n
    pend_g, pend_o = {}, {}
    with pkg.Router(n, 1 << 18) as r:
        for b in range(12):
            alive = (rng.random(n) > 0.3).astype(int).tolist()
            s = pkg.gen_stream(int(rng.integers(1000, 1 << 18)), [6, 64, 300, 1449], seed=100 + b, p_invalid=0.05)
            r.set_alive(alive)
            srt, pk, fill_g, _, _ = r.route_pack(s.data, fill_g)
            out_g, pend_g = oracle.materialize(s.data, srt, pk, pend_g, fill_g)
            recs, _, _ = oracle.route(s.data, n, alive)
            srt_o, pk_o, fill_o, _ = oracle.pack_packets(recs, n, fill_o, oracle.probed_dead(s.data, n, alive))
            out_o, pend_o = oracle.materialize(s.data, srt_o, pk_o, pend_o, fill_o)
            assert out_g == out_o
            assert pend_g == pend_o
            assert [len(pend_g.get(k, b"")) for k in range(n)] == list(map(int, fill_g))


def test_route_pack_submit_double_buffered(pkg, oracle):
    """sr_route_pack_submit / sr_route_pack_result on alternating slots, each result taken after the
    next batch was submitted, the pending bytes chained on the device (fill None) except where the
    host sets them: every batch equals the oracle's chain (records, descriptors, fills, probed dead)."""
    n = 7
    rng = np.random.default_rng(11)
    fill_o = [0] * n
    expect = []
    with pkg.Router(n, 1 << 18) as r:
        inflight = None
        for b in range(14):
            alive = (rng.random(n) > 0.3).astype(int).tolist()
            s = pkg.gen_stream(int(rng.integers(1, 1 << 18)), [6, 64, 300, 1449], seed=300 + b, p_invalid=0.05)
            host_fill = None
            if b in (0, 6):   # the host sets the pending bytes (a flush timer, a ping) now and then
                host_fill = rng.integers(0, 1451, n).tolist()
                if inflight is not None:   # the chain must be drained before the host's fills apply
                    got = r.route_pack_result(inflight[0])
                    assert_pack_equal(got, inflight[1])
                    inflight = None
                fill_o = host_fill
            r.set_alive(alive)
            slot = b % 2
            r.route_pack_submit(slot, s.data, host_fill)
            recs, _, _ = oracle.route(s.data, n, alive)
            probed = oracle.probed_dead(s.data, n, alive)
            srt_o, pk_o, fo_o, nv_o = oracle.pack_packets(recs, n, fill_o, probed)
            fill_o = list(map(int, fo_o))
            if inflight is not None:
                assert_pack_equal(r.route_pack_result(inflight[0]), inflight[1])
            inflight = (slot, (srt_o, pk_o, fo_o, nv_o, probed))
        assert_pack_equal(r.route_pack_result(inflight[0]), inflight[1])
        with pytest.raises(pkg.SrError):   # a slot's result is taken once
            r.route_pack_result(inflight[0])


def assert_pack_equal(got, want):
    srt, pk, fo, nv, pr = got
    srt_o, pk_o, fo_o, nv_o, probed = want
    assert pr.tolist() == probed.tolist()
    assert nv == nv_o
    assert np.array_equal(srt, srt_o), "sorted records differ"
    assert np.array_equal(pk.view(np.uint8), pk_o.view(np.uint8)), "packet descriptors differ"
    assert np.array_equal(fo, fo_o), "pending bytes after the batch differ"


def test_pack_packets_device_many(pkg, oracle, torch_stream):
    """Several batches routed in one sr_route_device_many launch (with probed-dead bitmaps), then
    sr_pack_packets per batch on device buffers, the pending bytes chained on the device."""
    import torch

    n, nb, size = 8, 5, 1 << 20
    alive = [1, 1, 0, 1, 1, 0, 1, 1]
    streams = [pkg.gen_stream(size, [64, 256, 1024], seed=700 + b, p_invalid=0.05) for b in range(nb)]
    cap = max(s.n_lines for s in streams)
    d_in = torch.zeros((nb, size), dtype=torch.uint8, device="cuda")
    for b, s in enumerate(streams):
        d_in[b, : s.data.size].copy_(torch.from_numpy(s.data))
    d_rec = torch.zeros((nb, cap), dtype=torch.int64, device="cuda")
    d_cnt = torch.zeros(nb, dtype=torch.int64, device="cuda")
    d_pd = torch.zeros((nb, 1), dtype=torch.int64, device="cuda")
    mp = pkg.max_packets(size, n)
    d_srt = torch.zeros((nb, cap), dtype=torch.int64, device="cuda")
    d_pk = torch.zeros((nb, mp * 2), dtype=torch.int64, device="cuda")
    d_counts = torch.zeros((nb, 3), dtype=torch.int64, device="cuda")
    d_fill = torch.zeros((nb + 1, n), dtype=torch.int16, device="cuda")
    d_fill[0] = torch.tensor([5, 1450, 0, 700, 64, 3, 1449, 0], dtype=torch.int16)
    with pkg.Router(n, size) as r:
        r.set_alive(alive)
        r.set_stream(torch_stream.cuda_stream)
        r.route_device_many([(d_in[b].data_ptr(), int(s.data.size), d_rec[b].data_ptr(), cap, None,
                              d_cnt[b].data_ptr(), d_pd[b].data_ptr()) for b, s in enumerate(streams)])
        for b in range(nb):
            r.pack_packets(d_rec[b].data_ptr(), d_cnt[b].data_ptr(), cap, d_fill[b].data_ptr(), d_pd[b].data_ptr(),
                           d_srt[b].data_ptr(), d_pk[b].data_ptr(), mp, d_counts[b].data_ptr(),
                           d_fill[b + 1].data_ptr())
        torch.cuda.synchronize()
    fill = d_fill[0].cpu().numpy().view(np.uint16).tolist()
    for b, s in enumerate(streams):
        recs, _, cnt = oracle.route(s.data, n, alive)
        probed = oracle.probed_dead(s.data, n, alive)
        pd = np.frombuffer(d_pd[b].cpu().numpy().tobytes(), dtype=np.uint64)
        assert pkg.bitmap_shards(pd, n).tolist() == probed.tolist()
        srt_o, pk_o, fill_o, nv = oracle.pack_packets(recs, n, fill, probed)
        np_, nv_g, nl = d_counts[b].cpu().tolist()
        assert (np_, nv_g, nl) == (len(pk_o), nv, cnt)
        srt = np.frombuffer(d_srt[b].cpu().numpy().tobytes(), dtype=pkg.RECORD_DTYPE)[:cnt]
        pk = np.frombuffer(d_pk[b].cpu().numpy().tobytes(), dtype=pkg.PACKET_DTYPE)[:np_]
        assert np.array_equal(srt, srt_o)
        assert np.array_equal(pk.view(np.uint8), pk_o.view(np.uint8))
        got_fill = d_fill[b + 1].cpu().numpy().view(np.uint16).tolist()
        assert got_fill == fill_o.tolist()
        fill = got_fill


def test_pack_packets_fill_in_place(pkg, oracle, torch_stream):
    """sr_pack_packets with d_fill_out aliasing d_fill_in (allowed by sr_route.h): the pending bytes
    are read before they are overwritten whichever chain path runs (mtu_emit's walk reads every
    shard's fill_in from every chunk, so an aliased launch takes mtu_chain instead)."""
    import torch

    for n, lens in ((8, [64, 256]), (3, [6, 7, 13])):
        s = pkg.gen_stream(1 << 19, lens, seed=900 + n, p_invalid=0.05)
        cap = s.n_lines
        mp = pkg.max_packets(1 << 19, n)
        d_in = torch.from_numpy(s.data.copy()).cuda()
        d_rec = torch.zeros(cap, dtype=torch.int64, device="cuda")
        d_cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        d_srt = torch.zeros(cap, dtype=torch.int64, device="cuda")
        d_pk = torch.zeros(mp * 2, dtype=torch.int64, device="cuda")
        d_counts = torch.zeros(3, dtype=torch.int64, device="cuda")
        fill = [(97 * k + 5) % 1451 for k in range(n)]
        d_fill = torch.tensor(np.array(fill, dtype=np.uint16).view(np.int16), device="cuda")
        with pkg.Router(n, 1 << 19) as r:
            r.set_stream(torch_stream.cuda_stream)
            r.route_device_many([(d_in.data_ptr(), int(s.data.size), d_rec.data_ptr(), cap, None, d_cnt.data_ptr())])
            r.pack_packets(d_rec.data_ptr(), d_cnt.data_ptr(), cap, d_fill.data_ptr(), 0, d_srt.data_ptr(),
                           d_pk.data_ptr(), mp, d_counts.data_ptr(), d_fill.data_ptr())
            torch.cuda.synchronize()
        recs, _, cnt = oracle.route(s.data, n, None)
        srt_o, pk_o, fill_o, nv = oracle.pack_packets(recs, n, fill)
        np_, nv_g, nl = d_counts.cpu().tolist()
        assert (np_, nv_g, nl) == (len(pk_o), nv, cnt)
        pk = np.frombuffer(d_pk.cpu().numpy().tobytes(), dtype=pkg.PACKET_DTYPE)[:np_]
        assert np.array_equal(pk.view(np.uint8), pk_o.view(np.uint8)), "packet descriptors differ"
        assert d_fill.cpu().numpy().view(np.uint16).tolist() == fill_o.tolist()


def test_route_pack_edges(pkg, oracle):
    """Exact-fit packets, carry-only flushes, empty and single-line batches."""
    n = 2
    with pkg.Router(n, 1 << 16) as r:
        cases = [
            b"",
            b"a:1|c\n",
            (b"x" * 1443 + b":1|c\n"),                    # 1449 bytes: one line per packet
            (b"y" * 720 + b":1|c\n") * 2,                 # two 726-byte lines: 1452 > 1450
            (b"z" * 719 + b":1|c\n") * 2,                 # two 725-byte lines: exactly 1450
            b"bad\n" + b"k:1|c\n" * 500 + b"nocolon_line\n",
        ]
        for data in cases:
            for fill in ([0, 0], [1450, 1450], [1449, 1], [725, 724]):
                if not data:
                    srt, pk, fo, nv, pr = r.route_pack(data, fill)
                    assert len(srt) == 0 and len(pk) == 0 and fo.tolist() == fill
                    continue
                _check_pack(pkg, oracle, data, n, None, fill, r)


def test_pack_packets_many_independent_batches(pkg, oracle, torch_stream):
    """sr_pack_packets_many: the batches of several data threads packed in one set of launches,
    each from its own pending bytes, equal the oracle batch by batch."""
    import torch

    n, nb, size = 16, 7, 1 << 19
    alive = [int(k % 6 != 2) for k in range(n)]
    rng = np.random.default_rng(17)
    streams = [pkg.gen_stream(size - 1000 * b, [[64], [256], [1024], [64, 256, 1024], [6, 13]][b % 5],
                              seed=1300 + b, p_invalid=0.05) for b in range(nb)]
    cap = max(s.n_lines for s in streams)
    d_in = torch.zeros((nb, size), dtype=torch.uint8, device="cuda")
    for b, s in enumerate(streams):
        d_in[b, : s.data.size].copy_(torch.from_numpy(s.data))
    d_rec = torch.zeros((nb, cap), dtype=torch.int64, device="cuda")
    d_cnt = torch.zeros(nb, dtype=torch.int64, device="cuda")
    d_pd = torch.zeros((nb, 1), dtype=torch.int64, device="cuda")
    mp = pkg.max_packets(size, n)
    d_srt = torch.zeros((nb, cap), dtype=torch.int64, device="cuda")
    d_pk = torch.zeros((nb, mp * 2), dtype=torch.int64, device="cuda")
    d_counts = torch.zeros((nb, 3), dtype=torch.int64, device="cuda")
    fills = rng.integers(0, 1451, (nb, n)).astype(np.uint16)
    d_fin = torch.from_numpy(fills.view(np.int16)).cuda()
    d_fout = torch.zeros((nb, n), dtype=torch.int16, device="cuda")
    with pkg.Router(n, size) as r:
        r.set_alive(alive)
        r.set_stream(torch_stream.cuda_stream)
        r.route_device_many([(d_in[b].data_ptr(), int(s.data.size), d_rec[b].data_ptr(), cap, None,
                              d_cnt[b].data_ptr(), d_pd[b].data_ptr()) for b, s in enumerate(streams)])
        r.pack_packets_many([(d_rec[b].data_ptr(), d_cnt[b].data_ptr(), cap, d_fin[b].data_ptr(), d_pd[b].data_ptr(),
                              d_srt[b].data_ptr(), d_pk[b].data_ptr(), mp, d_counts[b].data_ptr(),
                              d_fout[b].data_ptr()) for b in range(nb)])
        torch.cuda.synchronize()
    for b, s in enumerate(streams):
        recs, _, cnt = oracle.route(s.data, n, alive)
        probed = oracle.probed_dead(s.data, n, alive)
        srt_o, pk_o, fill_o, nv = oracle.pack_packets(recs, n, fills[b], probed)
        np_, nv_g, nl = d_counts[b].cpu().tolist()
        assert (np_, nv_g, nl) == (len(pk_o), nv, cnt), b
        srt = np.frombuffer(d_srt[b].cpu().numpy().tobytes(), dtype=pkg.RECORD_DTYPE)[:cnt]
        pk = np.frombuffer(d_pk[b].cpu().numpy().tobytes(), dtype=pkg.PACKET_DTYPE)[:np_]
        assert np.array_equal(srt, srt_o), b
        assert np.array_equal(pk.view(np.uint8), pk_o.view(np.uint8)), b
        assert d_fout[b].cpu().numpy().view(np.uint16).tolist() == fill_o.tolist(), b


def test_route_pack_threads_share_the_gpu(pkg, oracle):
    """Data threads share a GPU (the executable's threads_num > 1, bench.py's two_threads leg): four
    contexts, each driven by its own host thread (ctypes drops the GIL), route and pack their own
    streams of batches at the same time; every result equals the oracle's, so the contexts' device
    state (look-back granules, epochs, packing scratch) does not cross."""
    import threading

    shapes = [([64], 4, 0.0), ([64, 256, 1024], 64, 0.25), ([256], 4, 0.25), ([6, 7, 13], 3, 0.0)]
    errors = []

    def worker(k):
        lens, n, dead = shapes[k]
        alive = _dead(n, dead, 100 + k)
        try:
            with pkg.Router(n, 1 << 20) as r:
                r.set_alive(alive)
                for b in range(6):
                    s = pkg.gen_stream(1 << 20, lens, seed=0xBEEF + 97 * k + b, p_invalid=0.05)
                    _check_pack(pkg, oracle, s.data, n, alive, [b * 37 % 1451] * n, r)
        except Exception as e:   # reported from the main thread
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(len(shapes))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a data thread did not finish"
    assert not errors, errors
