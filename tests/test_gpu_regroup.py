"""GPU: sr_pack_by_owner (HIP) against the oracle's restatement, the Regrouper end to end on a one-rank
RCCL group, and the C exchange: the rebase kernel on a 3-source receive buffer and sr_exchange_run over
device memory with three ranks as threads (the multi-rank gloo exchange is in test_regroup_dist.py)."""
from __future__ import annotations

import importlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _route_on_gpu(pkg, router, data, torch):
    d_in = torch.from_numpy(np.ascontiguousarray(data) if data.size else np.zeros(1, np.uint8)).to("cuda")
    cap = max(int(data.size), 1)
    d_rec = torch.empty(cap, dtype=torch.int64, device="cuda")
    d_n = torch.zeros(1, dtype=torch.int64, device="cuda")
    router.route_device(d_in.data_ptr(), int(data.size), d_rec.data_ptr(), cap, None, d_n.data_ptr())
    return d_in, d_rec, d_n, cap


@pytest.mark.parametrize("G,n_shards,dead", [(1, 4, 0), (2, 64, 0), (3, 16, 2), (8, 64, 5), (64, 100, 0), (5, 3, 3)])
def test_pack_by_owner_matches_oracle(pkg, oracle, G, n_shards, dead, torch_stream):
    import torch

    alive = [0 if k < dead else 1 for k in range(n_shards)]
    data = pkg.gen_stream(3 << 20, [64, 256, 1024], seed=900 + G, p_invalid=0.1).data
    with pkg.Router(n_shards, 4 << 20) as r:
        r.set_alive(alive)
        r.set_stream(torch_stream.cuda_stream)
        d_in, d_rec, d_n, cap = _route_on_gpu(pkg, r, data, torch)
        out_cap = pkg.pack_capacity(int(data.size))
        d_pb = torch.full((out_cap,), 0xAB, dtype=torch.uint8, device="cuda")
        d_pr = torch.empty(cap, dtype=torch.int64, device="cuda")
        d_cnt = torch.empty((G, 2), dtype=torch.int64, device="cuda")
        r.pack_by_owner(d_in.data_ptr(), int(data.size), d_rec.data_ptr(), d_n.data_ptr(), cap, G,
                        d_pb.data_ptr(), out_cap, d_pr.data_ptr(), d_cnt.data_ptr())
        torch.cuda.synchronize()
        n = int(d_n.item())
        recs = d_rec.cpu().numpy().view(pkg.RECORD_DTYPE)[:n]
        eb, er, ec = oracle.pack_by_owner(data, recs, G)
        cnt = d_cnt.cpu().numpy()
        assert np.array_equal(cnt, ec), (cnt, ec)
        tot_l, tot_b = int(ec[:, 0].sum()), int(ec[:, 1].sum())
        got_r = d_pr.cpu().numpy().view(pkg.RECORD_DTYPE)[:tot_l]
        assert np.array_equal(got_r, er)
        got_b = d_pb.cpu().numpy()
        assert np.array_equal(got_b[:tot_b], eb)
        assert (got_b[tot_b:] == 0xAB).all()   # nothing written past the packed total


def test_regrouper_one_rank_rccl(pkg, oracle, torch_stream):
    import torch
    import torch.distributed as dist

    rg = importlib.import_module("statsd-router_amd.regroup")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    store = dist.TCPStore("127.0.0.1", 0, 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1)
    try:
        data = pkg.gen_stream(2 << 20, [64, 256], seed=31, p_invalid=0.05).data
        with pkg.Router(8, 4 << 20) as r:
            r.set_stream(torch_stream.cuda_stream)
            d_in, d_rec, d_n, cap = _route_on_gpu(pkg, r, data, torch)
            reg = rg.Regrouper(pkg, r, 4 << 20, cap)
            rb, rr, rc = reg(d_in.data_ptr(), int(data.size), d_rec.data_ptr(), d_n.data_ptr(), cap)
            torch.cuda.synchronize()
            recs, _, n = oracle.route(data, 8)
            eb, er, ec = oracle.pack_by_owner(data, recs, 1)
            assert np.array_equal(rb.cpu().numpy(), eb)
            assert np.array_equal(rr.cpu().numpy().view(pkg.RECORD_DTYPE), er)
            assert rc.cpu().tolist() == ec.tolist()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_regrouper_two_slots_pipelined(pkg, oracle, torch_stream):
    """start(i+1) before finish(i): the two slots' buffers stay apart (one-rank RCCL group)."""
    import torch
    import torch.distributed as dist

    rg = importlib.import_module("statsd-router_amd.regroup")
    store = dist.TCPStore("127.0.0.1", 0, 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1)
    try:
        streams = [pkg.gen_stream(1 << 20, [64, 256, 1024], seed=41 + k, p_invalid=0.1).data for k in range(4)]
        with pkg.Router(16, 2 << 20) as r:
            r.set_stream(torch_stream.cuda_stream)
            routed = [_route_on_gpu(pkg, r, d, torch) for d in streams]
            cap = max(x[3] for x in routed)
            reg = rg.Regrouper(pkg, r, 2 << 20, cap, slots=2)
            got = []
            for i in range(len(streams)):
                d_in, d_rec, d_n, c = routed[i]
                reg.start(i % 2, d_in.data_ptr(), int(streams[i].size), d_rec.data_ptr(), d_n.data_ptr(), c)
                if i:
                    got.append([t.cpu() for t in reg.finish((i - 1) % 2)])
            got.append([t.cpu() for t in reg.finish((len(streams) - 1) % 2)])
            torch.cuda.synchronize()
            for data, (rb, rr, rc) in zip(streams, got):
                recs, _, n = oracle.route(data, 16)
                eb, er, ec = oracle.pack_by_owner(data, recs, 1)
                assert np.array_equal(rb.numpy(), eb)
                assert np.array_equal(rr.numpy().view(pkg.RECORD_DTYPE), er)
                assert rc.tolist() == ec.tolist()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("G,n_shards,nb", [(1, 4, 3), (3, 16, 5), (8, 64, 8), (64, 100, 2)])
def test_pack_many_by_owner_matches_oracle(pkg, oracle, G, n_shards, nb, torch_stream):
    """sr_pack_many_by_owner over a launch's batches = the per-batch packs concatenated per owner."""
    import torch

    streams = [pkg.gen_stream(1 << 18, [64, 256, 1024], seed=900 + 7 * G + b, p_invalid=0.05) for b in range(nb)]
    alive = [int(k % 5 != 1) for k in range(n_shards)]
    cap = max(s.n_lines for s in streams)
    d_in = torch.zeros((nb, 1 << 18), dtype=torch.uint8, device="cuda")
    for b, s in enumerate(streams):
        d_in[b, : s.data.size].copy_(torch.from_numpy(s.data))
    d_rec = torch.zeros((nb, cap), dtype=torch.int64, device="cuda")
    d_n = torch.zeros(nb, dtype=torch.int64, device="cuda")
    total = sum(int(s.data.size) for s in streams)
    out_cap = pkg.pack_capacity(total)
    d_pb = torch.full((out_cap,), 0xAB, dtype=torch.uint8, device="cuda")
    d_pr = torch.zeros(nb * cap, dtype=torch.int64, device="cuda")
    d_cnt = torch.zeros((G, 2), dtype=torch.int64, device="cuda")
    with pkg.Router(n_shards, 1 << 18) as r:
        r.set_alive(alive)
        r.set_stream(torch_stream.cuda_stream)
        r.route_device_many([(d_in[b].data_ptr(), int(s.data.size), d_rec[b].data_ptr(), cap, None, d_n[b].data_ptr())
                             for b, s in enumerate(streams)])
        r.pack_many_by_owner([(d_in[b].data_ptr(), int(s.data.size), d_rec[b].data_ptr(), cap, d_n[b].data_ptr())
                              for b, s in enumerate(streams)], G, d_pb.data_ptr(), out_cap, d_pr.data_ptr(),
                             d_cnt.data_ptr())
        torch.cuda.synchronize()
    recs_list = [oracle.route(s.data, n_shards, alive)[0] for s in streams]
    eb, er, ec = oracle.pack_many_by_owner([s.data for s in streams], recs_list, G)
    assert d_cnt.cpu().numpy().tolist() == ec.tolist()
    assert np.array_equal(d_pb[: eb.size].cpu().numpy(), eb)
    got = np.frombuffer(d_pr[: len(er)].cpu().numpy().tobytes(), dtype=pkg.RECORD_DTYPE)
    assert np.array_equal(got, er)


def test_c_exchange_one_rank(pkg, oracle, torch_stream):
    """The C-ABI exchange (sr_comm_* / sr_exchange_sizes / sr_exchange_data over RCCL) on a one-rank
    communicator, without torch.distributed: the launch's packs come back rebased, equal to the
    oracle's pack."""
    import torch

    streams = [pkg.gen_stream(1 << 19, [64, 256, 1024], seed=700 + b, p_invalid=0.05) for b in range(3)]
    cap = max(s.n_lines for s in streams)
    d_in = torch.zeros((3, 1 << 19), dtype=torch.uint8, device="cuda")
    for b, s in enumerate(streams):
        d_in[b, : s.data.size].copy_(torch.from_numpy(s.data))
    d_rec = torch.zeros((3, cap), dtype=torch.int64, device="cuda")
    d_n = torch.zeros(3, dtype=torch.int64, device="cuda")
    total = sum(int(s.data.size) for s in streams)
    out_cap = pkg.pack_capacity(total)
    d_pb = torch.zeros(out_cap, dtype=torch.uint8, device="cuda")
    d_pr = torch.zeros(3 * cap, dtype=torch.int64, device="cuda")
    d_cnt = torch.zeros((1, 2), dtype=torch.int64, device="cuda")
    d_rc = torch.zeros((1, 2), dtype=torch.int64, device="cuda")
    comm = pkg.Comm(pkg.Comm.new_id(), 1, 0, 0)
    try:
        with pkg.Router(32, 1 << 19) as r:
            r.set_stream(torch_stream.cuda_stream)
            batches = [(d_in[b].data_ptr(), int(s.data.size), d_rec[b].data_ptr(), cap, d_n[b].data_ptr())
                       for b, s in enumerate(streams)]
            r.route_device_many([(db, nb, dr, mr, None, dn) for db, nb, dr, mr, dn in batches])
            r.pack_many_by_owner(batches, 1, d_pb.data_ptr(), out_cap, d_pr.data_ptr(), d_cnt.data_ptr())
            sent, received = r.exchange_sizes(comm, d_cnt.data_ptr(), d_rc.data_ptr())
            assert sent.tolist() == received.tolist()
            n_l, n_b = int(received[:, 0].sum()), int(received[:, 1].sum())
            rb = torch.full((n_b + 64,), 0xCD, dtype=torch.uint8, device="cuda")
            rr = torch.zeros(n_l, dtype=torch.int64, device="cuda")
            r.exchange_data(comm, d_pb.data_ptr(), d_pr.data_ptr(), sent, received, rb.data_ptr(), rr.data_ptr())
            r.sync()
    finally:
        comm.close()
    recs_list = [oracle.route(s.data, 32)[0] for s in streams]
    eb, er, ec = oracle.pack_many_by_owner([s.data for s in streams], recs_list, 1)
    assert received.astype(np.int64).tolist() == ec.tolist() == d_rc.cpu().numpy().tolist()
    got_b = rb.cpu().numpy()
    assert np.array_equal(got_b[:n_b], eb) and (got_b[n_b:] == 0xCD).all()
    assert np.array_equal(rr.cpu().numpy().view(pkg.RECORD_DTYPE), er)


def test_launch_regrouper_c_exchange(pkg, oracle, torch_stream):
    """LaunchRegrouper with a pkg.Comm made from the torch.distributed group (one rank here): the
    same result as the torch.distributed exchange."""
    import torch
    import torch.distributed as dist

    rg = importlib.import_module("statsd-router_amd.regroup")
    store = dist.TCPStore("127.0.0.1", 0, 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1)
    comm = None
    try:
        comm = pkg.Comm.from_group(0)
        streams = [pkg.gen_stream(1 << 19, [64, 1024], seed=800 + b, p_invalid=0.1) for b in range(4)]
        cap = max(s.n_lines for s in streams)
        d_in = torch.zeros((4, 1 << 19), dtype=torch.uint8, device="cuda")
        for b, s in enumerate(streams):
            d_in[b, : s.data.size].copy_(torch.from_numpy(s.data))
        d_rec = torch.zeros((4, cap), dtype=torch.int64, device="cuda")
        d_n = torch.zeros(4, dtype=torch.int64, device="cuda")
        total = sum(int(s.data.size) for s in streams)
        with pkg.Router(16, 1 << 19) as r:
            r.set_stream(torch_stream.cuda_stream)
            batches = [(d_in[b].data_ptr(), int(s.data.size), d_rec[b].data_ptr(), cap, d_n[b].data_ptr())
                       for b, s in enumerate(streams)]
            r.route_device_many([(db, nb, dr, mr, None, dn) for db, nb, dr, mr, dn in batches])
            out = {}
            for name, c in (("torch", None), ("c", comm)):
                reg = rg.LaunchRegrouper(pkg, r, total, 4 * cap, comm=c)
                rb, rr, rc = reg(batches)
                torch.cuda.synchronize()
                out[name] = (rb.cpu().numpy(), rr.cpu().numpy(), rc.cpu().numpy().tolist(), reg.last_received)
            # the C exchange orders itself on the router's stream: a router on another stream than
            # torch's current one is accepted there (the torch.distributed path refuses it)
            other = torch.cuda.Stream()
            r.set_stream(other.cuda_stream)
            d_rec.zero_()
            torch.cuda.synchronize()
            r.route_device_many([(db, nb, dr, mr, None, dn) for db, nb, dr, mr, dn in batches])
            with pytest.raises(RuntimeError):
                rg.LaunchRegrouper(pkg, r, total, 4 * cap)(batches)
            reg = rg.LaunchRegrouper(pkg, r, total, 4 * cap, comm=comm)
            rb, rr, rc = reg(batches)
            other.synchronize()
            out["c_other_stream"] = (rb.cpu().numpy(), rr.cpu().numpy(), rc.cpu().numpy().tolist(), reg.last_received)
        assert np.array_equal(out["c"][0], out["c_other_stream"][0])
        assert np.array_equal(out["c"][1], out["c_other_stream"][1])
        assert out["c"][2] == out["c_other_stream"][2] and out["c"][3] == out["c_other_stream"][3]
        assert np.array_equal(out["torch"][0], out["c"][0])
        assert np.array_equal(out["torch"][1], out["c"][1])
        assert out["torch"][2] == out["c"][2] and out["torch"][3] == out["c"][3]
        recs_list = [oracle.route(s.data, 16)[0] for s in streams]
        eb, er, ec = oracle.pack_many_by_owner([s.data for s in streams], recs_list, 1)
        assert np.array_equal(out["c"][0], eb)
        assert np.array_equal(out["c"][1].view(pkg.RECORD_DTYPE), er)
    finally:
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


def test_regroup_launch_one_call(pkg, oracle, torch_stream):
    """sr_regroup_launch (sizes, size exchange, own chunk scattered in place, exchange in one call) on a
    one-rank communicator: the oracle's launch pack; receive buffers too small give -ENOSPC with the
    sizes, and LaunchRegrouper then finishes in separate calls and grows its receive capacity."""
    import torch
    import torch.distributed as dist

    rg = importlib.import_module("statsd-router_amd.regroup")
    store = dist.TCPStore("127.0.0.1", 0, 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1)
    comm = None
    try:
        comm = pkg.Comm.from_group(0)
        streams = [pkg.gen_stream(1 << 19, [64, 256, 1024], seed=900 + b, p_invalid=0.1) for b in range(3)]
        cap = max(s.n_lines for s in streams)
        d_in = torch.zeros((3, 1 << 19), dtype=torch.uint8, device="cuda")
        for b, s in enumerate(streams):
            d_in[b, : s.data.size].copy_(torch.from_numpy(s.data))
        d_rec = torch.zeros((3, cap), dtype=torch.int64, device="cuda")
        d_n = torch.zeros(3, dtype=torch.int64, device="cuda")
        total = sum(int(s.data.size) for s in streams)
        recs_list = [oracle.route(s.data, 16)[0] for s in streams]
        eb, er, ec = oracle.pack_many_by_owner([s.data for s in streams], recs_list, 1)
        with pkg.Router(16, 1 << 19) as r:
            r.set_stream(torch_stream.cuda_stream)
            batches = [(d_in[b].data_ptr(), int(s.data.size), d_rec[b].data_ptr(), cap, d_n[b].data_ptr())
                       for b, s in enumerate(streams)]
            r.route_device_many([(db, nb, dr, mr, None, dn) for db, nb, dr, mr, dn in batches])
            pcap = pkg.pack_capacity(total)
            packed = torch.empty(pcap, dtype=torch.uint8, device="cuda")
            precs = torch.empty(3 * cap, dtype=torch.int64, device="cuda")
            counts = torch.empty((1, 2), dtype=torch.int64, device="cuda")
            rcv = torch.empty((1, 2), dtype=torch.int64, device="cuda")
            # too small: -ENOSPC, the sizes returned, nothing written
            rb = torch.full((16,), 0xCD, dtype=torch.uint8, device="cuda")
            rr = torch.zeros(4, dtype=torch.int64, device="cuda")
            fits, sent, received = r.regroup_launch(comm, batches, counts.data_ptr(), rcv.data_ptr(), packed.data_ptr(),
                                                    pcap, precs.data_ptr(), rb.data_ptr(), rb.numel(), rr.data_ptr(),
                                                    rr.numel())
            torch_stream.synchronize()
            assert not fits and received.astype(np.int64).tolist() == ec.tolist() == sent.astype(np.int64).tolist()
            assert (rb.cpu().numpy() == 0xCD).all()
            # large enough: the whole regroup in one call
            n_b, n_l = int(ec[:, 1].sum()), int(ec[:, 0].sum())
            rb = torch.full((n_b + 64,), 0xCD, dtype=torch.uint8, device="cuda")
            rr = torch.zeros(n_l + 3, dtype=torch.int64, device="cuda")
            fits, sent, received = r.regroup_launch(comm, r.owner_batches(batches), counts.data_ptr(), rcv.data_ptr(),
                                                    packed.data_ptr(), pcap, precs.data_ptr(), rb.data_ptr(),
                                                    rb.numel(), rr.data_ptr(), rr.numel())
            torch_stream.synchronize()
            assert fits and received.astype(np.int64).tolist() == ec.tolist()
            got_b = rb.cpu().numpy()
            assert np.array_equal(got_b[:n_b], eb) and (got_b[n_b:] == 0xCD).all()
            assert np.array_equal(rr.cpu().numpy()[:n_l].view(pkg.RECORD_DTYPE), er)
            assert rcv.cpu().numpy().tolist() == ec.tolist()
            # LaunchRegrouper: a receive capacity below the launch's finishes in separate calls, then fits
            reg = rg.LaunchRegrouper(pkg, r, total, 3 * cap, comm=comm)
            reg.recv_cap = (8, 1)
            for k in range(2):
                rb, rr, rc = reg(batches)
                torch_stream.synchronize()
                assert np.array_equal(rb.cpu().numpy(), eb), k
                assert np.array_equal(rr.cpu().numpy().view(pkg.RECORD_DTYPE), er), k
                assert rc.cpu().numpy().tolist() == ec.tolist()
                assert reg.recv_cap[0] >= n_b and reg.recv_cap[1] >= n_l
    finally:
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


def _three_rank_packs(pkg, oracle, world=3, n_shards=16):
    """The oracle's launch packs of `world` ranks (rank world-1 has nothing valid to send)."""
    alive = [0 if k % 7 == 3 else 1 for k in range(n_shards)]
    packs = []
    for r in range(world):
        if r == world - 1:
            datas = [np.frombuffer(pkg.frame_datagrams([b"no colon here\n", b"x\n"]), dtype=np.uint8)]
        else:
            datas = [pkg.gen_stream(1 << 18, [64, 256, 1024], seed=1300 + 10 * r + b, p_invalid=0.1).data
                     for b in range(2)]
        packs.append(oracle.pack_many_by_owner(datas, [oracle.route(d, n_shards, alive)[0] for d in datas], world))
    return packs


@pytest.mark.parametrize("owner", [0, 1, 2])
def test_exchange_rebase_kernel_three_sources(pkg, oracle, owner, torch_stream):
    """exchange_rebase_kernel (sr_exchange_rebase) on a synthetic 3-source receive buffer: the owner's
    chunks of three ranks' packs concatenated with their offsets still relative to each source's chunk;
    after the rebase every record addresses its line in the concatenated bytes."""
    import torch

    packs = _three_rank_packs(pkg, oracle)
    received = np.stack([p[2][owner] for p in packs]).astype(np.uint64)
    peers, tot = pkg.exchange_plan(3, owner, packs[owner][2].astype(np.uint64), received)
    chunks_b, chunks_r = [], []
    for s, (pb, pr, cnt) in enumerate(packs):
        l0, b0 = int(cnt[:owner, 0].sum()), int(cnt[:owner, 1].sum())
        chunks_b.append(pb[b0: b0 + int(cnt[owner, 1])])
        chunks_r.append(pr[l0: l0 + int(cnt[owner, 0])])
    rb = np.concatenate(chunks_b)
    raw = np.concatenate(chunks_r)
    assert int(tot[2]) == raw.size and int(tot[3]) == rb.size
    exp = raw.copy()
    for s in range(3):
        a, n = int(peers[s]["recv_line0"]), int(peers[s]["recv_lines"])
        exp["offset"][a: a + n] += np.uint32(sum(int(packs[q][2][owner, 1]) for q in range(s)))
    d = torch.from_numpy(raw.view(np.int64).copy()).to("cuda")
    with pkg.Router(16, 1 << 16) as r:
        r.set_stream(torch_stream.cuda_stream)
        r.exchange_rebase(d.data_ptr(), peers)
        r.sync()
    got = d.cpu().numpy().view(pkg.RECORD_DTYPE)
    assert np.array_equal(got, exp)
    # every rebased record addresses its own line (the oracle's per-owner stream, source by source)
    lines = [bytes(pb[int(cnt[:owner, 1].sum()) + x["offset"]:][: x["length"]])
             for pb, pr, cnt in packs for x in pr[int(cnt[:owner, 0].sum()):][: int(cnt[owner, 0])]]
    assert [bytes(rb[x["offset"]: x["offset"] + x["length"]]) for x in got] == lines


def test_exchange_run_device_three_ranks(pkg, oracle):
    """sr_exchange_run over device memory with three ranks as threads of one process (sends through
    host mailboxes by hipMemcpy, own chunk hipMemcpy, rebase = the shipped kernel via
    sr_exchange_rebase): every owner's receive buffers equal the oracle's per-owner stream."""
    import ctypes
    import threading

    import torch

    hip = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch (and libsr_route.so) already loaded
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    world = 3
    packs = _three_rank_packs(pkg, oracle, world)
    box, cond, out, errs = {}, threading.Condition(), {}, {}

    class DeviceMailbox(pkg.Transport):
        def __init__(self, rank, router):
            self.rank, self.router, self.posted = rank, router, []

        def group_start(self):
            self.posted = []

        def send(self, addr, n, peer, tag):
            blob = ctypes.create_string_buffer(n)
            assert hip.hipMemcpy(ctypes.addressof(blob), addr, n, 4) == 0
            with cond:
                box.setdefault((self.rank, peer, tag), []).append(blob)
                cond.notify_all()

        def recv(self, addr, n, peer, tag):
            self.posted.append((addr, n, peer, tag))

        def group_end(self):
            for addr, n, peer, tag in self.posted:
                with cond:
                    assert cond.wait_for(lambda: box.get((peer, self.rank, tag)), timeout=60)
                    blob = box[(peer, self.rank, tag)].pop(0)
                assert len(blob) == n and hip.hipMemcpy(addr, ctypes.addressof(blob), n, 4) == 0

        def copy(self, dst, src, n):
            assert hip.hipMemcpy(dst, src, n, 4) == 0

        def rebase(self, recs_addr, peers, n_lines):
            self.router.exchange_rebase(recs_addr, peers)
            self.router.sync()

    def rank_main(r):
        try:
            torch.cuda.set_device(0)
            pb, pr, cnt = packs[r]
            sent = cnt.astype(np.uint64)
            received = np.stack([packs[s][2][r] for s in range(world)]).astype(np.uint64)
            n_l, n_b = int(received[:, 0].sum()), int(received[:, 1].sum())
            d_pb = torch.from_numpy(np.concatenate([pb, np.zeros(4, np.uint8)])).to("cuda")
            d_pr = torch.from_numpy(np.concatenate([pr, np.zeros(1, pkg.RECORD_DTYPE)]).view(np.int64).copy()).to("cuda")
            d_rb = torch.full((n_b + 64,), 0xCD, dtype=torch.uint8, device="cuda")
            d_rr = torch.zeros(max(n_l, 1), dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            with pkg.Router(16, 1 << 16) as router:
                pkg.exchange_run(DeviceMailbox(r, router), world, r, sent, received, d_pb.data_ptr(),
                                 d_pr.data_ptr(), d_rb.data_ptr(), d_rr.data_ptr())
                router.sync()
            out[r] = (d_rb.cpu().numpy(), d_rr.cpu().numpy().view(pkg.RECORD_DTYPE)[:n_l], n_b)
        except Exception as e:   # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    for r in range(world):
        rb, rr, n_b = out[r]
        assert (rb[n_b:] == 0xCD).all()
        eb = np.concatenate([packs[s][0][int(packs[s][2][:r, 1].sum()):][: int(packs[s][2][r, 1])] for s in range(world)])
        assert np.array_equal(rb[:n_b], eb)
        lines = [bytes(pb[int(cnt[:r, 1].sum()) + x["offset"]:][: x["length"]])
                 for pb, pr, cnt in packs for x in pr[int(cnt[:r, 0].sum()):][: int(cnt[r, 0])]]
        assert [bytes(rb[x["offset"]: x["offset"] + x["length"]]) for x in rr] == lines


@pytest.mark.parametrize("G,own", [(1, 0), (3, 1), (8, 7), (8, 0)])
def test_pack_owner_split_matches_oracle(pkg, oracle, G, own, torch_stream):
    """sr_pack_owner_sizes + sr_pack_owner_scatter = sr_pack_many_by_owner, with owner `own`'s chunk in its
    own buffers (nothing of it in the packed buffer, nothing written past it); a scatter whose batches do not
    match the sizes call, or without one, is refused."""
    import torch

    nb, n_shards = 3, 64
    streams = [pkg.gen_stream(1 << 18, [64, 256, 1024], seed=1300 + 11 * G + b, p_invalid=0.05) for b in range(nb)]
    cap = max(s.n_lines for s in streams)
    d_in = torch.zeros((nb, 1 << 18), dtype=torch.uint8, device="cuda")
    for b, s in enumerate(streams):
        d_in[b, : s.data.size].copy_(torch.from_numpy(s.data))
    d_rec = torch.zeros((nb, cap), dtype=torch.int64, device="cuda")
    d_n = torch.zeros(nb, dtype=torch.int64, device="cuda")
    out_cap = pkg.pack_capacity(sum(int(s.data.size) for s in streams))
    d_pb = torch.full((out_cap,), 0xAB, dtype=torch.uint8, device="cuda")
    d_pr = torch.full((nb * cap,), -1, dtype=torch.int64, device="cuda")
    d_cnt = torch.zeros((G, 2), dtype=torch.int64, device="cuda")
    batches = [(d_in[b].data_ptr(), int(s.data.size), d_rec[b].data_ptr(), cap, d_n[b].data_ptr())
               for b, s in enumerate(streams)]
    with pkg.Router(n_shards, 1 << 18) as r:
        r.set_stream(torch_stream.cuda_stream)
        r.route_device_many([(db, n, dr, mr, None, dn) for db, n, dr, mr, dn in batches])
        with pytest.raises(pkg.SrError):   # no sizes call yet
            r.pack_owner_scatter(batches, G, own, d_pb.data_ptr(), d_pr.data_ptr(), d_pb.data_ptr(), out_cap,
                                 d_pr.data_ptr())
        r.pack_owner_sizes(batches, G, d_cnt.data_ptr())
        torch.cuda.synchronize()
        cnt = d_cnt.cpu().numpy()
        ob = torch.full((int(cnt[own, 1]) + 256,), 0xCD, dtype=torch.uint8, device="cuda")
        orr = torch.full((int(cnt[own, 0]) + 8,), -1, dtype=torch.int64, device="cuda")
        with pytest.raises(pkg.SrError):   # other batches than the sizes call's
            r.pack_owner_scatter(batches[:2], G, own, ob.data_ptr(), orr.data_ptr(), d_pb.data_ptr(), out_cap,
                                 d_pr.data_ptr())
        with pytest.raises(pkg.SrError):
            r.pack_owner_scatter(batches, G, G, ob.data_ptr(), orr.data_ptr(), d_pb.data_ptr(), out_cap, d_pr.data_ptr())
        r.pack_owner_scatter(batches, G, own, ob.data_ptr(), orr.data_ptr(), d_pb.data_ptr(), out_cap, d_pr.data_ptr())
        torch.cuda.synchronize()
    recs_list = [oracle.route(s.data, n_shards)[0] for s in streams]
    eb, er, ec = oracle.pack_many_by_owner([s.data for s in streams], recs_list, G)
    assert cnt.tolist() == ec.tolist()
    l0 = np.concatenate([[0], np.cumsum(ec[:, 0])]).astype(np.int64)
    b0 = np.concatenate([[0], np.cumsum(ec[:, 1])]).astype(np.int64)
    got_b = d_pb.cpu().numpy()
    got_r = np.frombuffer(d_pr.cpu().numpy().tobytes(), dtype=pkg.RECORD_DTYPE)
    for o in range(G):
        if o == own:
            assert (got_b[b0[o]: b0[o + 1]] == 0xAB).all()
            assert (d_pr.cpu().numpy()[l0[o]: l0[o + 1]] == -1).all()
        else:
            assert np.array_equal(got_b[b0[o]: b0[o + 1]], eb[b0[o]: b0[o + 1]])
            assert np.array_equal(got_r[l0[o]: l0[o + 1]], er[l0[o]: l0[o + 1]])
    mine_b = ob.cpu().numpy()
    assert np.array_equal(mine_b[: ec[own, 1]], eb[b0[own]: b0[own + 1]]) and (mine_b[ec[own, 1]:] == 0xCD).all()
    mine_r = orr.cpu().numpy()
    assert np.array_equal(mine_r[: ec[own, 0]].view(pkg.RECORD_DTYPE), er[l0[own]: l0[own + 1]])
    assert (mine_r[ec[own, 0]:] == -1).all()


def test_c_exchange_own_chunk_in_place(pkg, oracle, torch_stream):
    """One-rank RCCL exchange after sr_pack_owner_scatter into the receive buffers: sr_exchange_data
    does not copy the (never written) packed own chunk over it, and the result is the oracle's pack."""
    import torch

    streams = [pkg.gen_stream(1 << 19, [64, 256, 1024], seed=720 + b, p_invalid=0.05) for b in range(2)]
    cap = max(s.n_lines for s in streams)
    d_in = torch.zeros((2, 1 << 19), dtype=torch.uint8, device="cuda")
    for b, s in enumerate(streams):
        d_in[b, : s.data.size].copy_(torch.from_numpy(s.data))
    d_rec = torch.zeros((2, cap), dtype=torch.int64, device="cuda")
    d_n = torch.zeros(2, dtype=torch.int64, device="cuda")
    out_cap = pkg.pack_capacity(sum(int(s.data.size) for s in streams))
    d_pb = torch.full((out_cap,), 0xAB, dtype=torch.uint8, device="cuda")
    d_pr = torch.zeros(2 * cap, dtype=torch.int64, device="cuda")
    d_cnt = torch.zeros((1, 2), dtype=torch.int64, device="cuda")
    d_rc = torch.zeros((1, 2), dtype=torch.int64, device="cuda")
    comm = pkg.Comm(pkg.Comm.new_id(), 1, 0, 0)
    try:
        with pkg.Router(32, 1 << 19) as r:
            r.set_stream(torch_stream.cuda_stream)
            batches = [(d_in[b].data_ptr(), int(s.data.size), d_rec[b].data_ptr(), cap, d_n[b].data_ptr())
                       for b, s in enumerate(streams)]
            r.route_device_many([(db, nb, dr, mr, None, dn) for db, nb, dr, mr, dn in batches])
            r.pack_owner_sizes(batches, 1, d_cnt.data_ptr())
            sent, received = r.exchange_sizes(comm, d_cnt.data_ptr(), d_rc.data_ptr())
            n_l, n_b = int(received[:, 0].sum()), int(received[:, 1].sum())
            rb = torch.full((n_b + 64,), 0xCD, dtype=torch.uint8, device="cuda")
            rr = torch.zeros(n_l, dtype=torch.int64, device="cuda")
            peers, _ = pkg.exchange_plan(1, 0, sent, received)
            r.pack_owner_scatter(batches, 1, 0, rb.data_ptr() + int(peers[0]["recv_byte0"]),
                                 rr.data_ptr() + 8 * int(peers[0]["recv_line0"]), d_pb.data_ptr(), out_cap,
                                 d_pr.data_ptr())
            r.exchange_data(comm, d_pb.data_ptr(), d_pr.data_ptr(), sent, received, rb.data_ptr(), rr.data_ptr())
            r.sync()
    finally:
        comm.close()
    recs_list = [oracle.route(s.data, 32)[0] for s in streams]
    eb, er, ec = oracle.pack_many_by_owner([s.data for s in streams], recs_list, 1)
    got_b = rb.cpu().numpy()
    assert np.array_equal(got_b[:n_b], eb) and (got_b[n_b:] == 0xCD).all()
    assert np.array_equal(rr.cpu().numpy().view(pkg.RECORD_DTYPE), er)
    assert (d_pb.cpu().numpy() == 0xAB).all()   # the packed buffer was never needed


def _rank_inputs(pkg, oracle, rank, world, n_shards, nb=2):
    """Per-rank launch inputs of the multi-rank regroup tests: rank 0 has nothing valid (source 0 sends
    nothing, so every owner's first chunk is empty and its rebase starts past line 0); rank 1 routes with
    the shards it owns dead, so its own chunk is empty while the others send to it; the rest are mixed
    lengths with invalid lines and a few dead shards. Every batch's last line is a valid line ending at
    the batch's last byte (the owner scatter's piece that crosses the batch's end), the batch sizes
    varying mod 4."""
    if rank == 1 % world:
        alive = [int(k % world != 1 % world or world == 1) for k in range(n_shards)]
    else:
        alive = [int(k % 7 != 3) for k in range(n_shards)]
    datas = []
    for b in range(nb):
        if rank == 0 and world > 1:
            d = np.frombuffer(pkg.frame_datagrams([b"no colon here\n", b"x\n", b"AAAA" * 300]), dtype=np.uint8)
        else:
            d = pkg.gen_stream((1 << 17) + 4099 * rank + 1001 * b, [64, 256, 1024], seed=1700 + 17 * rank + b,
                               p_invalid=0.1).data
            tail = (b"tail.%d.%d:1|c" % (rank, b)) + b"z" * ((rank + b) % 4)
            d = np.concatenate([d, np.frombuffer(pkg.frame_datagrams([tail]), dtype=np.uint8)])
        datas.append(np.ascontiguousarray(d))
    recs = [oracle.route(d, n_shards, alive)[0] for d in datas]
    return datas, recs, alive


def _expected_receive(oracle, inputs, world, r):
    """Owner r's receive buffer: every source's chunk r of its oracle pack, source by source, with the
    records rebased into the concatenated bytes."""
    packs = [oracle.pack_many_by_owner(d, rc, world) for d, rc, _ in inputs]
    eb = np.concatenate([pb[int(cnt[:r, 1].sum()):][: int(cnt[r, 1])] for pb, pr, cnt in packs]) if packs else b""
    er, base = [], 0
    for pb, pr, cnt in packs:
        x = pr[int(cnt[:r, 0].sum()):][: int(cnt[r, 0])].copy()
        x["offset"] += np.uint32(base)
        er.append(x)
        base += int(cnt[r, 1])
    return np.asarray(eb, dtype=np.uint8), np.concatenate(er), np.stack([p[2][r] for p in packs])


@pytest.mark.parametrize("world,n_shards", [(2, 64), (3, 16), (8, 64), (3, 1)])
def test_regroup_run_device_ranks(pkg, oracle, world, n_shards):
    """sr_regroup_run — the sequence sr_regroup_launch runs on RCCL (pack sizes, size exchange, plan, own
    chunk scattered into its place in the receive buffers, exchange without the own chunk's copy, rebase)
    — with `world` ranks as threads of one process on one GPU, each its own context and stream, on a
    mailbox transport over device memory. Every rank's receive bytes, rebased records and received sizes
    equal the oracle's per-owner stream; the transport is never asked to copy the own chunk. Two
    launches per rank (the context's pack state reused); rank 0 sends nothing, rank 1's own chunk is
    empty; the last rank's first launch has receive buffers one line short (-ENOSPC) and finishes with
    sr_pack_owner_scatter (own -1) + sr_exchange_run while its peers' sends wait."""
    import ctypes
    import threading

    import torch

    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    D2H, H2D, D2D = 2, 1, 3
    inputs = [_rank_inputs(pkg, oracle, r, world, n_shards) for r in range(world)]
    box, cond, out, errs = {}, threading.Condition(), {}, {}

    class Mailbox(pkg.Transport):
        def __init__(self, rank, router):
            self.rank, self.router, self.posted, self.step, self.calls = rank, router, [], 0, []

        def _put(self, key, blob):
            with cond:
                box.setdefault(key, []).append(blob)
                cond.notify_all()

        def _take(self, key):
            with cond:
                assert cond.wait_for(lambda: box.get(key), timeout=90), key
                return box[key].pop(0)

        def sizes(self, d_cnt, d_rcv):
            self.calls.append("sizes")
            self.router.sync()
            sent = np.zeros((world, 2), np.uint64)
            assert hip.hipMemcpy(sent.ctypes.data, d_cnt, sent.nbytes, D2H) == 0
            for q in range(world):
                self._put(("sz", self.step, self.rank, q), sent[q].copy())
            received = np.stack([self._take(("sz", self.step, q, self.rank)) for q in range(world)])
            assert hip.hipMemcpy(d_rcv, received.ctypes.data, received.nbytes, H2D) == 0
            self.step += 1
            return sent, received

        def group_start(self):
            self.router.sync()   # the scatter wrote the packed chunks
            self.posted = []

        def send(self, addr, n, peer, tag):
            self.calls.append(("send", peer, tag))
            blob = ctypes.create_string_buffer(n)
            assert hip.hipMemcpy(ctypes.addressof(blob), addr, n, D2H) == 0
            self._put(("d", self.rank, peer, tag), blob)

        def recv(self, addr, n, peer, tag):
            self.calls.append(("recv", peer, tag))
            self.posted.append((addr, n, peer, tag))

        def group_end(self):
            for addr, n, peer, tag in self.posted:
                blob = self._take(("d", peer, self.rank, tag))
                assert len(blob) == n and hip.hipMemcpy(addr, ctypes.addressof(blob), n, H2D) == 0

        def copy(self, dst, src, n):
            self.calls.append("copy")
            assert hip.hipMemcpy(dst, src, n, D2D) == 0

        def rebase(self, recs_addr, peers, n_lines):
            self.router.exchange_rebase(recs_addr, peers)
            self.router.sync()

    def rank_main(r):
        try:
            torch.cuda.set_device(0)
            datas, _, alive = inputs[r]
            nb = len(datas)
            cap = max(d.size for d in datas)
            d_in = torch.zeros((nb, cap), dtype=torch.uint8, device="cuda")
            for b, d in enumerate(datas):
                d_in[b, : d.size].copy_(torch.from_numpy(d))
            d_rec = torch.zeros((nb, cap), dtype=torch.int64, device="cuda")
            d_n = torch.zeros(nb, dtype=torch.int64, device="cuda")
            total = sum(int(d.size) for d in datas)
            pcap = pkg.pack_capacity(total)
            packed = torch.zeros(pcap, dtype=torch.uint8, device="cuda")
            precs = torch.zeros(nb * cap, dtype=torch.int64, device="cuda")
            counts = torch.zeros((world, 2), dtype=torch.int64, device="cuda")
            rcv = torch.zeros((world, 2), dtype=torch.int64, device="cuda")
            eb, er, ec = _expected_receive(oracle, inputs, world, r)
            torch.cuda.synchronize()
            got = []
            with pkg.Router(n_shards, cap) as router:
                router.set_alive(alive)
                batches = [(d_in[b].data_ptr(), int(d.size), d_rec[b].data_ptr(), cap, d_n[b].data_ptr())
                           for b, d in enumerate(datas)]
                router.route_device_many([(db, n, dr, mr, None, dn) for db, n, dr, mr, dn in batches])
                t = Mailbox(r, router)
                for step in range(2):
                    short = step == 0 and r == world - 1 and world > 1 and len(er) > 0
                    nl = max(len(er) - (1 if short else 0), 1)
                    rb = torch.full((eb.size + 64,), 0xCD, dtype=torch.uint8, device="cuda")
                    rr = torch.full((nl,), -1, dtype=torch.int64, device="cuda")
                    torch.cuda.synchronize()
                    fits, sent, received = router.regroup_run(
                        t, world, r, batches, counts.data_ptr(), rcv.data_ptr(), packed.data_ptr(), pcap,
                        precs.data_ptr(), rb.data_ptr(), rb.numel(), rr.data_ptr(), nl)
                    assert fits == (not short), (r, step, fits)
                    if not fits:   # finish: everything packed, then the exchange with the own chunk copied
                        rr = torch.full((len(er),), -1, dtype=torch.int64, device="cuda")
                        torch.cuda.synchronize()
                        router.pack_owner_scatter(batches, world, -1, 0, 0, packed.data_ptr(), pcap,
                                                  precs.data_ptr())
                        pkg.exchange_run(t, world, r, sent, received, packed.data_ptr(), precs.data_ptr(),
                                         rb.data_ptr(), rr.data_ptr())
                    router.sync()
                    got.append((rb.cpu().numpy(), rr.cpu().numpy().view(pkg.RECORD_DTYPE)[: len(er)],
                                received.astype(np.int64), rcv.cpu().numpy(), fits))
            out[r] = (got, eb, er, ec, t.calls)
        except Exception as e:   # noqa: BLE001
            import traceback
            errs[r] = traceback.format_exc()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(240)
    assert not any(t.is_alive() for t in th), "a rank did not finish"
    assert not errs, "\n".join(f"rank {r}:\n{e}" for r, e in errs.items())
    for r in range(world):
        got, eb, er, ec, calls = out[r]
        for step, (rb, rr, received, rcv, fits) in enumerate(got):
            assert received.tolist() == ec.tolist() == rcv.tolist(), (r, step)
            assert np.array_equal(rb[: eb.size], eb), (r, step)
            assert (rb[eb.size:] == 0xCD).all(), (r, step)
            assert np.array_equal(rr, er), (r, step)
        # the own chunk is never copied by the one-call sequence (only by the -ENOSPC fallback)
        fell_back = any(not g[4] for g in got)
        assert calls.count("copy") == (2 if fell_back and ec[r, 0] else 0), calls
        assert all(c[1] != r for c in calls if isinstance(c, tuple)), "a send or recv to itself"


def _end_straddle_batches(pkg):
    """Batches whose valid last line ends at the batch's last byte, for every (line start % 4,
    nbytes % 4) and several last-line lengths (one to five 16-byte pieces): the owner scatter's piece
    that crosses the batch's end must come out byte-exact."""
    out = []
    for a in range(4):
        for b in range(4):
            first = b"first.%d%d" % (a, b)
            first += b"x" * ((a - 1 - len(first) - 4) % 4) + b":1|c"   # framed: len + 1 = a (mod 4)
            L = 24 + 16 * ((a + b) % 5) + ((b - a) % 4) + 4 * (a & 1)        # framed length = b - a (mod 4)
            body = b"last.%d.%d." % (a, b)
            last = body + b"y" * (L - 1 - len(body) - 4) + b":1|c"
            d = np.frombuffer(pkg.frame_datagrams([first, last]), dtype=np.uint8)
            assert (len(first) + 1) % 4 == a and d.size % 4 == b and d[-1] == 10
            out.append(np.ascontiguousarray(d))
    return out


@pytest.mark.parametrize("G,own", [(2, None), (2, 0), (3, 1), (1, 0)])
def test_owner_scatter_batch_end_piece(pkg, oracle, G, own, torch_stream):
    """The owner pack of 16 batches whose last line ends at the batch's end (every line start % 4 and
    nbytes % 4): packed bytes and records equal the oracle's, also with one owner's chunk scattered into
    its own buffer."""
    import torch

    datas = _end_straddle_batches(pkg)
    nb, n_shards = len(datas), 4
    cap = max(d.size for d in datas)
    d_in = torch.zeros((nb, cap), dtype=torch.uint8, device="cuda")
    for b, d in enumerate(datas):
        d_in[b, : d.size].copy_(torch.from_numpy(d))
    d_rec = torch.zeros((nb, cap), dtype=torch.int64, device="cuda")
    d_n = torch.zeros(nb, dtype=torch.int64, device="cuda")
    total = sum(int(d.size) for d in datas)
    pcap = pkg.pack_capacity(total)
    d_pb = torch.full((pcap,), 0xAB, dtype=torch.uint8, device="cuda")
    d_pr = torch.full((nb * cap,), -1, dtype=torch.int64, device="cuda")
    d_cnt = torch.zeros((G, 2), dtype=torch.int64, device="cuda")
    recs_list = [oracle.route(d, n_shards)[0] for d in datas]
    eb, er, ec = oracle.pack_many_by_owner(datas, recs_list, G)
    batches = [(d_in[b].data_ptr(), int(d.size), d_rec[b].data_ptr(), cap, d_n[b].data_ptr()) for b, d in enumerate(datas)]
    with pkg.Router(n_shards, cap) as r:
        r.set_stream(torch_stream.cuda_stream)
        r.route_device_many([(db, n, dr, mr, None, dn) for db, n, dr, mr, dn in batches])
        if own is None:
            r.pack_many_by_owner(batches, G, d_pb.data_ptr(), pcap, d_pr.data_ptr(), d_cnt.data_ptr())
        else:
            r.pack_owner_sizes(batches, G, d_cnt.data_ptr())
            ob = torch.full((int(ec[own, 1]) + 64,), 0xCD, dtype=torch.uint8, device="cuda")
            orr = torch.full((int(ec[own, 0]) + 1,), -1, dtype=torch.int64, device="cuda")
            r.pack_owner_scatter(batches, G, own, ob.data_ptr(), orr.data_ptr(), d_pb.data_ptr(), pcap, d_pr.data_ptr())
        torch_stream.synchronize()
    assert d_cnt.cpu().numpy().tolist() == ec.tolist()
    l0 = np.concatenate([[0], np.cumsum(ec[:, 0])]).astype(np.int64)
    b0 = np.concatenate([[0], np.cumsum(ec[:, 1])]).astype(np.int64)
    got_b = d_pb.cpu().numpy()
    got_r = np.frombuffer(d_pr.cpu().numpy().tobytes(), dtype=pkg.RECORD_DTYPE)
    for o in range(G):
        if o == own:
            mine_b, mine_r = ob.cpu().numpy(), orr.cpu().numpy()
            assert np.array_equal(mine_b[: ec[o, 1]], eb[b0[o]: b0[o + 1]]) and (mine_b[ec[o, 1]:] == 0xCD).all()
            assert np.array_equal(mine_r[: ec[o, 0]].view(pkg.RECORD_DTYPE), er[l0[o]: l0[o + 1]])
        else:
            assert np.array_equal(got_b[b0[o]: b0[o + 1]], eb[b0[o]: b0[o + 1]]), o
            assert np.array_equal(got_r[l0[o]: l0[o + 1]], er[l0[o]: l0[o + 1]]), o
