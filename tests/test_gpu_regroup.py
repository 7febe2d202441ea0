"""GPU: sr_pack_by_owner (HIP) against the oracle's restatement, and the Regrouper end to end on a
one-rank RCCL group (the multi-rank exchange is covered with gloo in test_regroup_dist.py)."""
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
