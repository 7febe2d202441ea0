"""The C ABI's exchange plan (sr_exchange_plan / sr_exchange_run, statsd-router_amd/csrc/exchange.hpp)
without a GPU: the per-peer offsets against the torch.distributed exchange's own arithmetic
(regroup._exchange_data: all_to_all_single splits + the exclusive-scan rebase), and whole exchanges
at world sizes 2, 3 and 8 in one process, every rank a thread running sr_exchange_run on a mailbox
transport over host memory, against the oracle's per-owner streams. The reference analogue is the
SO_REUSEPORT spread of datagrams over data threads (sr-main.c:253-271,363-367); the exchange regroups
their routed lines by owner GPU."""
from __future__ import annotations

import ctypes
import errno
import threading

import numpy as np
import pytest


def _size_matrix(rng, world):
    """M[src, dst] = {lines, bytes} of an all-to-all (bytes 4-aligned, >= 8 per line; some zero)."""
    m = np.zeros((world, world, 2), dtype=np.uint64)
    for s in range(world):
        for d in range(world):
            if rng.random() < 0.2:
                continue
            n = int(rng.integers(1, 5000))
            m[s, d] = (n, 4 * int(rng.integers(2 * n, 300 * n)))
    return m


def _python_plan(sent, received):
    """What regroup._exchange_data does: all_to_all_single input/output splits in rank order, and
    base[s] = bytes received from ranks before s."""
    ex = lambda v: np.concatenate([[0], np.cumsum(v)[:-1]]).astype(np.uint64)
    return {"send_line0": ex(sent[:, 0]), "send_byte0": ex(sent[:, 1]), "recv_line0": ex(received[:, 0]),
            "recv_byte0": ex(received[:, 1]), "send_lines": sent[:, 0], "send_bytes": sent[:, 1],
            "recv_lines": received[:, 0], "recv_bytes": received[:, 1]}


@pytest.mark.parametrize("world", [1, 2, 3, 8, 64])
def test_plan_matches_torch_exchange_arithmetic(pkg, world):
    rng = np.random.default_rng(world)
    m = _size_matrix(rng, world)
    for rank in range(world):
        sent, received = m[rank], m[:, rank]
        peers, tot = pkg.exchange_plan(world, rank, sent, received)
        exp = _python_plan(sent, received)
        for k, v in exp.items():
            assert np.array_equal(peers[k], v), (rank, k)
        assert tot.tolist() == [int(sent[:, 0].sum()), int(sent[:, 1].sum()), int(received[:, 0].sum()),
                                int(received[:, 1].sum())]


def test_plan_rejects_bad_input(pkg):
    ok = np.array([[3, 64], [2, 32]], dtype=np.uint64)
    pkg.exchange_plan(2, 0, ok, ok)
    with pytest.raises(pkg.SrError) as e:   # own chunk: sent and received sizes disagree
        pkg.exchange_plan(2, 0, ok, np.array([[4, 64], [2, 32]], dtype=np.uint64))
    assert e.value.errno == errno.EINVAL
    with pytest.raises(pkg.SrError):        # received bytes past the u32 record offsets
        pkg.exchange_plan(2, 0, ok, np.array([[3, 64], [1, 1 << 32]], dtype=np.uint64))
    with pytest.raises(pkg.SrError):        # rank out of range
        pkg.exchange_plan(2, 2, ok, ok)
    with pytest.raises(pkg.SrError):        # more than SR_MAX_OWNERS
        z = np.zeros((65, 2), dtype=np.uint64)
        pkg.exchange_plan(65, 0, z, z)


class MailboxTransport:
    """Ranks as threads of one process: a send deposits a copy of the bytes, a receive is completed at
    group_end from the peer's deposit (FIFO per (source, destination, tag))."""

    def __init__(self, pkg, box, cond, rank):
        self.pkg, self.box, self.cond, self.rank = pkg, box, cond, rank
        self.posted, self.calls = [], []

    def group_start(self):
        self.posted = []

    def send(self, addr, n, peer, tag):
        assert peer != self.rank
        self.calls.append(("send", peer, tag, n))
        with self.cond:
            self.box.setdefault((self.rank, peer, tag), []).append(ctypes.string_at(addr, n))
            self.cond.notify_all()

    def recv(self, addr, n, peer, tag):
        assert peer != self.rank
        self.calls.append(("recv", peer, tag, n))
        self.posted.append((addr, n, peer, tag))

    def group_end(self):
        for addr, n, peer, tag in self.posted:
            with self.cond:
                key = (peer, self.rank, tag)
                if not self.cond.wait_for(lambda: self.box.get(key), timeout=60):
                    raise TimeoutError(f"rank {self.rank}: nothing from {peer} tag {tag}")
                blob = self.box[key].pop(0)
            assert len(blob) == n, (len(blob), n)
            ctypes.memmove(addr, blob, n)

    def copy(self, dst, src, n):
        self.calls.append(("copy", -1, -1, n))
        ctypes.memmove(dst, src, n)

    def rebase(self, recs_addr, peers, n_lines):
        self.calls.append(("rebase", -1, -1, n_lines))
        self.pkg.Transport.rebase(self, recs_addr, peers, n_lines)


def _rank_packs(pkg, oracle, world, n_shards, nb, empty_rank):
    alive = [0 if k % 7 == 3 else 1 for k in range(n_shards)]
    packs, inputs = [], []
    for r in range(world):
        if r == empty_rank:   # nothing valid to send
            datas = [np.frombuffer(pkg.frame_datagrams([b"no colon here\n", b"x\n"]), dtype=np.uint8)]
        else:
            datas = [pkg.gen_stream(20_000 + 3_000 * r + 1_000 * b, [64, 256, 1024], seed=500 + 10 * r + b,
                                    p_invalid=0.1).data for b in range(nb)]
        recs = [oracle.route(d, n_shards, alive)[0] for d in datas]
        packs.append(oracle.pack_many_by_owner(datas, recs, world))
        inputs.append((datas, recs))
    return packs, inputs


def _expected_lines(inputs, world, owner):
    lines, routes = [], []
    for datas, recs in inputs:
        for d, rr in zip(datas, recs):
            for x in rr:
                if x["route"] < 0xFFFD and x["route"] % world == owner:
                    lines.append(bytes(d[x["offset"]: x["offset"] + x["length"]]))
                    routes.append(int(x["route"]))
    return lines, routes


@pytest.mark.parametrize("world,n_shards,nb", [(2, 64, 1), (3, 16, 2), (8, 64, 2), (8, 5, 1)])
def test_exchange_run_threads(pkg, oracle, world, n_shards, nb):
    packs, inputs = _rank_packs(pkg, oracle, world, n_shards, nb, empty_rank=world - 1 if world > 2 else -1)
    box, cond = {}, threading.Condition()
    out, errs = {}, {}

    def rank_main(r):
        try:
            pb, pr, cnt = packs[r]
            sent = cnt.astype(np.uint64)
            received = np.stack([packs[s][2][r] for s in range(world)]).astype(np.uint64)
            n_l, n_b = int(received[:, 0].sum()), int(received[:, 1].sum())
            rb = np.full(n_b + 16, 0xCD, dtype=np.uint8)
            rr = np.zeros(max(n_l, 1), dtype=pkg.RECORD_DTYPE)
            pb = np.ascontiguousarray(pb) if pb.size else np.zeros(1, np.uint8)
            pr = np.ascontiguousarray(pr) if pr.size else np.zeros(1, pkg.RECORD_DTYPE)
            t = MailboxTransport(pkg, box, cond, r)
            pkg.exchange_run(t, world, r, sent, received, pb.ctypes.data, pr.ctypes.data, rb.ctypes.data,
                             rr.ctypes.data)
            out[r] = (rb, rr[:n_l], received, t.calls)
        except Exception as e:   # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    for r in range(world):
        rb, rr, received, calls = out[r]
        n_b = int(received[:, 1].sum())
        assert (rb[n_b:] == 0xCD).all()   # nothing written past the received total
        exp_lines, exp_routes = _expected_lines(inputs, world, r)
        assert len(rr) == len(exp_lines)
        assert [bytes(rb[x["offset"]: x["offset"] + x["length"]]) for x in rr] == exp_lines
        assert rr["route"].tolist() == exp_routes
        assert all(x["offset"] % 4 == 0 for x in rr)
        # byte-exact against the oracle's packs concatenated source by source, offsets rebased
        eb = np.concatenate([packs[s][0][int(packs[s][2][:r, 1].sum()):][: int(packs[s][2][r, 1])]
                             for s in range(world)])
        assert np.array_equal(rb[:n_b], eb)
        # the plan's call sequence: every peer's posts in rank order, the own chunk, one rebase
        peers = [c[1] for c in calls if c[0] in ("send", "recv")]
        assert peers == sorted(peers) and r not in peers
        assert calls[-1][0] == "rebase" if len(rr) else all(c[0] != "rebase" for c in calls)


def test_exchange_run_reports_transport_errors(pkg):
    class Failing(pkg.Transport):
        def send(self, addr, n, peer, tag):
            raise RuntimeError("link down")

        def recv(self, addr, n, peer, tag):
            pass

    s = np.array([[1, 8], [1, 8]], dtype=np.uint64)
    buf = np.zeros(64, dtype=np.uint8)
    with pytest.raises(RuntimeError, match="link down"):
        pkg.exchange_run(Failing(), 2, 0, s, s, buf.ctypes.data, buf.ctypes.data, buf.ctypes.data, buf.ctypes.data)
