"""Multi-GPU regroup of routed lines by owner GPU.

Each GPU routes its own datagram batches (no exchange on that path). Shard s is owned by GPU
s % G, which is the one that sends its lines on to downstream s (push_to_downstream,
sr-main.c:73-83). The exchange:
  1. sr_pack_by_owner (HIP, libsr_route.so): valid lines packed by owner, 4-byte aligned, with
     one record per line and the per-owner {lines, bytes} split sizes;
  2. all-to-all of the split sizes, then of the packed bytes and of the records (RCCL over xGMI
     with the "nccl" backend; gloo in the CPU tests);
  3. the received records' offsets are rebased into the received byte buffer.
Per source GPU the order of every shard's lines is the input order, as one reference thread
pushes them.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def _exchange_sizes(owner_counts, both, group):
    """First half of an exchange: all-to-all of the split sizes into both[1] (both[0] = ours).
    both: int64 [2, G, 2] on the packing device."""
    G = dist.get_world_size(group)
    both[0].copy_(owner_counts.reshape(G, 2))
    dist.all_to_all_single(both[1], both[0], group=group)


def _exchange_data(packed_bytes, packed_recs, recv_counts, send, recv, group):
    """Second half: all-to-all of the packed lines and records with the host copies of the split
    sizes, then the offset rebase on the device from the received sizes (no host-built tensors)."""
    dev = packed_bytes.device
    in_l, in_b = [c[0] for c in send], [c[1] for c in send]
    out_l, out_b = [c[0] for c in recv], [c[1] for c in recv]
    n_l, n_b = sum(out_l), sum(out_b)
    recv_bytes = torch.empty(n_b, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv_bytes, packed_bytes[: sum(in_b)], out_b, in_b, group=group)
    recv_recs = torch.empty(n_l, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_recs, packed_recs[: sum(in_l)], out_l, in_l, group=group)
    if n_l:
        # record offset = low 32 bits (little-endian {u32 offset, u16 length, u16 route}); every
        # rebased offset stays below 2^32, so a 64-bit add never carries into length/route.
        # base[s] = bytes received from ranks before s (exclusive scan, on the device)
        base = torch.cumsum(recv_counts[:, 1], 0) - recv_counts[:, 1]
        recv_recs += torch.repeat_interleave(base, recv_counts[:, 0], output_size=n_l)
    return recv_bytes, recv_recs


def _exchange(packed_bytes, packed_recs, owner_counts, group):
    """exchange_packed, also returning the host copies of the split sizes ([G, 2] lists sent and
    received). One host round trip per exchange: the sent and received sizes come back in one copy."""
    G = dist.get_world_size(group)
    both = torch.empty((2, G, 2), dtype=torch.int64, device=packed_bytes.device)
    _exchange_sizes(owner_counts, both, group)
    send, recv = both.cpu().tolist()
    rb, rr = _exchange_data(packed_bytes, packed_recs, both[1], send, recv, group)
    return rb, rr, both[1], send, recv


def exchange_packed(packed_bytes: torch.Tensor, packed_recs: torch.Tensor, owner_counts: torch.Tensor,
                    group=None):
    """All-to-all of packed lines.

    packed_bytes: uint8 (at least the packed total); packed_recs: int64 view of the sr_records
    (at least the packed line count); owner_counts: int64 [G, 2] {lines, bytes} per owner.
    Returns (recv_bytes uint8, recv_recs int64 with offsets into recv_bytes, recv_counts [G, 2]
    = {lines, bytes} received from each source rank)."""
    return _exchange(packed_bytes, packed_recs, owner_counts, group)[:3]


class DistHostTransport:
    """sr_transport over torch.distributed point-to-point calls on HOST memory (gloo): the C ABI's
    exchange (sr_exchange_run: plan, grouped sends/receives, own chunk, rebase) with gloo in place of
    RCCL, so the CPU tests drive the same C plan as sr_exchange_data. Sends and receives are posted
    (isend/irecv) between group_start and group_end, which waits for all of them, like an RCCL group."""

    def __init__(self, pkg, group=None):
        self.pkg, self.group, self.pending = pkg, group, []
        self.calls = []   # (kind, peer, tag, nbytes): what the plan asked for, in order

    def _view(self, addr, n):
        import ctypes
        return torch.frombuffer((ctypes.c_uint8 * n).from_address(addr), dtype=torch.uint8)

    def _global(self, peer):
        return dist.get_global_rank(self.group, peer) if self.group is not None else peer

    def group_start(self):
        self.pending = []

    def group_end(self):
        for w in self.pending:
            w.wait()
        self.pending = []

    def send(self, addr, n, peer, tag):
        self.calls.append(("send", peer, tag, n))
        self.pending.append(dist.isend(self._view(addr, n), self._global(peer), group=self.group, tag=tag))

    def recv(self, addr, n, peer, tag):
        self.calls.append(("recv", peer, tag, n))
        self.pending.append(dist.irecv(self._view(addr, n), self._global(peer), group=self.group, tag=tag))

    def copy(self, dst, src, n):
        import ctypes
        self.calls.append(("copy", -1, -1, n))
        ctypes.memmove(dst, src, n)

    def rebase(self, recs_addr, peers, n_lines):
        self.calls.append(("rebase", -1, -1, n_lines))
        self.pkg.Transport.rebase(self, recs_addr, peers, n_lines)


def exchange_packed_c(pkg, packed_bytes: torch.Tensor, packed_recs: torch.Tensor, owner_counts: torch.Tensor,
                      group=None, transport=None):
    """exchange_packed through the C ABI's plan (sr_exchange_run) on host tensors: the split sizes by
    all-to-all, then sr_exchange_run on a DistHostTransport. Returns (recv_bytes, recv_recs,
    recv_counts [G, 2], transport)."""
    G = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sent = owner_counts.reshape(G, 2).contiguous()
    received = torch.empty_like(sent)
    dist.all_to_all_single(received, sent, group=group)
    s, r = sent.numpy().astype(np.uint64), received.numpy().astype(np.uint64)
    n_l, n_b = int(r[:, 0].sum()), int(r[:, 1].sum())
    rb = torch.zeros(max(n_b, 1), dtype=torch.uint8)
    rr = torch.zeros(max(n_l, 1), dtype=torch.int64)
    t = transport or DistHostTransport(pkg, group)
    pkg.exchange_run(t, G, rank, s, r, packed_bytes.data_ptr(), packed_recs.data_ptr(), rb.data_ptr(),
                     rr.data_ptr())
    return rb[:n_b], rr[:n_l], received, t


class Regrouper:
    """Pack (HIP) + exchange for one Router context; buffers sized for one batch per slot.

    Synchronous use: `reg(...)` packs and exchanges one batch. Pipelined use (two slots):
    `start(slot, ...)` packs a batch and launches the all-to-all of its split sizes plus their
    copy to pinned host memory; `finish(slot)` waits for that copy and exchanges the lines. Calling
    start(i+1) before finish(i) lets batch i+1's route and pack run on the GPU while the host waits
    for batch i's sizes. All calls go on the router's stream (= torch's current one), so a slot's
    buffers are rewritten only after its exchange in stream order."""

    def __init__(self, pkg, router, max_batch_bytes: int, max_records: int, group=None, slots: int = 1):
        self.pkg, self.router, self.group = pkg, router, group
        self.G = dist.get_world_size(group)
        if not 1 <= self.G <= pkg.SR_MAX_OWNERS:
            raise ValueError(f"regroup over {self.G} ranks: at most {pkg.SR_MAX_OWNERS}")
        dev = torch.device("cuda", router.device)
        self.cap = pkg.pack_capacity(max_batch_bytes)
        self.max_records = max_records
        self.slots = [self._slot(dev) for _ in range(max(slots, 1))]
        # host copies of the last exchange's split sizes ([G][lines, bytes] sent and received)
        self.last_sent: list = []
        self.last_received: list = []

    def _slot(self, dev):
        return {"bytes": torch.empty(self.cap, dtype=torch.uint8, device=dev),
                "recs": torch.empty(max(self.max_records, 1), dtype=torch.int64, device=dev),
                "counts": torch.zeros((self.G, 2), dtype=torch.int64, device=dev),
                "both": torch.empty((2, self.G, 2), dtype=torch.int64, device=dev),
                "h_both": torch.empty((2, self.G, 2), dtype=torch.int64, pin_memory=True),
                "ev": torch.cuda.Event()}

    @property
    def counts(self):
        return self.slots[0]["counts"]

    def _check_stream(self):
        # the collectives are ordered after torch's current stream; the pack must run on it too
        h = getattr(self.router, "stream_handle", 0)
        if h == 0 or h != torch.cuda.current_stream().cuda_stream:
            raise RuntimeError("Regrouper: router.set_stream(s.cuda_stream) with s = torch's current stream "
                               "(a non-default stream) is required")

    def pack(self, d_bytes: int, nbytes: int, d_recs: int, d_n_records: int, max_records: int,
             slot: int = 0) -> None:
        self._check_stream()
        if max_records > self.max_records:
            raise ValueError("max_records exceeds the regrouper's record buffer")
        sl = self.slots[slot]
        self.router.pack_by_owner(d_bytes, nbytes, d_recs, d_n_records, max_records, self.G,
                                  sl["bytes"].data_ptr(), self.cap, sl["recs"].data_ptr(),
                                  sl["counts"].data_ptr())

    def exchange(self, slot: int = 0):
        """Pack output -> all-to-all (call after pack, on the router's stream = torch's current one)."""
        sl = self.slots[slot]
        rb, rr, rc, self.last_sent, self.last_received = _exchange(sl["bytes"], sl["recs"], sl["counts"],
                                                                   self.group)
        return rb, rr, rc

    def start(self, slot: int, d_bytes: int, nbytes: int, d_recs: int, d_n_records: int, max_records: int):
        sl = self.slots[slot]
        self.pack(d_bytes, nbytes, d_recs, d_n_records, max_records, slot)
        _exchange_sizes(sl["counts"], sl["both"], self.group)
        sl["h_both"].copy_(sl["both"], non_blocking=True)
        sl["ev"].record()

    def finish(self, slot: int):
        sl = self.slots[slot]
        sl["ev"].synchronize()
        self.last_sent, self.last_received = sl["h_both"].tolist()
        rb, rr = _exchange_data(sl["bytes"], sl["recs"], sl["both"][1], self.last_sent, self.last_received,
                                self.group)
        return rb, rr, sl["both"][1].clone()

    def __call__(self, d_bytes: int, nbytes: int, d_recs: int, d_n_records: int, max_records: int):
        self.pack(d_bytes, nbytes, d_recs, d_n_records, max_records)
        return self.exchange()


class LaunchRegrouper:
    """Pack + exchange of a whole route launch (up to SR_MAX_BATCHES_PER_LAUNCH batches) at once:
    one sr_pack_many_by_owner (owner chunks hold batch 0's lines, then batch 1's, ...), one
    all-to-all of the split sizes with one host round trip, then the packed lines and the records
    (RCCL over xGMI with the "nccl" backend; gloo in the CPU tests). Same stream rule as Regrouper."""

    def __init__(self, pkg, router, max_total_bytes: int, max_total_records: int, group=None, comm=None,
                 own_in_place: bool = True, one_call: bool = True):
        """comm: a pkg.Comm for the C-ABI exchange (sr_exchange_sizes / sr_exchange_data over RCCL);
        None: torch.distributed collectives on `group` (gloo in the CPU tests, nccl on GPUs).
        own_in_place (C-ABI exchange): the pack writes the rank's own chunk straight into the receive
        buffers; False: one sr_pack_many_by_owner and a device copy of the own chunk (A/B runs).
        one_call (with own_in_place): the whole regroup in one sr_regroup_launch; False: the same work in
        separate calls (sizes, size exchange, plan, scatter, exchange) from Python (A/B runs)."""
        self.pkg, self.router, self.group, self.comm = pkg, router, group, comm
        self.own_in_place = own_in_place
        self.one_call = one_call
        self.G = dist.get_world_size(group)
        if not 1 <= self.G <= pkg.SR_MAX_OWNERS:
            raise ValueError(f"regroup over {self.G} ranks: at most {pkg.SR_MAX_OWNERS}")
        dev = torch.device("cuda", router.device)
        self.cap = pkg.pack_capacity(max_total_bytes)
        self.max_records = max_total_records
        self.bytes = torch.empty(self.cap, dtype=torch.uint8, device=dev)
        self.recs = torch.empty(max(max_total_records, 1), dtype=torch.int64, device=dev)
        self.counts = torch.zeros((self.G, 2), dtype=torch.int64, device=dev)
        self.last_sent: list = []
        self.last_received: list = []
        self.recv_cap = (max(self.cap, 4), max(max_total_records, 1))   # grown when a receive is larger
        self._streams: dict = {}

    def __call__(self, batches):
        """batches = [(d_bytes, nbytes, d_recs, max_records, d_n_records), ...] routed on the router's
        stream. Returns (recv_bytes, recv_recs (offsets into recv_bytes), recv_counts [G, 2]).

        torch.distributed exchange: the collectives are ordered after torch's current stream, so the
        router must launch on it. C-ABI exchange (comm): pack, sizes, sends, receives and rebase are
        all ordered on the router's own stream, which need not be torch's current one; the returned
        buffers are allocated for that stream and are ready once it has reached this point."""
        h = getattr(self.router, "stream_handle", 0)
        cur = torch.cuda.current_stream(self.bytes.device).cuda_stream
        if h == 0 or (self.comm is None and h != cur):
            raise RuntimeError("LaunchRegrouper: router.set_stream(s.cuda_stream) with s a non-default stream is "
                               "required (for the torch.distributed exchange: torch's current stream)")
        if sum(b[3] for b in batches) > self.max_records or self.pkg.pack_capacity(sum(b[1] for b in batches)) > self.cap:
            raise ValueError("launch larger than the regrouper's buffers")
        if self.comm is None:
            self.router.pack_many_by_owner(batches, self.G, self.bytes.data_ptr(), self.cap, self.recs.data_ptr(),
                                           self.counts.data_ptr())
            rb, rr, rc, self.last_sent, self.last_received = _exchange(self.bytes, self.recs, self.counts, self.group)
            return rb, rr, rc
        # the C ABI: the split sizes, one size exchange (one host round trip), then the scatter with the
        # rank's own chunk written straight into its place in the receive buffers (no local copy), the
        # grouped sends and the rebase; receive buffers from the caching allocator's pool of the router's
        # stream. own_in_place: all of it in one sr_regroup_launch into receive buffers allocated before the
        # sizes are known (the largest receive so far); a receive that does not fit finishes in separate calls
        rs = self._streams.get(h)
        if rs is None:
            rs = torch.cuda.ExternalStream(h, device=self.bytes.device) if h != cur else torch.cuda.current_stream()
            self._streams[h] = rs
        dev = self.bytes.device
        if self.own_in_place:
            with torch.cuda.stream(rs):
                rc = torch.empty((self.G, 2), dtype=torch.int64, device=dev)
                rb = torch.empty(self.recv_cap[0], dtype=torch.uint8, device=dev)
                rr = torch.empty(self.recv_cap[1], dtype=torch.int64, device=dev)
            if self.one_call:
                fits, sent, received = self.router.regroup_launch(
                    self.comm, batches, self.counts.data_ptr(), rc.data_ptr(), self.bytes.data_ptr(), self.cap,
                    self.recs.data_ptr(), rb.data_ptr(), rb.numel(), rr.data_ptr(), rr.numel())
            else:
                self.router.pack_owner_sizes(batches, self.G, self.counts.data_ptr())
                sent, received = self.router.exchange_sizes(self.comm, self.counts.data_ptr(), rc.data_ptr())
                fits = False
            n_l, n_b = int(received[:, 0].sum()), int(received[:, 1].sum())
            if not fits:
                if n_b > rb.numel() or n_l > rr.numel():
                    self.recv_cap = (max(self.recv_cap[0], n_b + n_b // 4 + 4),
                                     max(self.recv_cap[1], n_l + n_l // 4 + 1))
                    with torch.cuda.stream(rs):
                        rb = torch.empty(self.recv_cap[0], dtype=torch.uint8, device=dev)
                        rr = torch.empty(self.recv_cap[1], dtype=torch.int64, device=dev)
                peers, _ = self.pkg.exchange_plan(self.G, self.comm.rank, sent, received)
                me = peers[self.comm.rank]
                self.router.pack_owner_scatter(batches, self.G, self.comm.rank, rb.data_ptr() + int(me["recv_byte0"]),
                                               rr.data_ptr() + 8 * int(me["recv_line0"]), self.bytes.data_ptr(),
                                               self.cap, self.recs.data_ptr())
                self.router.exchange_data(self.comm, self.bytes.data_ptr(), self.recs.data_ptr(), sent, received,
                                          rb.data_ptr(), rr.data_ptr())
        else:
            self.router.pack_many_by_owner(batches, self.G, self.bytes.data_ptr(), self.cap, self.recs.data_ptr(),
                                           self.counts.data_ptr())
            with torch.cuda.stream(rs):
                rc = torch.empty((self.G, 2), dtype=torch.int64, device=dev)
                sent, received = self.router.exchange_sizes(self.comm, self.counts.data_ptr(), rc.data_ptr())
                n_l, n_b = int(received[:, 0].sum()), int(received[:, 1].sum())
                rb = torch.empty(max(n_b, 1), dtype=torch.uint8, device=dev)
                rr = torch.empty(max(n_l, 1), dtype=torch.int64, device=dev)
            self.router.exchange_data(self.comm, self.bytes.data_ptr(), self.recs.data_ptr(), sent, received,
                                      rb.data_ptr(), rr.data_ptr())
        self.last_sent, self.last_received = sent.astype(np.int64).tolist(), received.astype(np.int64).tolist()
        return rb[:n_b], rr[:n_l], rc
