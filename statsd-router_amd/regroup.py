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

import torch
import torch.distributed as dist


def _exchange(packed_bytes, packed_recs, owner_counts, group):
    """exchange_packed, also returning the host copies of the split sizes ([G, 2] lists sent and
    received). One host round trip per exchange: the sent and received sizes come back in one copy,
    and the offset rebase runs on the device from the received sizes (no host-built tensors)."""
    G = dist.get_world_size(group)
    dev = packed_bytes.device
    both = torch.empty((2, G, 2), dtype=torch.int64, device=dev)
    both[0].copy_(owner_counts.reshape(G, 2))
    dist.all_to_all_single(both[1], both[0], group=group)
    send, recv = both.cpu().tolist()
    in_l, in_b = [c[0] for c in send], [c[1] for c in send]
    out_l, out_b = [c[0] for c in recv], [c[1] for c in recv]
    n_l, n_b = sum(out_l), sum(out_b)
    recv_bytes = torch.empty(n_b, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv_bytes, packed_bytes[: sum(in_b)], out_b, in_b, group=group)
    recv_recs = torch.empty(n_l, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_recs, packed_recs[: sum(in_l)], out_l, in_l, group=group)
    recv_counts = both[1]
    if n_l:
        # record offset = low 32 bits (little-endian {u32 offset, u16 length, u16 route}); every
        # rebased offset stays below 2^32, so a 64-bit add never carries into length/route.
        # base[s] = bytes received from ranks before s (exclusive scan, on the device)
        base = torch.cumsum(recv_counts[:, 1], 0) - recv_counts[:, 1]
        recv_recs += torch.repeat_interleave(base, recv_counts[:, 0], output_size=n_l)
    return recv_bytes, recv_recs, recv_counts, send, recv


def exchange_packed(packed_bytes: torch.Tensor, packed_recs: torch.Tensor, owner_counts: torch.Tensor,
                    group=None):
    """All-to-all of packed lines.

    packed_bytes: uint8 (at least the packed total); packed_recs: int64 view of the sr_records
    (at least the packed line count); owner_counts: int64 [G, 2] {lines, bytes} per owner.
    Returns (recv_bytes uint8, recv_recs int64 with offsets into recv_bytes, recv_counts [G, 2]
    = {lines, bytes} received from each source rank)."""
    return _exchange(packed_bytes, packed_recs, owner_counts, group)[:3]


class Regrouper:
    """Pack (HIP) + exchange for one Router context; buffers sized for one batch."""

    def __init__(self, pkg, router, max_batch_bytes: int, max_records: int, group=None):
        self.pkg, self.router, self.group = pkg, router, group
        self.G = dist.get_world_size(group)
        if not 1 <= self.G <= pkg.SR_MAX_OWNERS:
            raise ValueError(f"regroup over {self.G} ranks: at most {pkg.SR_MAX_OWNERS}")
        dev = torch.device("cuda", router.device)
        self.cap = pkg.pack_capacity(max_batch_bytes)
        self.max_records = max_records
        self.out_bytes = torch.empty(self.cap, dtype=torch.uint8, device=dev)
        self.out_recs = torch.empty(max(max_records, 1), dtype=torch.int64, device=dev)
        self.counts = torch.zeros((self.G, 2), dtype=torch.int64, device=dev)
        # host copies of the last exchange's split sizes ([G][lines, bytes] sent and received)
        self.last_sent: list = []
        self.last_received: list = []

    def pack(self, d_bytes: int, nbytes: int, d_recs: int, d_n_records: int, max_records: int) -> None:
        if max_records > self.max_records:
            raise ValueError("max_records exceeds the regrouper's record buffer")
        self.router.pack_by_owner(d_bytes, nbytes, d_recs, d_n_records, max_records, self.G,
                                  self.out_bytes.data_ptr(), self.cap, self.out_recs.data_ptr(),
                                  self.counts.data_ptr())

    def exchange(self):
        """Pack output -> all-to-all (call after pack, on the router's stream = torch's current one)."""
        rb, rr, rc, self.last_sent, self.last_received = _exchange(self.out_bytes, self.out_recs, self.counts,
                                                                   self.group)
        return rb, rr, rc

    def __call__(self, d_bytes: int, nbytes: int, d_recs: int, d_n_records: int, max_records: int):
        self.pack(d_bytes, nbytes, d_recs, d_n_records, max_records)
        return self.exchange()
