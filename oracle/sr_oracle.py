"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes view of the CPU restatement (oracle/sr_oracle.c -> oracle/_build/libsr_oracle.so) and a
runner for the compiled reference harness (oracle/_ref/sr_ref_harness, built from the reference's
own sources by `make -C oracle ref`). Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module; the product never does.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess
import tempfile
from typing import Sequence

import numpy as np

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(ORACLE_DIR, "_build", "libsr_oracle.so")
REF_HARNESS = os.path.join(ORACLE_DIR, "_ref", "sr_ref_harness")
REF_ROUTER = os.path.join(ORACLE_DIR, "_ref", "sr_ref_router")
REF_TEST_HOSTNAME = "sr-test-host"   # what ref_router_harness.c makes gethostname() return

RECORD_DTYPE = np.dtype([("offset", "<u4"), ("length", "<u2"), ("route", "<u2")])
PACKET_DTYPE = np.dtype([("first", "<u4"), ("nlines", "<u2"), ("shard", "<u2"), ("length", "<u2"),
                         ("carry", "<u2"), ("open", "<u4")])
REF_EVENT_DTYPE = np.dtype([("verdict", "u1"), ("zero", "u1"), ("route", "<u2"), ("length", "<i4"),
                            ("hash", "<u8")])

_LIB = None


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        if not os.path.exists(ORACLE_LIB):
            raise ImportError(f"{ORACLE_LIB} missing: run `make -C oracle`")
        L = ctypes.CDLL(ORACLE_LIB)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.sro_frame_datagram.restype, L.sro_frame_datagram.argtypes = sz, [vp, vp, sz]
        L.sro_hash.restype, L.sro_hash.argtypes = ctypes.c_int, [vp, sz, ctypes.POINTER(ctypes.c_uint64)]
        L.sro_find_downstream.restype = ctypes.c_int
        L.sro_find_downstream.argtypes = [ctypes.c_uint64, ctypes.c_uint32, vp]
        L.sro_route_batch.restype = sz
        L.sro_route_batch.argtypes = [vp, sz, ctypes.c_uint32, vp, vp, sz, vp]
        L.sro_probed_dead.restype = None
        L.sro_probed_dead.argtypes = [vp, sz, ctypes.c_uint32, vp, vp]
        L.sro_pack_packets.restype = ctypes.c_int
        L.sro_pack_packets.argtypes = [vp, sz, ctypes.c_uint32, vp, vp, vp, vp, sz, ctypes.POINTER(sz),
                                       ctypes.POINTER(sz), vp]
        L.sro_bench.restype = ctypes.c_int
        L.sro_bench.argtypes = [vp, vp, sz, ctypes.c_uint32, vp, ctypes.c_int, ctypes.c_double,
                                ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                ctypes.POINTER(ctypes.c_double)]
        _LIB = L
    return _LIB


def alive_words(n: int, alive) -> np.ndarray:
    nw = max((n + 63) // 64, 1)
    w = np.zeros(nw, dtype=np.uint64)
    bits = np.ones(n, dtype=bool) if alive is None else np.asarray(list(alive), dtype=bool)
    for k in np.nonzero(bits)[0]:
        w[k >> 6] |= np.uint64(1) << np.uint64(k & 63)
    return w


def frame(dgram: bytes) -> bytes:
    """sr-main.c:163-173."""
    out = ctypes.create_string_buffer(len(dgram) + 2)
    n = lib().sro_frame_datagram(out, dgram, len(dgram))
    return out.raw[:n]


def hash_line(line: bytes):
    """sr-main.c:120-134: the sdbm hash, or None if the line has no ':'."""
    h = ctypes.c_uint64(0)
    rc = lib().sro_hash(line, len(line), ctypes.byref(h))
    return None if rc else h.value


def find_downstream(h: int, n: int, alive=None) -> int:
    w = alive_words(n, alive)
    return lib().sro_find_downstream(h, n, w.ctypes.data)


def route(data, n_downstreams: int, alive=None, max_records: int | None = None):
    """Records (structured array), hashes, and the line count for a framed batch."""
    buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, dtype=np.uint8)
    cap = buf.size if max_records is None else max_records
    out = np.zeros(max(cap, 1), dtype=RECORD_DTYPE)
    hs = np.zeros(max(cap, 1), dtype=np.uint64)
    w = alive_words(n_downstreams, alive)
    n = lib().sro_route_batch(buf.ctypes.data, buf.size, n_downstreams, w.ctypes.data, out.ctypes.data,
                              cap, hs.ctypes.data)
    k = min(n, cap)
    return out[:k], hs[:k], n


def probed_dead(data, n_downstreams: int, alive) -> np.ndarray:
    """Shard ids of the dead downstreams the batch's probes visit (sr-main.c:106)."""
    buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, dtype=np.uint8)
    w = alive_words(n_downstreams, alive)
    out = np.zeros(max((n_downstreams + 63) // 64, 1), dtype=np.uint64)
    lib().sro_probed_dead(buf.ctypes.data, buf.size, n_downstreams, w.ctypes.data, out.ctypes.data)
    bits = np.unpackbits(out.view(np.uint8), bitorder="little")[:n_downstreams]
    return np.nonzero(bits)[0]


def pack_packets(recs: np.ndarray, n_downstreams: int, fill_in=None, probed=()):
    """push_to_downstream + ds_schedule_flush (sr-main.c:49-83) over routed records, in the form of
    sr_pack_packets. Returns (sorted records, packets (PACKET_DTYPE), fill_out u16[N], n_valid)."""
    recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
    n = len(recs)
    fin = np.zeros(max(n_downstreams, 1), dtype=np.uint16)
    if fill_in is not None:
        fin[:n_downstreams] = np.asarray(fill_in, dtype=np.uint16)
    pw = np.zeros(max((n_downstreams + 63) // 64, 1), dtype=np.uint64)
    for k in probed:
        pw[int(k) >> 6] |= np.uint64(1) << np.uint64(int(k) & 63)
    sorted_ = np.zeros(max(n, 1), dtype=RECORD_DTYPE)
    cap = 2 * n + 5 * n_downstreams + 4
    pk = np.zeros(cap, dtype=PACKET_DTYPE)
    fout = np.zeros(max(n_downstreams, 1), dtype=np.uint16)
    npk, nv = ctypes.c_size_t(), ctypes.c_size_t()
    rc = lib().sro_pack_packets(recs.ctypes.data, n, n_downstreams, fin.ctypes.data, pw.ctypes.data,
                                sorted_.ctypes.data, pk.ctypes.data, cap, ctypes.byref(npk), ctypes.byref(nv),
                                fout.ctypes.data)
    if rc:
        raise RuntimeError("sro_pack_packets: descriptor room")
    return sorted_[:n], pk[: npk.value], fout[:n_downstreams], nv.value


def materialize(data, sorted_recs: np.ndarray, packets: np.ndarray, pending: dict, fill_out=None):
    """Packet bytes from descriptors: {shard: [flushed packet bytes, ...]} and the new pending
    buffers {shard: bytes}. pending: {shard: bytes pending before the batch}; fill_out (optional):
    the pending lengths after the batch (a shard without descriptors whose fill_out is 0 was
    probed dead: its pending bytes are dropped, sr-main.c:106)."""
    raw = bytes(data)
    out, new_pending = {}, dict(pending)
    if fill_out is not None:
        for s, f in enumerate(fill_out):
            if int(f) == 0:
                new_pending[s] = b""
    for p in packets:
        s = int(p["shard"])
        body = b"".join(raw[int(r["offset"]): int(r["offset"]) + int(r["length"])]
                        for r in sorted_recs[int(p["first"]): int(p["first"]) + int(p["nlines"])])
        assert len(body) == int(p["length"])
        lead = pending.get(s, b"")[: int(p["carry"])]
        assert len(lead) == int(p["carry"])
        if int(p["open"]):
            new_pending[s] = lead + body
        else:
            out.setdefault(s, []).append(lead + body)
    return out, new_pending


def pack_many_by_owner(datas, recs_list, n_owners: int):
    """sr_pack_many_by_owner restated from pack_by_owner: per owner, batch 0's chunk, then batch 1's, ...;
    record offsets relative to the owner's chunk. Returns (packed bytes, packed records, counts[G, 2])."""
    parts = [pack_by_owner(d, r, n_owners) for d, r in zip(datas, recs_list)]
    out_b, out_r = [], []
    counts = np.zeros((n_owners, 2), dtype=np.int64)
    for o in range(n_owners):
        shift = 0
        for pb, pr, pc in parts:
            l0 = int(pc[:o, 0].sum())
            b0 = int(pc[:o, 1].sum())
            nl, nb = int(pc[o, 0]), int(pc[o, 1])
            out_b.append(pb[b0: b0 + nb])
            rr = pr[l0: l0 + nl].copy()
            rr["offset"] = rr["offset"] + shift
            out_r.append(rr)
            shift += nb
            counts[o] += (nl, nb)
    cat_b = np.concatenate(out_b) if out_b else np.zeros(0, np.uint8)
    cat_r = np.concatenate(out_r) if out_r else np.zeros(0, RECORD_DTYPE)
    return cat_b, cat_r, counts


def bench(batches: Sequence[np.ndarray], n_downstreams: int, alive, threads: int, seconds: float):
    """Time the restatement (the reference's serial per-line loop) on host cores.
    Returns (lines, bytes, wall_seconds)."""
    arrs = [np.ascontiguousarray(b, dtype=np.uint8) for b in batches]
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    sizes = (ctypes.c_size_t * len(arrs))(*[a.size for a in arrs])
    w = alive_words(n_downstreams, alive)
    lines, nbytes, wall = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_double()
    rc = lib().sro_bench(ptrs, sizes, len(arrs), n_downstreams, w.ctypes.data, threads, seconds,
                         ctypes.byref(lines), ctypes.byref(nbytes), ctypes.byref(wall))
    if rc:
        raise RuntimeError("sro_bench failed")
    return lines.value, nbytes.value, wall.value


def have_reference() -> bool:
    return os.path.exists(REF_HARNESS)


def run_reference(dgrams: Sequence[bytes], n_downstreams: int, alive=None, probed: bool = False):
    """Feed raw datagrams through the REFERENCE's udp_read_cb (compiled from /root/reference) and
    return its per-line events (REF_EVENT_DTYPE); with probed=True also the shard ids of the dead
    downstreams whose pending buffer the reference dropped (sr-main.c:106)."""
    w = alive_words(n_downstreams, alive)
    with tempfile.TemporaryDirectory() as td:
        fin, fout, fpr = os.path.join(td, "in.bin"), os.path.join(td, "out.bin"), os.path.join(td, "pr.bin")
        with open(fin, "wb") as f:
            for d in dgrams:
                f.write(struct.pack("<I", len(d)))
                f.write(d)
        hexw = ",".join(f"{int(x):x}" for x in w)
        subprocess.run([REF_HARNESS, str(n_downstreams), hexw, fin, fout] + ([fpr] if probed else []), check=True)
        ev = np.fromfile(fout, dtype=REF_EVENT_DTYPE)
        if not probed:
            return ev
        pw = np.fromfile(fpr, dtype=np.uint64)
        bits = np.unpackbits(pw.view(np.uint8), bitorder="little")[:n_downstreams] if pw.size else np.zeros(0)
        return ev, np.nonzero(bits)[0]


# ---- one reference data thread driven by scripted events (oracle/ref_router_harness.c) ---------
EV_ALIVE, EV_FLUSH, EV_PING = 0xFFFFFFF1, 0xFFFFFFF2, 0xFFFFFFF3


def write_events(path: str, events, n_downstreams: int) -> None:
    """events: ("dgram", bytes) | ("alive", [0/1 per downstream]) | ("flush",) | ("ping",)."""
    with open(path, "wb") as f:
        for e in events:
            if e[0] == "dgram":
                f.write(struct.pack("<I", len(e[1])))
                f.write(e[1])
            elif e[0] == "alive":
                f.write(struct.pack("<I", EV_ALIVE))
                f.write(alive_words(n_downstreams, e[1]).tobytes())
            elif e[0] == "flush":
                f.write(struct.pack("<I", EV_FLUSH))
            elif e[0] == "ping":
                f.write(struct.pack("<I", EV_PING))
            else:
                raise ValueError(e)


def parse_router_output(blob: bytes):
    """-> {"packets": {ds: [bytes]}, "logs": [(level, text bytes)], "final": {ds: (pending, traffic, packets)}}"""
    res = {"packets": {}, "logs": [], "final": {}}
    i = 0
    while i < len(blob):
        t = blob[i]
        if t == 1:
            d, l = struct.unpack_from("<HH", blob, i + 1)
            res["packets"].setdefault(d, []).append(blob[i + 5: i + 5 + l])
            i += 5 + l
        elif t == 2:
            lv, l = struct.unpack_from("<BH", blob, i + 1)
            res["logs"].append((lv, blob[i + 4: i + 4 + l]))
            i += 4 + l
        elif t == 3:
            d, l = struct.unpack_from("<HH", blob, i + 1)
            pend = blob[i + 5: i + 5 + l]
            tr, pk = struct.unpack_from("<II", blob, i + 5 + l)
            res["final"][d] = (pend, tr, pk)
            i += 13 + l
        else:
            raise ValueError(f"bad event type {t} at {i}")
    return res


def have_reference_router() -> bool:
    return os.path.exists(REF_ROUTER)


def run_reference_router(config_text: str, events, n_downstreams: int):
    """Run the REFERENCE data thread (init_config + udp_read_cb + ds_flush_timer_cb + ping_cb +
    ds_flush_cb, compiled from /root/reference) over scripted events."""
    with tempfile.TemporaryDirectory() as td:
        cfg, fin, fout = (os.path.join(td, x) for x in ("sr.conf", "in.bin", "out.bin"))
        with open(cfg, "w") as f:
            f.write(config_text)
        write_events(fin, events, n_downstreams)
        subprocess.run([REF_ROUTER, cfg, fin, fout], check=True)
        with open(fout, "rb") as f:
            return parse_router_output(f.read())


def pack_by_owner(data, recs: np.ndarray, n_owners: int):
    """Restatement of sr_pack_by_owner (include/sr_route.h), numpy, test-only.

    Valid lines (route < 0xFFFD) grouped by owner = route % n_owners, input order within an owner;
    each line starts at a 4-byte aligned position, zero fill in between. Returns
    (packed bytes, packed records with offsets relative to the owner's chunk, counts[G, 2] =
    {lines, bytes} per owner). Parity unpinned against the reference, which has no multi-GPU
    path: what is pinned is the per-shard line sequence, compared with the oracle's routing."""
    buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.asarray(data, np.uint8)
    route = recs["route"].astype(np.int64)
    valid = route < 0xFFFD
    owner = np.where(valid, route % n_owners, -1)
    idx = np.nonzero(valid)[0]
    order = idx[np.argsort(owner[idx], kind="stable")]
    lens = recs["length"][order].astype(np.int64)
    len4 = (lens + 3) & ~3
    pos = np.cumsum(len4) - len4                      # global position in the packed buffer
    own = owner[order]
    lines = np.bincount(own, minlength=n_owners).astype(np.int64)
    nbytes = np.bincount(own, weights=len4, minlength=n_owners).astype(np.int64)
    start = np.cumsum(nbytes) - nbytes
    total = int(len4.sum())
    out = np.zeros(total, dtype=np.uint8)
    if lens.size:
        seg = np.cumsum(lens) - lens
        j = np.arange(int(lens.sum()), dtype=np.int64) - np.repeat(seg, lens)
        out[np.repeat(pos, lens) + j] = buf[np.repeat(recs["offset"][order].astype(np.int64), lens) + j]
    out_recs = recs[order].copy()
    out_recs["offset"] = (pos - start[own]).astype(np.uint32)
    return out, out_recs, np.stack([lines, nbytes], axis=1)
