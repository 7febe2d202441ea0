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

RECORD_DTYPE = np.dtype([("offset", "<u4"), ("length", "<u2"), ("route", "<u2")])
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


def run_reference(dgrams: Sequence[bytes], n_downstreams: int, alive=None) -> np.ndarray:
    """Feed raw datagrams through the REFERENCE's udp_read_cb (compiled from /root/reference) and
    return its per-line events (REF_EVENT_DTYPE)."""
    w = alive_words(n_downstreams, alive)
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fin, "wb") as f:
            for d in dgrams:
                f.write(struct.pack("<I", len(d)))
                f.write(d)
        hexw = ",".join(f"{int(x):x}" for x in w)
        subprocess.run([REF_HARNESS, str(n_downstreams), hexw, fin, fout], check=True)
        return np.fromfile(fout, dtype=REF_EVENT_DTYPE)


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
