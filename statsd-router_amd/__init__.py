"""statsd-router_amd — MI355X-native statsd-router hot path.

Python view of the C ABI in ``include/sr_route.h`` (ctypes; the product is the C library
``lib/libsr_route.so`` built from ``csrc/sr_route.hip``). The reference has no Python API; this
module exists so tests and ``bench.py`` can drive the same C entry points a C host (the router's
``udp_read_cb`` replacement) calls. Names follow the reference's domain: datagrams, lines,
downstreams (shards), the alive bitmap.

Loading is strict: if ``libsr_route.so`` is missing or lacks a symbol, importing raises. There is
no CPU fallback of the hot path anywhere in this package.

Import with ``importlib.import_module("statsd-router_amd")`` (the directory name has a hyphen).
"""
from __future__ import annotations

import ctypes
import errno
import os
from dataclasses import dataclass
from typing import Iterable, Sequence

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_DIR = os.path.join(PKG_DIR, "lib")
# SR_ROUTE_LIB: another build of the same library (same-box A/B runs of kernel variants, tools/ab_kernels.sh)
ROUTE_LIB = os.environ.get("SR_ROUTE_LIB") or os.path.join(LIB_DIR, "libsr_route.so")
GEN_LIB = os.path.join(LIB_DIR, "libsr_gen.so")
HEADER = os.path.join(REPO_DIR, "include", "sr_route.h")

# ---- constants mirrored from include/sr_route.h (checked against the header by tests) --------
SR_DATA_BUF_SIZE = 4096
SR_MAX_DATAGRAM = 4095
SR_DOWNSTREAM_BUF_SIZE = 1450
SR_MIN_LINE_LENGTH = 6
SR_MAX_LINE_LENGTH = 1449
SR_MAX_DOWNSTREAMS = 65533
SR_VALID, SR_INVALID_LENGTH, SR_INVALID_FORMAT, SR_ALL_DEAD = 0, 1, 2, 3
SR_ROUTE_INVALID_LENGTH = 0xFFFD
SR_ROUTE_INVALID_FORMAT = 0xFFFE
SR_ROUTE_ALL_DEAD = 0xFFFF

RECORD_DTYPE = np.dtype([("offset", "<u4"), ("length", "<u2"), ("route", "<u2")])
assert RECORD_DTYPE.itemsize == 8

# every function the header declares (tests check the library exports exactly these)
ABI_FUNCTIONS = (
    "sr_frame_datagram", "sr_frame_datagrams", "sr_open", "sr_set_alive", "sr_set_stream", "sr_set_layout",
    "sr_last_layout",
    "sr_route_batch", "sr_last_probed_dead", "sr_route_device", "sr_route_device_many", "sr_pack_by_owner",
    "sr_pack_many_by_owner", "sr_pack_packets", "sr_pack_packets_many", "sr_route_pack_batch", "sr_alloc_host", "sr_free_host", "sr_sync", "sr_close", "sr_version",
    "sr_pack_owner_sizes", "sr_pack_owner_scatter", "sr_regroup_launch",
    "sr_comm_id", "sr_comm_open", "sr_comm_close", "sr_exchange_sizes", "sr_exchange_data",
    "sr_exchange_plan", "sr_exchange_run", "sr_exchange_rebase", "sr_route_pack_submit", "sr_route_pack_result",
    "sr_set_trace", "sr_route_pack_trace", "sr_set_knob", "sr_route_pack_many", "sr_regroup_run",
)
SR_MAX_PACK_DOWNSTREAMS = 4096
SR_LAYOUT_AUTO, SR_LAYOUT_UNIFORM, SR_LAYOUT_SEGMENTS, SR_LAYOUT_CHUNKS = 0, 1, 2, 3
SR_COMM_ID_BYTES = 128
# sr_set_knob (developer / test knobs of one context; none changes a result)
SR_KNOB_LB_SPIN, SR_KNOB_DEFER_PICKS, SR_KNOB_MTU_CHUNK, SR_KNOB_MTU_XCD, SR_KNOB_MTU_WALK = 1, 2, 3, 4, 5
SR_KNOB_HIST, SR_KNOB_PREFETCH, SR_KNOB_FUSE_DEFER = 7, 8, 9
LAYOUT_NAMES = {0: "none", 1: "uniform", 2: "segments", 3: "chunks"}
PACKET_DTYPE = np.dtype([("first", "<u4"), ("nlines", "<u2"), ("shard", "<u2"), ("length", "<u2"),
                         ("carry", "<u2"), ("open", "<u4")])
assert PACKET_DTYPE.itemsize == 16


def max_packets(nbytes: int, n_downstreams: int) -> int:
    """SR_MAX_PACKETS: descriptor room that always suffices."""
    return 2 * nbytes // 1450 + 5 * n_downstreams + 4
SR_MAX_OWNERS = 64


def pack_capacity(nbytes: int) -> int:
    """SR_PACK_CAPACITY: packed-bytes room that always suffices for a batch of nbytes."""
    return nbytes + nbytes // 2 + 4
SR_MAX_BATCHES_PER_LAUNCH = 32


class SrBatch(ctypes.Structure):
    """struct sr_batch (include/sr_route.h): one device-resident batch of sr_route_device_many."""
    _fields_ = [
        ("d_bytes", ctypes.c_void_p), ("nbytes", ctypes.c_size_t), ("d_out", ctypes.c_void_p),
        ("max_records", ctypes.c_size_t), ("d_hashes", ctypes.c_void_p), ("d_n_records", ctypes.c_void_p),
        ("d_probed_dead", ctypes.c_void_p),
    ]


class SrPackBatch(ctypes.Structure):
    """struct sr_pack_batch (include/sr_route.h): one batch of sr_pack_packets_many."""
    _fields_ = [
        ("d_recs", ctypes.c_void_p), ("d_n_records", ctypes.c_void_p), ("max_records", ctypes.c_size_t),
        ("d_fill_in", ctypes.c_void_p), ("d_probed_dead", ctypes.c_void_p), ("d_sorted", ctypes.c_void_p),
        ("d_packets", ctypes.c_void_p), ("max_packets", ctypes.c_size_t), ("d_counts", ctypes.c_void_p),
        ("d_fill_out", ctypes.c_void_p),
    ]


class SrPackResult(ctypes.Structure):
    """struct sr_pack_result (include/sr_route.h): the outputs of a sr_route_pack_submit slot."""
    _fields_ = [("sorted", ctypes.c_void_p), ("n_records", ctypes.c_size_t), ("n_valid", ctypes.c_size_t),
                ("packets", ctypes.c_void_p), ("n_packets", ctypes.c_size_t), ("fill", ctypes.c_void_p),
                ("probed_dead", ctypes.c_void_p)]


class SrExchangePeer(ctypes.Structure):
    """struct sr_exchange_peer (include/sr_route.h): one peer's share of an exchange plan."""
    _fields_ = [(n, ctypes.c_uint64) for n in ("send_line0", "send_lines", "send_byte0", "send_bytes",
                                               "recv_line0", "recv_lines", "recv_byte0", "recv_bytes")]


PEER_DTYPE = np.dtype([(n, "<u8") for n, _ in SrExchangePeer._fields_])

_GROUP_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
_SEND_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                            ctypes.c_int)
_COPY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
_REBASE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(SrExchangePeer),
                              ctypes.c_int, ctypes.c_uint64)
_SIZES_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p)


class SrTransport(ctypes.Structure):
    """struct sr_transport (include/sr_route.h)."""
    _fields_ = [("user", ctypes.c_void_p), ("group_start", _GROUP_FN), ("group_end", _GROUP_FN),
                ("send", _SEND_FN), ("recv", _SEND_FN), ("copy", _COPY_FN), ("rebase", _REBASE_FN)]


class SrError(OSError):
    """A negative errno returned by the C ABI."""


def _check(rc: int, what: str) -> int:
    if rc < 0:
        raise SrError(-rc, f"{what}: {os.strerror(-rc)}")
    return rc


def verdicts(routes: np.ndarray) -> np.ndarray:
    """Map the record ``route`` field to sr_verdict values (sr_record_verdict in the header)."""
    r = np.asarray(routes, dtype=np.uint16)
    v = np.zeros(r.shape, dtype=np.uint8)
    bad = r >= SR_ROUTE_INVALID_LENGTH
    v[bad] = (r[bad].astype(np.int32) - 0xFFFC).astype(np.uint8)
    return v


def _load_route_lib() -> ctypes.CDLL:
    # One HIP runtime per process: PyTorch-ROCm wheels bundle their own libamdhip64.so.7 /
    # libhsa-runtime64.so.1 (same sonames as /opt/rocm's). If torch is importable, load it first
    # so libsr_route.so binds to the runtime torch already uses (a second HSA runtime in the same
    # process cannot open the GPUs).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(ROUTE_LIB):
        raise ImportError(
            f"{ROUTE_LIB} is missing: build it with __graft_entry__.build() or `make -C statsd-router_amd`"
        )
    lib = ctypes.CDLL(ROUTE_LIB)
    c_size_p = ctypes.POINTER(ctypes.c_size_t)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    vp = ctypes.c_void_p
    sig = {
        "sr_frame_datagram": (ctypes.c_size_t, [vp, vp, ctypes.c_size_t]),
        "sr_frame_datagrams": (ctypes.c_size_t, [vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t]),
        "sr_open": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_size_t, ctypes.c_uint32]),
        "sr_set_alive": (ctypes.c_int, [vp, u64p]),
        "sr_set_stream": (ctypes.c_int, [vp, vp]),
        "sr_set_layout": (ctypes.c_int, [vp, ctypes.c_int]),
        "sr_last_layout": (ctypes.c_int, [vp]),
        "sr_route_batch": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, c_size_p, vp]),
        "sr_last_probed_dead": (ctypes.c_int, [vp, u64p]),
        "sr_route_device": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp, vp]),
        "sr_route_device_many": (ctypes.c_int, [vp, ctypes.POINTER(SrBatch), ctypes.c_size_t]),
        "sr_pack_by_owner": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, ctypes.c_uint32,
                                            vp, ctypes.c_size_t, vp, vp]),
        "sr_pack_many_by_owner": (ctypes.c_int, [vp, ctypes.POINTER(SrBatch), ctypes.c_size_t, ctypes.c_uint32, vp,
                                                 ctypes.c_size_t, vp, vp]),
        "sr_pack_owner_sizes": (ctypes.c_int, [vp, ctypes.POINTER(SrBatch), ctypes.c_size_t, ctypes.c_uint32, vp]),
        "sr_pack_owner_scatter": (ctypes.c_int, [vp, ctypes.POINTER(SrBatch), ctypes.c_size_t, ctypes.c_uint32,
                                                 ctypes.c_int, vp, vp, vp, ctypes.c_size_t, vp]),
        "sr_pack_packets": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t, vp, vp, vp, vp, ctypes.c_size_t, vp, vp]),
        "sr_pack_packets_many": (ctypes.c_int, [vp, ctypes.POINTER(SrPackBatch), ctypes.c_size_t]),
        "sr_route_pack_batch": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, c_size_p, c_size_p,
                                               vp, ctypes.c_size_t, c_size_p, vp]),
        "sr_alloc_host": (vp, [ctypes.c_size_t]),
        "sr_free_host": (None, [vp]),
        "sr_sync": (ctypes.c_int, [vp]),
        "sr_close": (None, [vp]),
        "sr_version": (ctypes.c_char_p, []),
        "sr_comm_id": (ctypes.c_int, [vp]),
        "sr_comm_open": (ctypes.c_int, [ctypes.POINTER(vp), vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
        "sr_comm_close": (None, [vp]),
        "sr_exchange_sizes": (ctypes.c_int, [vp, vp, vp, vp, vp, vp]),
        "sr_exchange_data": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp]),
        "sr_exchange_plan": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, vp, vp, vp, vp]),
        "sr_exchange_run": (ctypes.c_int, [ctypes.POINTER(SrTransport), ctypes.c_int, ctypes.c_int, vp, vp, vp, vp,
                                           vp, vp]),
        "sr_exchange_rebase": (ctypes.c_int, [vp, vp, vp, ctypes.c_int]),
        "sr_regroup_launch": (ctypes.c_int, [vp, vp, ctypes.POINTER(SrBatch), ctypes.c_size_t, vp, vp, vp,
                                             ctypes.c_size_t, vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp, vp]),
        "sr_route_pack_submit": (ctypes.c_int, [vp, ctypes.c_int, vp, ctypes.c_size_t, vp]),
        "sr_route_pack_result": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(SrPackResult)]),
        "sr_set_trace": (ctypes.c_int, [vp, ctypes.c_int]),
        "sr_route_pack_trace": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp), c_size_p]),
        "sr_set_knob": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int64]),
        "sr_route_pack_many": (ctypes.c_int, [vp, ctypes.POINTER(SrBatch), ctypes.POINTER(SrPackBatch), ctypes.c_size_t]),
        "sr_regroup_run": (ctypes.c_int, [vp, ctypes.POINTER(SrTransport), _SIZES_FN, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(SrBatch), ctypes.c_size_t, vp, vp, vp, ctypes.c_size_t, vp, vp,
                                          ctypes.c_size_t, vp, ctypes.c_size_t, vp, vp]),
    }
    for name in ABI_FUNCTIONS:
        if os.environ.get("SR_ROUTE_LIB") and not hasattr(lib, name):
            continue   # an older build under A/B (SR_ROUTE_LIB) may lack entry points added since
        fn = getattr(lib, name)  # raises AttributeError if the export is missing
        fn.restype, fn.argtypes = sig[name]
    return lib


_LIB: ctypes.CDLL | None = None
_GEN: ctypes.CDLL | None = None


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        _LIB = _load_route_lib()
    return _LIB


def gen_lib() -> ctypes.CDLL:
    global _GEN
    if _GEN is None:
        if not os.path.exists(GEN_LIB):
            raise ImportError(f"{GEN_LIB} is missing: build with __graft_entry__.build()")
        g = ctypes.CDLL(GEN_LIB)
        g.sr_gen_stream.restype = ctypes.c_size_t
        g.sr_gen_stream.argtypes = [
            ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_double,
            ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
            ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t),
        ]
        _GEN = g
    return _GEN


# ---- framing (host, no GPU) -----------------------------------------------------------------
def frame_datagrams(dgrams: Sequence[bytes]) -> bytes:
    """Frame datagrams as udp_read_cb does (sr-main.c:163-173) and concatenate them."""
    L = lib()
    cap = sum(min(len(d), SR_MAX_DATAGRAM) + 1 for d in dgrams)
    out = ctypes.create_string_buffer(max(cap, 1))
    bufs = [ctypes.create_string_buffer(bytes(d), max(len(d), 1)) for d in dgrams]
    ptrs = (ctypes.c_void_p * max(len(dgrams), 1))(*[ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_size_t * max(len(dgrams), 1))(*[len(d) for d in dgrams])
    n = L.sr_frame_datagrams(out, cap, ptrs, lens, len(dgrams))
    if n == ctypes.c_size_t(-1).value:
        raise SrError(errno.ENOSPC, "sr_frame_datagrams")
    return out.raw[:n]


# ---- synthetic traffic ------------------------------------------------------------------------
GEN_FIXED, GEN_TEST_SHAPE = 0, 1


@dataclass
class Stream:
    data: np.ndarray          # uint8, concatenated framed datagrams
    dgram_lens: np.ndarray    # uint32
    n_lines: int


def gen_stream(nbytes: int, line_lens: Iterable[int], seed: int, p_invalid: float = 0.0,
               kind: int = GEN_FIXED, max_dgram: int = SR_MAX_DATAGRAM) -> Stream:
    """Seeded synthetic stream (statsd-router_amd/csrc/sr_gen.c) of at most nbytes bytes."""
    g = gen_lib()
    lens = np.ascontiguousarray(np.array(list(line_lens), dtype=np.uint32))
    out = np.zeros(max(nbytes, 1), dtype=np.uint8)
    dcap = nbytes // 6 + 2
    dl = np.zeros(dcap, dtype=np.uint32)
    nd, nl = ctypes.c_size_t(0), ctypes.c_size_t(0)
    n = g.sr_gen_stream(seed, kind, lens.ctypes.data, len(lens), float(p_invalid), max_dgram,
                        out.ctypes.data, nbytes, dl.ctypes.data, dcap, ctypes.byref(nd), ctypes.byref(nl))
    return Stream(out[:n], dl[: min(nd.value, dcap)].copy(), nl.value)


def bitmap_shards(words, n: int) -> np.ndarray:
    """Shard ids whose bit is set in a ceil(n/64)-word bitmap."""
    w = np.asarray(words, dtype=np.uint64)
    bits = np.unpackbits(w.view(np.uint8), bitorder="little")[:n]
    return np.nonzero(bits)[0]


# ---- the router context -------------------------------------------------------------------------
def alive_words(n_downstreams: int, alive: Iterable[int] | np.ndarray | None) -> np.ndarray:
    """Bitmap words from a 0/1 sequence (None = all alive)."""
    nw = max((n_downstreams + 63) // 64, 1)
    w = np.zeros(nw, dtype=np.uint64)
    bits = np.ones(n_downstreams, dtype=bool) if alive is None else np.asarray(list(alive), dtype=bool)
    for k in np.nonzero(bits)[0]:
        w[k >> 6] |= np.uint64(1) << np.uint64(k & 63)
    return w


class Router:
    """One sr_ctx: a HIP stream's worth of routing state on one GPU (sr_open .. sr_close)."""

    def __init__(self, n_downstreams: int, max_batch_bytes: int, device: int = 0):
        self._lib = lib()
        self.n_downstreams = n_downstreams
        self.max_batch_bytes = max_batch_bytes
        self.device = device
        h = ctypes.c_void_p()
        _check(self._lib.sr_open(ctypes.byref(h), device, max_batch_bytes, n_downstreams), "sr_open")
        self._h = h

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def close(self) -> None:
        if self._h:
            self._lib.sr_close(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_alive(self, alive) -> None:
        """alive: 0/1 per downstream, or a uint64 word array."""
        a = np.asarray(alive)
        w = a.astype(np.uint64) if a.dtype == np.uint64 else alive_words(self.n_downstreams, alive)
        w = np.ascontiguousarray(w)
        _check(self._lib.sr_set_alive(self._h, w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))), "sr_set_alive")

    def set_stream(self, stream_handle: int | None) -> None:
        """Launch on this HIP stream from now on. 0/None = the context's own non-blocking stream
        (sr_set_stream's NULL), which is NOT the HIP null stream: work on torch's default stream
        is not ordered with it."""
        _check(self._lib.sr_set_stream(self._h, ctypes.c_void_p(stream_handle or 0)), "sr_set_stream")
        self.stream_handle = int(stream_handle or 0)

    def set_layout(self, layout: int) -> None:
        """sr_set_layout: SR_LAYOUT_AUTO (default), SR_LAYOUT_UNIFORM, SR_LAYOUT_SEGMENTS or
        SR_LAYOUT_CHUNKS (the route kernel's lane layout; records are identical either way)."""
        _check(self._lib.sr_set_layout(self._h, int(layout)), "sr_set_layout")

    def set_knob(self, knob: int, value: int) -> None:
        """sr_set_knob: a developer / test knob of this context (SR_KNOB_*); results never change."""
        _check(self._lib.sr_set_knob(self._h, int(knob), int(value)), "sr_set_knob")

    def set_trace(self, on: bool = True) -> None:
        """sr_set_trace: later route + pack submissions also return input-order records and hashes."""
        _check(self._lib.sr_set_trace(self._h, 1 if on else 0), "sr_set_trace")

    def route_pack_trace(self, slot: int):
        """sr_route_pack_trace after route_pack_result(slot) (slot 2: the last route_pack): (records in
        input order, per-line hashes), copied."""
        r, h, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_size_t()
        _check(self._lib.sr_route_pack_trace(self._h, slot, ctypes.byref(r), ctypes.byref(h), ctypes.byref(n)),
               "sr_route_pack_trace")
        k = n.value
        if not k:
            return np.zeros(0, RECORD_DTYPE), np.zeros(0, np.uint64)
        recs = np.frombuffer((ctypes.c_uint8 * (8 * k)).from_address(r.value), dtype=RECORD_DTYPE).copy()
        hs = np.frombuffer((ctypes.c_uint8 * (8 * k)).from_address(h.value), dtype=np.uint64).copy()
        return recs, hs

    def last_layout(self) -> int:
        """sr_last_layout: the lane layout of the context's last route launch (1 uniform, 2 segments,
        3 chunks)."""
        return _check(self._lib.sr_last_layout(self._h), "sr_last_layout")

    def route(self, data: bytes | np.ndarray, max_records: int | None = None, want_hashes: bool = False):
        """sr_route_batch on host memory. Returns (records[n] structured array, hashes or None, n)."""
        buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, dtype=np.uint8)
        nbytes = int(buf.size)
        cap = nbytes if max_records is None else max_records
        out = np.zeros(max(cap, 1), dtype=RECORD_DTYPE)
        hashes = np.zeros(max(cap, 1), dtype=np.uint64) if want_hashes else None
        n = ctypes.c_size_t(0)
        rc = self._lib.sr_route_batch(self._h, buf.ctypes.data if nbytes else None, nbytes, out.ctypes.data,
                                      cap, ctypes.byref(n), hashes.ctypes.data if want_hashes else None)
        if rc not in (0, -errno.ENOSPC):
            _check(rc, "sr_route_batch")
        k = min(n.value, cap)
        return out[:k], (hashes[:k] if want_hashes else None), n.value

    def last_probed_dead(self) -> np.ndarray:
        """sr_last_probed_dead: the dead downstreams probed by the last route() (sr-main.c:106) as
        a sorted array of shard ids."""
        nw = max((self.n_downstreams + 63) // 64, 1)
        w = np.zeros(nw, dtype=np.uint64)
        _check(self._lib.sr_last_probed_dead(self._h, w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))),
               "sr_last_probed_dead")
        return bitmap_shards(w, self.n_downstreams)

    def route_device(self, d_bytes: int, nbytes: int, d_out: int, max_records: int,
                     d_hashes: int | None, d_count: int) -> None:
        """sr_route_device with raw device pointers (e.g. torch tensors' data_ptr())."""
        _check(self._lib.sr_route_device(self._h, ctypes.c_void_p(d_bytes), nbytes, ctypes.c_void_p(d_out),
                                         max_records, ctypes.c_void_p(d_hashes or 0), ctypes.c_void_p(d_count)),
               "sr_route_device")

    def route_device_many(self, batches) -> None:
        """sr_route_device_many: batches = [(d_bytes, nbytes, d_out, max_records, d_hashes, d_count
        [, d_probed_dead]), ...]."""
        arr = (SrBatch * max(len(batches), 1))()
        for i, b in enumerate(batches):
            db, nb, do, mr, dh, dc = b[:6]
            dp = b[6] if len(b) > 6 else None
            arr[i] = SrBatch(db, nb, do, mr, dh or None, dc, dp or None)
        _check(self._lib.sr_route_device_many(self._h, arr, len(batches)), "sr_route_device_many")

    def pack_by_owner(self, d_bytes: int, nbytes: int, d_recs: int, d_n_records: int, max_records: int,
                      n_owners: int, d_out_bytes: int, out_cap: int, d_out_recs: int, d_owner_counts: int) -> None:
        """sr_pack_by_owner with raw device pointers (asynchronous on the context's stream)."""
        vp = ctypes.c_void_p
        _check(self._lib.sr_pack_by_owner(self._h, vp(d_bytes), nbytes, vp(d_recs), vp(d_n_records), max_records,
                                          n_owners, vp(d_out_bytes), out_cap, vp(d_out_recs), vp(d_owner_counts)),
               "sr_pack_by_owner")

    def route_pack(self, data, fill=None):
        """sr_route_pack_batch on host memory: route + per-downstream MTU packing. fill: pending
        bytes per downstream before the batch (None = 0). Returns (sorted records, packets,
        fill after, n_valid, probed-dead shard ids)."""
        buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, dtype=np.uint8)
        nbytes, n = int(buf.size), self.n_downstreams
        f = np.zeros(max(n, 1), dtype=np.uint16)
        if fill is not None:
            f[:n] = np.asarray(fill, dtype=np.uint16)
        srt = np.zeros(max(nbytes, 1), dtype=RECORD_DTYPE)
        mp = max_packets(nbytes, n)
        pk = np.zeros(mp, dtype=PACKET_DTYPE)
        pw = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
        nr, nv, npk = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        _check(self._lib.sr_route_pack_batch(self._h, buf.ctypes.data if nbytes else None, nbytes, f.ctypes.data,
                                             srt.ctypes.data, srt.size, ctypes.byref(nr), ctypes.byref(nv),
                                             pk.ctypes.data, mp, ctypes.byref(npk), pw.ctypes.data),
               "sr_route_pack_batch")
        return srt[: nr.value], pk[: npk.value], f[:n].copy(), nv.value, bitmap_shards(pw, n)

    def route_pack_submit(self, slot: int, data, fill=None) -> None:
        """sr_route_pack_submit (asynchronous). data must stay alive and unchanged until
        route_pack_result(slot): keep a reference (e.g. a pinned or numpy buffer). fill None = chain
        from the previous submission's pending bytes on the device."""
        buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, dtype=np.uint8)
        f = None
        if fill is not None:
            f = np.zeros(max(self.n_downstreams, 1), dtype=np.uint16)
            f[: self.n_downstreams] = np.asarray(fill, dtype=np.uint16)
        self._pending = getattr(self, "_pending", {})
        self._pending[slot] = buf
        _check(self._lib.sr_route_pack_submit(self._h, slot, buf.ctypes.data if buf.size else None, int(buf.size),
                                              f.ctypes.data if f is not None else None), "sr_route_pack_submit")

    def route_pack_result(self, slot: int):
        """sr_route_pack_result: (sorted records, packets, fill after, n_valid, probed-dead shard ids),
        copied out of the slot."""
        r = SrPackResult()
        _check(self._lib.sr_route_pack_result(self._h, slot, ctypes.byref(r)), "sr_route_pack_result")
        n = self.n_downstreams
        take = lambda addr, count, dt: (np.frombuffer((ctypes.c_uint8 * (count * dt.itemsize)).from_address(addr),
                                                      dtype=dt).copy() if count else np.zeros(0, dt))
        srt = take(r.sorted, r.n_records, RECORD_DTYPE)
        pk = take(r.packets, r.n_packets, PACKET_DTYPE)
        fill = take(r.fill, n, np.dtype(np.uint16))
        pw = take(r.probed_dead, max((n + 63) // 64, 1), np.dtype(np.uint64))
        getattr(self, "_pending", {}).pop(slot, None)
        return srt, pk, fill, int(r.n_valid), bitmap_shards(pw, n)

    def pack_packets(self, d_recs: int, d_n_records: int, max_records: int, d_fill_in: int | None,
                     d_probed_dead: int | None, d_sorted: int, d_packets: int, max_pk: int, d_counts: int,
                     d_fill_out: int) -> None:
        """sr_pack_packets with raw device pointers (asynchronous on the context's stream)."""
        vp = ctypes.c_void_p
        _check(self._lib.sr_pack_packets(self._h, vp(d_recs), vp(d_n_records), max_records, vp(d_fill_in or 0),
                                         vp(d_probed_dead or 0), vp(d_sorted), vp(d_packets), max_pk, vp(d_counts),
                                         vp(d_fill_out)), "sr_pack_packets")

    @staticmethod
    def owner_batches(batches):
        """The sr_batch array of [(d_bytes, nbytes, d_recs, max_records, d_n_records), ...] (reusable)."""
        arr = (SrBatch * max(len(batches), 1))()
        for i, (db, nb, dr, mr, dn) in enumerate(batches):
            arr[i] = SrBatch(db, nb, dr, mr, None, dn, None)
        return arr

    _owner_batches = owner_batches

    def pack_many_by_owner(self, batches, n_owners: int, d_out_bytes: int, out_cap: int, d_out_recs: int,
                           d_owner_counts: int) -> None:
        """sr_pack_many_by_owner: batches = [(d_bytes, nbytes, d_recs, max_records, d_n_records), ...]."""
        vp = ctypes.c_void_p
        _check(self._lib.sr_pack_many_by_owner(self._h, self._owner_batches(batches), len(batches), n_owners,
                                               vp(d_out_bytes), out_cap, vp(d_out_recs), vp(d_owner_counts)),
               "sr_pack_many_by_owner")

    def pack_owner_sizes(self, batches, n_owners: int, d_owner_counts: int) -> None:
        """sr_pack_owner_sizes: the split sizes of sr_pack_many_by_owner alone (batches as there)."""
        _check(self._lib.sr_pack_owner_sizes(self._h, self._owner_batches(batches), len(batches), n_owners,
                                             ctypes.c_void_p(d_owner_counts)), "sr_pack_owner_sizes")

    def pack_owner_scatter(self, batches, n_owners: int, own: int, d_own_bytes: int, d_own_recs: int,
                           d_out_bytes: int, out_cap: int, d_out_recs: int) -> None:
        """sr_pack_owner_scatter: the rest of the pack after pack_owner_sizes, owner `own`'s chunk written to
        d_own_bytes / d_own_recs (e.g. its place in the exchange's receive buffers)."""
        vp = ctypes.c_void_p
        _check(self._lib.sr_pack_owner_scatter(self._h, self._owner_batches(batches), len(batches), n_owners, own,
                                               vp(d_own_bytes), vp(d_own_recs), vp(d_out_bytes), out_cap,
                                               vp(d_out_recs)), "sr_pack_owner_scatter")

    def pack_packets_many(self, batches) -> None:
        """sr_pack_packets_many: batches = [(d_recs, d_n_records, max_records, d_fill_in, d_probed_dead,
        d_sorted, d_packets, max_packets, d_counts, d_fill_out), ...] (raw device pointers, 0 = NULL)."""
        arr = (SrPackBatch * max(len(batches), 1))()
        for i, b in enumerate(batches):
            arr[i] = SrPackBatch(*[x or None if j not in (2, 7) else x for j, x in enumerate(b)])
        _check(self._lib.sr_pack_packets_many(self._h, arr, len(batches)), "sr_pack_packets_many")

    def route_pack_many(self, batches) -> None:
        """sr_route_pack_many: batches = [(d_bytes, nbytes, d_out, max_records, d_hashes, d_n_records,
        d_probed_dead, d_fill_in, d_sorted, d_packets, max_packets, d_counts, d_fill_out), ...]: each routed
        into d_out, then packed from it (raw device pointers, 0 = NULL)."""
        n = max(len(batches), 1)
        ra, pa = (SrBatch * n)(), (SrPackBatch * n)()
        for i, b in enumerate(batches):
            db, nb, do, mr, dh, dc, dp, fi, ds, dpk, mp, dcnt, fo = b
            ra[i] = SrBatch(db, nb, do, mr, dh or None, dc, dp or None)
            pa[i] = SrPackBatch(do, dc, mr, fi or None, dp or None, ds, dpk, mp, dcnt, fo)
        _check(self._lib.sr_route_pack_many(self._h, ra, pa, len(batches)), "sr_route_pack_many")

    def exchange_sizes(self, comm: "Comm", d_owner_counts: int, d_recv_counts: int):
        """sr_exchange_sizes: returns (sent, received) as u64 [world, 2] {lines, bytes} arrays."""
        sent = np.zeros((comm.world, 2), dtype=np.uint64)
        received = np.zeros((comm.world, 2), dtype=np.uint64)
        vp = ctypes.c_void_p
        _check(self._lib.sr_exchange_sizes(self._h, comm.handle, vp(d_owner_counts), vp(d_recv_counts),
                                           sent.ctypes.data, received.ctypes.data), "sr_exchange_sizes")
        return sent, received

    def regroup_launch(self, comm: "Comm", batches, d_owner_counts: int, d_recv_counts: int, d_packed: int,
                       packed_cap: int, d_packed_recs: int, d_recv_bytes: int, recv_bytes_cap: int, d_recv_recs: int,
                       recv_recs_cap: int):
        """sr_regroup_launch (batches as pack_many_by_owner's, or an array from owner_batches()): returns
        (fits, sent, received); fits False = -ENOSPC: the sizes are exchanged, nothing scattered or sent yet
        (finish with pack_owner_scatter and exchange_data into buffers of the received totals)."""
        sent = np.zeros((comm.world, 2), dtype=np.uint64)
        received = np.zeros((comm.world, 2), dtype=np.uint64)
        arr = batches if isinstance(batches, ctypes.Array) else self._owner_batches(batches)
        n = len(batches)
        vp = ctypes.c_void_p
        rc = self._lib.sr_regroup_launch(self._h, comm.handle, arr, n, vp(d_owner_counts), vp(d_recv_counts),
                                         vp(d_packed), packed_cap, vp(d_packed_recs), vp(d_recv_bytes),
                                         recv_bytes_cap, vp(d_recv_recs), recv_recs_cap, sent.ctypes.data,
                                         received.ctypes.data)
        if rc == -errno.ENOSPC:
            return False, sent, received
        _check(rc, "sr_regroup_launch")
        return True, sent, received

    def regroup_run(self, transport: "Transport", world: int, rank: int, batches, d_owner_counts: int,
                    d_recv_counts: int, d_packed: int, packed_cap: int, d_packed_recs: int, d_recv_bytes: int,
                    recv_bytes_cap: int, d_recv_recs: int, recv_recs_cap: int):
        """sr_regroup_run: regroup_launch's sequence on a Python transport whose sizes(d_owner_counts,
        d_recv_counts) does the size exchange (returns (sent, received) [world, 2] and writes d_recv_counts).
        Returns (fits, sent, received) as regroup_launch."""
        sent = np.zeros((world, 2), dtype=np.uint64)
        received = np.zeros((world, 2), dtype=np.uint64)
        err = []
        cb = _transport_struct(transport, err)

        def sizes(_u, d_cnt, d_rcv, h_s, h_r):
            try:
                s_, r_ = transport.sizes(int(d_cnt or 0), int(d_rcv or 0))
                hs = np.frombuffer((ctypes.c_uint8 * (16 * world)).from_address(h_s), dtype=np.uint64)
                hr = np.frombuffer((ctypes.c_uint8 * (16 * world)).from_address(h_r), dtype=np.uint64)
                hs[:] = np.asarray(s_, dtype=np.uint64).reshape(-1)
                hr[:] = np.asarray(r_, dtype=np.uint64).reshape(-1)
                return 0
            except Exception as e:   # noqa: BLE001 - reported after the C call returns
                err.append(e)
                return -errno.EIO

        sizes_fn = _SIZES_FN(sizes)
        arr = batches if isinstance(batches, ctypes.Array) else self._owner_batches(batches)
        vp = ctypes.c_void_p
        rc = self._lib.sr_regroup_run(self._h, ctypes.byref(cb), sizes_fn, world, rank, arr, len(batches),
                                      vp(d_owner_counts), vp(d_recv_counts), vp(d_packed), packed_cap,
                                      vp(d_packed_recs), vp(d_recv_bytes), recv_bytes_cap, vp(d_recv_recs),
                                      recv_recs_cap, sent.ctypes.data, received.ctypes.data)
        if err:
            raise err[0]
        if rc == -errno.ENOSPC:
            return False, sent, received
        _check(rc, "sr_regroup_run")
        return True, sent, received

    def exchange_data(self, comm: "Comm", d_packed: int, d_packed_recs: int, sent: np.ndarray,
                      received: np.ndarray, d_recv_bytes: int, d_recv_recs: int) -> None:
        """sr_exchange_data (asynchronous on the router's stream)."""
        sent = np.ascontiguousarray(sent, dtype=np.uint64)
        received = np.ascontiguousarray(received, dtype=np.uint64)
        vp = ctypes.c_void_p
        _check(self._lib.sr_exchange_data(self._h, comm.handle, vp(d_packed), vp(d_packed_recs), sent.ctypes.data,
                                          received.ctypes.data, vp(d_recv_bytes), vp(d_recv_recs)),
               "sr_exchange_data")

    def exchange_rebase(self, d_recv_recs: int, peers: np.ndarray) -> None:
        """sr_exchange_rebase: the exchange's record rebase alone (asynchronous on the router's stream)."""
        p = np.ascontiguousarray(peers, dtype=PEER_DTYPE)
        _check(self._lib.sr_exchange_rebase(self._h, ctypes.c_void_p(d_recv_recs), p.ctypes.data, int(p.size)),
               "sr_exchange_rebase")

    def sync(self) -> None:
        _check(self._lib.sr_sync(self._h), "sr_sync")


class Comm:
    """An RCCL communicator of the C ABI (sr_comm_open): `world` ranks, one GPU each."""

    def __init__(self, comm_id: bytes, world: int, rank: int, device: int):
        self._lib = lib()
        if len(comm_id) != SR_COMM_ID_BYTES:
            raise ValueError("communicator id must be SR_COMM_ID_BYTES bytes")
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(comm_id), SR_COMM_ID_BYTES)
        _check(self._lib.sr_comm_open(ctypes.byref(h), buf, world, rank, device), "sr_comm_open")
        self.handle, self.world, self.rank, self.device = h, world, rank, device

    @staticmethod
    def new_id() -> bytes:
        buf = ctypes.create_string_buffer(SR_COMM_ID_BYTES)
        _check(lib().sr_comm_id(buf), "sr_comm_id")
        return buf.raw

    @classmethod
    def from_group(cls, device: int, group=None) -> "Comm":
        """Every rank of a torch.distributed group joins one communicator (rank 0 makes the id)."""
        import torch.distributed as dist
        box = [None]
        if dist.get_rank(group) == 0:   # a failure here still reaches every rank (no rank left waiting)
            try:
                box[0] = cls.new_id()
            except (OSError, RuntimeError) as e:
                box[0] = f"{type(e).__name__}: {e}"
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        if isinstance(box[0], str):
            raise RuntimeError(f"rank 0 could not make the communicator id: {box[0]}")
        return cls(box[0], dist.get_world_size(group), dist.get_rank(group), device)

    def close(self) -> None:
        if self.handle:
            self._lib.sr_comm_close(self.handle)
            self.handle = ctypes.c_void_p()


def exchange_plan(world: int, rank: int, sent, received):
    """sr_exchange_plan (host only): returns (peers: PEER_DTYPE [world], totals: u64 [4] = {lines sent,
    bytes sent, lines received, bytes received})."""
    s = np.ascontiguousarray(sent, dtype=np.uint64).reshape(-1)
    r = np.ascontiguousarray(received, dtype=np.uint64).reshape(-1)
    if s.size != 2 * world or r.size != 2 * world:
        raise ValueError("split sizes must be [world, 2]")
    peers = np.zeros(max(world, 1), dtype=PEER_DTYPE)
    tot = np.zeros(4, dtype=np.uint64)
    _check(lib().sr_exchange_plan(world, rank, s.ctypes.data, r.ctypes.data, peers.ctypes.data, tot.ctypes.data),
           "sr_exchange_plan")
    return peers, tot


class Transport:
    """A transport for sr_exchange_run written in Python (override the methods; raise to fail).
    Addresses are plain integers; what they address (host or device memory) is the transport's business."""

    def group_start(self) -> None:
        pass

    def group_end(self) -> None:
        pass

    def send(self, addr: int, nbytes: int, peer: int, tag: int) -> None:
        raise NotImplementedError

    def recv(self, addr: int, nbytes: int, peer: int, tag: int) -> None:
        raise NotImplementedError

    def copy(self, dst: int, src: int, nbytes: int) -> None:
        ctypes.memmove(dst, src, nbytes)

    def sizes(self, d_owner_counts: int, d_recv_counts: int):
        """sr_regroup_run's size exchange: returns (sent, received) u64 [world, 2] and writes the received
        sizes to d_recv_counts."""
        raise NotImplementedError

    def rebase(self, recs_addr: int, peers: np.ndarray, n_lines: int) -> None:
        """Host memory: records [recv_line0, +recv_lines) of every source move by its recv_byte0."""
        recs = host_records(recs_addr, n_lines)
        for p in peers:
            a, n = int(p["recv_line0"]), int(p["recv_lines"])
            recs["offset"][a: a + n] += np.uint32(p["recv_byte0"])


def host_records(addr: int, n: int) -> np.ndarray:
    """A writable RECORD_DTYPE view of n records at a host address."""
    if n == 0:
        return np.zeros(0, dtype=RECORD_DTYPE)
    return np.frombuffer((ctypes.c_uint8 * (8 * n)).from_address(addr), dtype=RECORD_DTYPE)


def _transport_struct(transport: Transport, err: list) -> SrTransport:
    """An SrTransport whose callbacks call the Python transport; exceptions go to err (the callback
    returns -EIO). Keep the returned structure alive for the duration of the C call."""
    def wrap(fn):
        def call(*a):
            try:
                fn(*a)
                return 0
            except Exception as e:   # noqa: BLE001 - reported after the C call returns
                err.append(e)
                return -errno.EIO
        return call

    def rebase(_u, recs, peers_p, w, n):
        arr = np.ctypeslib.as_array(ctypes.cast(peers_p, ctypes.POINTER(ctypes.c_uint64)), shape=(w * 8,))
        transport.rebase(recs, arr.copy().view(PEER_DTYPE), int(n))

    return SrTransport(None,
                       _GROUP_FN(wrap(lambda _u: transport.group_start())),
                       _GROUP_FN(wrap(lambda _u: transport.group_end())),
                       _SEND_FN(wrap(lambda _u, b, n, p, t: transport.send(b, n, p, t))),
                       _SEND_FN(wrap(lambda _u, b, n, p, t: transport.recv(b, n, p, t))),
                       _COPY_FN(wrap(lambda _u, d, s, n: transport.copy(d, s, n))),
                       _REBASE_FN(wrap(rebase)))


def exchange_run(transport: Transport, world: int, rank: int, sent, received, packed: int, packed_recs: int,
                 recv_bytes: int, recv_recs: int) -> None:
    """sr_exchange_run: the C exchange plan and its calls, on a Python transport."""
    err = []
    cb = _transport_struct(transport, err)
    s = np.ascontiguousarray(sent, dtype=np.uint64).reshape(-1)
    r = np.ascontiguousarray(received, dtype=np.uint64).reshape(-1)
    if s.size != 2 * world or r.size != 2 * world:
        raise ValueError("split sizes must be [world, 2]")
    vp = ctypes.c_void_p
    rc = lib().sr_exchange_run(ctypes.byref(cb), world, rank, s.ctypes.data, r.ctypes.data, vp(packed),
                               vp(packed_recs), vp(recv_bytes), vp(recv_recs))
    if err:
        raise err[0]
    _check(rc, "sr_exchange_run")


def version() -> str:
    return lib().sr_version().decode()
