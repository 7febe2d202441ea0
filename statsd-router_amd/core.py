"""ctypes view of one router data thread (include/sr_router.h, lib/libsr_router.so).

The product is the C library (host/sr_core.c over libsr_route.so); this module lets tests and the
bench drive it with Python callbacks. Loading is strict, like the package's.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import LIB_DIR, SrError, _check, alive_words, lib

ROUTER_LIB = os.path.join(LIB_DIR, "libsr_router.so")
SR_TRACE, SR_DEBUG, SR_INFO, SR_WARN, SR_ERROR = range(5)


class IoVec(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("len", ctypes.c_size_t)]


class CoreConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("max_batch_bytes", ctypes.c_size_t), ("n_downstreams", ctypes.c_uint32),
                ("ds_hosts", ctypes.POINTER(ctypes.c_char_p)), ("ds_data_ports", ctypes.POINTER(ctypes.c_char_p)),
                ("ping_prefix", ctypes.c_char_p), ("hostname", ctypes.c_char_p), ("data_port", ctypes.c_int),
                ("log_level", ctypes.c_int)]


EMIT_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(IoVec), ctypes.c_int, ctypes.c_size_t)
LOG_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t)
FLUSH_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p)

_RLIB = None


def router_lib() -> ctypes.CDLL:
    global _RLIB
    if _RLIB is None:
        lib()   # libsr_route.so first (one HIP runtime per process)
        if not os.path.exists(ROUTER_LIB):
            raise ImportError(f"{ROUTER_LIB} is missing: build it with __graft_entry__.build()")
        L = ctypes.CDLL(ROUTER_LIB)
        vp = ctypes.c_void_p
        L.sr_core_open.restype = ctypes.c_int
        L.sr_core_open.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(CoreConfig), EMIT_FN, LOG_FN, FLUSH_FN, vp]
        L.sr_core_set_alive.restype, L.sr_core_set_alive.argtypes = ctypes.c_int, [vp, vp]
        L.sr_core_batch_buffer.restype = vp
        L.sr_core_batch_buffer.argtypes = [vp, ctypes.POINTER(ctypes.c_size_t)]
        L.sr_core_route.restype, L.sr_core_route.argtypes = ctypes.c_int, [vp, vp, ctypes.c_size_t]
        L.sr_core_slot_buffer.restype = vp
        L.sr_core_slot_buffer.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]
        L.sr_core_submit.restype, L.sr_core_submit.argtypes = ctypes.c_int, [vp, ctypes.c_int, ctypes.c_size_t]
        L.sr_core_drain.restype, L.sr_core_drain.argtypes = ctypes.c_int, [vp]
        L.sr_core_in_flight.restype, L.sr_core_in_flight.argtypes = ctypes.c_int, [vp]
        L.sr_core_flush_timer.restype, L.sr_core_flush_timer.argtypes = ctypes.c_int, [vp]
        L.sr_core_ping.restype, L.sr_core_ping.argtypes = ctypes.c_int, [vp]
        L.sr_core_state.restype = ctypes.c_int
        L.sr_core_state.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t),
                                    ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
        L.sr_core_metric_name.restype = ctypes.c_char_p
        L.sr_core_metric_name.argtypes = [vp, ctypes.c_uint32, ctypes.c_int]
        L.sr_core_close.restype, L.sr_core_close.argtypes = None, [vp]
        L.sr_core_route_datagrams.restype = ctypes.c_int
        L.sr_core_route_datagrams.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t]
        L.sr_core_submit_datagrams.restype = ctypes.c_int
        L.sr_core_submit_datagrams.argtypes = [vp, ctypes.c_int, ctypes.c_size_t, vp, ctypes.c_size_t]
        L.sr_core_context.restype, L.sr_core_context.argtypes = vp, [vp]
        L.sr_core_inject_faults.restype = ctypes.c_int
        L.sr_core_inject_faults.argtypes = [vp, ctypes.c_uint, ctypes.c_uint]
        _RLIB = L
    return _RLIB


class Core:
    """One data thread: packets and log lines are collected in Python lists
    (packets[ds] = [bytes, ...]; logs = [(level, text bytes), ...])."""

    def __init__(self, n_downstreams: int, ds_hosts, ds_data_ports, ping_prefix: str, hostname: str,
                 data_port: int, max_batch_bytes: int = 1 << 20, device: int = 0, log_level: int = SR_WARN):
        self._L = router_lib()
        self.n = n_downstreams
        self.packets: dict[int, list[bytes]] = {}
        self.logs: list[tuple[int, bytes]] = []
        self.flushes = 0
        hosts = (ctypes.c_char_p * n_downstreams)(*[h.encode() for h in ds_hosts])
        ports = (ctypes.c_char_p * n_downstreams)(*[p.encode() for p in ds_data_ports])
        self._keep = (hosts, ports, ping_prefix.encode(), hostname.encode())
        cfg = CoreConfig(device, max_batch_bytes, n_downstreams, hosts, ports, self._keep[2], self._keep[3],
                         data_port, log_level)

        def emit(_u, ds, iov, cnt, nbytes):
            b = b"".join(ctypes.string_at(iov[i].base, iov[i].len) for i in range(cnt))
            assert len(b) == nbytes
            self.packets.setdefault(int(ds), []).append(b)

        def log(_u, level, msg, n):
            self.logs.append((int(level), ctypes.string_at(msg, n)))

        def flush(_u):
            self.flushes += 1

        self._cb = (EMIT_FN(emit), LOG_FN(log), FLUSH_FN(flush))
        h = ctypes.c_void_p()
        _check(self._L.sr_core_open(ctypes.byref(h), ctypes.byref(cfg), *self._cb, None), "sr_core_open")
        self._h = h

    def close(self):
        if self._h:
            self._L.sr_core_close(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_alive(self, alive) -> None:
        w = np.ascontiguousarray(alive_words(self.n, alive))
        _check(self._L.sr_core_set_alive(self._h, w.ctypes.data), "sr_core_set_alive")

    @staticmethod
    def _ends(ends):
        """Datagram end offsets as a u32 array (None: no boundaries)."""
        if ends is None:
            return None, 0
        a = np.ascontiguousarray(np.asarray(ends, dtype=np.uint32))
        return a, int(a.size)

    def route(self, framed: bytes, ends=None) -> None:
        """sr_core_route (ends: the framed datagrams' end offsets, for TRACE: sr_core_route_datagrams)."""
        buf = ctypes.create_string_buffer(bytes(framed), max(len(framed), 1))
        a, n = self._ends(ends)
        _check(self._L.sr_core_route_datagrams(self._h, buf, len(framed), a.ctypes.data if n else None, n),
               "sr_core_route")

    def route_in_place(self, framed: bytes, ends=None) -> None:
        """Frame into the core's page-locked batch buffer first (what a C caller does)."""
        cap = ctypes.c_size_t()
        p = self._L.sr_core_batch_buffer(self._h, ctypes.byref(cap))
        if len(framed) > cap.value:
            raise SrError(28, "batch larger than the core's buffer")
        ctypes.memmove(p, bytes(framed), len(framed))
        a, n = self._ends(ends)
        _check(self._L.sr_core_route_datagrams(self._h, p, len(framed), a.ctypes.data if n else None, n),
               "sr_core_route")

    def submit(self, framed: bytes, ends=None) -> None:
        """Double-buffered: frame into the next slot's buffer and sr_core_submit it (the previous
        batch completes here, the new one stays in flight until the next submit or drain)."""
        slot = getattr(self, "_slot", 0)
        cap = ctypes.c_size_t()
        p = self._L.sr_core_slot_buffer(self._h, slot, ctypes.byref(cap))
        if len(framed) > cap.value:
            raise SrError(28, "batch larger than the core's buffer")
        ctypes.memmove(p, bytes(framed), len(framed))
        a, n = self._ends(ends)
        rc = self._L.sr_core_submit_datagrams(self._h, slot, len(framed), a.ctypes.data if n else None, n)
        if self._L.sr_core_in_flight(self._h) == slot:
            self._slot = slot ^ 1   # taken, even when completing the previous batch failed
        _check(rc, "sr_core_submit")

    def inject_faults(self, fail_submit: int = 0, fail_finish: int = 0) -> None:
        """sr_core_inject_faults (test hook)."""
        _check(self._L.sr_core_inject_faults(self._h, fail_submit, fail_finish), "sr_core_inject_faults")

    def set_layout(self, layout: int) -> None:
        """sr_set_layout on the core's device context (sr_core_context)."""
        _check(lib().sr_set_layout(self._L.sr_core_context(self._h), int(layout)), "sr_set_layout")

    def in_flight(self) -> int:
        """sr_core_in_flight: the slot whose batch is on the GPU, or -1."""
        return self._L.sr_core_in_flight(self._h)

    def drain(self) -> None:
        _check(self._L.sr_core_drain(self._h), "sr_core_drain")

    def flush_timer(self) -> None:
        _check(self._L.sr_core_flush_timer(self._h), "sr_core_flush_timer")

    def ping(self) -> None:
        _check(self._L.sr_core_ping(self._h), "sr_core_ping")

    def state(self, ds: int):
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        tr, pk = ctypes.c_int32(), ctypes.c_int32()
        _check(self._L.sr_core_state(self._h, ds, ctypes.byref(p), ctypes.byref(n), ctypes.byref(tr),
                                     ctypes.byref(pk)), "sr_core_state")
        return ctypes.string_at(p.value, n.value) if n.value else b"", tr.value, pk.value

    def metric_name(self, ds: int, which: int) -> bytes:
        return self._L.sr_core_metric_name(self._h, ds, which)
