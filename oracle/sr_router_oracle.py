"""ORACLE — TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of one reference data thread (hulu/statsd-router v0.0.16), line by line
and in the reference's order, for small scripted sessions:
  udp_read_cb        sr-main.c:149-191   framing, line split, length gate, WARN texts, TRACE "got packet"
  process_data_line  sr-main.c:137-147   ':' verdict (hash via sr_oracle.hash_line, sr-main.c:120-134)
  find_downstream    sr-main.c:86-117    probe, with the drop of every probed dead buffer (:106), TRACE
                                         hash / pick lines (:91,102)
  log_msg            sr-util.c:18-20     messages below the configured log_level are dropped
  push_to_downstream sr-main.c:73-83     1450-byte active buffer, flush when the line does not fit
  ds_schedule_flush  sr-main.c:49-71     packet and traffic counters (the ring never fills here:
                                         it is drained after every event, like the harness does)
  ds_flush_timer_cb  sr-main.c:194-204
  ping_cb            sr-main.c:206-235   names as built by sr-init.c:57,90-118
Pinned by tests/test_oracle_router.py against tests/golden/router_*.json, which the compiled
reference produced (tests/golden/make_router_golden.py, oracle/ref_router_harness.c).
"""
from __future__ import annotations

import sr_oracle as O

CAP = 1450            # DOWNSTREAM_BUF_SIZE, sr-types.h:30
METRIC_SIZE = 256     # sr-types.h:32


def _int32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def _cstr(b: bytes) -> bytes:
    """What printf's %s / %.*s prints of b: up to its first NUL."""
    return b.split(b"\0", 1)[0]


class DataThread:
    def __init__(self, n, ds_hosts, ds_data_ports, ping_prefix, hostname, data_port, log_level=3):
        self.n = n
        self.log_level = log_level
        self.alive = [0] * n                      # health clients start dead (sr-init.c:85)
        self.pending = [b""] * n
        self.traffic = [0] * n
        self.npackets = [0] * n
        self.packets: dict[int, list[bytes]] = {}
        self.logs: list[tuple[int, bytes]] = []
        self.alive_metric = f"{ping_prefix}.{hostname}-{data_port}.healthy_downstreams".encode()
        mh = bytearray(METRIC_SIZE)              # sr-init.c:90-96: shared, never terminated
        self.conn, self.traffic_name, self.packet_name = [], [], []
        for i in range(n):
            h = ds_hosts[i].encode()
            mh[: len(h)] = h.replace(b".", b"_")
            name = bytes(mh).split(b"\0", 1)[0]
            port = ds_data_ports[i].encode()
            p = ping_prefix.encode()
            self.conn.append(b"%s.%s-%d-%s-%s.connections:1|c\n%s.%s-%s.connections:1|c\n"
                             % (p, hostname.encode(), data_port, name, port, p, name, port))
            self.traffic_name.append(b"%s.%s-%s.traffic" % (p, name, port))
            self.packet_name.append(b"%s.%s-%s.packets" % (p, name, port))

    # ---- the reference functions ------------------------------------------------------------
    def _log(self, level: int, text: bytes):   # log_msg (sr-util.c:18-20)
        if level >= self.log_level:
            self.logs.append((level, text))

    def _warn(self, text: bytes):
        self._log(3, text)

    def _flush(self, s):                          # ds_schedule_flush
        self.npackets[s] += 1
        self.traffic[s] += len(self.pending[s])
        self.packets.setdefault(s, []).append(self.pending[s])
        self.pending[s] = b""

    def _push(self, s, line: bytes):              # push_to_downstream
        if len(self.pending[s]) + len(line) > CAP:
            self._flush(s)
        self.pending[s] += line

    def _find_downstream(self, h: int, line: bytes):
        self._log(0, b"find_downstream: hash = %x, length = %d, line = " % (h, len(line)) + _cstr(line))   # :91
        idx = list(range(self.n))
        for i in range(self.n, 0, -1):
            j = h % i
            k = idx[j]
            if self.alive[k]:
                self._log(0, b"find_downstream: pushing to downstream %d" % k)                        # :102
                self._push(k, line)
                return
            self.pending[k] = b""                  # :106
            if j != i - 1:
                idx[j], idx[i - 1] = idx[i - 1], k
            h = ((h * 7 + 5) & 0xFFFFFFFFFFFFFFFF) // 3
        self._warn(b"find_downstream: all downstreams are dead")

    def _process_data_line(self, line: bytes):
        h = O.hash_line(line)
        if h is None:
            self._warn(b"process_data_line: invalid metric " + _cstr(line[:-1]))
            return
        self._find_downstream(h, line)

    def datagram(self, d: bytes):                 # udp_read_cb
        buf = O.frame(d)
        if buf:
            self._log(0, b"udp_read_cb: got packet " + _cstr(buf))                                   # :174
        while buf:
            k = buf.index(b"\n") + 1
            line, buf = buf[:k], buf[k:]
            if 5 < len(line) < CAP:
                self._process_data_line(line)
            else:
                self._warn(b"udp_read_cb: invalid length %d of metric " % len(line) + _cstr(line))

    def set_alive(self, alive):
        self.alive = [int(a) for a in alive]

    def flush_timer(self):                        # ds_flush_timer_cb
        for s in range(self.n):
            if self.pending[s]:
                self._flush(s)

    def ping(self):                               # ping_cb
        count = 0
        for i in range(self.n):
            if self.alive[i]:
                self._push(i, self.conn[i])
                count += 1
            tr, pk = self.traffic[i], self.npackets[i]
            self.traffic[i] = self.npackets[i] = 0
            self._process_data_line(b"%s:%d|c\n%s:%d|c\n" % (self.traffic_name[i], _int32(tr), self.packet_name[i],
                                                             _int32(pk)))
        self._process_data_line(b"%s:%d|g\n" % (self.alive_metric, count))

    def run(self, events):
        for e in events:
            if e[0] == "dgram":
                self.datagram(e[1])
            elif e[0] == "alive":
                self.set_alive(e[1])
            elif e[0] == "flush":
                self.flush_timer()
            elif e[0] == "ping":
                self.ping()
        return self

    def final(self):
        return {s: (self.pending[s], _int32(self.traffic[s]), _int32(self.npackets[s])) for s in range(self.n)}
