"""GPU: statsd-router-mi355x end to end over loopback, the reference test suite's way
(statsd-router-test-lib.rb): real UDP datagrams in, mock downstreams (tools/loopback/sr_sink: UDP data
+ TCP health) out, WARN lines checked on the router's stdout.

Checks, for the reference test catalogue's line shapes (test/003-019):
  - every line a downstream receives is one the oracle routes to that downstream (all alive);
  - per downstream, the multiset of received data lines equals what the reference's data thread
    (oracle/sr_router_oracle.py, pinned to the compiled reference) pushes there;
  - the WARN lines are exactly the reference's texts, in order;
  - and, when the reference executable was built (oracle/_ref/statsd-router), it receives the same
    per-downstream multisets when run the same way.
"""
from __future__ import annotations

import os
import random
import socket
import subprocess
import time
from collections import Counter

import pytest

from router_proc import OURS, REFERENCE, REPO, Router, config_text, free_ports

pytestmark = pytest.mark.gpu

SINK = os.path.join(REPO, "tools", "loopback", "sr_sink")
PREFIX = "statsd-e2e"


def valid_metric(r: random.Random, n: int) -> bytes:   # statsd-router-test-lib.rb:232-250
    num = str(r.randrange(100))
    name = "statsd-cluster.count" + "X" * max(0, n - 20 - len(num)) + num
    return f"{name}:{r.randrange(1000)}|c".encode()


def invalid_metric(r: random.Random, n: int) -> bytes:  # :253-267 (n-1 letters, the '\n' is added on send)
    return bytes(r.choice(b"ABCDEFGHIJKLMNOPQRSTUVWXYZ") for _ in range(n - 1))


def catalogue(seed=11):
    r = random.Random(seed)
    dg = []
    for n in (64, 256, 1024):
        for _ in range(30):
            dg.append(valid_metric(r, n) + b"\n")                  # 003-005 (006 sends valid 64 too)
    for n in (256, 1024, 32):
        for _ in range(10):
            dg.append(invalid_metric(r, n) + b"\n")                # 007, 008
    for n in (32, 256, 1024):
        for _ in range(10):
            dg.append(invalid_metric(r, n) + b"\n" + valid_metric(r, n) + b"\n")   # 009-014
            dg.append(valid_metric(r, n) + b"\n" + invalid_metric(r, n) + b"\n")
    dg.append(b"\n".join(invalid_metric(r, 128) for _ in range(10)) + b"\n")      # 017
    dg.append(b"\n".join(valid_metric(r, 128) for _ in range(10)) + b"\n")        # 018
    dg.append(invalid_metric(r, 4) + b"\n")                                        # 019
    dg.append(invalid_metric(r, 1600) + b"\n")
    for _ in range(200):                                                           # bulk, several packets
        dg.append(b"\n".join(valid_metric(r, r.choice((64, 100, 200))) for _ in range(12)) + b"\n")
    return dg


def run_router(exe, datagrams, n_ds, tmp, threads=1, log_level=1, messages=False):
    base = free_ports(4 + 2 * n_ds)
    data_port, ctl, sink_base = base, base + 1, base + 4
    ds = [(sink_base + 2 * i, sink_base + 2 * i + 1) for i in range(n_ds)]
    dump = os.path.join(tmp, f"dump-{os.path.basename(exe)}.bin")
    sink = subprocess.Popen([SINK, str(sink_base), str(n_ds), "60", "3.0", dump], stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE)
    assert sink.stderr.readline().strip() == b"ready"
    r = Router(exe, config_text(data_port, ctl, ds, log_level=log_level, threads=threads, flush=0.1, health=0.1,
                                ping=1000.0, prefix=PREFIX), tmp)
    try:
        for i in range(n_ds):
            assert r.wait_for(lambda lv, m, i=i: m == b"ds_health_read_cb downstream %d is up" % i, 20), r.raw[-20:]
        time.sleep(0.3)   # every data thread has seen the alive bits
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        for d in datagrams:
            s.sendto(d, ("127.0.0.1", data_port))
            time.sleep(0.0005)
        s.close()
        out, _ = sink.communicate(timeout=90)
    finally:
        r.stop()
        if sink.poll() is None:
            sink.kill()
    got = {i: Counter() for i in range(n_ds)}
    with open(dump, "rb") as f:
        blob = f.read()
    i = 0
    while i < len(blob):
        d, l = int.from_bytes(blob[i:i + 2], "little"), int.from_bytes(blob[i + 2:i + 4], "little")
        pkt = blob[i + 4:i + 4 + l]
        i += 4 + l
        assert len(pkt) <= 1450 and pkt.endswith(b"\n")
        for line in pkt.split(b"\n")[:-1]:
            if not line.startswith(PREFIX.encode()):
                got[d][line + b"\n"] += 1
    data_path = (b"udp_read_cb:", b"process_data_line:", b"find_downstream:")
    if messages:   # every data-path message (TRACE included), whole
        return got, [(lv, m) for lv, m in r.messages() if m.startswith(data_path)]
    warns = [m for lv, m in r.lines if lv == "WARN" and m.startswith(data_path)]
    return got, warns


def expected(datagrams, n_ds):
    import sr_router_oracle as RO

    t = RO.DataThread(n_ds, ["127.0.0.1"] * n_ds, [str(9000 + i) for i in range(n_ds)], PREFIX, "h", 1)
    t.set_alive([1] * n_ds)
    for d in datagrams:
        t.datagram(d)
    t.flush_timer()
    want = {i: Counter() for i in range(n_ds)}
    for s, pkts in t.packets.items():
        for p in pkts:
            for line in p.split(b"\n")[:-1]:
                want[s][line + b"\n"] += 1
    # the router's log is read line by line: an invalid-length line's own '\n' ends the message
    return want, [m[:-1] if m.endswith(b"\n") else m for lv, m in t.logs if lv == 3]


@pytest.mark.parametrize("n_ds", [1, 3])
def test_router_end_to_end_loopback(tmp_path, n_ds, oracle):
    dg = catalogue()
    want, want_warns = expected(dg, n_ds)
    got, warns = run_router(OURS, dg, n_ds, str(tmp_path))
    assert warns == want_warns
    for k in range(n_ds):
        for line in got[k]:
            h = oracle.hash_line(line)
            assert oracle.find_downstream(h, n_ds) == k
    assert got == want


@pytest.mark.skipif(not os.path.exists(REFERENCE), reason="reference executable not built (make -C oracle ref)")
def test_router_matches_reference_executable(tmp_path):
    dg = catalogue(seed=12)
    ours, w1 = run_router(OURS, dg, 3, str(tmp_path))
    ref, w2 = run_router(REFERENCE, dg, 3, str(tmp_path))
    assert ours == ref
    assert w1 == w2


def test_timers_run_while_the_socket_never_drains(tmp_path):
    """Two blasters saturate the data port for 3 s: the read event hands back to the loop after a few
    batches (sr_router_main.c), so the ping timer (0.3 s) still fires and its self-metrics reach the
    downstream among the data packets, as the reference's one-datagram reads let its timers run."""
    blast = os.path.join(REPO, "tools", "loopback", "sr_blast")
    base = free_ports(6)
    data_port, ctl, sink_base = base, base + 1, base + 2
    dump = os.path.join(str(tmp_path), "dump-saturated.bin")
    sink = subprocess.Popen([SINK, str(sink_base), "1", "12", "1.5", dump], stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE)
    assert sink.stderr.readline().strip() == b"ready"
    r = Router(OURS, config_text(data_port, ctl, [(sink_base, sink_base + 1)], log_level=1, flush=1.0, health=0.2,
                                 ping=0.3, prefix=PREFIX), str(tmp_path))
    try:
        assert r.wait_for(lambda lv, m: m == b"ds_health_read_cb downstream 0 is up", 20), r.raw[-20:]
        time.sleep(0.5)
        bl = [subprocess.Popen([blast, str(data_port), "3", "0", "1400", str(40 + k)], stdout=subprocess.PIPE)
              for k in range(2)]
        for b in bl:
            b.communicate(timeout=60)
        sink.communicate(timeout=60)
    finally:
        r.stop()
        if sink.poll() is None:
            sink.kill()
    with open(dump, "rb") as f:
        blob = f.read()
    seq, i = [], 0   # per datagram: (data lines, healthy_downstreams gauge lines)
    while i < len(blob):
        l = int.from_bytes(blob[i + 2:i + 4], "little")
        lines = blob[i + 4:i + 4 + l].split(b"\n")[:-1]
        i += 4 + l
        seq.append((sum(not x.startswith(PREFIX.encode()) for x in lines),
                    sum(x.startswith(PREFIX.encode()) and b"healthy_downstreams" in x for x in lines)))
    data_idx = [k for k, (d, _) in enumerate(seq) if d]
    assert len(data_idx) > 1000, "the blast never reached the downstream"
    first, last = data_idx[0], data_idx[-1]
    during = sum(g for d, g in seq[first:last + 1])
    assert during >= 4, f"only {during} ping gauges among {last - first + 1} datagrams of a 3 s blast (ping 0.3 s)"


@pytest.mark.skipif(not os.path.exists(REFERENCE), reason="reference executable not built (make -C oracle ref)")
def test_trace_log_matches_reference_executable(tmp_path):
    """log_level=0 (the reference's default, sr-init.c:252): the executable prints the reference's
    TRACE lines (sr-main.c:91,102,174) between its WARN lines, message for message and in order, as
    the reference executable does for the same datagrams; the packets are unchanged."""
    dg = catalogue(seed=13)[:260]
    ours, m1 = run_router(OURS, dg, 3, str(tmp_path), log_level=0, messages=True)
    ref, m2 = run_router(REFERENCE, dg, 3, str(tmp_path), log_level=0, messages=True)
    assert ours == ref
    assert sum(lv == "TRACE" for lv, _ in m2) > 2 * len(dg)
    assert m1 == m2
