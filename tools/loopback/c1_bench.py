#!/usr/bin/env python3
"""Config C1 (BASELINE.json configs[0]): a router over loopback, 1 downstream, 64-byte valid metrics
(test/003 shape), driven flat out by sr_blast; delivered lines/s counted by the mock downstream
sr_sink. Runs statsd-router-mi355x and, when built, the reference executable
(oracle/_ref/statsd-router) the same way, one after the other.

  python tools/loopback/c1_bench.py [--seconds 3] [--threads 1] [--rate 0] [--dgram 1400]

Prints one JSON line per router: offered (sent) and delivered datagrams / lines per second.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
from router_proc import OURS, REFERENCE, Router, config_text, free_ports  # noqa: E402

BLAST = os.path.join(HERE, "sr_blast")
SINK = os.path.join(HERE, "sr_sink")


def run(exe, seconds, threads, rate, dgram, tmp, env=None, nblast=1):
    base = free_ports(6)
    data_port, ctl, sink_base = base, base + 1, base + 2
    sink = subprocess.Popen([SINK, str(sink_base), "1", str(seconds + 30), "1.5"], stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE)
    assert sink.stderr.readline().strip() == b"ready"
    r = Router(exe, config_text(data_port, ctl, [(sink_base, sink_base + 1)], log_level=1, threads=threads,
                                flush=1.0, health=0.2, ping=1000.0), tmp, env=env)
    try:
        if not r.wait_for(lambda lv, m: m == b"ds_health_read_cb downstream 0 is up", 30):
            raise RuntimeError(f"{exe}: downstream never came up: {r.raw[-10:]}")
        time.sleep(0.5)
        blasters = [subprocess.Popen([BLAST, str(data_port), str(seconds), str(rate), str(dgram), str(17 + k)],
                                     stdout=subprocess.PIPE) for k in range(nblast)]
        outs = [json.loads(b.communicate(timeout=seconds + 30)[0]) for b in blasters]
        sent = {k: sum(o[k] for o in outs) for k in ("datagrams", "lines", "bytes")}
        sent["seconds"] = max(o["seconds"] for o in outs)
        out, _ = sink.communicate(timeout=seconds + 60)
        got = json.loads(out)
    finally:
        r.stop()
        if sink.poll() is None:
            sink.kill()
    span = max(got["last"] - got["first"], 1e-9)
    return {
        "router": os.path.basename(exe), "threads_num": threads, "blasters": nblast, "seconds": sent["seconds"],
        "offered_lines_per_s": round(sent["lines"] / sent["seconds"], 1),
        "offered_datagrams_per_s": round(sent["datagrams"] / sent["seconds"], 1),
        "delivered_lines": got["lines"], "delivered_lines_per_s": round(got["lines"] / span, 1),
        # lines delivered per second of sending (the socket buffer and the pending buffers hold only a few
        # datagrams past the blast; the sink's span also covers the last flush-timer tick)
        "delivered_lines_per_blast_s": round(got["lines"] / sent["seconds"], 1),
        "delivered_fraction": round(got["lines"] / max(sent["lines"], 1), 4),
        # the sink's first / last datagram against the first sender's start and the last sender's end
        # (one CLOCK_MONOTONIC): the span's head and the tail after the blast (flush-timer ticks)
        "sink_head_s": round(got["first_abs"] - min(o["start_abs"] for o in outs), 4) if "first_abs" in got else None,
        "sink_tail_s": round(got["last_abs"] - max(o["end_abs"] for o in outs), 4) if "last_abs" in got else None,
        "downstream_packets": got["datagrams"],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--rate", type=float, default=0.0)
    ap.add_argument("--dgram", type=int, default=1400)
    ap.add_argument("--only", choices=["ours", "reference"], default=None)
    ap.add_argument("--blasters", type=int, default=1, help="sender processes")
    ap.add_argument("--exe", action="append", default=[],
                    help="tag=path of another router executable to run the same way (A/B of builds)")
    ap.add_argument("--var", action="append", default=[],
                    help="tag:K=V,K=V - this build again with environment settings (A/B of data-thread modes)")
    a = ap.parse_args()
    import tempfile

    with tempfile.TemporaryDirectory() as tmp:
        exes = [("ours", OURS)] + ([("reference", REFERENCE)] if os.path.exists(REFERENCE) else [])
        exes = [(t, e, None) for t, e in exes] + [tuple(e.split("=", 1)) + (None,) for e in a.exe]
        for v in a.var:
            tag, kv = v.split(":", 1)
            env = dict(os.environ, **dict(x.split("=", 1) for x in kv.split(",") if x))
            exes.append((tag, OURS, env))
        extra = {e[0] for e in exes[2:]}
        for tag, exe, env in exes:
            if a.only and tag != a.only and tag not in extra:
                continue
            print(json.dumps(dict(run(exe, a.seconds, a.threads, a.rate, a.dgram, tmp, env=env, nblast=a.blasters),
                                  kind=tag)), flush=True)


if __name__ == "__main__":
    main()
