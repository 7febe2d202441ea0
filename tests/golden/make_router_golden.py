#!/usr/bin/env python3
"""Fixtures for the router-level side effects, produced by the REFERENCE compiled from
/root/reference (oracle/Makefile `ref`; run in the build container only):

  probed_dead.json   per golden case (tests/golden/*.npz): the dead downstreams whose pending
                     buffer the reference drops while routing the case (sr-main.c:106), read from
                     oracle/_ref/sr_ref_harness's 5th output;
  router_*.json      scripted data-thread sessions (datagrams, alive snapshots, flush and ping
                     ticks) run through oracle/_ref/sr_ref_router: every packet each downstream
                     received (flush ring drained by the reference's ds_flush_cb), every log line at or
                     above the session's log_level (3: WARN and ERROR; 0: also the TRACE lines of
                     sr-main.c:91,102,174), the final pending buffers and counters. Inputs are stored
                     with the outputs.

Writes only what the oracle's restatement also reproduces (checked here) for probed_dead.
"""
from __future__ import annotations

import base64
import glob
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import sr_oracle as O  # noqa: E402
from conftest import load_case  # noqa: E402


def bits(words, n):
    return [int((int(words[k >> 6]) >> (k & 63)) & 1) for k in range(n)]


def probed_fixtures():
    out = {}
    for p in sorted(glob.glob(os.path.join(HERE, "*.npz"))):
        name = os.path.basename(p)[:-4]
        c = load_case(name)
        n = c["n"]
        alive = bits(c["alive"], n)
        _, probed = O.run_reference(c["dgrams"], n, alive, probed=True)
        framed = b"".join(O.frame(d) for d in c["dgrams"])
        mine = O.probed_dead(framed, n, alive) if n else np.zeros(0, dtype=np.int64)
        assert mine.tolist() == probed.tolist(), (name, mine, probed)
        out[name] = probed.tolist()
    with open(os.path.join(HERE, "probed_dead.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(f"probed_dead.json: {len(out)} cases")


CONFIG = """# router fixture config (sr-init.c keys)
data_port={port}
control_port=9001
downstream_flush_interval=2.0
downstream_health_check_interval=2.0
downstream_ping_interval=10.0
ping_prefix={prefix}
downstream={downstreams}
log_level={log_level}
threads_num=1
"""


def session(seed: int, n: int, steps: int, max_lines: int = 120, nul: bool = False):
    r = random.Random(seed)
    events = [("alive", [1] * n)]
    names = [f"svc{r.randrange(40)}.req.{r.choice(['a', 'bb', 'ccc'])}{r.randrange(999)}" for _ in range(300)]
    for _ in range(steps):
        k = r.random()
        if k < 0.65:
            lines = []
            for _ in range(r.randrange(1, max_lines)):
                q = r.random()
                if q < 0.85:
                    lines.append(f"{r.choice(names)}:{r.randrange(1000)}|{r.choice('cgm')}".encode() + b"x" * r.choice([0, 0, 40, 300]))
                    if nul and r.random() < 0.05:   # printf's %.*s stops at a NUL (sr-main.c:91,174)
                        k = r.randrange(len(lines[-1]) + 1)
                        lines[-1] = lines[-1][:k] + b"\0" + lines[-1][k:]
                elif q < 0.91:
                    lines.append(b"nocolon" + b"Z" * r.randrange(0, 60))
                elif q < 0.95:
                    lines.append(b"ab" if r.random() < 0.8 else b"L" * 1500 + b":1|c")
                else:
                    lines.append(b"")
            d = b"\n".join(lines)
            if r.random() < 0.5:
                d += b"\n"
            events.append(("dgram", d[: r.choice([4095, 4095, 5000])]))
        elif k < 0.80:
            events.append(("alive", [int(r.random() > 0.35) for _ in range(n)]))
        elif k < 0.90:
            events.append(("flush",))
        else:
            events.append(("ping",))
    return events


def router_fixtures():
    specs = [
        # seed, downstreams, steps, ping prefix, data port, log_level, lines per datagram below, NULs
        (1, 3, 160, "statsd-cluster-test", 9000, 3, 120, False),
        (2, 1, 100, "sr", 8125, 3, 120, False),
        (3, 7, 200, "statsd-cluster-test", 9000, 3, 120, False),
        (4, 16, 160, "pfx.x", 9300, 3, 120, False),
        # log_level 0, the reference's default (sr-init.c:252): TRACE lines too
        (5, 5, 90, "statsd-cluster-test", 9000, 0, 30, True),
    ]
    for seed, n, steps, prefix, port, level, max_lines, nul in specs:
        downstreams = ",".join(f"127.0.0.{1 + (i % 9)}:{9100 + 2 * i}:{9101 + 2 * i}" for i in range(n))
        cfg = CONFIG.format(port=port, prefix=prefix, downstreams=downstreams, log_level=level)
        events = session(seed, n, steps, max_lines, nul)
        res = O.run_reference_router(cfg, events, n)
        enc = lambda b: base64.b64encode(b).decode()  # noqa: E731
        doc = {
            "config": cfg, "n_downstreams": n, "hostname": O.REF_TEST_HOSTNAME,
            "ds_hosts": [f"127.0.0.{1 + (i % 9)}" for i in range(n)],
            "ds_data_ports": [str(9100 + 2 * i) for i in range(n)],
            "ping_prefix": prefix, "data_port": port, "log_level": level,
            "events": [[e[0], enc(e[1])] if e[0] == "dgram" else ([e[0], e[1]] if e[0] == "alive" else [e[0]])
                       for e in events],
            "packets": {str(k): [enc(p) for p in v] for k, v in res["packets"].items()},
            "logs": [[lv, enc(t)] for lv, t in res["logs"]],
            "final": {str(k): [enc(v[0]), v[1], v[2]] for k, v in res["final"].items()},
        }
        name = f"router_s{seed}_n{n}.json" if level == 3 else f"router_s{seed}_n{n}_level{level}.json"
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(doc, f)
        npk = sum(len(v) for v in res["packets"].values())
        print(f"{name}: {len(events)} events, {npk} packets, {len(res['logs'])} log lines")


if __name__ == "__main__":
    if not (O.have_reference() and O.have_reference_router()):
        sys.exit("build the reference harnesses first: make -C oracle ref")
    probed_fixtures()
    router_fixtures()
