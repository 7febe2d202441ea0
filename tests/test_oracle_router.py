"""CPU: the pure-Python data-thread restatement (oracle/sr_router_oracle.py) reproduces every
packet, log line (WARN, and TRACE at log_level 0) and final buffer the compiled reference produced for the scripted sessions in
tests/golden/router_*.json (push_to_downstream / flush / dead drop / flush timer / ping)."""
from __future__ import annotations

import pytest

from conftest import load_router_fixture, router_fixtures


@pytest.mark.parametrize("name", router_fixtures())
def test_router_oracle_matches_reference(name):
    import sr_router_oracle as RO

    f = load_router_fixture(name)
    t = RO.DataThread(f["n"], f["ds_hosts"], f["ds_data_ports"], f["ping_prefix"], f["hostname"], f["data_port"],
                      log_level=f["log_level"])
    t.run(f["events"])
    assert t.logs == f["logs"]
    assert {k: v for k, v in t.packets.items() if v} == f["packets"]
    assert t.final() == f["final"]


def test_probed_dead_fixtures_match_oracle(oracle):
    import json
    import os

    from conftest import GOLDEN, load_case

    want = json.load(open(os.path.join(GOLDEN, "probed_dead.json")))
    for name, probed in want.items():
        c = load_case(name)
        n = c["n"]
        alive = [int((int(c["alive"][k >> 6]) >> (k & 63)) & 1) for k in range(n)]
        framed = b"".join(oracle.frame(d) for d in c["dgrams"])
        got = oracle.probed_dead(framed, n, alive).tolist() if n else []
        assert got == probed, name
