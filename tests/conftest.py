"""Shared fixtures. `-m "not gpu"` runs on the CPU build container; `-m gpu` on an MI355X."""
from __future__ import annotations

import glob
import importlib
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session")
def pkg():
    m = importlib.import_module("statsd-router_amd")
    _force_layout(m)
    return m


def _force_layout(m):
    """SR_TEST_LAYOUT=<n> (test runs only): every context the tests open starts in lane layout n
    (sr_set_layout), e.g. the parity, MTU and router-core suites all in the chunk layout (3). The
    library itself reads no environment variable."""
    lay = os.environ.get("SR_TEST_LAYOUT")
    if not lay or getattr(m.Router, "_layout_forced", False):
        return
    layout = int(lay)
    r_init = m.Router.__init__

    def router_init(self, *a, **k):
        r_init(self, *a, **k)
        self.set_layout(layout)

    m.Router.__init__ = router_init
    m.Router._layout_forced = True
    core = importlib.import_module("statsd-router_amd.core")
    c_init = core.Core.__init__

    def core_init(self, *a, **k):
        c_init(self, *a, **k)
        self.set_layout(layout)

    core.Core.__init__ = core_init


@pytest.fixture(scope="session")
def oracle():
    import sr_oracle

    return sr_oracle


def golden_cases():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def load_case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))  # allow_pickle=False (default)
    raw = z["dgram_bytes"].tobytes()
    lens = z["dgram_lens"].astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)]).tolist()
    dgrams = [raw[offs[i]:offs[i + 1]] for i in range(len(lens))]
    return {
        "dgrams": dgrams,
        "alive": z["alive"],
        "n": int(z["n_downstreams"][0]),
        "records": z["records"],
        "hashes": z["hashes"],
    }


def load_digests():
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)


@pytest.fixture
def torch_stream():
    """A fresh torch stream made current for the test: the router is set to it, so torch's copies
    and fills, the HIP kernels and the collectives are ordered on one stream. (Router.set_stream(0)
    means the context's own non-blocking stream, not torch's default stream.)"""
    import torch

    prev = torch.cuda.current_stream()
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    try:
        yield s
    finally:
        torch.cuda.synchronize()
        torch.cuda.set_stream(prev)


def router_fixtures():
    return sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN, "router_*.json")))


def load_router_fixture(name):
    """A scripted data-thread session and what the compiled reference did with it
    (tests/golden/make_router_golden.py)."""
    import base64

    with open(os.path.join(GOLDEN, name + ".json")) as f:
        d = json.load(f)
    dec = base64.b64decode
    events = []
    for e in d["events"]:
        if e[0] == "dgram":
            events.append(("dgram", dec(e[1])))
        elif e[0] == "alive":
            events.append(("alive", e[1]))
        else:
            events.append((e[0],))
    return {
        "n": d["n_downstreams"], "ds_hosts": d["ds_hosts"], "ds_data_ports": d["ds_data_ports"],
        "ping_prefix": d["ping_prefix"], "hostname": d["hostname"], "data_port": d["data_port"],
        "log_level": d.get("log_level", 3),
        "events": events,
        "packets": {int(k): [dec(p) for p in v] for k, v in d["packets"].items()},
        "logs": [(lv, dec(t)) for lv, t in d["logs"]],
        "final": {int(k): (dec(v[0]), v[1], v[2]) for k, v in d["final"].items()},
    }
