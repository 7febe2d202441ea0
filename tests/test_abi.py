"""The C-ABI library loads and exports exactly what include/*.h declares; host-only entry points
(framing, generator) behave. CPU only: no GPU compute is called here."""
from __future__ import annotations

import ctypes
import glob
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO


def declared_functions(header="sr_route.h"):
    names = set()
    src = open(os.path.join(REPO, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    for m in re.finditer(r"^(?!\s*static)[A-Za-z_][\w \t\*]*?\b(sr_\w+)\s*\(", src, flags=re.M):
        names.add(m.group(1))
    return names


def test_headers_are_the_two_libraries():
    assert sorted(os.path.basename(h) for h in glob.glob(os.path.join(REPO, "include", "*.h"))) == \
        ["sr_route.h", "sr_router.h"]


def test_header_declares_the_python_abi_list(pkg):
    assert declared_functions() == set(pkg.ABI_FUNCTIONS)


def _exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_library_exports_every_declared_symbol(pkg):
    lib = ctypes.CDLL(pkg.ROUTE_LIB)
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert declared_functions() <= _exported(pkg.ROUTE_LIB)


def test_router_library_exports_sr_router_h(pkg):
    """libsr_router.so (host/sr_core.c) exports exactly the functions include/sr_router.h declares."""
    import importlib

    core = importlib.import_module("statsd-router_amd.core")
    core.router_lib()
    declared = declared_functions("sr_router.h")
    assert declared and declared == {n for n in _exported(core.ROUTER_LIB) if n.startswith("sr_")}


def test_header_constants_match_python(pkg):
    src = open(pkg.HEADER).read()

    def val(name):
        m = re.search(r"#define\s+%s\s+\(?([0-9xA-Fa-f]+)u?" % name, src)
        return int(m.group(1), 0)

    assert val("SR_DATA_BUF_SIZE") == pkg.SR_DATA_BUF_SIZE
    assert val("SR_DOWNSTREAM_BUF_SIZE") == pkg.SR_DOWNSTREAM_BUF_SIZE
    assert val("SR_MIN_LINE_LENGTH") == pkg.SR_MIN_LINE_LENGTH
    assert val("SR_MAX_DOWNSTREAMS") == pkg.SR_MAX_DOWNSTREAMS
    assert val("SR_ROUTE_INVALID_LENGTH") == pkg.SR_ROUTE_INVALID_LENGTH
    assert val("SR_ROUTE_INVALID_FORMAT") == pkg.SR_ROUTE_INVALID_FORMAT
    assert val("SR_ROUTE_ALL_DEAD") == pkg.SR_ROUTE_ALL_DEAD


def test_record_layout(pkg):
    assert pkg.RECORD_DTYPE.itemsize == 8
    assert [pkg.RECORD_DTYPE.fields[f][1] for f in ("offset", "length", "route")] == [0, 4, 6]
    v = pkg.verdicts(np.array([0, 7, 0xFFFC, 0xFFFD, 0xFFFE, 0xFFFF], dtype=np.uint16))
    assert v.tolist() == [0, 0, 0, 1, 2, 3]


def test_version_string(pkg):
    assert "gfx950" in pkg.version()


@pytest.mark.parametrize("seed", range(5))
def test_frame_datagrams_matches_oracle(pkg, oracle, seed):
    rng = np.random.default_rng(seed)
    dgrams = []
    for _ in range(50):
        n = int(rng.choice([0, 1, 5, 100, 4094, 4095, 4096, 5000]))
        d = bytes(rng.integers(0, 256, n, dtype=np.uint8))
        if rng.random() < 0.5 and n:
            d = d[:-1] + b"\n"
        dgrams.append(d)
    assert pkg.frame_datagrams(dgrams) == b"".join(oracle.frame(d) for d in dgrams)


def test_generator_is_deterministic_and_framed(pkg, oracle):
    a = pkg.gen_stream(1 << 20, [64], seed=7)
    b = pkg.gen_stream(1 << 20, [64], seed=7)
    c = pkg.gen_stream(1 << 20, [64], seed=8)
    assert np.array_equal(a.data, b.data) and not np.array_equal(a.data, c.data)
    assert a.data.size == 1 << 20 and a.n_lines == (1 << 20) // 64
    assert int(a.dgram_lens.sum()) == a.data.size and int(a.dgram_lens.max()) <= 4095
    # every datagram already framed: framing is the identity
    offs = np.concatenate([[0], np.cumsum(a.dgram_lens.astype(np.int64))])
    raw = a.data.tobytes()
    for i in range(0, len(a.dgram_lens), 37):
        d = raw[offs[i]:offs[i + 1]]
        assert oracle.frame(d) == d
    m = pkg.gen_stream(1 << 20, [64, 256, 1024], seed=9, p_invalid=0.1)
    recs, _, n = oracle.route(m.data, 4)
    lens = set(recs["length"].tolist())
    assert lens == {64, 256, 1024} and n == m.n_lines
    frac_bad = float((pkg.verdicts(recs["route"]) == 2).mean())
    assert 0.07 < frac_bad < 0.13


def test_product_library_has_only_the_product_route_kernels(pkg):
    """Ablation variants (some write wrong records by design) never ship: the product library holds
    exactly the three lane layouts, KV_UNIFORM (0), KV_SEGMENTS (4194304) and KV_CHUNKS (8388608,
    route_chunk_kernel), each also as KV_ALIVE (+268435456: launches with every shard alive), the
    first two also as KV_PICKS (+536870912: probes that end after their first picks), and the dead-shard
    specialisations KV_DEFER1 (+2147483648: one pick, then the deferral) and KV_DEAD1 (+134217728:
    exactly one dead shard; with KV_HIST1, +1048576, for route + pack launches), which write identical
    records (tests/test_gpu_layout.py, tests/test_gpu_bench_shape.py); ablations live in tools/ and
    `make VARIANTS=1` builds only."""
    out = subprocess.run(["nm", "-C", pkg.ROUTE_LIB], capture_output=True, text=True).stdout
    kernels = {l.split(" ", 2)[-1] for l in out.splitlines()
               if ("route_kernel<" in l or "route_chunk_kernel<" in l) and "__device_stub__" not in l}
    assert kernels == {"void srk::route_kernel<256, 0u>(srk::RouteParams)",
                       "void srk::route_kernel<256, 4194304u>(srk::RouteParams)",
                       "void srk::route_kernel<256, 268435456u>(srk::RouteParams)",     # KV_ALIVE
                       "void srk::route_kernel<256, 272629760u>(srk::RouteParams)",     # KV_SEGMENTS | KV_ALIVE
                       "void srk::route_kernel<256, 536870912u>(srk::RouteParams)",     # KV_PICKS
                       "void srk::route_kernel<256, 541065216u>(srk::RouteParams)",     # KV_SEGMENTS | KV_PICKS
                       "void srk::route_kernel<256, 2684354560u>(srk::RouteParams)",    # KV_PICKS | KV_DEFER1
                       "void srk::route_kernel<256, 2688548864u>(srk::RouteParams)",    # KV_SEGMENTS | KV_PICKS | KV_DEFER1
                       "void srk::route_kernel<256, 671088640u>(srk::RouteParams)",     # KV_PICKS | KV_DEAD1
                       "void srk::route_kernel<256, 675282944u>(srk::RouteParams)",     # KV_SEGMENTS | KV_PICKS | KV_DEAD1
                       "void srk::route_kernel<256, 672137216u>(srk::RouteParams)",     # ... | KV_HIST1
                       "void srk::route_kernel<256, 676331520u>(srk::RouteParams)",     # KV_SEGMENTS ... | KV_HIST1
                       "void srk::route_chunk_kernel<8388608u>(srk::RouteParams)",
                       "void srk::route_chunk_kernel<276824064u>(srk::RouteParams)",    # | KV_ALIVE
                       "void srk::route_chunk_kernel<2155872256u>(srk::RouteParams)",   # | KV_DEFER1
                       "void srk::route_chunk_kernel<142606336u>(srk::RouteParams)"}, kernels   # | KV_DEAD1
    assert b"SR_VARIANT" not in open(pkg.ROUTE_LIB, "rb").read()
