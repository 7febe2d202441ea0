"""The CPU oracle against the reference's own outputs (tests/golden, made by make_golden.py from
the compiled reference). CPU only."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import golden_cases, load_case, load_digests


def _bitmap_bits(words, n):
    return [int((int(words[k >> 6]) >> (k & 63)) & 1) for k in range(n)]


@pytest.mark.parametrize("name", golden_cases())
def test_oracle_reproduces_reference_fixture(oracle, name):
    c = load_case(name)
    framed = b"".join(oracle.frame(d) for d in c["dgrams"])
    recs, hs, n = oracle.route(framed, c["n"], _bitmap_bits(c["alive"], c["n"]))
    assert n == len(c["records"])
    assert np.array_equal(recs, c["records"])
    assert np.array_equal(hs, c["hashes"])


def test_oracle_full_config_digests(oracle, pkg):
    """Full-size BASELINE configs: regenerate the inputs and compare SHA-256 of the oracle's
    record/hash arrays with the reference's (digests.json)."""
    for key, d in sorted(load_digests().items()):
        s = pkg.gen_stream(d["nbytes"], d["line_lens"], seed=d["seed"], p_invalid=d["p_invalid"])
        assert s.data.size == d["n_bytes_generated"], key
        words = np.array([int(x, 16) for x in d["alive"]], dtype=np.uint64)
        recs, hs, n = oracle.route(s.data, d["n_downstreams"], _bitmap_bits(words, d["n_downstreams"]))
        assert n == d["n_lines"], key
        assert hashlib.sha256(recs.tobytes()).hexdigest() == d["sha256_records"], key
        assert hashlib.sha256(hs.tobytes()).hexdigest() == d["sha256_hashes"], key


def test_survey_known_answers(oracle):
    """hashes verified against the reference binary."""
    assert oracle.hash_line(b"foo.bar:1|c\n") == 0xC6AADFE5F2B2ED2B
    assert oracle.hash_line(b"x:1|c\n") == 0x78
    assert oracle.hash_line(b"\xc3\xa9n:1|c\n") == 0xFFFFFFC2E19F3948  # signed char
    assert oracle.hash_line(b":12|c\n") == 0
    assert oracle.hash_line(b"nocolon\n") is None


def test_oracle_framing(oracle):
    assert oracle.frame(b"") == b""
    assert oracle.frame(b"a") == b"a\n"
    assert oracle.frame(b"a\n") == b"a\n"
    assert oracle.frame(b"x" * 5000) == b"x" * 4095 + b"\n"
    assert oracle.frame(b"x" * 4094 + b"\n") == b"x" * 4094 + b"\n"
    assert oracle.frame(b"x" * 4095 + b"\n") == b"x" * 4095 + b"\n"   # '\n' cut off, re-appended
