"""Pins taken from the reference's own black-box test library
(/root/reference/test/statsd-router-test-lib.rb), restated here as data + a few lines of Python.
CPU only.

The Ruby `hashring` (statsd-router-test-lib.rb:213-229) hashes unsigned bytes and never wraps
`(hash*7+5)/3` to 64 bits, so it only agrees with the C router (sr-main.c:98-113) on the FIRST
choice, and for ASCII names. The tests below use it exactly where it is a valid oracle:
  * all downstreams alive  -> shard == hashring(name)[0]
  * one downstream alive   -> shard == that downstream
"""
from __future__ import annotations

import random

DOWNSTREAM_NUM = 3                # statsd-router-test-lib.rb:7
MIN_METRICS_LENGTH = 6            # :40
MAX_METRICS_LENGTH = 1450         # :41


def ruby_hashring(name: bytes, n: int = DOWNSTREAM_NUM):
    """statsd-router-test-lib.rb:213-229, restated (bignum semantics kept)."""
    h = 0
    for b in name:
        h = ((h << 6) + (h << 16) - h + b) & 0xFFFFFFFFFFFFFFFF
    a = list(range(n))
    for i in reversed(range(n)):
        j = h % (i + 1)
        k = a[j]
        if j != i:
            a[j] = a[i]
            a[i] = k
        h = (h * 7 + 5) // 3
    return list(reversed(a))


def valid_metric_name(rng: random.Random, length: int) -> bytes:
    """statsd-router-test-lib.rb:232-240."""
    name = b"statsd-cluster.count"
    number = str(rng.randrange(100)).encode()
    if len(name) + len(number) < length:
        name += b"X" * (length - len(name) - len(number)) + number
    return name


def test_first_choice_matches_test_library(oracle):
    rng = random.Random(3)
    for length in (32, 64, 128, 256, 1024):
        for _ in range(200):
            name = valid_metric_name(rng, length)
            h = oracle.hash_line(name + b":1|c\n")
            assert oracle.find_downstream(h, DOWNSTREAM_NUM) == ruby_hashring(name)[0]


def test_single_alive_downstream_gets_everything(oracle):
    rng = random.Random(4)
    for alive_k in range(DOWNSTREAM_NUM):
        alive = [int(k == alive_k) for k in range(DOWNSTREAM_NUM)]
        for _ in range(100):
            name = valid_metric_name(rng, 64)
            h = oracle.hash_line(name + b":1|c\n")
            assert oracle.find_downstream(h, DOWNSTREAM_NUM, alive) == alive_k


def test_length_bounds_match_test_library(oracle):
    """MIN/MAX_METRICS_LENGTH (:40-41) and invalid_metric (:253-267): a line of L bytes (incl. '\\n')
    is length-valid iff MIN <= L < MAX; test/019 sends invalid_metric(4) and (1600)."""
    for L in (1, 4, 5, 6, 7, 1448, 1449, 1450, 1600):
        line = b"A" * (L - 1) + b"\n"
        recs, _, n = oracle.route(line, 3)
        assert n == 1
        expect_len_ok = MIN_METRICS_LENGTH <= L < MAX_METRICS_LENGTH
        route = int(recs["route"][0])
        assert (route != 0xFFFD) == expect_len_ok, L
        if expect_len_ok:
            assert route == 0xFFFE   # no ':' -> "invalid metric"
