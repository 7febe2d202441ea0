"""CPU: the host surface of statsd-router-mi355x (config file, logger, control port, downstream
health checks; host/sr_config.c, host/sr_health.c) behaves like the reference executable compiled
from /root/reference (oracle/_ref/statsd-router): same exit codes and log messages for bad configs,
same control-port replies (test/020-health-check-test.rb), same up/down health events
(statsd-router-test-lib.rb:389-411). No GPU is touched: on a CPU box the data threads fail to open
their GPU context and say so; the main thread's services run regardless."""
from __future__ import annotations

import os
import time

import pytest

from router_proc import OURS, REFERENCE, HealthServer, Router, config_text, control, free_ports, wait_control

BOTH = [OURS] + ([REFERENCE] if os.path.exists(REFERENCE) else [])
# on a CPU box our data threads cannot open a GPU context: keep the main thread's services running
NO_GPU = {"SR_REQUIRE_GPU": "0"}


def _msgs(r):
    return [(lv, m) for lv, m in r.lines]


def test_usage():
    import subprocess

    for exe in BOTH:
        p = subprocess.run([exe], capture_output=True, timeout=10)
        assert p.returncode == 1
        assert p.stdout == b"Usage: %s config.file\n" % exe.encode()


BAD = {
    "empty_line": "data_port=9000\n\ncontrol_port=9001\n",
    "unknown_key": "data_port=9000\nfoo=1\n",
    "no_equals": "data_port\n",
    "threads_zero": "threads_num=0\n",
    "missing_everything": "# nothing but a comment\n",
    "bad_log_level": ("data_port=9000\ncontrol_port=9001\ndownstream_flush_interval=1\n"
                      "downstream_health_check_interval=1\ndownstream_ping_interval=1\nping_prefix=p\n"
                      "downstream=127.0.0.1:9100:9101\nlog_level=9\n"),
    "no_data_port_in_downstream": ("data_port=9000\ncontrol_port=9001\ndownstream_flush_interval=1\n"
                                   "downstream_health_check_interval=1\ndownstream_ping_interval=1\nping_prefix=p\n"
                                   "downstream=127.0.0.1\nlog_level=0\n"),
    "no_health_port": ("data_port=9000\ncontrol_port=9001\ndownstream_flush_interval=1\n"
                       "downstream_health_check_interval=1\ndownstream_ping_interval=1\nping_prefix=p\n"
                       "downstream=127.0.0.1:9100\nlog_level=0\n"),
    "zero_intervals": ("data_port=9000\ncontrol_port=9001\ndownstream_flush_interval=0\n"
                       "downstream_health_check_interval=-1\ndownstream_ping_interval=0\nping_prefix=p\n"
                       "downstream=127.0.0.1:9100:9101\n"),
}


@pytest.mark.skipif(not os.path.exists(REFERENCE), reason="reference executable not built (make -C oracle ref)")
@pytest.mark.parametrize("name", sorted(BAD))
def test_bad_config_same_as_reference(tmp_path, name):
    out = {}
    for exe in (OURS, REFERENCE):
        r = Router(exe, BAD[name], str(tmp_path), env=NO_GPU)
        rc = r.wait_exit(10)
        out[exe] = (rc, _msgs(r))
    assert out[OURS] == out[REFERENCE]
    assert out[OURS][0] == 1


def test_bad_config_messages(tmp_path):
    r = Router(OURS, BAD["empty_line"], str(tmp_path), env=NO_GPU)
    assert r.wait_exit(10) == 1
    assert ("ERROR", b'process_config_line: bad line in config ""') in r.lines
    assert ("ERROR", b"init_config: failed to load config file") in r.lines
    assert ("ERROR", b"main: init_config() failed") in r.lines


@pytest.mark.parametrize("exe", BOTH)
def test_control_port_health_replies(tmp_path, exe):
    """test/020: health -> "health: up"; "health down" sets a sticky reply; unknown -> nothing."""
    base = free_ports(4)
    r = Router(exe, config_text(base, base + 1, [(base + 2, base + 3)], log_level=3), str(tmp_path), env=NO_GPU)
    try:
        assert wait_control(base + 1)
        assert control(base + 1, b"health\n") == b"health: up\n"
        assert control(base + 1, b"health down\n") == b"health: down\n"
        assert control(base + 1, b"health\n") == b"health: down\n"
        assert control(base + 1, b"health up") == b"health: up\n"
        assert control(base + 1, b"health  \n") == b"health: up\n"
        assert control(base + 1, b"status\n") == b""
        assert r.wait_for(lambda lv, m: m == b"control_write_cb: nothing to send", 5)
    finally:
        r.stop()


@pytest.mark.parametrize("exe", BOTH)
def test_downstream_health_toggles(tmp_path, exe):
    """statsd-router-test-lib.rb:389-411: the router logs DEBUG up/down events as the mocks' health
    servers start and stop."""
    base = free_ports(8)
    ds = [(base + 2 + 2 * i, base + 3 + 2 * i) for i in range(3)]
    hs = [HealthServer(h) for _, h in ds]
    r = Router(exe, config_text(base, base + 1, ds, log_level=1, health=0.1), str(tmp_path), env=NO_GPU)
    try:
        for i in (0, 2):
            hs[i].start()
            assert r.wait_for(lambda lv, m, i=i: (lv, m) == ("DEBUG", b"ds_health_read_cb downstream %d is up" % i), 10)
        hs[0].stop()
        assert r.wait_for(lambda lv, m: (lv, m) == ("DEBUG", b"ds_mark_down downstream 0 is down"), 10)
        hs[1].start()
        assert r.wait_for(lambda lv, m: (lv, m) == ("DEBUG", b"ds_health_read_cb downstream 1 is up"), 10)
        ups = [m for lv, m in r.lines if lv == "DEBUG" and m.endswith(b"is up")]
        assert ups.count(b"ds_health_read_cb downstream 2 is up") == 1   # logged on the transition only
    finally:
        r.stop()
        for h in hs:
            h.stop()


@pytest.mark.parametrize("exe", BOTH)
def test_sighup_sigint(tmp_path, exe):
    """sr-init.c:177-185,290-297: SIGHUP is logged at INFO and the router keeps serving; SIGINT is logged
    and the process exits with status 0. Same lines from both executables."""
    import signal

    base = free_ports(4)
    r = Router(exe, config_text(base, base + 1, [(base + 2, base + 3)], log_level=2), str(tmp_path), env=NO_GPU)
    try:
        assert wait_control(base + 1)
        # (both signals before any control request: the reference logs from its signal handler, which is
        # not safe while its main loop is itself logging, e.g. a control connection's lines)
        r.p.send_signal(signal.SIGHUP)
        assert r.wait_for(lambda lv, m: (lv, m) == ("INFO", b"on_sighup: sighup received"), 5)
        assert r.p.poll() is None
        r.p.send_signal(signal.SIGHUP)
        end = time.monotonic() + 5   # the second line (the log is read by a thread of the test)
        while sum(m == b"on_sighup: sighup received" for _, m in r.lines) < 2 and time.monotonic() < end:
            time.sleep(0.05)
        assert sum(m == b"on_sighup: sighup received" for _, m in r.lines) == 2
        assert r.p.poll() is None
        assert control(base + 1, b"health\n") == b"health: up\n"   # still serving
        time.sleep(0.2)   # its control lines written before the next signal
        r.p.send_signal(signal.SIGINT)
        assert r.wait_exit(10) == 0
        assert ("INFO", b"on_sigint: sigint received") in r.lines
    finally:
        r.stop()


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="needs a box without a GPU")
def test_data_thread_without_gpu_ends_the_process(tmp_path):
    """A data thread that cannot open its GPU context must not leave its SO_REUSEPORT share of the
    data port unread while the control port answers "health: up": the process exits with status 1."""
    base = free_ports(4)
    r = Router(OURS, config_text(base, base + 1, [(base + 2, base + 3)], log_level=3), str(tmp_path))
    try:
        assert r.wait_exit(30) == 1
        assert any(lv == "ERROR" and m.startswith(b"data_pipe_thread: sr_core_open() failed") for lv, m in r.lines)
    finally:
        r.stop()
