"""bench.py --gpus N without WORLD_SIZE re-launches itself as N ranks (torch.distributed.run,
127.0.0.1) before anything touches a GPU. CPU only: --dry-ranks makes each rank report its env."""
from __future__ import annotations

import json
import os
import subprocess
import sys

from conftest import REPO


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=240)


def test_gpus_n_spawns_n_ranks():
    p = _run(["--gpus", "3", "--dry-ranks"])
    assert p.returncode == 0, p.stderr[-2000:]
    ranks = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert sorted(int(r["RANK"]) for r in ranks) == [0, 1, 2]
    assert sorted(int(r["LOCAL_RANK"]) for r in ranks) == [0, 1, 2]
    assert {r["WORLD_SIZE"] for r in ranks} == {"3"} and {r["MASTER_ADDR"] for r in ranks} == {"127.0.0.1"}


def test_one_gpu_runs_in_process():
    p = _run(["--gpus", "1", "--dry-ranks"])
    assert p.returncode == 0
    ranks = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert ranks == [{"RANK": None, "LOCAL_RANK": None, "WORLD_SIZE": None, "MASTER_ADDR": None}]


def test_gpus_must_match_world_size():
    p = _run(["--gpus", "4", "--dry-ranks"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=2" in (p.stderr + p.stdout)
