#!/usr/bin/env python3
"""Device-resident throughput of the statsd-router hot path on MI355X.

The hot path: newline tokenise -> length / ':' validate -> sdbm name hash ->
consistent-hash shard pick, one sr_record per line (sr-main.c:86-191), over synthetic framed
datagrams already resident in HBM.

One STEP = one route_kernel launch over SR_MAX_BATCHES_PER_LAUNCH (32) distinct 16 MiB batches
(512 MiB of framed datagrams at C2 = BASELINE.json configs[1]: 64-byte valid metrics, 4 downstream
shards). Consecutive steps alternate over a rotating set of 64 distinct batches (1 GiB per GPU,
4x the 256 MiB Infinity Cache), each launch replayed from its captured HIP graph. The timed
region is exactly K steps bracketed by barrier + synchronize; warm-up is W steps and at least
--min-warmup-ms of back-to-back launches (the clocks settle). roofline.achieved is the timed
region's bytes over the timed region's GPU time (HIP events on the launch stream).

After timing, the timed configuration itself is checked: one more replay of launch 0, then batch
0's records are SHA-256 compared with tests/golden/digests.json (the compiled reference's output
for the same seed) and the launch's last batch is compared record for record with the C oracle.

  python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c4|c5]
  --gpus N > 1 without WORLD_SIZE: re-launches itself under torch.distributed.run (N ranks, one per
  GPU; each rank routes its own batches: weak scaling, no collective on the classify path) plus a
  classify + regroup leg over RCCL on C5-shaped batches.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import hashlib
import importlib
import json
import os
import platform
import socket
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (description, batch bytes, line lengths, p_invalid, shards, seed base, digest key)
    "c2": ("C2: 16 MiB batches of 64-byte valid metrics, 4 downstream shards", 16 << 20, [64], 0.0, 4, 0x5EED0002,
           "c2_64B_n4"),
    "c3": ("C3: 16 MiB batches of 256-byte metrics, 10% invalid lines, 4 shards", 16 << 20, [256], 0.10, 4,
           0x5EED0003, "c3_256B_10pct_invalid_n4"),
    "c4": ("C4: 16 MiB batches of 1024-byte metrics, 16 downstream shards", 16 << 20, [1024], 0.0, 16, 0x5EED0004,
           "c4_1024B_n16"),
    "c5": ("C5: 16 MiB batches of mixed 64/256/1024-byte metrics, 64 shards", 16 << 20, [64, 256, 1024], 0.0, 64,
           0x5EED0005, "c5_mixed_n64"),
    # not a BASELINE configuration: statsd-sized lines whose ends fall anywhere in a 64-byte chunk
    # (lane-layout A/B only; verified against the oracle, no reference digest)
    "u1": ("U1: 16 MiB batches of 40/70/100/130-byte metrics, 16 shards", 16 << 20, [40, 70, 100, 130], 0.0, 16,
           0x5EED0011, "u1_unaligned_n16"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200, help="timed launches (32 x 16 MiB batches each)")
    ap.add_argument("--warmup", type=int, default=20, help="untimed launches first")
    ap.add_argument("--min-warmup-ms", type=float, default=60.0,
                    help="keep warming up until this much time has passed (clocks settle)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batches", type=int, default=64, help="distinct batches in the rotating set")
    ap.add_argument("--per-launch", type=int, default=32, help="batches per route_kernel launch (one step)")
    ap.add_argument("--dead", type=float, default=0.0,
                    help="fraction of dead downstreams (0.25 uses the digest's alive mask)")
    ap.add_argument("--regroup", default="auto", choices=["auto", "on", "off"],
                    help="classify + all-to-all regroup leg (auto: on when more than one GPU)")
    ap.add_argument("--regroup-config", default="c5", choices=sorted(CONFIGS))
    ap.add_argument("--regroup-steps", type=int, default=8)
    ap.add_argument("--regroup-batches", type=int, default=32, help="batches per regroup step (one route launch)")
    ap.add_argument("--regroup-timeout", type=float, default=240.0,
                    help="seconds the regroup leg may take before every rank gives it up (the main line is still printed)")
    ap.add_argument("--exchange", default="c", choices=["c", "torch"],
                    help="regroup transport: the C ABI's RCCL exchange or torch.distributed")
    ap.add_argument("--regroup-copy-own", action="store_true",
                    help="developer A/B: pack the own chunk into the packed buffer and copy it (round-4 path)")
    ap.add_argument("--regroup-split-calls", action="store_true",
                    help="developer A/B: the regroup's calls one by one from Python instead of sr_regroup_launch")
    ap.add_argument("--regroup-slots", type=int, default=2, choices=[1, 2],
                    help="regroup steps alternating over this many contexts and streams (2: step i + 1's route "
                         "overlaps step i's scatter and exchange)")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-pack", action="store_true", help="skip the route + MTU packing leg")
    ap.add_argument("--pack-threads", type=int, default=1, choices=[1, 2],
                    help="2: also time two data threads' route + pack graphs running concurrently (their "
                         "route launches overlap: a rocprof mean over the run then mixes in stretched launches)")
    ap.add_argument("--layout", default="auto", choices=["auto", "uniform", "segments", "chunks"],
                    help="route kernel lane layout (sr_set_layout; records identical either way)")
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                    help="sr_set_knob on the bench's contexts (A/B runs): lb_spin, defer_picks, mtu_chunk, mtu_xcd, "
                         "mtu_walk (results never change)")
    ap.add_argument("--dry-ranks", action="store_true",
                    help="each rank prints its RANK / LOCAL_RANK / WORLD_SIZE and exits (launcher test; no GPU)")
    # the PMC counter bytes of the dominant kernel (tools/pmc_summary.py): at the top of the tree so
    # that it travels to the GPU box with the library it was measured on (profiles/ does not)
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "bench_traffic.json"))
    return ap.parse_args(argv)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(args_argv, n):
    """torch.distributed.run command line re-running this script with N ranks (one per GPU)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
            os.path.abspath(__file__)] + list(args_argv)


def maybe_spawn(args, argv) -> int | None:
    """--gpus N > 1 outside a torch.distributed launch: start the N ranks as child processes
    (before this process touches the GPU) and return their exit code. None = run here."""
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if args.gpus not in (1, world):
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
        return None
    if args.gpus <= 1:
        return None
    return subprocess.run(launcher_cmd(argv, args.gpus)).returncode


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    rc = maybe_spawn(args, argv)
    if rc is not None:
        sys.exit(rc)
    if args.dry_ranks:
        # one write(2) per rank: the ranks share the pipe, and a short write is atomic on it
        line = json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")})
        os.write(1, (line + "\n").encode())
        return

    import numpy as np
    import torch
    import torch.distributed as dist

    # The contract is ONE JSON line on stdout. Libraries (RCCL's version banner, HIP runtime notes)
    # write to fd 1 as well: point fd 1 at stderr and keep a private handle for the result line.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    sys.stdout = sys.stderr
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)   # before the process group: its collectives run on this rank's GPU
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    pkg = importlib.import_module("statsd-router_amd")
    digests = json.load(open(os.path.join(REPO, "tests", "golden", "digests.json")))

    desc, batch_bytes, lens, p_inv, shards, seed0, dkey = CONFIGS[args.config]
    alive, alive_tag = [1] * shards, "all"
    if args.dead > 0:
        alive_tag = "dead25" if abs(args.dead - 0.25) < 1e-9 else None
        if alive_tag and f"{dkey}/{alive_tag}" in digests:
            words = [int(w, 16) for w in digests[f"{dkey}/{alive_tag}"]["alive"]]
            alive = [(words[k >> 6] >> (k & 63)) & 1 for k in range(shards)]
        else:
            rng = np.random.default_rng(seed0 + 7919 * rank)
            for k in rng.choice(shards, max(1, int(round(args.dead * shards))), replace=False):
                alive[int(k)] = 0

    # ---- rotating set of distinct batches, resident in HBM -------------------------------------
    B = args.batches
    M = max(1, min(args.per_launch, pkg.SR_MAX_BATCHES_PER_LAUNCH, B))
    B -= B % M                                  # whole launches only
    ng = B // M                                 # launch groups in the rotating set
    host = [pkg.gen_stream(batch_bytes, lens, seed=seed0 + 1_000_003 * rank + 65_537 * b, p_invalid=p_inv)
            for b in range(B)]
    sizes = [int(s.data.size) for s in host]
    lines = [int(s.n_lines) for s in host]
    d_in = torch.empty((B, batch_bytes), dtype=torch.uint8, device=dev)
    for b, s in enumerate(host):
        d_in[b, : sizes[b]].copy_(torch.from_numpy(s.data))
    max_lines = max(lines)
    # one record array per batch slot of a launch (batches of one launch never share records)
    d_out = torch.empty((M, max_lines * 8), dtype=torch.uint8, device=dev)
    d_cnt = torch.zeros(B, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(device=dev)
    router = pkg.Router(shards, batch_bytes, device=local)
    router.set_alive(alive)
    router.set_stream(stream.cuda_stream)
    apply_knobs(pkg, router, args.knob)
    router.set_layout({"auto": pkg.SR_LAYOUT_AUTO, "uniform": pkg.SR_LAYOUT_UNIFORM,
                       "segments": pkg.SR_LAYOUT_SEGMENTS, "chunks": pkg.SR_LAYOUT_CHUNKS}[args.layout])
    in_ptr, out_ptr, cnt_ptr = d_in.data_ptr(), d_out.data_ptr(), d_cnt.data_ptr()

    def launch(gi):
        """One step: launch group gi (batches gi*M .. gi*M+M-1) in ONE route_kernel launch."""
        router.route_device_many([(in_ptr + b * batch_bytes, sizes[b], out_ptr + m * max_lines * 8, max_lines, None,
                                   cnt_ptr + 8 * b) for m, b in enumerate(range(gi * M, gi * M + M))])

    group_bytes = [sum(sizes[gi * M: gi * M + M]) for gi in range(ng)]
    group_lines = [sum(lines[gi * M: gi * M + M]) for gi in range(ng)]
    K = max(1, args.steps)
    with torch.cuda.stream(stream):
        for gi in range(ng):                    # eager once (allocations, code load)
            launch(gi)
        stream.synchronize()
        graphs = []
        for gi in range(ng):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                launch(gi)
            graphs.append(g)
        captured_layout = pkg.LAYOUT_NAMES.get(router.last_layout(), "?")
        # warm-up: W launches, and at least --min-warmup-ms of back-to-back launches
        t_w = time.perf_counter()
        w_done = 0
        while w_done < args.warmup or (time.perf_counter() - t_w) * 1e3 < args.min_warmup_ms:
            for _ in range(16):
                graphs[w_done % ng].replay()
                w_done += 1
            stream.synchronize()

        # ---- timed region: exactly K steps ------------------------------------------------------
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        for i in range(K):
            graphs[i % ng].replay()
        ev1.record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        region_ms = ev0.elapsed_time(ev1)

    counts = d_cnt.cpu().numpy()
    assert all(int(counts[b]) == lines[b] for b in range(B)), "line counts differ from the generator"
    verify = None if args.no_verify else verify_timed_launch(pkg, graphs[0], stream, d_out, host, M, max_lines,
                                                             shards, alive, rank, digests, dkey, alive_tag)

    ceiling = read_ceiling(d_in, stream)
    wall = t1 - t0
    steps_lines = sum(group_lines[i % ng] for i in range(K))
    steps_bytes = sum(group_bytes[i % ng] for i in range(K))
    t = torch.tensor([wall, region_ms / 1e3], dtype=torch.float64, device=dev)
    tot = torch.tensor([steps_lines, steps_bytes], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    wall_max, region_max = float(t[0]), float(t[1])
    total_lines, total_bytes = float(tot[0]), float(tot[1])

    result = None
    if rank == 0:
        # the dominant kernel's achieved HBM rate: algorithmic bytes (the framed bytes, read once)
        # of the timed launches on this GPU over their GPU time
        achieved = steps_bytes / (region_ms * 1e-3) / 1e9
        kernel_name = "route_chunk_kernel" if captured_layout == "chunks" else "route_kernel"
        traffic, traffic_src = None, None
        tj = args.traffic_json
        if tj and os.path.exists(tj):
            with open(tj) as f:
                tr = json.load(f)
            # counter bytes of a rocprofv3 --pmc run (tools/pmc_summary.py) count only when they were
            # measured on this very build of the library and configuration
            lib_sha = hashlib.sha256(open(pkg.ROUTE_LIB, "rb").read()).hexdigest()
            if (tr.get("config") == args.config and tr.get("lib_sha256") == lib_sha
                    and tr.get("kernel") == kernel_name):   # the kernel named explicitly, no default
                traffic = tr.get("hbm_bytes_per_launch")
                traffic_src = f"{os.path.relpath(tj, REPO)} (rocprofv3 --pmc of this build, lib sha256 {lib_sha[:12]})"
            else:
                traffic_src = (f"{os.path.relpath(tj, REPO)} is for config {tr.get('config')} / kernel "
                               f"{tr.get('kernel')} / lib {str(tr.get('lib_sha256'))[:12]}, not this build: not reported")
        result = {
            "metric": "M metrics/s parsed+hashed, device-resident (GiB/s and HBM roofline alongside)",
            "value": round(total_lines / wall_max / 1e6, 3),
            "unit": "M metrics/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "warmup_launches_run": w_done,
            "ms_per_step": round(wall_max * 1e3 / K, 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": f"synthetic: seeded sr_gen streams, {B} distinct framed 16 MiB batches per GPU resident in HBM",
            "config": {
                "workload": desc,
                "step": f"one {kernel_name} launch over {M} distinct batches ({group_bytes[0]} B at group 0)",
                "batch_bytes": batch_bytes,
                "line_bytes": lens,
                "p_invalid": p_inv,
                "shards": shards,
                "alive": f"{sum(alive)}/{shards}",
                "rotating_batches": B,
                "parallelism": f"dp{world} (independent datagram batches per GPU)",
                "batches_per_launch": M,
                "launch": f"hipGraph replay, one graph per launch of {M} batches, {ng} graphs alternating",
                "lane_layout": f"{captured_layout} (sr_set_layout {args.layout})",
            },
            "gib_per_s": round(total_bytes / wall_max / 2**30, 3),
            "gpu_region_ms": round(region_max * 1e3, 4),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": kernel_name,
                "read_ceiling": dict(ceiling, frac_of_ceiling=round(achieved / ceiling["achieved"], 4))
                if ceiling.get("achieved") else ceiling,
                "bytes_per_launch": steps_bytes / K,
                "launch_us": round(region_ms * 1e3 / K, 3),
                "launch_timing": (f"timed region: {K} back-to-back launches between two HIP events on the launch "
                                  "stream; achieved = the region's framed bytes / the region's event time"),
            },
            "verify": verify,
            "cpu_baseline": None,
        }

        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(host, shards, alive, args.cpu_seconds)
        if not args.no_e2e:
            result["e2e"] = e2e(pkg, router, stream, host, sizes, lines, batch_bytes, dev, M)
        if not args.no_pack:
            result["route_pack"] = pack_leg(pkg, router, stream, d_in, sizes, lines, batch_bytes, shards, M, dev,
                                            dead=sum(alive) < shards, alive=alive, threads=args.pack_threads,
                                            host=None if args.no_verify else host, knobs=args.knob,
                                            min_warmup_ms=args.min_warmup_ms)
        if args.knob:
            result["config"]["knobs"] = args.knob
    router.close()
    del d_in, d_out
    torch.cuda.empty_cache()
    emitted = threading.Lock()   # held by whoever prints the line (once)

    def emit(res):
        if emitted.acquire(blocking=False):
            if rank == 0:
                print(json.dumps(res), file=json_out, flush=True)
            return True
        return False

    dog = None
    if args.regroup == "on" or (args.regroup == "auto" and world > 1):
        # a collective that never completes (a peer lost, a transport stuck) must not take the main
        # line with it: past the deadline every rank prints what it has and leaves
        def give_up():
            print(f"bench.py rank {rank}: regroup leg timed out after {args.regroup_timeout:.0f} s", file=sys.stderr)
            if rank == 0:
                result["regroup"] = {"error": f"timed out after {args.regroup_timeout:.0f} s"}
            emit(result)
            sys.stderr.flush()
            json_out.flush()
            os._exit(3)   # the line is out; the exit status still says the run did not finish cleanly

        dog = threading.Timer(args.regroup_timeout, give_up)
        dog.daemon = True
        dog.start()
        try:   # a failing regroup leg must not take the main line with it
            rg = regroup_leg(pkg, dev, local, world, rank, args.regroup_config, args.regroup_steps,
                             per_step=args.regroup_batches, exchange=args.exchange,
                             own_in_place=not args.regroup_copy_own, one_call=not args.regroup_split_calls,
                             slots=args.regroup_slots)
        except (RuntimeError, OSError, ValueError) as e:
            rg = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0:
            result["regroup"] = rg
    emit(result)
    if dist.is_initialized():
        dist.destroy_process_group()
    if dog is not None:
        dog.cancel()


def apply_knobs(pkg, router, knobs):
    """--knob NAME=VALUE: sr_set_knob (SR_KNOB_<NAME>) on a context."""
    for kv in knobs:
        name, _, val = kv.partition("=")
        router.set_knob(getattr(pkg, "SR_KNOB_" + name.upper()), int(val, 0))


def read_ceiling(d_in, stream, reps=20):
    """SURVEY.md §8d's measured streaming-read ceiling: a read-only kernel (tools/hbm/hbm_read.hip,
    16 B per lane, 8 loads in flight) over the same resident batches, timed with HIP events on the
    launch stream. Returns {"achieved": GB/s, ...} or a note when the tool library is absent."""
    import ctypes
    import torch

    path = os.path.join(REPO, "tools", "hbm", "libsr_hbm.so")
    if not os.path.exists(path):
        return {"note": f"{path} not built"}
    lib = ctypes.CDLL(path)
    lib.sr_hbm_read.restype = ctypes.c_int
    lib.sr_hbm_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    n = d_in.numel() & ~15
    blocks = 4096
    out = torch.empty(blocks, dtype=torch.int32, device=d_in.device)
    with torch.cuda.stream(stream):
        for _ in range(3):
            lib.sr_hbm_read(d_in.data_ptr(), n, out.data_ptr(), blocks, stream.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            lib.sr_hbm_read(d_in.data_ptr(), n, out.data_ptr(), blocks, stream.cuda_stream)
        e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return {"achieved": round(n / (ms * 1e-3) / 1e9, 1), "unit": "GB/s", "bytes": int(n),
            "kernel": "tools/hbm/hbm_read.hip: read-only, nontemporal 16-B loads, 4096 x 256 threads"}


def verify_timed_launch(pkg, graph, stream, d_out, host, M, max_lines, shards, alive, rank, digests, dkey, tag):
    """Replay launch 0 of the timed set once more; batch 0's records against the reference digest
    (rank 0: same seed as tests/golden/digests.json), the last batch of the launch against the
    oracle record for record. Raises on any difference."""
    import numpy as np

    graph.replay()
    stream.synchronize()
    out = {}
    n0 = host[0].n_lines
    r0 = d_out[0, : n0 * 8].cpu().numpy().tobytes()
    key = f"{dkey}/{tag}" if tag else None
    if rank == 0 and key in digests and digests[key]["nbytes"] == host[0].data.size:
        want = digests[key]["sha256_records"]
        got = hashlib.sha256(r0).hexdigest()
        if got != want:
            raise SystemExit(f"batch 0 records differ from the reference digest {key}: {got} != {want}")
        out["digest"] = f"{key}: batch 0 records sha256 match the compiled reference"
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import sr_oracle

    m = M - 1
    crecs, _, cn = sr_oracle.route(host[m].data, shards, alive)
    got = np.frombuffer(d_out[m, : cn * 8].cpu().numpy().tobytes(), dtype=pkg.RECORD_DTYPE)
    if cn != host[m].n_lines or not np.array_equal(got, crecs):
        raise SystemExit(f"batch {m} of the timed launch differs from the oracle")
    out["oracle"] = f"batch {m} of launch 0 ({cn} lines) equals the C oracle record for record"
    return out


def cpu_baseline(host, shards, alive, seconds):
    """The reference's own read callback (oracle/_ref/sr_ref_bench: sr-main.c's udp_read_cb compiled
    unmodified from /root/reference, log_level ERROR, lines pushed into real downstream buffers,
    each datagram through a socketpair recv) on this host's CPUs: one process alone, then one per
    CPU of the process's share in parallel, each a reference data thread (threads_num,
    sr-main.c:363-367). Without that binary, the C restatement (oracle/sr_oracle.c, measured
    1.3-1.6x faster than the reference) is timed instead ("kind": "port")."""
    import struct
    import subprocess
    import tempfile

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import sr_oracle

    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    cores = min(affinity, share) if share > 0 else affinity
    common = {"cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
              "cores_note": (f"threads = the process's CPU share (sched_getaffinity {affinity}, OMP_NUM_THREADS "
                             f"{share or 'unset'}); on the GPU box that share is 16 CPUs per GPU")}
    ref = os.path.join(REPO, "oracle", "_ref", "sr_ref_bench")
    if os.path.exists(ref):
        h = host[0]
        with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
            off = 0
            for l in h.dgram_lens.tolist():
                f.write(struct.pack("<I", l))
                f.write(h.data[off:off + l].tobytes())
                off += l
            path = f.name
        try:
            def launch(k):
                return [subprocess.Popen([ref, str(shards), path, str(seconds)], stdout=subprocess.PIPE) for _ in range(k)]

            def collect(ps):
                return [json.loads(p.communicate(timeout=4 * seconds + 60)[0]) for p in ps]

            one = collect(launch(1))[0]
            many = collect(launch(cores))
        finally:
            os.unlink(path)
        lines_bytes = h.data.size / max(h.n_lines, 1)
        tot = sum(r["reference_lines_per_s"] for r in many)
        return dict({
            "value": round(tot / 1e6, 3),
            "unit": "M metrics/s",
            "cores": cores,
            "kind": "reference",
            "sample": (f"one 16 MiB batch of the same workload ({h.n_lines} lines in {len(h.dgram_lens)} datagrams) "
                       f"replayed through the reference's udp_read_cb (oracle/_ref/sr_ref_bench), {cores} processes x "
                       f"{seconds:.1f} s = {cores * seconds:.0f} core-seconds"),
            "single_thread": round(one["reference_lines_per_s"] / 1e6, 3),
            "single_thread_gib_per_s": round(one["reference_lines_per_s"] * lines_bytes / 2**30, 3),
            "gib_per_s": round(tot * lines_bytes / 2**30, 3),
            "restatement_single_thread": round(one["restatement_lines_per_s"] / 1e6, 3),
            "restatement_over_reference": one["restatement_over_reference"],
        }, **common)

    sample = [host[b].data for b in range(min(4, len(host)))]
    l1, b1, w1 = sr_oracle.bench(sample, shards, alive, 1, seconds)
    lm, bm, wm = sr_oracle.bench(sample, shards, alive, cores, seconds)
    return dict({
        "value": round(lm / wm / 1e6, 3),
        "unit": "M metrics/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"{len(sample)} x 16 MiB batches of the same workload routed repeatedly by the C restatement "
                   f"(oracle/sr_oracle.c: memchr + serial sdbm + probe, like sr-main.c:175-189), "
                   f"{cores} threads x {seconds:.1f} s = {cores * seconds:.0f} core-seconds"),
        "single_thread": round(l1 / w1 / 1e6, 3),
        "single_thread_gib_per_s": round(b1 / w1 / 2**30, 3),
        "gib_per_s": round(bm / wm / 2**30, 3),
    }, **common)


def regroup_leg(pkg, dev, local, world, rank, cfg, steps, per_step=8, exchange="c", own_in_place=True,
                one_call=True, slots=2):
    """Classify + regroup on its own batches of config `cfg` (C5 by default: mixed
    lengths, 64 shards). One step = one route launch of `per_step` batches, then ONE pack of all of
    them by owner GPU (shard % G) and ONE exchange: an all-to-all of the split sizes (the step's single
    host round trip), of the packed lines and of the records (RCCL over xGMI). Timed like the main
    region (barrier + synchronize, max over ranks).

    slots = 2 (the C exchange): consecutive steps alternate between two router contexts, each with its
    own stream, communicator, records and receive buffers, so step i + 1's route launch and split sizes
    run while step i's scatter and exchange move its payload (the host's wait for step i + 1's sizes
    overlaps step i's transfer); slots = 1: every step on one stream, strictly in sequence."""
    import torch
    import torch.distributed as dist

    rg_mod = importlib.import_module("statsd-router_amd.regroup")
    if world == 1 and not dist.is_initialized():
        dist.init_process_group("nccl", store=dist.TCPStore("127.0.0.1", 0, 1, True), rank=0, world_size=1)
    desc, batch_bytes, lens, p_inv, shards, seed0, _ = CONFIGS[cfg]
    nb = per_step
    host = [pkg.gen_stream(batch_bytes, lens, seed=seed0 + 1_000_003 * rank + 65_537 * b, p_invalid=p_inv)
            for b in range(nb)]
    sizes = [int(s.data.size) for s in host]
    lines = [int(s.n_lines) for s in host]
    max_lines = max(lines)
    d_in = torch.empty((nb, batch_bytes), dtype=torch.uint8, device=dev)
    for b, s in enumerate(host):
        d_in[b, : sizes[b]].copy_(torch.from_numpy(s.data))
    base = d_in.data_ptr()
    if exchange != "c" or not own_in_place or not one_call:
        slots = 1   # the developer A/B paths stay on one stream

    def open_comm():
        err, comm = "", None
        try:
            comm = pkg.Comm.from_group(local)
        except (OSError, RuntimeError) as e:
            err = str(e)
        ok = torch.tensor([0.0 if comm is None else 1.0], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)   # every rank on the same transport
        if ok.item() != 1.0 and comm is not None:
            comm.close()
            comm = None
        return comm, err

    class Slot:   # one router context: stream, records, communicator, regrouper
        def __init__(self):
            self.stream = torch.cuda.Stream(device=dev)
            self.router = pkg.Router(shards, batch_bytes, device=local)
            self.router.set_stream(self.stream.cuda_stream)
            self.d_rec = torch.empty((nb, max_lines), dtype=torch.int64, device=dev)
            self.d_n = torch.zeros(nb, dtype=torch.int64, device=dev)
            self.route_descs = [(base + b * batch_bytes, sizes[b], self.d_rec[b].data_ptr(), max_lines, None,
                                 self.d_n[b].data_ptr()) for b in range(nb)]
            self.pack_descs = [(base + b * batch_bytes, sizes[b], self.d_rec[b].data_ptr(), max_lines,
                                self.d_n[b].data_ptr()) for b in range(nb)]
            self.comm = None

    ss = [Slot() for _ in range(max(1, slots))]
    transport = "torch.distributed all_to_all_single (nccl)"
    if exchange == "c":   # the C ABI's RCCL exchange (sr_exchange_sizes / sr_exchange_data)
        errs = []
        for sl in ss:
            sl.comm, err = open_comm()
            errs.append(err)
        if all(sl.comm is not None for sl in ss):
            transport = "C ABI sr_regroup_launch (RCCL)" + (f", {len(ss)} communicators" if len(ss) > 1 else "")
        else:
            for sl in ss:
                if sl.comm is not None:
                    sl.comm.close()
                    sl.comm = None
            transport += f" (sr_comm_open failed on some rank{': ' + ' '.join(e for e in errs if e) if any(errs) else ''})"
    for sl in ss:
        with torch.cuda.stream(sl.stream):
            sl.reg = rg_mod.LaunchRegrouper(pkg, sl.router, sum(sizes), nb * max_lines, comm=sl.comm,
                                            own_in_place=own_in_place, one_call=one_call)

    def step(i):
        sl = ss[i % len(ss)]
        with torch.cuda.stream(sl.stream):
            sl.router.route_device_many(sl.route_descs)
            rb, rr, _ = sl.reg(sl.pack_descs)
        sent = sum(c[1] for c in sl.reg.last_sent) - sl.reg.last_sent[rank][1]
        return int(rr.numel()), int(rb.numel()), sent

    for i in range(2 * len(ss)):
        step(i)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    acc = [0, 0, 0]
    for i in range(steps):
        acc = [a + x for a, x in zip(acc, step(i))]
    torch.cuda.synchronize()
    dist.barrier()
    wall = time.perf_counter() - t0
    for sl in ss:
        sl.router.close()
        if sl.comm is not None:
            sl.comm.close()
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    tot = torch.tensor([sum(lines) * steps, acc[0], acc[1], acc[2]], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    w = float(t[0])
    comm = ss[0].comm
    return {"value": round(float(tot[0]) / w / 1e6, 3), "unit": "M metrics/s", "workload": desc,
            "steps_per_gpu": steps, "batches_per_step": nb, "ms_per_step": round(w * 1e3 / steps, 4),
            "slots": len(ss),
            "lines_regrouped": int(tot[1]), "bytes_regrouped": int(tot[2]),
            "bytes_sent_to_other_gpus_per_s": round(float(tot[3]) / w / 1e9, 3), "exchange": transport,
            "note": (f"route launch of {nb} x 16 MiB batches + one pack by owner + one exchange (split sizes, "
                     f"packed lines, records) per step over {world} GPU(s); owner = shard % {world}; one host round "
                     f"trip per step for the split sizes; "
                     + (f"steps alternate over {len(ss)} contexts and streams (step i + 1's route overlaps step i's "
                        "scatter and exchange); " if len(ss) > 1 else "")
                     + (("sr_regroup_launch: " if one_call else "")
                        + "sr_pack_owner_sizes, then sr_pack_owner_scatter with the rank's own chunk written straight "
                        "into the receive buffers (no local copy)" if comm is not None and own_in_place
                        else "sr_pack_many_by_owner"))}


def verify_pack(pkg, th, host, M, max_lines, shards, alive):
    """After the route_pack leg's timing: replay its graph once more, then batch M - 1 of the launch
    (sorted records, packet descriptors, counts, pending bytes out, probed-dead bitmap) against the
    C oracle's push_to_downstream restatement. Raises on any difference."""
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import sr_oracle

    with torch.cuda.stream(th.st):
        th.g_all.replay()
    th.st.synchronize()
    m = M - 1
    s = host[th.first + m]
    recs, _, cn = sr_oracle.route(s.data, shards, alive)
    probed = sr_oracle.probed_dead(s.data, shards, alive)
    fill_in = th.fill[m].cpu().numpy().view(np.uint16)
    srt_o, pk_o, fo_o, nv_o = sr_oracle.pack_packets(recs, shards, fill_in, probed)
    np_, nv, nl = (int(x) for x in th.counts[m].cpu().tolist())
    srt = np.frombuffer(th.srt[m].cpu().numpy().tobytes(), dtype=pkg.RECORD_DTYPE)[:nl]
    pk = np.frombuffer(th.pk[m].cpu().numpy().tobytes(), dtype=pkg.PACKET_DTYPE)[:np_]
    fo = th.fout[m].cpu().numpy().view(np.uint16)
    pd = pkg.bitmap_shards(np.frombuffer(th.pd[m].cpu().numpy().tobytes(), dtype=np.uint64), shards)
    if ((np_, nv, nl) != (len(pk_o), nv_o, cn) or not np.array_equal(srt, srt_o)
            or not np.array_equal(pk.view(np.uint8), pk_o.view(np.uint8)) or fo.tolist() != fo_o.tolist()
            or pd.tolist() != probed.tolist()):
        raise SystemExit(f"route_pack leg: batch {m} of the timed graph differs from the oracle")
    return (f"batch {m} of the timed route + pack graph ({cn} lines, {np_} packets) equals the C oracle: sorted "
            "records, descriptors, counts, pending bytes out, probed-dead bitmap")


def pack_leg(pkg, router, stream, d_in, sizes, lines, batch_bytes, shards, M, dev, dead=False, reps=20,
             alive=None, threads=2, host=None, knobs=(), min_warmup_ms=60.0):
    """The router's device data path: one route launch over M batches (the
    batches of M data threads), then the per-downstream MTU packing of all of them in one
    sr_pack_packets_many (sorted records + packet descriptors, each batch from its own pending
    bytes), captured in one graph and replayed back to back. Reported: lines/s through route +
    packing, and the packing's own time. Then the same with two contexts on two streams (two
    router data threads sharing the GPU, as `threads_num` > 1 does): each replays its own
    route + pack graph over its own M batches, and one context's packing runs beside the other's
    route launch."""
    import torch

    max_lines = max(lines)
    mp = pkg.max_packets(batch_bytes, shards)
    base = d_in.data_ptr()
    nsets = max(1, len(sizes) // M)

    class Thread:   # one data thread's device state: its context, stream, buffers and graphs
        def __init__(self, rt, st, first):
            self.rt, self.st, self.first = rt, st, first
            self.rec = torch.empty((M, max_lines), dtype=torch.int64, device=dev)
            self.cnt = torch.zeros(M, dtype=torch.int64, device=dev)
            self.srt = torch.empty((M, max_lines), dtype=torch.int64, device=dev)
            self.pk = torch.empty((M, mp * 2), dtype=torch.int64, device=dev)
            self.counts = torch.zeros((M, 3), dtype=torch.int64, device=dev)
            self.fill = torch.zeros((M, shards), dtype=torch.int16, device=dev)
            self.fout = torch.zeros((M, shards), dtype=torch.int16, device=dev)
            # the probed-dead bitmap of every batch, as the router asks for it (sr-main.c:106)
            self.pd = torch.zeros((M, max((shards + 63) // 64, 1)), dtype=torch.int64, device=dev)
            # with dead shards the router has the route kernel write the hashes (the replay reads them)
            self.h = torch.empty((M, max_lines), dtype=torch.int64, device=dev) if dead else None

        def route(self):
            self.rt.route_device_many([(base + (self.first + b) * batch_bytes, sizes[self.first + b],
                                        self.rec[b].data_ptr(), max_lines,
                                        self.h[b].data_ptr() if dead else None, self.cnt[b].data_ptr(),
                                        self.pd[b].data_ptr()) for b in range(M)])

        def route_pack(self):   # sr_route_pack_many: the route kernel's tile histograms feed the sort
            self.rt.route_pack_many([(base + (self.first + b) * batch_bytes, sizes[self.first + b],
                                      self.rec[b].data_ptr(), max_lines, self.h[b].data_ptr() if dead else None,
                                      self.cnt[b].data_ptr(), self.pd[b].data_ptr(), self.fill[b].data_ptr(),
                                      self.srt[b].data_ptr(), self.pk[b].data_ptr(), mp, self.counts[b].data_ptr(),
                                      self.fout[b].data_ptr()) for b in range(M)])

        def capture(self):
            with torch.cuda.stream(self.st):
                self.route_pack()                            # eager once: the packing scratch is allocated here
                self.st.synchronize()
                self.g_all, self.g_route = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.g_all, stream=self.st):
                    self.route_pack()
                with torch.cuda.graph(self.g_route, stream=self.st):
                    self.route()

    def replay(th, attr):   # a graph replays on the current stream: the thread's own
        with torch.cuda.stream(th.st):
            getattr(th, attr).replay()

    def timed(threads, attr):
        # the main leg's warm-up rule: back-to-back replays for at least min_warmup_ms (the clocks settle)
        t_w = time.perf_counter()
        while (time.perf_counter() - t_w) * 1e3 < min_warmup_ms:
            for _ in range(8):
                for th in threads:
                    replay(th, attr)
            torch.cuda.synchronize()
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(threads[0].st)
        for th in threads[1:]:
            th.st.wait_event(a)
        for _ in range(reps):
            for th in threads:
                replay(th, attr)
        for th in threads[1:]:
            e = torch.cuda.Event()
            e.record(th.st)
            threads[0].st.wait_event(e)
        z.record(threads[0].st)
        z.synchronize()
        return a.elapsed_time(z) / reps

    t1 = Thread(router, stream, 0)
    t1.capture()
    res = {"route_pack": timed([t1], "g_all"), "route_only": timed([t1], "g_route")}
    verify = None if host is None else verify_pack(pkg, t1, host, M, max_lines, shards, alive)
    packets = int(t1.counts[:, 0].sum())
    tot_lines = sum(lines[:M])
    out = {"value": round(tot_lines / (res["route_pack"] * 1e-3) / 1e6, 3), "unit": "M metrics/s",
           "ms_per_launch": round(res["route_pack"], 4), "route_only_ms": round(res["route_only"], 4),
           "packing_ms": round(res["route_pack"] - res["route_only"], 4),
           "packets_per_launch": packets,
           "probed_dead_shards": int(sum(bin(int(w) & (2**64 - 1)).count("1") for w in t1.pd[0].tolist())),
           "verify": verify,
           "note": (f"sr_route_pack_many: one route launch over {M} batches with their probed-dead bitmaps "
                    f"(sr-main.c:106; all alive with <= 16 shards: also each tile's per-shard line counts) + the "
                    f"packing of all of them (regroup by downstream, next-fit 1450-byte packets), one graph, {reps} "
                    f"replays; packing_ms = that graph - the route launch's graph")}
    if threads < 2:
        return out
    # two data threads on one GPU: a second context on its own stream over the next M batches
    r2 = pkg.Router(shards, batch_bytes, device=dev.index)
    try:
        r2.set_alive(alive if alive is not None else [1] * shards)
        apply_knobs(pkg, r2, knobs)
        s2 = torch.cuda.Stream(device=dev)
        r2.set_stream(s2.cuda_stream)
        t2 = Thread(r2, s2, M if nsets > 1 else 0)
        t2.capture()
        two = timed([t1, t2], "g_all")
        lines2 = tot_lines + sum(lines[t2.first:t2.first + M])
        out["two_threads"] = {
            "value": round(lines2 / (two * 1e-3) / 1e6, 3), "unit": "M metrics/s",
            "ms_per_round": round(two, 4), "packets_per_launch": [packets, int(t2.counts[:, 0].sum())],
            "note": ("two router contexts (two data threads sharing the GPU), each with its own stream replaying "
                     f"its own route + pack graph over its own {M} batches; the streams run concurrently, so one "
                     "thread's packing overlaps the other's route launch; rate = both threads' lines / round")}
    finally:
        r2.close()
    return out


def e2e(pkg, router, stream, host, sizes, lines, batch_bytes, dev, M, groups=24):
    """Host memory -> H2D -> route -> D2H records with pinned buffers ("end to end").

    Groups of M batches, double-buffered: the H2D copy of group g+1 (copy stream) overlaps the
    route launch of group g (the context's stream, M batches per launch as in the timed region)
    and the D2H of group g-1's records (third stream)."""
    import torch

    nb = min(len(host), 2 * M)
    pinned = [torch.from_numpy(host[b].data).pin_memory() for b in range(nb)]
    max_lines = max(lines)
    out_pinned = [torch.empty((M, max_lines * 8), dtype=torch.uint8).pin_memory() for _ in range(2)]
    d_buf = [torch.empty((M, batch_bytes), dtype=torch.uint8, device=dev) for _ in range(2)]
    d_out = [torch.empty((M, max_lines * 8), dtype=torch.uint8, device=dev) for _ in range(2)]
    d_cnt = torch.zeros((2, M), dtype=torch.int64, device=dev)
    h2d, d2h = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    ev_in = [torch.cuda.Event() for _ in range(2)]
    ev_done = [torch.cuda.Event() for _ in range(2)]
    ev_out = [torch.cuda.Event() for _ in range(2)]
    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    warm = 2
    tot_lines = tot_bytes = 0
    torch.cuda.synchronize()
    for g in range(groups + warm):
        if g == warm:
            torch.cuda.synchronize()
            a.record(h2d)
            tot_lines = tot_bytes = 0
        k = g % 2
        bs = [(g * M + m) % nb for m in range(M)]
        with torch.cuda.stream(h2d):
            h2d.wait_event(ev_done[k])          # the route of group g-2 has consumed d_buf[k]
            for m, b in enumerate(bs):
                d_buf[k][m, : sizes[b]].copy_(pinned[b], non_blocking=True)
            ev_in[k].record(h2d)
        stream.wait_event(ev_in[k])
        stream.wait_event(ev_out[k])            # group g-2's records have left d_out[k]
        router.route_device_many([(d_buf[k][m].data_ptr(), sizes[b], d_out[k][m].data_ptr(), max_lines, None,
                                   d_cnt[k, m].data_ptr()) for m, b in enumerate(bs)])
        ev_done[k].record(stream)
        with torch.cuda.stream(d2h):
            d2h.wait_event(ev_done[k])
            for m, b in enumerate(bs):
                out_pinned[k][m, : lines[b] * 8].copy_(d_out[k][m, : lines[b] * 8], non_blocking=True)
            ev_out[k].record(d2h)
        tot_lines += sum(lines[b] for b in bs)
        tot_bytes += sum(sizes[b] for b in bs)
    z.record(d2h)
    torch.cuda.synchronize()
    ms = a.elapsed_time(z)
    return {"value": round(tot_lines / (ms * 1e-3) / 1e6, 3), "unit": "M metrics/s",
            "gib_per_s": round(tot_bytes / (ms * 1e-3) / 2**30, 3),
            "note": (f"pinned host batches -> H2D -> route_kernel ({M} batches per launch) -> D2H 8-B records; "
                     "double-buffered on three streams (copy in / route / copy out)")}


if __name__ == "__main__":
    main()
