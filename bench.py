#!/usr/bin/env python3
"""Device-resident throughput of the statsd-router hot path on MI355X.

One step = one pass of the hot path (frame-free tokenise -> length/':' validate -> sdbm name hash
-> consistent-hash shard pick, one sr_record per line) over one 16 MiB batch of synthetic framed
datagrams already resident in HBM (BASELINE.json configs[1], "C2": 64-byte valid metrics, 4
downstream shards). The timed region cycles through a rotating set of distinct batches (default
64 x 16 MiB = 1 GiB per GPU, well past the 256 MiB Infinity Cache) launched back to back from a
captured HIP graph.

  python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c4|c5]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N  (one rank per GPU,
  each routing its own datagram batches: weak scaling, no data-path collective)

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (description, batch bytes, line lengths, p_invalid, shards, seed base)
    "c2": ("C2: 16 MiB batch of 64-byte valid metrics, 4 downstream shards", 16 << 20, [64], 0.0, 4, 0x5EED0002),
    "c3": ("C3: 16 MiB batch of 256-byte metrics, 10% invalid lines, 4 shards", 16 << 20, [256], 0.10, 4, 0x5EED0003),
    "c4": ("C4: 16 MiB batch of 1024-byte metrics, 16 downstream shards", 16 << 20, [1024], 0.0, 16, 0x5EED0004),
    "c5": ("C5: 16 MiB batch of mixed 64/256/1024-byte metrics, 64 shards", 16 << 20, [64, 256, 1024], 0.0, 64, 0x5EED0005),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2048)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batches", type=int, default=64, help="distinct batches in the rotating set")
    ap.add_argument("--dead", type=float, default=0.0, help="fraction of dead downstreams")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pkg = importlib.import_module("statsd-router_amd")

    desc, batch_bytes, lens, p_inv, shards, seed0 = CONFIGS[args.config]
    rng = np.random.default_rng(seed0 + 7919 * rank)
    alive = [1] * shards
    if args.dead > 0:
        for k in rng.choice(shards, max(1, int(round(args.dead * shards))), replace=False):
            alive[int(k)] = 0

    # ---- rotating set of distinct batches, resident in HBM -------------------------------------
    B = args.batches
    host = []
    for b in range(B):
        s = pkg.gen_stream(batch_bytes, lens, seed=seed0 + 1_000_003 * rank + 65_537 * b, p_invalid=p_inv)
        host.append(s)
    sizes = [int(s.data.size) for s in host]
    lines = [int(s.n_lines) for s in host]
    d_in = torch.empty((B, batch_bytes), dtype=torch.uint8, device=dev)
    for b, s in enumerate(host):
        d_in[b, : sizes[b]].copy_(torch.from_numpy(s.data))
    max_lines = max(lines)
    d_out = torch.empty(max_lines * 8, dtype=torch.uint8, device=dev)
    d_cnt = torch.zeros(B, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(device=dev)
    router = pkg.Router(shards, batch_bytes, device=local)
    router.set_alive(alive)
    router.set_stream(stream.cuda_stream)
    in_ptr, out_ptr, cnt_ptr = d_in.data_ptr(), d_out.data_ptr(), d_cnt.data_ptr()

    def launch(b):
        router.route_device(in_ptr + b * batch_bytes, sizes[b], out_ptr, max_lines, None, cnt_ptr + 8 * b)

    with torch.cuda.stream(stream):
        for i in range(max(args.warmup, 1)):
            launch(i % B)
        stream.synchronize()
        # capture the rotating set as one graph (+ a tail graph so exactly K steps are timed)
        K = args.steps
        g_full = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_full, stream=stream):
            for b in range(B):
                launch(b)
        g_tail = None
        if K % B:
            g_tail = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_tail, stream=stream):
                for b in range(K % B):
                    launch(b)
        g_full.replay()
        stream.synchronize()

        # ---- timed region: exactly K steps ------------------------------------------------------
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(K // B):
            g_full.replay()
        if g_tail is not None:
            g_tail.replay()
        ev1.record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        region_ms = ev0.elapsed_time(ev1)

        # per-launch durations (HIP events on the launch stream), outside the timed region
        nprobe = min(K, 512)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nprobe)]
        for i, (a, z) in enumerate(evs):
            a.record(stream)
            launch(i % B)
            z.record(stream)
        stream.synchronize()
        launch_ms = float(np.mean([a.elapsed_time(z) for a, z in evs]))

    counts = d_cnt.cpu().numpy()
    assert all(int(counts[b]) == lines[b] for b in range(B)), "line counts differ from the generator"

    wall = t1 - t0
    steps_lines = sum(lines[i % B] for i in range(K))
    steps_bytes = sum(sizes[i % B] for i in range(K))
    t = torch.tensor([wall, region_ms / 1e3], dtype=torch.float64, device=dev)
    tot = torch.tensor([steps_lines, steps_bytes], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    wall_max, region_max = float(t[0]), float(t[1])
    total_lines, total_bytes = float(tot[0]), float(tot[1])

    result = None
    if rank == 0:
        bytes_per_launch = float(np.mean(sizes))
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        traffic = None
        tj = args.traffic_json
        if tj and os.path.exists(tj):
            with open(tj) as f:
                tr = json.load(f)
            if tr.get("config") == args.config:
                traffic = tr.get("hbm_bytes_per_launch")
        result = {
            "metric": "M metrics/s parsed+hashed, device-resident (GiB/s and HBM roofline alongside)",
            "value": round(total_lines / wall_max / 1e6, 3),
            "unit": "M metrics/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max * 1e3 / K, 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": f"synthetic: seeded sr_gen streams, {B} distinct framed batches per GPU resident in HBM",
            "config": {
                "workload": desc,
                "batch_bytes": batch_bytes,
                "line_bytes": lens,
                "p_invalid": p_inv,
                "shards": shards,
                "alive": f"{sum(alive)}/{shards}",
                "rotating_batches": B,
                "parallelism": f"dp{world} (independent datagram batches per GPU)",
                "launch": "hipGraph replay of back-to-back route_kernel launches",
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
                "kernel": "route_kernel",
                "bytes_per_launch": bytes_per_launch,
                "launch_us": round(launch_ms * 1e3, 3),
                "launch_timing": "mean of 512 eager launches, each bracketed by HIP events on its stream",
            },
            "cpu_baseline": None,
        }

        if world == 1 and not args.no_cpu:
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import sr_oracle

            sample = [host[b].data for b in range(min(4, B))]
            cores = min(16, os.cpu_count() or 1)
            l1, b1, w1 = sr_oracle.bench(sample, shards, alive, 1, args.cpu_seconds)
            lm, bm, wm = sr_oracle.bench(sample, shards, alive, cores, args.cpu_seconds)
            result["cpu_baseline"] = {
                "value": round(lm / wm / 1e6, 3),
                "unit": "M metrics/s",
                "cores": cores,
                "kind": "port",
                "sample": (f"{len(sample)} x 16 MiB batches of the same workload routed repeatedly by the C "
                           f"restatement (oracle/sr_oracle.c: memchr + serial sdbm + probe, like sr-main.c:175-189), "
                           f"{cores} threads x {args.cpu_seconds:.1f} s"),
                "single_thread": round(l1 / w1 / 1e6, 3),
                "single_thread_gib_per_s": round(b1 / w1 / 2**30, 3),
                "gib_per_s": round(bm / wm / 2**30, 3),
            }

        if not args.no_e2e:
            result["e2e"] = e2e(pkg, router, stream, host, sizes, lines, batch_bytes, dev)
    router.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def e2e(pkg, router, stream, host, sizes, lines, batch_bytes, dev, iters=64):
    """Host memory -> H2D -> route -> D2H records, pinned buffers, one stream."""
    nb = min(8, len(host))
    pinned = [torch.from_numpy(host[b].data).pin_memory() for b in range(nb)]
    max_lines = max(lines)
    out_pinned = torch.empty(max_lines * 8, dtype=torch.uint8).pin_memory()
    d_buf = torch.empty(batch_bytes, dtype=torch.uint8, device=dev)
    d_out = torch.empty(max_lines * 8, dtype=torch.uint8, device=dev)
    d_cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    with torch.cuda.stream(stream):
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tot_lines = tot_bytes = 0
        for it in range(iters + 4):
            if it == 4:
                stream.synchronize()
                a.record(stream)
                tot_lines = tot_bytes = 0
            b = it % nb
            d_buf[: sizes[b]].copy_(pinned[b], non_blocking=True)
            router.route_device(d_buf.data_ptr(), sizes[b], d_out.data_ptr(), max_lines, None, d_cnt.data_ptr())
            out_pinned[: lines[b] * 8].copy_(d_out[: lines[b] * 8], non_blocking=True)
            tot_lines += lines[b]
            tot_bytes += sizes[b]
        z.record(stream)
        stream.synchronize()
    ms = a.elapsed_time(z)
    return {"value": round(tot_lines / (ms * 1e-3) / 1e6, 3), "unit": "M metrics/s",
            "gib_per_s": round(tot_bytes / (ms * 1e-3) / 2**30, 3),
            "note": "pinned host batch -> H2D -> route_kernel -> D2H 8-B records, serial on one stream"}


if __name__ == "__main__":
    main()
