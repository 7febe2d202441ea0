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
    ap.add_argument("--steps", type=int, default=4096)
    ap.add_argument("--warmup", type=int, default=2048,
                    help="untimed steps first (about 12 ms at C2: the clocks settle)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batches", type=int, default=64, help="distinct batches in the rotating set")
    ap.add_argument("--per-launch", type=int, default=32,
                    help="batches routed per kernel launch (sr_route_device_many; 1 = sr_route_device)")
    ap.add_argument("--dead", type=float, default=0.0, help="fraction of dead downstreams")
    ap.add_argument("--regroup", default="auto", choices=["auto", "on", "off"],
                    help="classify + all-to-all regroup leg (auto: on when more than one GPU)")
    ap.add_argument("--regroup-steps", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def main():
    args = parse()
    # The contract is ONE JSON line on stdout. Libraries (RCCL's version banner, HIP runtime notes)
    # write to fd 1 as well: point fd 1 at stderr and keep a private handle for the result line.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    sys.stdout = sys.stderr
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
    M = max(1, min(args.per_launch, pkg.SR_MAX_BATCHES_PER_LAUNCH, B))
    # one record array per batch slot of a launch (batches of one launch never share records)
    d_out = torch.empty((M, max_lines * 8), dtype=torch.uint8, device=dev)
    d_cnt = torch.zeros(B, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(device=dev)
    router = pkg.Router(shards, batch_bytes, device=local)
    router.set_alive(alive)
    router.set_stream(stream.cuda_stream)
    in_ptr, out_ptr, cnt_ptr = d_in.data_ptr(), d_out.data_ptr(), d_cnt.data_ptr()

    def launch_range(i0, i1):
        """Steps i0 .. i1-1 (batch i % B each), M batches per kernel launch."""
        for j0 in range(i0, i1, M):
            descs = []
            for m, i in enumerate(range(j0, min(j0 + M, i1))):
                b = i % B
                descs.append((in_ptr + b * batch_bytes, sizes[b], out_ptr + m * max_lines * 8, max_lines, None,
                              cnt_ptr + 8 * b))
            if M == 1:
                router.route_device(*descs[0])
            else:
                router.route_device_many(descs)

    def launch(i):   # one launch: steps i*M .. i*M+M-1
        launch_range(i * M, i * M + M)

    with torch.cuda.stream(stream):
        launch_range(0, max(args.warmup, 1))
        stream.synchronize()
        # capture the rotating set as one graph (+ a tail graph so exactly K steps are timed)
        K = args.steps
        g_full = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_full, stream=stream):
            launch_range(0, B)
        g_tail = None
        if K % B:
            g_tail = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_tail, stream=stream):
                launch_range(0, K % B)
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
        nprobe = max(1, min(K, 512) // M)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nprobe)]
        probe_bytes = 0
        for i, (a, z) in enumerate(evs):
            a.record(stream)
            launch(i)
            z.record(stream)
            probe_bytes += sum(sizes[j % B] for j in range(i * M, i * M + M))
        stream.synchronize()
        launch_ms = float(np.mean([a.elapsed_time(z) for a, z in evs]))
        bytes_per_launch = probe_bytes / nprobe

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
                "batches_per_launch": M,
                "launch": f"hipGraph replay of back-to-back route_kernel launches, {M} batches each",
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
                "launch_timing": f"mean of {nprobe} eager launches ({M} batches each), each bracketed by HIP events "
                                 "on its stream",
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
            result["e2e"] = e2e(pkg, router, stream, host, sizes, lines, batch_bytes, dev, M)
    if args.regroup == "on" or (args.regroup == "auto" and world > 1):
        rg = regroup_leg(pkg, router, stream, d_in, sizes, lines, batch_bytes, B, max_lines, dev, world,
                         args.regroup_steps)
        if rank == 0:
            result["regroup"] = rg
    router.close()
    if rank == 0:
        print(json.dumps(result), file=json_out, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def regroup_leg(pkg, router, stream, d_in, sizes, lines, batch_bytes, B, max_lines, dev, world, steps):
    """Classify + regroup: per batch, route, pack by owner GPU (shard % G) and
    all-to-all the packed lines and records (RCCL over xGMI). Not graph-captured: the split sizes
    go through the host. Timed like the main region (barrier + synchronize, max over ranks)."""
    rg_mod = importlib.import_module("statsd-router_amd.regroup")
    if world == 1 and not dist.is_initialized():
        dist.init_process_group("nccl", store=dist.TCPStore("127.0.0.1", 0, 1, True), rank=0, world_size=1)
    reg = rg_mod.Regrouper(pkg, router, batch_bytes, max_lines, slots=2)
    d_rec = torch.empty(max_lines, dtype=torch.int64, device=dev)
    d_n = torch.zeros(1, dtype=torch.int64, device=dev)
    base = d_in.data_ptr()
    rank = dist.get_rank()

    def start(i):
        b = i % B
        router.route_device(base + b * batch_bytes, sizes[b], d_rec.data_ptr(), max_lines, None, d_n.data_ptr())
        reg.start(i % 2, base + b * batch_bytes, sizes[b], d_rec.data_ptr(), d_n.data_ptr(), max_lines)

    def finish(i):
        rb, rr, _ = reg.finish(i % 2)
        # bytes this rank sent to the other ranks, from the host copy the exchange already made
        sent = sum(c[1] for c in reg.last_sent) - reg.last_sent[rank][1]
        return int(rr.numel()), int(rb.numel()), sent

    def run(n):
        # two slots: batch i+1 is routed and packed while the host waits for batch i's split sizes
        acc = [0, 0, 0]
        start(0)
        for i in range(n):
            if i + 1 < n:
                start(i + 1)
            acc = [a + x for a, x in zip(acc, finish(i))]
        return acc

    with torch.cuda.stream(stream):
        run(2)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        recv_lines, recv_bytes, sent_off = run(steps)
        torch.cuda.synchronize()
        dist.barrier()
        wall = time.perf_counter() - t0
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    tot = torch.tensor([sum(lines[i % B] for i in range(steps)), recv_lines, recv_bytes, sent_off],
                       dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    w = float(t[0])
    return {"value": round(float(tot[0]) / w / 1e6, 3), "unit": "M metrics/s",
            "steps_per_gpu": steps, "ms_per_step": round(w * 1e3 / steps, 4),
            "lines_regrouped": int(tot[1]), "bytes_regrouped": int(tot[2]),
            "bytes_sent_to_other_gpus_per_s": round(float(tot[3]) / w / 1e9, 3),
            "note": (f"route + sr_pack_by_owner + all-to-all (split sizes, packed lines, records) per 16 MiB batch "
                     f"over {world} GPU(s); owner = shard % {world}; host round trip for the split sizes, "
                     f"two slots: batch i+1 routed and packed while batch i's sizes come back")}


def e2e(pkg, router, stream, host, sizes, lines, batch_bytes, dev, M, groups=24):
    """Host memory -> H2D -> route -> D2H records with pinned buffers ("end to end").

    Groups of M batches, double-buffered: the H2D copy of group g+1 (copy stream) overlaps the
    route launch of group g (the context's stream, M batches per launch as in the timed region)
    and the D2H of group g-1's records (third stream)."""
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
