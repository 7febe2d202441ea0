"""Developer timeline of the MTU chunk kernels (a -DSR_MTU_STAMPS build of libsr_route.so, selected
with SR_ROUTE_LIB): per chunk, s_memrealtime at the phase boundaries of mtu_table and mtu_emit, for
one pack of 32 C2 batches. Prints phase medians, the spans and the mean chunks resident.
  SR_ROUTE_LIB=<dir>/libsr_route.so python tools/mtu_stamps.py [config]"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("statsd-router_amd")
cfg = {"c2": ([64], 4), "c5": ([64, 256, 1024], 64), "c4": ([1024], 16)}[sys.argv[1] if len(sys.argv) > 1 else "c2"]
M, BB = 32, 16 << 20
streams = [pkg.gen_stream(BB, cfg[0], seed=0x5EED0002 + 65537 * b) for b in range(M)]
lines = [s.n_lines for s in streams]
ml = max(lines)
d_in = torch.zeros((M, BB), dtype=torch.uint8, device="cuda")
for b, s in enumerate(streams):
    d_in[b, : s.data.size].copy_(torch.from_numpy(s.data))
shards = cfg[1]
d_rec = torch.empty((M, ml), dtype=torch.int64, device="cuda")
d_cnt = torch.zeros(M, dtype=torch.int64, device="cuda")
mp = pkg.max_packets(BB, shards)
d_srt = torch.empty((M, ml), dtype=torch.int64, device="cuda")
d_pk = torch.empty((M, mp * 2), dtype=torch.int64, device="cuda")
d_counts = torch.zeros((M, 3), dtype=torch.int64, device="cuda")
d_fill = torch.zeros((M, shards), dtype=torch.int16, device="cuda")
d_fout = torch.zeros((M, shards), dtype=torch.int16, device="cuda")
s = torch.cuda.Stream()
with pkg.Router(shards, BB) as r, torch.cuda.stream(s):
    r.set_stream(s.cuda_stream)
    r.route_device_many([(d_in[b].data_ptr(), int(streams[b].data.size), d_rec[b].data_ptr(), ml, None,
                          d_cnt[b].data_ptr()) for b in range(M)])
    for _ in range(3):
        r.pack_packets_many([(d_rec[b].data_ptr(), d_cnt[b].data_ptr(), ml, d_fill[b].data_ptr(), 0, d_srt[b].data_ptr(),
                              d_pk[b].data_ptr(), mp, d_counts[b].data_ptr(), d_fout[b].data_ptr()) for b in range(M)])
    r.sync()
lib = pkg.lib()
lib.sr_mtu_stamps.restype = ctypes.c_size_t
lib.sr_mtu_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros((1 << 16, 8), dtype=np.uint64)
n = lib.sr_mtu_stamps(buf.ctypes.data, buf.shape[0])
st = buf[:n].astype(np.float64) * 0.01   # us
live = st[:, 0] > 0
st = st[live]
print(f"chunks with lines: {len(st)}")
names = ["prefix", "next", "doubling", "xloop"]
for i, nm in enumerate(names):
    print(f"table {nm:9s} median {np.median(st[:, i + 1] - st[:, i]):.2f} us  p90 {np.percentile(st[:, i + 1] - st[:, i], 90):.2f}")
print(f"table chunk lifetime median {np.median(st[:, 4] - st[:, 0]):.2f} us; span {st[:, 4].max() - st[:, 0].min():.1f} us; "
      f"mean resident {np.sum(st[:, 4] - st[:, 0]) / (st[:, 4].max() - st[:, 0].min()):.0f}")
e = st[st[:, 7] > 0]
print(f"emit prefix+nx {np.median(e[:, 6] - e[:, 5]):.2f} us, walk {np.median(e[:, 7] - e[:, 6]):.2f} us (p90 {np.percentile(e[:, 7] - e[:, 6], 90):.2f}); "
      f"span {e[:, 7].max() - e[:, 5].min():.1f} us; mean resident {np.sum(e[:, 7] - e[:, 5]) / (e[:, 7].max() - e[:, 5].min()):.0f}")
