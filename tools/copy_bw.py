import torch, time, json
n = 537 * 1024 * 1024
a = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
b = torch.empty_like(a)
for _ in range(5): b.copy_(a)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20): b.copy_(a)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(json.dumps({"bytes": n, "ms": ms, "copy_TBps_rw": 2 * n / ms / 1e9}))
# int4 view copy
a4 = a.view(torch.int32); b4 = b.view(torch.int32)
e0.record()
for _ in range(20): b4.copy_(a4)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(json.dumps({"int32_ms": ms, "copy_TBps_rw": 2 * n / ms / 1e9}))
