import ctypes, os, sys, torch
REPO = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
lib = ctypes.CDLL(os.path.join(REPO, "tools/hbm/libsr_hbm.so"))
lib.sr_hbm_read_mode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
n = 1 << 30
d = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
out = torch.zeros(1 << 17, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
for mode in (0, 1, 2, 1, 2):
    for _ in range(3): lib.sr_hbm_read_mode(d.data_ptr(), n, out.data_ptr(), 4096, s.cuda_stream, mode)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): lib.sr_hbm_read_mode(d.data_ptr(), n, out.data_ptr(), 4096, s.cuda_stream, mode)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(mode, round(n / ms / 1e6, 1), "GB/s")
