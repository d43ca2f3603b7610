import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import custom_go_client_benchmark_amd as pkg
n = pkg._native
name = "princer_100M_files/file_0"
for sz in [(13 << 20) + 777, (16 << 20) + 16, (20 << 20) + 4321, 64 << 20, (256 << 20) + 3]:
    t = torch.empty(sz, dtype=torch.uint8, device="cuda")
    n.gpu_fill_pattern(0, t.data_ptr(), sz, name, 0)
    ok = bytes(t[: 1 << 20].cpu().numpy()) == n.object_bytes(name, 0, 1 << 20)
    res = [n.gpu_verify_pattern(0, t.data_ptr(), sz, name, 0) for _ in range(3)]
    t[sz // 2] ^= 1
    res2 = n.gpu_verify_pattern(0, t.data_ptr(), sz, name, 0)
    print("size", sz, "prefix_ok", ok, "clean", res, "one-flip", res2, "expect first", sz // 2)
