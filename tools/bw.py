"""Diagnostics: achievable HBM read rate on this box (torch reductions) for reference."""
import torch

dev = torch.device("cuda", 0)
for mb in (268, 1024):
    x = torch.ones(mb * 2**20 // 4, dtype=torch.float32, device=dev)
    for _ in range(3):
        x.sum()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        x.sum()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 20
    print("sum %d MB: %.1f us  %.2f TB/s" % (mb, ms * 1e3, x.numel() * 4 / ms / 1e9), flush=True)
