"""Practical HBM bandwidth on this box for the activation sizes of the bench (torch copy / read-reduce)."""
import torch

dev = torch.device("cuda:0")
for mb in (26, 52, 105, 210, 420, 1680):
    n = mb * 1024 * 1024 // 2
    a = torch.empty(n, dtype=torch.float16, device=dev).uniform_()
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20
    e0.record()
    for _ in range(20):
        s = a.sum(dtype=torch.float32)
    e1.record()
    torch.cuda.synchronize()
    t2 = e0.elapsed_time(e1) / 20
    print(f"{mb:5d} MB: copy {2 * mb * 1.048576 / t:8.0f} GB/s ({t * 1e3:.1f} us)   read-sum {mb * 1.048576 / t2:8.0f} GB/s", flush=True)
