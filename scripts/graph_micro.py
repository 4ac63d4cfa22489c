"""Per-kernel device cost of dependent tiny kernels: 200 in-stream launches vs the same 200 replayed as
one captured hipGraph (torch.cuda.CUDAGraph), timed with events over 50 repetitions."""
import torch

dev = torch.device("cuda:0")
x = torch.zeros(256, device=dev)
s = torch.cuda.Stream(dev)
K, R = 200, 50


def body():
    for _ in range(K):
        x.add_(1.0)


with torch.cuda.stream(s):
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        body()
    torch.cuda.synchronize()
    for mode in ("direct", "graph", "direct", "graph"):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(R):
            if mode == "graph":
                g.replay()
            else:
                body()
        e1.record(s)
        torch.cuda.synchronize()
        print(f"{mode}: {e0.elapsed_time(e1) * 1e3 / (R * K):.2f} us per dependent kernel", flush=True)
