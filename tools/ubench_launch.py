"""Back-to-back dependent kernel launches on one stream: per-kernel wall time of eager
launches vs the same sequence replayed from a captured HIP graph (torch.cuda.CUDAGraph).
Prices the inter-kernel gap that a build of ~15-19 kernels pays.
  python tools/ubench_launch.py"""
import time

import torch

x = torch.zeros(1024, device="cuda")
K, REP = 20, 200


def seq():
    for _ in range(K):
        x.add_(1.0)


for _ in range(10):
    seq()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(REP):
    seq()
torch.cuda.synchronize()
eager = (time.perf_counter() - t0) / (REP * K) * 1e6

s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    seq()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        seq()
torch.cuda.synchronize()
for _ in range(10):
    g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(REP):
    g.replay()
torch.cuda.synchronize()
graph = (time.perf_counter() - t0) / (REP * K) * 1e6
print(f"per dependent kernel: eager {eager:.2f} us, graph replay {graph:.2f} us")
