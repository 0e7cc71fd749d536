#!/usr/bin/env python3
"""Does replaying a HIP graph whose previous replay is still running block the host?  (It decides whether
the engine can queue decode step N+1 behind step N.)  Prints host time of each replay call."""
import time

import torch

x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
y = torch.empty_like(x)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
  for _ in range(2):
    torch.matmul(x, x, out=y)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
  for _ in range(20):
    torch.matmul(x, x, out=y)
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
  for _ in range(20):
    torch.matmul(x, x, out=y)
torch.cuda.synchronize()
t0 = time.perf_counter(); g.replay(); t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
print(f"one replay: host {1e3 * (t1 - t0):.2f} ms, GPU {1e3 * (t2 - t0):.2f} ms")
t0 = time.perf_counter(); g.replay(); t1 = time.perf_counter(); g.replay(); t2 = time.perf_counter()
torch.cuda.synchronize(); t3 = time.perf_counter()
print(f"same graph twice: first call {1e3 * (t1 - t0):.2f} ms, second call {1e3 * (t2 - t1):.2f} ms, total {1e3 * (t3 - t0):.2f} ms")
t0 = time.perf_counter(); g.replay(); t1 = time.perf_counter(); g2.replay(); t2 = time.perf_counter()
torch.cuda.synchronize(); t3 = time.perf_counter()
print(f"two graphs: first call {1e3 * (t1 - t0):.2f} ms, second call {1e3 * (t2 - t1):.2f} ms, total {1e3 * (t3 - t0):.2f} ms")
ev = torch.cuda.Event(); 
t0 = time.perf_counter(); g.replay(); ev.record(); t1 = time.perf_counter(); ev.synchronize(); t2 = time.perf_counter()
print(f"event after replay: record {1e3 * (t1 - t0):.2f} ms, sync {1e3 * (t2 - t1):.2f} ms")
h = torch.zeros(64, dtype=torch.int32).pin_memory(); d = torch.zeros(64, dtype=torch.int32, device="cuda")
t0 = time.perf_counter(); g.replay(); t1 = time.perf_counter(); d.copy_(h, non_blocking=True); t2 = time.perf_counter()
p = torch.tensor(list(range(64)), dtype=torch.int32); d.copy_(p, non_blocking=True); t3 = time.perf_counter()
torch.cuda.synchronize()
print(f"after replay: pinned H2D {1e3 * (t2 - t1):.3f} ms, pageable H2D non_blocking {1e3 * (t3 - t2):.3f} ms")
