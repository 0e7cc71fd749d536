"""Find which FP8 stream GEMM configuration crashes (diagnostic)."""
import sys
import torch
sys.path.insert(0, ".")
from xotorch_support_jetson_amd.ops._ext import require
from xotorch_support_jetson_amd.ops.weights_layout import quantize_fp8_rows, shuffle_for_stream8

dev = torch.device("cuda", 0)
M, N, K = 1, 1024, 2048
w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) / 32
q, sc = quantize_fp8_rows(w)
w8 = shuffle_for_stream8(q)
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
b = torch.randn(N, device=dev, dtype=torch.bfloat16)
ws1 = torch.empty(8 * M * N, device=dev, dtype=torch.float32)
for odt in (torch.float32, torch.bfloat16):
  for bias in (b, None):
    for ws in (ws1, None):
      y = torch.empty(M, N, device=dev, dtype=odt)
      print(odt, bias is not None, ws is not None, flush=True)
      require().gemm_stream8(x, w8, sc, y, bias, None, ws, 0, 1, 1)
      torch.cuda.synchronize()
      print("  ok", flush=True)
