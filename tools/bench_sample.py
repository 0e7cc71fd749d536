"""Sampling kernel timing (top-k 35, temperature 0.7) for B = 1 / 128 / 512 rows of 128256 logits."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xotorch_support_jetson_amd.ops import kernels as K  # noqa: E402


def main():
  dev = torch.device("cuda:0")
  so = torch.tensor([1, 0], dtype=torch.int64, device=dev)
  for B in (1, 128, 512):
    logits = torch.randn(B, 128256, device=dev) * 3
    temps = torch.full((B,), 0.7, device=dev)
    tok = torch.empty(B, dtype=torch.int32, device=dev)
    for _ in range(3):
      K.sample(logits, temps, 35, so, tok)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(20):
      K.sample(logits, temps, 35, so, tok)
    en.record()
    en.synchronize()
    print(json.dumps({"sample_topk35": B, "us": st.elapsed_time(en) * 1e3 / 20}))


if __name__ == "__main__":
  main()
