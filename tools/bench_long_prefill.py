#!/usr/bin/env python3
"""Long-context prefill on one peer: time to first token of one prompt of --tokens synthetic ids, prefilled
in MAX_STEP_TOKENS chunks through the paged cache (chunked prefill), then --decode decode steps at that
context.  The reference's engine sizes its KV cache at prompt + 1024 tokens and ships an O(T^2) mask
per hop; here the context is bounded by the KV pool only.
  python tools/bench_long_prefill.py --model llama-3-8b --tokens 32768"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--model", default="llama-3-8b")
  ap.add_argument("--tokens", type=int, default=32768)
  ap.add_argument("--chunk", type=int, default=8192)
  ap.add_argument("--decode", type=int, default=32)
  a = ap.parse_args()
  from xotorch_support_jetson_amd.inference.shard import Shard
  from xotorch_support_jetson_amd.models.config import preset
  from xotorch_support_jetson_amd.runtime.runner import ShardRunner
  c = preset(a.model)
  dev = torch.device("cuda", 0)
  sh = Shard(a.model, 0, c.num_layers - 1, c.num_layers)
  r = ShardRunner(c, sh, dev, max_batch=1, max_ctx=a.tokens + a.decode + 64, seed=0)
  ids = torch.randint(0, c.vocab_size, (a.tokens,), generator=torch.Generator().manual_seed(0)).to(torch.int32)

  def prefill(rid):
    out = None
    for lo in range(0, a.tokens, a.chunk):
      x = ids[lo:lo + a.chunk].to(dev)
      out = r.forward([rid], [x.numel()], x)
    return out
  prefill("warm")  # GEMM policy tuning for the chunk shapes
  r.free("warm")
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  out = prefill("q")
  torch.cuda.synchronize()
  ttft = time.perf_counter() - t0
  tok = out.argmax(-1).to(torch.int32).view(1)
  for _ in range(3):  # graph capture + warm-up at this context
    tok = r.forward(["q"], [1], tok).argmax(-1).to(torch.int32).view(1)
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for _ in range(a.decode):
    tok = r.forward(["q"], [1], tok).argmax(-1).to(torch.int32).view(1)
  torch.cuda.synchronize()
  dec = (time.perf_counter() - t0) / a.decode
  flops = 2 * a.tokens * c.params_per_layer(0) * c.num_layers + 2 * a.tokens ** 2 * c.num_heads * c.head_dim * c.num_layers
  print(json.dumps({"model": a.model, "prompt_tokens": a.tokens, "chunk": a.chunk, "ttft_s": round(ttft, 3),
                    "prefill_tok_s": round(a.tokens / ttft, 1), "prefill_TFLOPs": round(flops / ttft / 1e12, 1),
                    "decode_ms_at_context": round(dec * 1e3, 3), "dtype": "bf16",
                    "data": "random-init weights, synthetic ids"}), flush=True)


if __name__ == "__main__":
  main()
