#!/usr/bin/env python3
"""Host overhead of one engine decode step (ShardedInferenceEngine._infer_batch) vs. the runner's forward
alone, at serving batch sizes, on one GPU: python tools/diag/prof_engine_step.py [B ...]"""
import asyncio
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


async def main(bs):
  from xotorch_support_jetson_amd.download.shard_download import NoopShardDownloader
  from xotorch_support_jetson_amd.inference import sharded_engine as se
  from xotorch_support_jetson_amd.inference.shard import Shard
  os.environ["XOT_MAX_BATCH"] = str(max(bs))
  eng = se.ShardedInferenceEngine(NoopShardDownloader())
  shard = Shard("llama-3-8b", 0, 31, 32)
  await eng.ensure_shard(shard)
  state = {"temperature": 0.6, "top_k": 35}
  for B in bs:
    pre = [(f"b{B}r{i}", np.arange(100, dtype=np.int64).reshape(1, -1) + i, state) for i in range(B)]
    eng._infer_batch(pre)
    dec = [(f"b{B}r{i}", np.asarray([[7]], dtype=np.int64), state, True) for i in range(B)]  # engine-loop items
    for _ in range(3):
      eng._infer_batch(dec)
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
      eng._infer_batch(dec)
    t_eng = (time.perf_counter() - t0) / n
    rids = [it[0] for it in dec]
    x = torch.full((B,), 7, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
      eng.runner.forward(rids, [1] * B, x)
    torch.cuda.synchronize()
    t_fwd = (time.perf_counter() - t0) / n
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
      eng._infer_batch(dec)
    pr.disable()
    print(f"B={B}: engine step {t_eng * 1e3:.2f} ms, runner forward alone {t_fwd * 1e3:.2f} ms", flush=True)
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
    for rid in rids:
      eng.runner.free(rid)


if __name__ == "__main__":
  asyncio.run(main([int(a) for a in sys.argv[1:]] or [64, 256]))
