"""One pp-N ring stage of the headline on ONE GPU: the work a rank of `bench.py --gpus N` does per decode tick,
measured without the other ranks (the driver's multi-GPU run is the only place they exist together).

For each requested rank r of an N-GPU ring (layer ranges from the same partitioner bench.py uses) this builds
that rank's shard, prefills `--batch` sequences of `--prompt-len` tokens through it (synthetic hidden states for
non-first stages), then times decode ticks exactly as RingStage.decode_tick runs them on that rank:
  first stage   embedding + its layers, and (split LM head) the head rows [Vs, V) + the sampler over the
                candidates handed over by the last stage
  middle stage  its layers
  last stage    its layers + final norm + head rows [0, Vs) + top-k candidates
Reported per rank: device ms per tick (one micro-batch through the stage).  With N micro-batches in flight the
ring's round time is N x the slowest stage's tick (plus any hand-off the compute does not hide), so

  predicted node tok/s = N * batch / (N * max_stage_ms)  = batch / max_stage_ms

  python tools/bench_stage.py --world 8 --ranks 0,3,7 [--batch 512] [--steps 10] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--model", default="llama-3-70b")
  ap.add_argument("--world", type=int, default=8)
  ap.add_argument("--ranks", default="0,7")
  ap.add_argument("--batch", type=int, default=512)
  ap.add_argument("--prompt-len", type=int, default=512)
  ap.add_argument("--steps", type=int, default=10)
  ap.add_argument("--warmup", type=int, default=4)
  ap.add_argument("--json", default=None)
  args = ap.parse_args()

  from xotorch_support_jetson_amd.models.config import preset
  from xotorch_support_jetson_amd.ops import kernels as K
  from xotorch_support_jetson_amd.parallel.comm import LoopbackTransport
  from xotorch_support_jetson_amd.parallel.pipeline import KC, MicroBatch, RingStage
  from xotorch_support_jetson_amd.runtime.runner import ShardRunner
  from xotorch_support_jetson_amd.topology.ring_memory_weighted_partitioning_strategy import equal_layer_shards

  dev = torch.device("cuda:0")
  cfg = preset(args.model)
  shards = equal_layer_shards(args.model, cfg.num_layers, args.world)
  B, L, D = args.batch, args.prompt_len, cfg.hidden_size
  max_ctx = L + args.warmup + args.steps + 8
  rows = []
  for r in [int(x) for x in args.ranks.split(",")]:
    sh = shards[r]
    t0 = time.time()
    runner = ShardRunner(cfg, sh, dev, num_pages=B * (-(-max_ctx // 64)) + 16, max_batch=B, max_ctx=max_ctx, seed=0)
    stage = RingStage(runner, r, args.world, LoopbackTransport(r, args.world))
    rids = [f"r{i}" for i in range(B)]
    mb = MicroBatch(rids, prompt=None, temps=torch.full((B,), 0.6, device=dev))
    g = torch.Generator(device=dev).manual_seed(r)
    per = max(1, 8192 // L)
    for lo in range(0, B, per):  # prefill in 8192-token chunks of whole sequences, as RingStage.prefill does
      n = min(per, B - lo)
      if stage.first:
        x = torch.randint(0, cfg.vocab_size, (n * L,), device=dev, dtype=torch.int32, generator=g)
      else:
        x = (torch.randn(n * L, D, device=dev, generator=g) * 0.5).to(torch.bfloat16)
      runner.forward(rids[lo:lo + n], [L] * n, x)
    torch.cuda.synchronize()
    t_pref = time.time() - t0

    # what this rank receives per tick
    if stage.first:
      item = (torch.randn(B, D, device=dev, generator=g).to(torch.bfloat16),
              torch.randn(B, KC, device=dev, generator=g).sort(dim=1, descending=True).values,
              torch.randint(0, stage.vs, (B, KC), device=dev, dtype=torch.int32, generator=g)) if stage.split else None
      ids = torch.randint(0, cfg.vocab_size, (B,), device=dev, dtype=torch.int32, generator=g)
    else:
      xin = (torch.randn(B, D, device=dev, generator=g) * 0.5).to(torch.bfloat16)

    def tick():
      if stage.first:
        x = stage._finish_head(*item, mb.temps) if stage.split else ids
      else:
        x = xin
      y = runner.forward(rids, [1] * B, x)
      if stage.last:
        stage._head_part(y) if stage.split else K.sample(y, mb.temps, 35, stage.seed_off)

    for _ in range(args.warmup):
      tick()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(args.steps):
      tick()
    en.record()
    en.synchronize()
    ms = st.elapsed_time(en) / args.steps
    row = dict(rank=r, world=args.world, layers=f"{sh.start_layer}-{sh.end_layer}", batch=B,
               first=stage.first, last=stage.last, split_head=stage.split, stage_ms=round(ms, 3),
               prefill_s=round(t_pref, 1))
    print(json.dumps(row), flush=True)
    rows.append(row)
    del stage, runner, mb
    torch.cuda.empty_cache()
  worst = max(x["stage_ms"] for x in rows)
  summary = dict(model=args.model, world=args.world, batch_per_gpu=B, max_stage_ms=worst,
                 predicted_node_tok_s=round(B / worst * 1e3, 1), stages=rows)
  print(json.dumps(summary), flush=True)
  if args.json:
    with open(args.json, "w") as f:
      json.dump(summary, f, indent=1)


if __name__ == "__main__":
  main()
