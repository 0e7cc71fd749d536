#!/usr/bin/env python3
"""BASELINE config 5: Llama-3-8B fine-tune pipeline-sharded across N peers (one per GPU).

  python tools/bench_train.py [--model llama-3-8b] [--seq 2048] [--mb 1] [--microbatches M]
  torchrun --nproc-per-node N tools/bench_train.py --gpus N [--parallel pp|dp]

Each rank holds 32/N layers as a ShardTrainer (HIP RMSNorm/SiLU/RoPE/cross-entropy fwd+bwd kernels,
fused AdamW on fp32 master weights, hipBLASLt GEMMs, flash-style HIP attention fwd/bwd); activations go forward and
gradients backward over RCCL p2p in a GPipe schedule (parallel/pipeline_train.py).  Synthetic token
data, random-init weights of the exact architecture.  Prints one JSON line: trained tokens/s of the
whole job (max step time over ranks), plus the loss curve.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sync():
  if torch.cuda.is_available():
    torch.cuda.synchronize()


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--gpus", type=int, default=1)
  ap.add_argument("--model", default="llama-3-8b")
  ap.add_argument("--layers", type=int, default=0,
                  help="stage-sized run: only this many layers (e.g. one pp8 stage's share); labelled in the output")
  ap.add_argument("--seq", type=int, default=2048)
  ap.add_argument("--mb", type=int, default=1, help="sequences per micro-batch")
  ap.add_argument("--microbatches", type=int, default=0, help="micro-batches per step (default max(8, 4N))")
  ap.add_argument("--steps", type=int, default=4)
  ap.add_argument("--warmup", type=int, default=1)
  ap.add_argument("--lr", type=float, default=1e-5)
  ap.add_argument("--parallel", choices=("pp", "dp"), default="pp",
                  help="pp: layer pipeline (the reference's strategy); dp: full replica per GPU, bucketed "
                       "all-reduce overlapped with backward (parallel/data_parallel.py)")
  ap.add_argument("--schedule", choices=("gpipe", "1f1b"), default="gpipe", help="pp micro-batch order")
  ap.add_argument("--torch-prof", default="",
                  help="after the timed steps, profile one more step with torch.profiler and write the per-op table "
                       "(device time of the torch ops that are not own kernels, with their Python call sites) here")
  args = ap.parse_args()

  import torch.distributed as dist
  from xotorch_support_jetson_amd.models.config import preset
  from xotorch_support_jetson_amd.models.weights import random_weights
  from xotorch_support_jetson_amd.parallel.comm import P2PTransport, init_distributed
  from xotorch_support_jetson_amd.parallel.pipeline_train import PipelineTrainer, TrainBatch
  from xotorch_support_jetson_amd.topology.ring_memory_weighted_partitioning_strategy import equal_layer_shards
  from xotorch_support_jetson_amd.train.trainer import ShardTrainer

  rank, world, dev = init_distributed()
  if world != args.gpus:
    raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
  cfg = preset(args.model)
  if args.layers:
    cfg = cfg.with_layers(args.layers)
  dp = args.parallel == "dp"
  if dp:
    from xotorch_support_jetson_amd.inference.shard import Shard
    from xotorch_support_jetson_amd.parallel.data_parallel import DataParallelTrainer
    shard = Shard(args.model, 0, cfg.num_layers - 1, cfg.num_layers)
    M = args.microbatches or 8  # per rank
  else:
    shard = equal_layer_shards(args.model, cfg.num_layers, world)[rank]
    M = args.microbatches or max(8, 4 * world)
  t0 = time.time()
  tr = ShardTrainer(random_weights(cfg, shard, dev, seed=0), dev, lr=args.lr, max_seq=args.seq)
  pt = DataParallelTrainer(tr, rank, world) if dp else PipelineTrainer(tr, rank, world, P2PTransport(rank, world),
                                                                      schedule=args.schedule)
  sync()
  print(f"[rank {rank}] layers {shard.start_layer}-{shard.end_layer} init {time.time() - t0:.1f}s", file=sys.stderr)

  g = torch.Generator().manual_seed(1234)

  def batches():
    out = []
    for _ in range(M):
      x = torch.randint(0, cfg.vocab_size, (args.mb, args.seq), generator=g)
      out.append(TrainBatch(x, torch.roll(x, -1, 1), torch.full((args.mb,), args.seq)))
    return out

  losses = []
  for _ in range(args.warmup):
    losses.append(pt.step(batches()))
  data = [batches() for _ in range(args.steps)]
  if world > 1:
    dist.barrier()
  sync()
  t0 = time.perf_counter()
  for b in data:
    losses.append(pt.step(b))
  sync()
  if world > 1:
    dist.barrier()
  el = time.perf_counter() - t0
  if world > 1:
    e = torch.tensor([el], dtype=torch.float64, device=dev)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    el = float(e)
  tokens = args.steps * M * args.mb * args.seq * (world if dp else 1)
  if rank == 0:
    print(json.dumps({
      "metric": (f"training tokens/sec (whole node) {args.model} data-parallel across {world} MI355X" if dp else
                 f"training tokens/sec (whole node) {args.model} pipeline-sharded across {world} MI355X"),
      "value": round(tokens / el, 1), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
      "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 1), "higher_is_better": True,
      "scaling": "weak" if args.microbatches == 0 else "strong", "dtype": "bf16 (fp32 master + AdamW)",
      "data": "synthetic tokens, random-init weights", "losses": [round(l, 4) for l in losses],
      "config": {"model": args.model + (f" ({args.layers} of {preset(args.model).num_layers} layers)" if args.layers else ""), "seq_len": args.seq, "micro_batch": args.mb, "micro_batches": M,
                 "global_batch_tokens": M * args.mb * args.seq * (world if dp else 1),
                 "parallelism": (f"dp{world} (bucketed all-reduce overlapped with backward)" if dp else
                                 f"pp{world} ({args.schedule}, RCCL p2p)")},
    }), flush=True)
  if args.torch_prof and rank == 0:
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
      pt.step(batches())
      sync()
    with open(args.torch_prof, "w") as f:
      f.write(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=60) + "\n")
      f.write(prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=40) + "\n")
  if world > 1:
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
  main()
