#!/usr/bin/env python3
"""Headline benchmark: output tokens/sec (whole node), Llama-3-70B ring-sharded across N MI355X.

  python bench.py --gpus N --steps K --warmup W            (N=1 runs in-process)
  torchrun --nproc-per-node N bench.py --gpus N ...         (one rank per GPU, RCCL p2p ring)

Each rank holds 80/N consecutive layers (ring memory-weighted partitioner).  The node serves
N x --batch-per-gpu sequences (weak scaling: per-GPU work per step is fixed: 80 layer-passes x batch-per-gpu
tokens) as N micro-batches (or --micro-batches K >= N of N x batch-per-gpu / K each), so the ring is full and
all GPUs work concurrently.
Prompts (--prompt-len tokens, synthetic ids) are prefilled through the real model, then W untimed
decode rounds, then K timed rounds; one round = every sequence in the node generates one token
(sampled on device with temperature / top-k 35, the reference's sampler).  Weights are random-init
bf16 with the exact Llama-3-70B architecture (no checkpoint download on the GPU box).
Timing: barrier + device sync on both sides of the K rounds, max over ranks.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def log(*a):
  print(*a, file=sys.stderr, flush=True)


def cfg_name(model: str) -> str:
  return {"llama-3-70b": "Llama-3-70B"}.get(model, model)


def sync():
  if torch.cuda.is_available():
    torch.cuda.synchronize()


class ClockSampler:
  """Board power / shader clock of this rank's GPU over the timed rounds (rocm-smi, read-only, ~0.3 s apart): a
  decode step is GEMM-bound at the board power cap, so a slow box shows up here (a lower sclk at the same cap)."""

  def __init__(self, device_index: int, enabled: bool = True):
    import shutil
    import threading
    self.idx = device_index
    self.samples = []
    self._stop = threading.Event()
    on = enabled and shutil.which("rocm-smi") is not None
    self._t = threading.Thread(target=self._run, daemon=True) if on else None

  def _one(self):
    import re
    import subprocess
    r = subprocess.run(["rocm-smi", "-d", str(self.idx), "--showpower", "--showclocks", "--json"],
                       capture_output=True, text=True, timeout=10)
    card = next(iter(json.loads(r.stdout).values()))
    power = sclk = None
    for k, v in card.items():
      if "Power" in k and power is None:
        try:
          power = float(str(v).split()[0])
        except ValueError:
          pass
      if "sclk" in k.lower() and sclk is None:  # ("sclk clock speed:" "(2100Mhz)"; the level key has no MHz)
        m = re.search(r"(\d+)\s*Mhz", str(v), re.I)
        sclk = float(m.group(1)) if m else None
    return power, sclk

  def _run(self):
    while not self._stop.is_set():
      try:
        self.samples.append(self._one())
      except Exception:  # noqa: BLE001 - diagnostics only
        pass
      self._stop.wait(0.3)

  def __enter__(self):
    if self._t is not None:
      self._t.start()
    return self

  def __exit__(self, *exc):
    self._stop.set()
    if self._t is not None:
      self._t.join(15)

  def summary(self) -> dict:
    ps = [p for p, _ in self.samples if p is not None]
    cs = [c for _, c in self.samples if c is not None]
    mean = lambda xs: round(sum(xs) / len(xs), 1) if xs else None  # noqa: E731
    return {"samples": len(self.samples), "power_w_mean": mean(ps), "power_w_max": max(ps) if ps else None,
            "sclk_mhz_mean": mean(cs), "sclk_mhz_min": min(cs) if cs else None}


def gemm_choices(batch: int) -> dict:
  """The GEMM configuration the warmup tuner chose for each decode projection shape of this batch (kernel, tile
  code | n-tiles, K split): what a fresh box picked, so a slow record can be told from a different tile pick."""
  from xotorch_support_jetson_amd.ops import linear as L
  mb = L._m_bucket(batch)
  out = {"_source": "seed table (ops/gemm_seed_mi355x.json) under the box's own" if L.policy.seeded else "tuned"}
  for k, v in L.policy.table.items():
    if len(k) >= 5 and k[0] == "sh" and k[1] == mb:
      out[f"N{k[2]} K{k[3]} {k[4]}"] = list(v) if isinstance(v, tuple) else v
  return out


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--gpus", type=int, default=1)
  ap.add_argument("--steps", type=int, default=16)
  ap.add_argument("--warmup", type=int, default=3)
  ap.add_argument("--model", default="llama-3-70b")
  ap.add_argument("--batch-per-gpu", type=int, default=int(os.environ.get("XOT_BENCH_BATCH", 512)))
  ap.add_argument("--micro-batches", type=int, default=0,
                  help="micro-batches circulating in the ring (default: one per stage).  The node's batch stays "
                       "gpus x batch-per-gpu; 2 x gpus micro-batches of half the size give every stage a spare "
                       "micro-batch to run while a hand-off is in flight (hop latency / stage jitter slack)")
  ap.add_argument("--prompt-len", type=int, default=512)
  ap.add_argument("--temperature", type=float, default=0.6)
  ap.add_argument("--layers", type=int, default=0, help="debug only: truncate the model (result marked invalid)")
  ap.add_argument("--dump-tokens", default=None,
                  help="tests: the sampling rank writes micro-batch 0's generated ids (JSON) to this path; the "
                       "per-step host reads make the timing meaningless")
  ap.add_argument("--weight-dtype", default="bf16", choices=["bf16", "fp8"],
                  help="fp8: weight-only e4m3 projections (a separate, reduced-precision measurement; the headline "
                       "is bf16)")
  args = ap.parse_args()
  os.environ["XOT_WEIGHT_DTYPE"] = args.weight_dtype

  from xotorch_support_jetson_amd.models.config import preset
  from xotorch_support_jetson_amd.parallel.comm import P2PTransport, init_distributed
  from xotorch_support_jetson_amd.parallel.pipeline import MicroBatch, RingStage, run_decode_steps
  from xotorch_support_jetson_amd.runtime.runner import ShardRunner
  from xotorch_support_jetson_amd.topology.ring_memory_weighted_partitioning_strategy import equal_layer_shards
  import torch.distributed as dist

  rank, world, dev = init_distributed()
  if world != args.gpus:
    raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
  cfg = preset(args.model)
  if args.layers:
    cfg = cfg.with_layers(args.layers)
  shards = equal_layer_shards(args.model, cfg.num_layers, world)
  assert len(shards) == world, shards
  shard = shards[rank]
  M = args.micro_batches or world  # micro-batches in flight >= stages, so the ring is always full
  if M < world or (args.batch_per_gpu * world) % M:
    raise SystemExit(f"--micro-batches {M}: needs >= {world} and to divide {args.batch_per_gpu * world} sequences")
  B = args.batch_per_gpu * world // M  # sequences per micro-batch
  max_ctx = args.prompt_len + args.warmup + args.steps + 8
  pages_per_seq = -(-max_ctx // 64)
  t0 = time.time()
  runner = ShardRunner(cfg, shard, dev, num_pages=M * B * pages_per_seq + 16, max_batch=B, max_ctx=max_ctx,
                       seed=0)
  sync()
  t_init = time.time() - t0
  log(f"[rank {rank}] shard {shard.start_layer}-{shard.end_layer} weights {runner.weights.nbytes() / 1e9:.1f} GB "
      f"kv {runner.kv.nbytes() / 1e9:.1f} GB init {t_init:.1f}s")

  transport = P2PTransport(rank, world)
  stage = RingStage(runner, rank, world, transport)
  g = torch.Generator().manual_seed(1234)
  mbs = []
  for m in range(M):
    rids = [f"mb{m}-r{i}" for i in range(B)]
    prompt = torch.randint(0, cfg.vocab_size, (B, args.prompt_len), generator=g, dtype=torch.int32)
    mbs.append(MicroBatch(rids, prompt=prompt, temps=torch.full((B,), args.temperature, device=dev)))

  # ---- prefill (real forward through every stage)
  if world > 1:
    dist.barrier()
  sync()
  t0 = time.time()
  first = [stage.prefill(mb) for mb in mbs]
  transport.drain()
  sync()
  t_prefill = time.time() - t0
  log(f"[rank {rank}] prefill {M * B} x {args.prompt_len} tokens in {t_prefill:.1f}s")

  # ---- warmup rounds (graph capture + GEMM policy tuning happen here)
  rec = args.dump_tokens is not None
  toks = run_decode_steps(stage, mbs, args.warmup, first_tokens=first if stage.last else None, record=rec)
  transport.drain()
  sync()
  log(f"[rank {rank}] warmup done")

  # ---- timed rounds
  if world > 1:
    dist.barrier()
  sync()
  stage.start_timing()  # device events around each tick: stage work vs. waiting for the previous stage
  sent0 = transport.sent_bytes
  clocks = ClockSampler(dev.index or 0, enabled=dev.type == "cuda")
  with clocks:
    t0 = time.perf_counter()
    toks = run_decode_steps(stage, mbs, args.steps, first_tokens=toks if stage.last else None, record=rec)
    transport.drain()
    sync()
    if world > 1:
      dist.barrier()
    elapsed = time.perf_counter() - t0
  if world > 1:
    e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    elapsed = float(e.item())

  # per-rank diagnostics (after the timed region): a multi-GPU run that under-delivers shows which stage is
  # the slow one (stage_ms) and where the ring starves (recv_wait_ms)
  mine = dict(rank=rank, layers=f"{shard.start_layer}-{shard.end_layer}", **stage.timing(),
              send_mb_per_step=round((transport.sent_bytes - sent0) / args.steps / 1e6, 3),
              gpu=clocks.summary(), gemm=gemm_choices(B))
  per_rank = [mine]
  if world > 1:
    per_rank = [None] * world
    dist.all_gather_object(per_rank, mine)

  if rec and stage.samples:
    with open(args.dump_tokens, "w") as f:
      json.dump(mbs[0].tokens, f)
  total_tokens = args.steps * M * B
  tps = total_tokens / elapsed
  ms_step = elapsed / args.steps * 1e3
  if rank == 0:
    out = {
      "metric": ("output tokens/sec (whole node) Llama-3-70B ring-sharded across 1/2/4/8 MI355X"
                 if args.model == "llama-3-70b" else f"output tokens/sec (whole node) {args.model} ring-sharded"),
      "value": round(tps, 2),
      "unit": "tokens/s",
      "n_gpus": world,
      "steps": args.steps,
      "warmup": args.warmup,
      "ms_per_step": round(ms_step, 3),
      "higher_is_better": True,
      "scaling": "weak",
      "vs_baseline": None,
      "dtype": "bf16" if args.weight_dtype == "bf16" else "bf16 activations, fp8-e4m3 weights (NOT the headline)",
      "data": f"synthetic prompts, random-init weights (exact {cfg_name(args.model)} architecture)",
      "config": {
        "model": args.model if not args.layers else f"{args.model}-TRUNCATED-{args.layers}L-INVALID",
        "global_batch": M * B,
        "seq_len": args.prompt_len,
        "parallelism": f"pp{world} (ring, {M} micro-batches x {B})",
        "batch_per_gpu": args.batch_per_gpu,
        "micro_batches": M,
        "micro_batch_size": B,
        "decode_context": f"{args.prompt_len + args.warmup}..{args.prompt_len + args.warmup + args.steps}",
        "sampling": f"temperature {args.temperature}, top-k 35 (on-device)",
        "weight_dtype": args.weight_dtype,
      },
      "extra": {"prefill_s": round(t_prefill, 2), "init_s": round(t_init, 2),
                "tokens_per_s_per_gpu": round(tps / world, 2),
                "reference_derived_ceiling_tok_s": 0.57 if world == 8 else (2.3 if world == 2 else None),
                "per_rank": per_rank},
    }
    print(json.dumps(out), flush=True)
  if world > 1:
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
  main()
