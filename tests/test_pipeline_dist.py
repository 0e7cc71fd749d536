"""Ring pipeline across processes (gloo on CPU; the same code runs RCCL p2p on MI355X): 2 ranks, each
holding half of the layers, M=2 micro-batches in flight; greedy tokens must equal a single-process
full-model run, with the LM head on the last stage or split between the last and the first stage."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.models.config import PRESETS
from xotorch_support_jetson_amd.parallel.comm import P2PTransport
from xotorch_support_jetson_amd.parallel.pipeline import MicroBatch, RingStage, run_decode_steps
from xotorch_support_jetson_amd.runtime.runner import ShardRunner
from xotorch_support_jetson_amd.topology.ring_memory_weighted_partitioning_strategy import equal_layer_shards

MODEL = "tiny-llama"
B, L, STEPS = 3, 10, 5


def _prompts(m):
  g = torch.Generator().manual_seed(100 + m)
  return torch.randint(0, PRESETS[MODEL].vocab_size, (B, L), generator=g, dtype=torch.int32)


def _run(stage, n_mb):
  mbs = [MicroBatch([f"m{m}r{b}" for b in range(B)], prompt=_prompts(m), temps=torch.zeros(B)) for m in range(n_mb)]
  first = [stage.prefill(mb) for mb in mbs]
  for mb, t in zip(mbs, first):
    if t is not None and not stage.split:  # split head: the prefill token is drawn by the first stage
      mb.tokens.append(t.tolist())
  run_decode_steps(stage, mbs, STEPS, first_tokens=first if stage.last else None, record=True)
  return [mb.tokens for mb in mbs]


def _worker(rank, world, port, q, split):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    c = PRESETS[MODEL]
    shard = equal_layer_shards(MODEL, c.num_layers, world)[rank]
    runner = ShardRunner(c, shard, "cpu", max_batch=8, max_ctx=64)
    stage = RingStage(runner, rank, world, P2PTransport(rank, world), split_head=split)
    assert stage.split == split
    toks = _run(stage, 2)
    stage.t.drain()
    dist.barrier()
    if stage.samples:
      q.put(toks)
  finally:
    dist.destroy_process_group()


def _free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


@pytest.mark.parametrize("split", [False, True])
def test_two_rank_ring_matches_single_process(split):
  c = PRESETS[MODEL]
  full = ShardRunner(c, Shard(MODEL, 0, c.num_layers - 1, c.num_layers), "cpu", max_batch=8, max_ctx=64)
  from xotorch_support_jetson_amd.parallel.comm import LoopbackTransport
  ref = _run(RingStage(full, 0, 1, LoopbackTransport(0, 1)), 2)
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_worker, args=(r, 2, port, q, split)) for r in range(2)]
  for p in procs:
    p.start()
  try:
    got = q.get(timeout=240)
  finally:
    for p in procs:
      p.join(timeout=60)
      if p.is_alive():
        p.kill()
  assert all(p.exitcode == 0 for p in procs)
  assert len(ref[0]) == STEPS + 1
  if split:  # a round's tokens are drawn at the start of the next round: STEPS tokens, prefill's included
    assert got == [r[:STEPS] for r in ref]
  else:
    assert got == ref
