"""Pipeline training over a 2-rank gloo ring (the same code runs RCCL p2p on MI355X): loss and
updated weights after two optimizer steps equal a single-process run of the full model with the
same micro-batches (GPipe accumulation == one big batch)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.models.config import PRESETS
from xotorch_support_jetson_amd.models.weights import random_weights
from xotorch_support_jetson_amd.parallel.comm import LoopbackTransport, P2PTransport
from xotorch_support_jetson_amd.parallel.pipeline_train import PipelineTrainer, TrainBatch
from xotorch_support_jetson_amd.topology.ring_memory_weighted_partitioning_strategy import equal_layer_shards
from xotorch_support_jetson_amd.train.trainer import ShardTrainer



def _batches(step):
  g = torch.Generator().manual_seed(7 + step)
  out = []
  for m in range(3):
    x = torch.randint(0, 512, (2, 12), generator=g)
    y = torch.roll(x, -1, 1)
    out.append(TrainBatch(x, y, torch.tensor([12, 7 + m])))
  return out


def _run(trainer, rank, world, transport, schedule="gpipe"):
  pt = PipelineTrainer(trainer, rank, world, transport, schedule=schedule)
  return [pt.step(_batches(s)) for s in range(2)]


def _worker(rank, world, port, q, MODEL, schedule):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    c = PRESETS[MODEL]
    shard = equal_layer_shards(MODEL, c.num_layers, world)[rank]
    tr = ShardTrainer(random_weights(c, shard, "cpu", seed=3), "cpu", lr=1e-3)
    losses = _run(tr, rank, world, P2PTransport(rank, world), schedule)
    # numpy, not torch tensors: a queued tensor is an fd into this process, gone once it exits
    q.put((rank, losses, {k: v.detach().float().numpy().copy() for k, v in tr.master.items()}))
    dist.barrier()
  finally:
    dist.destroy_process_group()


def _port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


# untied / tied embeddings; 1F1B over 3 ranks (warm-up forwards 2 / 1 / 0)
@pytest.mark.parametrize("MODEL,world,schedule", [("tiny-llama", 2, "gpipe"), ("tiny-llama-d64", 2, "gpipe"),
                                                  ("tiny-llama", 3, "1f1b")])
def test_pipeline_training_two_ranks_matches_single(MODEL, world, schedule):
  c = PRESETS[MODEL]
  full = ShardTrainer(random_weights(c, Shard(MODEL, 0, c.num_layers - 1, c.num_layers), "cpu", seed=3), "cpu",
                      lr=1e-3)
  ref_losses = _run(full, 0, 1, LoopbackTransport(0, 1))
  assert ref_losses[1] < ref_losses[0] + 1.0
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _port()
  procs = [ctx.Process(target=_worker, args=(r, world, port, q, MODEL, schedule)) for r in range(world)]
  for p in procs:
    p.start()
  try:
    res = {}
    for _ in range(world):
      r, losses, master = q.get(timeout=240)
      res[r] = (losses, master)
  finally:
    for p in procs:
      p.join(timeout=60)
      if p.is_alive():
        p.kill()
  assert all(p.exitcode == 0 for p in procs)
  # tied embeddings: one bf16 grad summed by autograd vs two bf16 grads summed in fp32 -> rounding-level
  # grad differences, which early Adam steps (update ~ lr * sign(g)) can turn into <= 2 lr per element
  tol = 1e-3 if c.tie_word_embeddings else 1e-4
  for r in range(world):
    for a, b in zip(res[r][0], ref_losses):
      assert abs(a - b) < tol, (r, res[r][0], ref_losses)
  merged = {k: torch.from_numpy(v) for r in range(world) for k, v in res[r][1].items()}
  for k, v in full.master.items():
    assert torch.allclose(v, merged[k], atol=1e-6 if tol < 1e-3 else 2e-3, rtol=1e-5), k
  if c.tie_word_embeddings:  # the last stage's head copy took the same update as the embedding
    assert torch.allclose(merged["lm_head"], torch.from_numpy(res[0][1]["embed"]), atol=1e-7)


def _worker_gpu(rank, world, port, q, MODEL):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    c = PRESETS[MODEL]
    shard = equal_layer_shards(MODEL, c.num_layers, world)[rank]
    dev = torch.device("cuda", 0)  # both ranks on the box's GPU, hand-offs staged through the host
    tr = ShardTrainer(random_weights(c, shard, dev, seed=3), dev, lr=1e-3)
    losses = _run(tr, rank, world, P2PTransport(rank, world))
    q.put((rank, losses, {k: v.detach().float().cpu().numpy().copy() for k, v in tr.master.items()},
           sorted(tr.acc)))
    dist.barrier()
  finally:
    dist.destroy_process_group()


@pytest.mark.gpu
def test_pipeline_tied_embedding_gpu_grad_acc():
  """On the GPU the embedding (first stage) and its head copy (last stage) accumulate their gradients in fp32
  GradAcc buffers (EMBED_ACC / the fused-CE dHead), not p.grad: the tied sum must read and write those, so both
  copies take the same update and match the single-GPU run of the whole model."""
  MODEL, world = "tiny-llama-d64", 2
  c = PRESETS[MODEL]
  dev = torch.device("cuda", 0)
  full = ShardTrainer(random_weights(c, Shard(MODEL, 0, c.num_layers - 1, c.num_layers), dev, seed=3), dev, lr=1e-3)
  init = full.master["embed"].float().cpu().clone()
  ref_losses = _run(full, 0, 1, LoopbackTransport(0, 1))
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _port()
  procs = [ctx.Process(target=_worker_gpu, args=(r, world, port, q, MODEL)) for r in range(world)]
  for p in procs:
    p.start()
  try:
    res = {}
    for _ in range(world):
      r, losses, master, accs = q.get(timeout=100)
      res[r] = (losses, master, accs)
  finally:
    for p in procs:
      p.join(timeout=60)
      if p.is_alive():
        p.kill()
  assert "embed" in res[0][2]  # the GradAcc path is the one under test
  assert torch.allclose(torch.from_numpy(res[1][1]["lm_head"]), torch.from_numpy(res[0][1]["embed"]), atol=1e-7)
  for r in range(world):
    for a, b in zip(res[r][0], ref_losses):
      assert abs(a - b) < 2e-2, (r, res[r][0], ref_losses)
  d_ref = full.master["embed"].float().cpu() - init
  d_got = torch.from_numpy(res[0][1]["embed"]) - init
  rel = float((d_got - d_ref).abs().mean() / d_ref.abs().mean())
  print(f"tied embedding update: mean relative difference {rel:.4f}")
  assert rel < 0.10, rel  # bf16 GEMMs on both sides: the update, not bit patterns
