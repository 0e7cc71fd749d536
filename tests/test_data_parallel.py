"""Data parallelism (2 ranks, gloo on CPU; the same code runs RCCL on MI355X): one optimizer step over
2 x 2 micro-batches with bucketed all-reduce from backward hooks == a single process stepping on all 4
micro-batches (loss normalised by the global token count, so the summed gradients are the same)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.models.config import PRESETS
from xotorch_support_jetson_amd.models.weights import random_weights
from xotorch_support_jetson_amd.parallel.pipeline_train import PipelineTrainer, TrainBatch
from xotorch_support_jetson_amd.train.trainer import ShardTrainer

MODEL = "tiny-llama"
LR = 1e-3


def _batches(n, seed):
  g = torch.Generator().manual_seed(seed)
  c = PRESETS[MODEL]
  out = []
  for _ in range(n):
    x = torch.randint(0, c.vocab_size, (2, 16), generator=g)
    out.append(TrainBatch(x, torch.roll(x, -1, 1), torch.tensor([16, 11])))
  return out


def _trainer():
  c = PRESETS[MODEL]
  sh = Shard(MODEL, 0, c.num_layers - 1, c.num_layers)
  return ShardTrainer(random_weights(c, sh, "cpu", seed=3), "cpu", lr=LR)


def _worker(rank, world, port, q, split=(2, 2)):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    from xotorch_support_jetson_amd.parallel.data_parallel import DataParallelTrainer
    tr = _trainer()
    dp = DataParallelTrainer(tr, rank, world, bucket_mb=0.25)  # small buckets: several all-reduces
    assert len(dp.buckets) > 2
    allb = _batches(sum(split), 7)
    lo = sum(split[:rank])
    losses = [dp.step(allb[lo:lo + split[rank]]) for _ in range(2)]
    if rank == 0:
      q.put((losses, {k: v.clone().numpy() for k, v in tr.master.items()}))
  finally:
    dist.destroy_process_group()


def _free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


@pytest.mark.parametrize("split", [(2, 2), (3, 1), (1, 0), (0, 2)])
def test_data_parallel_matches_single_process(split):
  """Even and uneven micro-batch counts per rank, including a rank with none (buckets fill in
  a different order on a rank with no backward, so launches must follow the bucket list, not readiness)."""
  ref = _trainer()
  from xotorch_support_jetson_amd.parallel.comm import LoopbackTransport
  pt = PipelineTrainer(ref, 0, 1, LoopbackTransport(0, 1))
  allb = _batches(sum(split), 7)
  ref_losses = [pt.step(allb) for _ in range(2)]
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_worker, args=(r, 2, port, q, split)) for r in range(2)]
  for p in procs:
    p.start()
  try:
    losses, master = q.get(timeout=240)
  finally:
    for p in procs:
      p.join(timeout=60)
      if p.is_alive():
        p.kill()
  assert all(p.exitcode == 0 for p in procs)
  for a, b in zip(losses, ref_losses):
    assert abs(a - b) < 1e-3 * max(1.0, abs(b)), (losses, ref_losses)
  init = _trainer().master
  for k, v in ref.master.items():
    d_ref = v - init[k]
    d_dp = torch.from_numpy(master[k]) - init[k]
    # AdamW's first steps move every weight by ~lr * sign(grad): compare the updates in bulk (elements
    # whose tiny gradient differs in sign between the two bf16 accumulation orders flip individually)
    rel = ((d_dp - d_ref).abs().mean() / (d_ref.abs().mean() + 1e-12)).item()
    assert rel < 0.05, (k, rel)


@pytest.mark.gpu
def test_data_parallel_gpu_side_stream_matches_pipeline(monkeypatch):
  """On the GPU the projections' weight gradients (and the untied LM head's) accumulate on a side stream
  (train/autograd_ops.py DW_STREAM); the data-parallel buckets copy them out in the last micro-batch's backward,
  after joining that stream.  One rank's DataParallelTrainer == the pipeline trainer (side stream on and off)."""
  from xotorch_support_jetson_amd.parallel.comm import LoopbackTransport
  from xotorch_support_jetson_amd.parallel.data_parallel import DataParallelTrainer
  import xotorch_support_jetson_amd.train.autograd_ops as A
  dev = torch.device("cuda", 0)
  c = PRESETS[MODEL]
  sh = Shard(MODEL, 0, c.num_layers - 1, c.num_layers)

  def run(kind, side):
    monkeypatch.setattr(A, "DW_STREAM", side)
    tr = ShardTrainer(random_weights(c, sh, "cpu", seed=3), dev, lr=LR)
    assert "lm_head" in tr.acc or "lm_head" not in tr.params
    pt = DataParallelTrainer(tr, 0, 1, bucket_mb=0.25) if kind == "dp" else PipelineTrainer(tr, 0, 1, LoopbackTransport(0, 1))
    losses = [pt.step(_batches(3, 7)) for _ in range(2)]
    torch.cuda.synchronize()
    return losses, {k: v.float().cpu() for k, v in tr.master.items()}

  init = _trainer().master
  ref_l, ref_m = run("pp", False)
  for kind, side in (("dp", True), ("pp", True), ("dp", False)):
    got_l, got_m = run(kind, side)
    for a, b in zip(got_l, ref_l):
      assert abs(a - b) < 1e-3 * max(1.0, abs(b)), (kind, side, got_l, ref_l)
    for k, v in ref_m.items():
      d_ref, d = v - init[k], got_m[k] - init[k]
      rel = ((d - d_ref).abs().mean() / (d_ref.abs().mean() + 1e-12)).item()
      assert rel < 0.05, (kind, side, k, rel)
