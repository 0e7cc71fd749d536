"""`xot train|eval <model> --gpus N --ring [--parallel pp|dp]`: training / evaluation on the local GPUs
over RCCL / xGMI instead of gRPC SendExample hops: the layer pipeline (parallel/pipeline_train.py) or
data-parallel replicas (parallel/data_parallel.py; each rank takes every world-th micro-batch).

Same data (`--data` JSONL dir, `batch_with_lengths`), same checkpoint files as the Node path
(`train/checkpoint.py` names, HF tensor names, optimizer sidecars) so a ring-trained checkpoint
loads into `xot run` on any partitioning and `--resume-checkpoint` works both ways.
"""
from __future__ import annotations

import os
import socket
from pathlib import Path
from typing import Optional

import torch


def _free_port() -> int:
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


def _model_dir(model_id: str) -> Optional[Path]:
  from ..helpers import xot_home
  from ..models import registry
  repo = registry.get_repo(model_id, "ShardedInferenceEngine")
  if repo is None:
    return None
  p = xot_home() / "downloads" / repo.replace("/", "--")
  return p if (p / "config.json").exists() else None


def _worker(rank: int, world: int, port: int, a: dict) -> None:
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                    LOCAL_RANK=str(rank))
  import torch.distributed as dist
  from ..inference.tokenizers import _resolve_tokenizer
  from ..models import registry
  from ..models.config import load_config, preset
  from ..models.weights import load_hf_weights, random_weights
  from ..parallel.comm import P2PTransport, init_distributed
  from ..parallel.pipeline_train import PipelineTrainer, TrainBatch
  from ..topology.ring_memory_weighted_partitioning_strategy import equal_layer_shards
  from ..train import checkpoint as ck
  from ..train.dataset import DEFAULT_DATA, iterate_batches, load_dataset
  from ..train.trainer import ShardTrainer

  rank, world, dev = init_distributed()
  model = a["model"]
  mdir = _model_dir(model)
  cfg = load_config(mdir) if mdir is not None else preset(model)
  dp = a.get("parallel") == "dp"
  if dp:
    from ..inference.shard import Shard
    shard = Shard(model, 0, cfg.num_layers - 1, cfg.num_layers)
  else:
    shard = equal_layer_shards(model, cfg.num_layers, world)[rank]
  if mdir is not None and any(mdir.glob("*.safetensors")):
    w = load_hf_weights(mdir, cfg, shard, dev)
  else:
    w = random_weights(cfg, shard, dev, seed=0)
  if a.get("resume") and ck.list_checkpoints(a["resume"], model):
    latest, files = ck.select_checkpoint_files(a["resume"], shard)  # one partition, no overlapping files
    sd = ck._gather_tensors(files, shard, cfg.tie_word_embeddings)
    from ..models.weights import copy_weights_into, from_hf_state_dict
    copy_weights_into(w, from_hf_state_dict(sd, cfg, shard, device=dev))
    if rank == 0:
      print(f"resumed {model} from iteration {latest}", flush=True)
  tr = ShardTrainer(w, dev, lr=a["lr"], max_seq=4096)
  if a.get("resume"):  # optimizer state of this exact shard, when the partitioning is unchanged
    files = ck.list_checkpoints(a["resume"], model)
    if files:
      side = ck.checkpoint_path(a["resume"], shard, files[-1][0])
      side = side.with_name(side.name.replace(".safetensors", ".optim.safetensors"))
      if side.exists():
        from safetensors.torch import load_file
        tr.load_state_dict({k: v.to(dev) for k, v in load_file(str(side)).items()})
  if dp:
    from ..parallel.data_parallel import DataParallelTrainer
    pt = DataParallelTrainer(tr, rank, world)
  else:
    mon = None
    if world > 1 and os.environ.get("XOT_HEARTBEAT", "1") == "1":  # parallel/health.py
      from ..parallel.health import HealthMonitor
      mon = HealthMonitor(rank, world, timeout=float(os.environ.get("XOT_HEARTBEAT_TIMEOUT", "30"))).start()
    pt = PipelineTrainer(tr, rank, world, P2PTransport(rank, world, monitor=mon), schedule=a.get("schedule", "gpipe"))
  tok = _resolve_tokenizer(mdir if mdir is not None else (registry.get_repo(model, "ShardedInferenceEngine") or "byte"),
                           cfg.vocab_size)
  train, valid, test = load_dataset(a["data"] or DEFAULT_DATA, lambda s: tok.encode(s))
  bs, mb = a["batch_size"], max(1, a["micro_batch"])

  def to_micro(batch):
    x, y, ln = batch
    lo, hi = 0, x.shape[0]
    if dp:  # data parallel: this rank's contiguous share of the rows (sizes differ by at most one; a
      # batch with fewer rows than ranks leaves some ranks without work -- they still join every
      # all-reduce, in the same order, with zero gradients: parallel/data_parallel.py)
      lo, hi = rank * x.shape[0] // world, (rank + 1) * x.shape[0] // world
    out = []
    for i in range(lo, hi, mb):
      j = min(i + mb, hi)
      out.append(TrainBatch(torch.from_numpy(x[i:j]), torch.from_numpy(y[i:j]), torch.from_numpy(ln[i:j])))
    return out

  class _Shim:  # save_shard_checkpoint wants engine.runner.weights / engine.trainer
    pass

  if a["command"] == "eval":
    tot, n = 0.0, 0
    for batch in iterate_batches(test, bs):
      micro = to_micro(batch)
      loss = _eval_dp(pt, micro) if dp else _eval(pt, micro)
      tot += loss * float(batch[2].sum())
      n += int(batch[2].sum())
    if rank == 0:
      print(f"eval | loss={tot / max(n, 1):.4f} tokens={n}", flush=True)
  else:
    try:
      _train_epochs(a, pt, tr, w, shard, rank, world, dp, train, bs, to_micro, _Shim)
    except Exception as e:
      from ..parallel.health import PeerFailure
      if not isinstance(e, PeerFailure):
        raise
      # a ring peer died or wedged: its layers (and the in-flight step) are gone.  Exit without the
      # closing barrier; `xot train --resume-checkpoint DIR` re-partitions the last saved iteration
      # (HF key names, any layer split) over the peers that are left.
      print(f"[rank {rank}] {e}; stopping, resume from the last checkpoint", flush=True)
      os._exit(75)
  if world > 1:
    if not dp and pt.t.monitor is not None:
      pt.t.monitor.stop()  # orderly exit: peers must not flag it
    dist.barrier()
    dist.destroy_process_group()


def _train_epochs(a, pt, tr, w, shard, rank, world, dp, train, bs, to_micro, _Shim):
  from ..train import checkpoint as ck
  from ..train.dataset import iterate_batches
  for epoch in range(a["iters"]):
    tot, n = 0.0, 0
    for batch in iterate_batches(train, bs, train=True, seed=epoch):
      loss = pt.step(to_micro(batch))
      tot += loss * float(batch[2].sum())
      n += int(batch[2].sum())
    if rank == 0:
      print(f"epoch {epoch + 1}/{a['iters']}\t| loss: {tot / max(n, 1):.4f}, tokens: {n}", flush=True)
    if a["save_every"] > 0 and (epoch + 1) % a["save_every"] == 0 and a["save_dir"] and (rank == 0 or not dp):
      tr.sync_to_inference()
      shim = _Shim()
      shim.runner = type("R", (), {"weights": w})()
      shim.trainer = tr
      path = ck.checkpoint_path(a["save_dir"], shard, epoch + 1)
      ck.save_shard_checkpoint(shim, shard, path)
      print(f"[rank {rank}] saved {path}", flush=True)


@torch.no_grad()
def _eval(pt, micro) -> float:
  """Forward-only pass of the pipeline; mean loss on the last stage, broadcast over the ring."""
  import torch.distributed as dist
  tr = pt.tr
  denom = float(sum(int(b.lengths.sum()) for b in micro))
  total = torch.zeros(1, device=pt.dev)
  for b in micro:
    mbs, L = b.x.shape
    if pt.first:
      inp = b.x.to(pt.dev)
    else:
      inp = torch.empty(mbs, L, pt.D, dtype=torch.bfloat16, device=pt.dev)
      pt.t.irecv(inp, pt.prev).wait()
    out = tr.forward(inp if pt.first else inp.to(torch.bfloat16))
    if pt.last:
      loss, _ = tr.loss_of(out, b.y, b.lengths, denom)
      total += loss.float()
    else:
      pt.t.isend(out.contiguous(), pt.next)
  pt.t.drain()
  if pt.world > 1:
    dist.all_reduce(total)
  return float(total)


@torch.no_grad()
def _eval_dp(pt, micro) -> float:
  """Data-parallel evaluation: each rank its micro-batches, token-weighted losses summed over ranks."""
  import torch.distributed as dist
  tr = pt.tr
  denom = pt._global_tokens(micro)
  total = torch.zeros(1, device=pt.dev)
  for b in micro:
    out = tr.forward(b.x.to(pt.dev))
    loss, _ = tr.loss_of(out, b.y, b.lengths, denom)
    total += loss.float()
  if pt.world > 1:
    total = total if dist.get_backend() == "nccl" else total.cpu()
    dist.all_reduce(total)
  return float(total)


def run_ring(args) -> int:
  """Spawn one training process per GPU (torch.multiprocessing, RCCL process group)."""
  import torch.multiprocessing as mp
  n = args.gpus or max(1, torch.cuda.device_count())
  a = {"model": args.model_name or args.default_model, "command": args.command, "data": args.data,
       "batch_size": args.batch_size, "micro_batch": getattr(args, "micro_batch", 1), "iters": args.iters,
       "save_every": args.save_every, "save_dir": args.save_checkpoint_dir, "resume": args.resume_checkpoint,
       "lr": args.lr, "parallel": getattr(args, "parallel", "pp"), "schedule": getattr(args, "schedule", "gpipe")}
  if not a["model"]:
    print("Error: model name is required")
    return 1
  port = _free_port()
  if n == 1:
    _worker(0, 1, port, a)
    return 0
  ctx = mp.get_context("spawn")
  procs = [ctx.Process(target=_worker, args=(r, n, port, a)) for r in range(n)]
  for p in procs:
    p.start()
  rc = 0
  for p in procs:
    p.join()
    rc = rc or (p.exitcode or 0)
  return rc
