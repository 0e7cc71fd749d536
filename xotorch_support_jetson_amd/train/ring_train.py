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


def _load_stage(a: dict, cfg, mdir, shard, dev, src_dir: Optional[str], rank: int, iteration: Optional[int] = None):
  """Weights of `shard` (HF files or random init, then the newest complete checkpoint in `src_dir` if any)
  and its ShardTrainer (optimizer moments merged from every sidecar of that iteration: after a re-partition
  a stage's layers come from several old stages' files).  `iteration`: the one iteration every stage loads
  (chosen once for the whole model by the caller); None picks the newest complete one.  Returns (weights,
  trainer, iteration or 0)."""
  from ..models.weights import copy_weights_into, from_hf_state_dict, load_hf_weights, random_weights
  from ..train import checkpoint as ck
  from ..train.trainer import ShardTrainer
  model = a["model"]
  if mdir is not None and any(mdir.glob("*.safetensors")):
    w = load_hf_weights(mdir, cfg, shard, dev)
  else:
    w = random_weights(cfg, shard, dev, seed=0)
  it, files = 0, []
  if src_dir and ck.list_checkpoints(src_dir, model):
    it, files = ck.select_checkpoint_files(src_dir, shard, iteration)  # one partition, no overlapping files
    sd = ck._gather_tensors(files, shard, cfg.tie_word_embeddings)
    copy_weights_into(w, from_hf_state_dict(sd, cfg, shard, device=dev))
    if rank == 0:
      print(f"resumed {model} from iteration {it}", flush=True)
  tr = ShardTrainer(w, dev, lr=a["lr"], max_seq=4096)
  if files:
    from safetensors.torch import load_file
    state = {}
    for f in files:
      side = f.with_name(f.name.replace(".safetensors", ".optim.safetensors"))
      if side.exists():
        state.update({k: v.to(dev) for k, v in load_file(str(side)).items()})
    if state:
      tr.load_state_dict(state)
  return w, tr, it


def _failed_peers(e: BaseException, mon) -> Optional[list]:
  """The dead ranks behind a training exception, or None if it is not a peer failure.  A collective
  (gloo all-reduce) on a closed peer fails with a backend error before the heartbeat times out: wait for
  the monitor's verdict."""
  from ..parallel.health import PeerFailure
  if isinstance(e, PeerFailure):
    return list(e.dead)
  if isinstance(e, RuntimeError) and mon is not None and mon.failed.wait(mon.timeout + 4 * mon.interval + 1):
    return sorted(mon.dead)
  return None


def _worker(rank: int, world: int, port: int, a: dict) -> None:
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                    LOCAL_RANK=str(rank))
  import torch.distributed as dist
  from ..inference.shard import Shard
  from ..inference.tokenizers import _resolve_tokenizer
  from ..models import registry
  from ..models.config import load_config, preset
  from ..parallel.comm import P2PTransport, init_distributed
  from ..parallel.health import FaultInjector, HealthMonitor, reform_ring
  from ..parallel.pipeline_train import PipelineTrainer, TrainBatch
  from ..parallel.ring_serve import control_group, ring_shards
  from ..train.dataset import DEFAULT_DATA, load_dataset

  rank, world, dev = init_distributed()
  backend = dist.get_backend() if world > 1 else None
  model = a["model"]
  mdir = _model_dir(model)
  cfg = load_config(mdir) if mdir is not None else preset(model)
  dp = a.get("parallel") == "dp"
  tok = _resolve_tokenizer(mdir if mdir is not None else (registry.get_repo(model, "ShardedInferenceEngine") or "byte"),
                           cfg.vocab_size)
  train, valid, test = load_dataset(a["data"] or DEFAULT_DATA, lambda s: tok.encode(s))
  bs, mb = a["batch_size"], max(1, a["micro_batch"])
  hb_timeout = float(os.environ.get("XOT_HEARTBEAT_TIMEOUT", "30"))
  injector = None  # the environment's (tests) on the first ring; none after a re-form
  generation, src_dir, first_epoch = 0, a.get("resume"), 0
  src_it = None  # the iteration every stage loads after a re-form (picked once, for the whole model)

  class _Shim:  # save_shard_checkpoint wants engine.runner.weights / engine.trainer
    pass

  while True:
    if dp:
      shard = Shard(model, 0, cfg.num_layers - 1, cfg.num_layers)
    else:  # memory-weighted layer ranges in ring order (parallel/ring_serve.py:ring_shards)
      shard = ring_shards(model, cfg.num_layers, world, control_group() if world > 1 else None)[rank]
    w, tr, _ = _load_stage(a, cfg, mdir, shard, dev, src_dir, rank, src_it)
    mon = None
    if dp:
      from ..parallel.data_parallel import DataParallelTrainer
      pt = DataParallelTrainer(tr, rank, world)
    else:
      if world > 1 and os.environ.get("XOT_HEARTBEAT", "1") == "1":  # parallel/health.py
        mon = HealthMonitor(rank, world, timeout=hb_timeout, generation=generation).start()
      t = P2PTransport(rank, world, monitor=mon, injector=injector)
      pt = PipelineTrainer(tr, rank, world, t, schedule=a.get("schedule", "gpipe"))

    def to_micro(batch, rank=rank, world=world):
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

    if a["command"] == "eval":
      _run_eval(pt, test, bs, to_micro, dp, rank)
      break
    try:
      _train_epochs(a, pt, tr, w, shard, rank, world, dp, train, bs, to_micro, _Shim, first_epoch)
      break
    except Exception as e:
      dead = _failed_peers(e, mon)
      if dead is None or dp or 0 in dead or rank in dead:
        raise
      # a ring peer died or wedged: its layers and the in-flight step are gone.  The survivors re-form a
      # dense ring, re-partition the layers over it and reload the last complete checkpoint in place
      # (the reference re-partitions on the next request after a peer drops: orchestration/node.py:455-460).
      alive = [r for r in range(world) if r not in set(dead)]
      if mon is not None:
        mon.stop()
      generation += 1
      print(f"[rank {rank}] peer(s) {dead} failed: re-forming the training ring over {alive} "
            f"(generation {generation})", flush=True)
      del pt, tr, w
      if torch.cuda.is_available():
        torch.cuda.empty_cache()
      rank, world = reform_ring(alive, rank, generation, backend=backend)
      injector = FaultInjector("", rank)
      from ..train import checkpoint as ck
      save = a.get("save_dir")
      if save and ck.list_checkpoints(save, model):
        # one iteration for every stage and for the epoch counter: the newest that covers the WHOLE model
        # (a peer that died mid-save leaves the newest iteration with a gap another stage would not see)
        src_dir = save
        src_it = first_epoch = ck.select_checkpoint_files(save, Shard(model, 0, cfg.num_layers - 1, cfg.num_layers))[0]
      else:  # nothing saved by this run yet: restart it from its initial weights
        first_epoch, src_it = 0, None
      if rank == 0:
        print(f"restarting at epoch {first_epoch + 1} on {world} rank(s)", flush=True)
  if world > 1:
    if not dp and pt.t.monitor is not None:
      pt.t.monitor.stop()  # orderly exit: peers must not flag it
    dist.barrier()
    dist.destroy_process_group()


def _run_eval(pt, test, bs, to_micro, dp, rank) -> None:
  from ..train.dataset import iterate_batches
  tot, n = 0.0, 0
  for batch in iterate_batches(test, bs):
    micro = to_micro(batch)
    loss = _eval_dp(pt, micro) if dp else _eval(pt, micro)
    tot += loss * float(batch[2].sum())
    n += int(batch[2].sum())
  if rank == 0:
    print(f"eval | loss={tot / max(n, 1):.4f} tokens={n}", flush=True)


def _train_epochs(a, pt, tr, w, shard, rank, world, dp, train, bs, to_micro, _Shim, first_epoch: int = 0):
  from ..train import checkpoint as ck
  from ..train.dataset import iterate_batches
  for epoch in range(first_epoch, a["iters"]):
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
  for p in procs:
    p.join()
  rc = procs[0].exitcode or 0
  for r, p in enumerate(procs[1:], 1):
    if not p.exitcode:
      continue
    if _peer_failure_exit(p.exitcode):  # the survivors re-formed the ring without it
      print(f"training rank {r} died (exit {p.exitcode}); the ring recovered without it", flush=True)
    else:  # a crash (uncaught exception ...) is a failure of the run even if the survivors finished
      print(f"training rank {r} failed with exit code {p.exitcode}", flush=True)
      rc = rc or p.exitcode
  return rc


def _peer_failure_exit(code: int) -> bool:
  """Exit codes of a rank that vanished (killed by a signal, or the test fault injector's hard exit 17:
  parallel/health.py) -- what the ring's recovery is for -- as opposed to a rank that raised."""
  return code < 0 or code == 17
