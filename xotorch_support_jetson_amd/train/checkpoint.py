"""Per-shard checkpoints (reference design: node.py:230-252 + the unimplemented save_checkpoint).

File: {dir}/{model_id}/{start:03d}-{end:03d}-of-{n:03d}-{iteration:06d}.safetensors with HF tensor names
(un-shuffled, gate/up split), so a checkpoint written by one partition can be loaded by any other:
loading picks every tensor of the requested layer range from the shard files of the newest complete\niteration.
Those files must form ONE partition of the model (disjoint layer ranges, same layer count): files of
the same iteration left by an earlier run with a different layer split would otherwise override each
other's overlapping layers in sort order, so an overlap is an error, as is a gap in the requested layers.
Optimizer state (fp32 master weights + AdamW moments + step) goes to a `.optim.safetensors` sidecar.
`--resume-checkpoint DIR` (parsed but never read by the reference) resumes from the newest iteration.
"""
from __future__ import annotations

import re
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import torch

from ..inference.shard import Shard

_NAME = re.compile(r"^(\d{3})-(\d{3})-of-(\d{3})-(\d{6})\.safetensors$")


def checkpoint_path(directory: str | Path, shard: Shard, iteration: int) -> Path:
  return (Path(directory) / shard.model_id /
          f"{shard.start_layer:03d}-{shard.end_layer:03d}-of-{shard.n_layers:03d}-{iteration:06d}.safetensors")


def list_checkpoints(directory: str | Path, model_id: str) -> List[Tuple[int, int, int, int, Path]]:
  d = Path(directory) / model_id
  out = []
  if d.exists():
    for p in d.iterdir():
      m = _NAME.match(p.name)
      if m:
        s, e, n, it = map(int, m.groups())
        out.append((it, s, e, n, p))
  return sorted(out)


def _check_iteration(cks, it: int, shard: Shard) -> List[Path]:
  """Files of iteration `it` if they form ONE partition (disjoint layer ranges of one model size) covering
  the shard's layers; else ValueError (mixed / overlapping) or FileNotFoundError (a gap)."""
  parts = sorted((s, e, n, p) for i, s, e, n, p in cks if i == it)
  ns = {n for _, _, n, _ in parts}
  if len(ns) != 1:
    raise ValueError(f"iteration {it} of {shard.model_id} mixes models of {sorted(ns)} layers: {[p.name for *_, p in parts]}")
  for (s0, e0, _, p0), (s1, e1, _, p1) in zip(parts, parts[1:]):
    if s1 <= e0:
      raise ValueError(f"iteration {it} of {shard.model_id}: {p0.name} and {p1.name} overlap (layers {s1}-{min(e0, e1)}); "
                       "they come from runs with different layer splits -- keep one partition's files")
  have = {l for s, e, _, _ in parts for l in range(s, e + 1)}
  missing = [l for l in shard.layers() if l not in have]
  if missing:
    raise FileNotFoundError(f"iteration {it} of {shard.model_id} has no file for layers {missing[0]}..{missing[-1]}")
  return [p for *_, p in parts]


def select_checkpoint_files(directory: str | Path, shard: Shard, iteration: Optional[int] = None) -> Tuple[int, List[Path]]:
  """(iteration, files) to load `shard` from: one partition of the model whose layer ranges are pairwise
  disjoint.  With `iteration` given, exactly that iteration (ValueError / FileNotFoundError if it does not
  cover the shard).  Otherwise the newest iteration that covers the WHOLE model -- so every stage of a ring
  loading from a shared directory picks the same iteration, even when a peer died mid-save and left the
  newest one with a gap outside this shard -- and, when no iteration covers the whole model (each host of a
  multi-host ring saved only its own layers locally), the newest one that covers this shard.  Skipped
  iterations are reported; if none qualifies, the newest one's error is raised."""
  cks = list_checkpoints(directory, shard.model_id)
  if not cks:
    raise FileNotFoundError(f"no checkpoints for {shard.model_id} under {directory}")
  if iteration is not None:
    return iteration, _check_iteration(cks, iteration, shard)
  whole = Shard(shard.model_id, 0, shard.n_layers - 1, shard.n_layers)
  its = sorted({c[0] for c in cks}, reverse=True)
  for it in its:
    try:
      return it, _check_iteration(cks, it, whole)
    except (ValueError, FileNotFoundError):
      continue
  first_err = None
  for it in its:
    try:
      files = _check_iteration(cks, it, shard)
    except (ValueError, FileNotFoundError) as e:
      first_err = first_err or e
      print(f"checkpoint: skipping incomplete iteration {it}: {e}")
      continue
    return it, files
  raise first_err


def save_shard_checkpoint(engine, shard: Shard, path: str | Path) -> Path:
  from safetensors.torch import save_file
  path = Path(path)
  path.parent.mkdir(parents=True, exist_ok=True)
  trainer = getattr(engine, "trainer", None)
  if trainer is not None:
    trainer.sync_to_inference()
  sd = {k: v.detach().to("cpu").contiguous() for k, v in engine.runner.weights.to_hf_state_dict().items()}
  save_file(sd, str(path), metadata={"format": "pt", "shard": shard.key()})
  if trainer is not None:
    osd = {k: v.detach().to("cpu").contiguous() for k, v in trainer.state_dict().items()}
    save_file(osd, str(path.with_name(path.name.replace(".safetensors", ".optim.safetensors"))))
  return path


def _gather_tensors(files: List[Path], shard: Shard, tie: bool) -> Dict[str, torch.Tensor]:
  from safetensors import safe_open
  want: Dict[str, torch.Tensor] = {}
  for f in files:
    with safe_open(str(f), framework="pt") as sf:
      for k in sf.keys():
        if k.startswith("model.layers."):
          if int(k.split(".")[2]) in shard.layers():
            want[k] = sf.get_tensor(k)
        elif k.startswith("model.embed_tokens"):
          if shard.is_first_layer() or (shard.is_last_layer() and tie):
            want[k] = sf.get_tensor(k)
        elif (k.startswith("model.norm") or k.startswith("lm_head")) and shard.is_last_layer():
          want[k] = sf.get_tensor(k)
  return want


def load_shard_checkpoint(engine, shard: Shard, path: str | Path) -> None:
  from ..models.weights import copy_weights_into, from_hf_state_dict
  path = Path(path)
  cfg = engine.runner.config
  m = _NAME.match(path.name)
  if path.is_dir():
    _, files = select_checkpoint_files(path, shard)
  elif m and (not path.exists() or not (int(m.group(1)) <= shard.start_layer and shard.end_layer <= int(m.group(2)))):
    # a file name that does not cover the shard (or was never written as one file) names an iteration: take that
    # iteration's partition from its directory (e.g. a checkpoint a federated box saved as one file per local
    # sub-range, loaded under another split)
    _, files = select_checkpoint_files(path.parent.parent, shard, iteration=int(m.group(4)))
  else:
    files = [path]
  sd = _gather_tensors(files, shard, cfg.tie_word_embeddings)
  w = from_hf_state_dict(sd, cfg, shard, device=engine.runner.device)
  copy_weights_into(engine.runner.weights, w)  # in place: captured decode graphs keep their addresses
  engine.trainer = None
  # optimizer sidecar for this exact shard, if present
  for f in files:
    side = f.with_name(f.name.replace(".safetensors", ".optim.safetensors"))
    m = _NAME.match(f.name)
    if side.exists() and m and (int(m.group(1)), int(m.group(2))) == (shard.start_layer, shard.end_layer):
      from safetensors.torch import load_file
      tr = engine._get_trainer()
      tr.load_state_dict({k: v.to(tr.device) for k, v in load_file(str(side)).items()})
