"""Batch-1 fused-norm decode vs unfused, per step and per deferral site (diagnostic; prints max |diff|)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import xotorch_support_jetson_amd.models.transformer as TM  # noqa: E402
from xotorch_support_jetson_amd.inference.shard import Shard  # noqa: E402
from xotorch_support_jetson_amd.models.config import preset  # noqa: E402
from xotorch_support_jetson_amd.models.weights import random_weights  # noqa: E402
from xotorch_support_jetson_amd.ops import linear as L  # noqa: E402
from xotorch_support_jetson_amd.runtime.runner import ShardRunner  # noqa: E402

gpu = torch.device("cuda", 0)
c = preset("llama-3-8b").with_layers(2)
sh = Shard("llama-3-8b", 0, 1, 2)
w = random_weights(c, sh, gpu, seed=5)
ids = torch.randint(0, c.vocab_size, (12,), generator=torch.Generator().manual_seed(1), dtype=torch.int32)
orig_lrn = L.linear_resid_norm


RUNS = [0]
_orig_run = L.PendingNorm.run


def _counted(self, *a, **k):
  RUNS[0] += 1
  return _orig_run(self, *a, **k)


L.PendingNorm.run = _counted


def run(fuse, sites, graphs=False):
  L.FUSE_NORM = TM.FUSE_NORM = fuse

  def lrn(*a, defer_to=None, **k):
    site = "down" if a[1] is not None and any(a[1] is lw.down_w for lw in w.layers.values()) else "o"
    return orig_lrn(*a, defer_to=defer_to if site in sites else None, **k)

  TM.linear_resid_norm = lrn
  r = ShardRunner(c, sh, gpu, weights=w, max_batch=4, max_ctx=128, use_graphs=graphs)
  out = [r.forward(["a"], [12], ids).clone()]  # graph replays reuse the output buffer
  tok = out[0].argmax(-1).int()
  for _ in range(3):
    out.append(r.forward(["a"], [1], tok).clone())
    tok = out[-1].argmax(-1).int()
  return out


ref = run(False, ())
ref2 = run(False, ())
print("unfused twice:", [round((a - b).abs().max().item(), 4) for a, b in zip(ref, ref2)], flush=True)
for graphs in (False, True):
  for sites in (("o",), ("down",), ("o", "down")):
    RUNS[0] = 0
    got = run(True, sites, graphs)
    print("graphs" if graphs else "eager", sites, "fused GEMMs", RUNS[0],
          [round((a - b).abs().max().item(), 4) for a, b in zip(ref, got)], flush=True)
refg = run(False, (), True)
print("unfused graphs:", [round((a - b).abs().max().item(), 4) for a, b in zip(ref, refg)], flush=True)
