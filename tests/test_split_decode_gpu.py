"""Split decode step (models/transformer.py:_forward_split): two half-batches on two streams, captured into
one HIP graph, give the same logits as the single-stream step on the same weights and cache contents."""
import pytest
import torch

from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.models import transformer
from xotorch_support_jetson_amd.models.config import preset
from xotorch_support_jetson_amd.runtime.runner import ShardRunner

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("offset", [False, True])
def test_split_decode_matches_single_stream(gpu, monkeypatch, graphs, offset):
  name = "tiny-llama-d64"
  c = preset(name)
  L = c.num_layers
  sh = Shard(name, 0, L - 1, L)
  ref = ShardRunner(c, sh, gpu, max_batch=8, max_ctx=512, use_graphs=graphs)
  monkeypatch.setattr(transformer, "SPLIT_DECODE_MIN", 4)
  monkeypatch.setattr(transformer, "SPLIT_OFFSET", offset)
  spl = ShardRunner(c, sh, gpu, max_batch=8, max_ctx=512, use_graphs=graphs)
  assert spl.model.side is not None and ref.model.side is None
  g = torch.Generator().manual_seed(1)
  rids = [f"r{i}" for i in range(8)]
  q = [3 + 5 * i for i in range(8)]
  ids = torch.randint(0, c.vocab_size, (sum(q),), generator=g, dtype=torch.int32)
  a, b = ref.forward(rids, q, ids), spl.forward(rids, q, ids)  # prefill: not split
  torch.testing.assert_close(a, b)
  tok = a.argmax(-1).int()
  for _ in range(4):
    a = ref.forward(rids, [1] * 8, tok)
    b = spl.forward(rids, [1] * 8, tok)
    assert (a - b).abs().max().item() <= 2e-2 * max(1.0, a.abs().max().item())
    assert torch.equal(a.argmax(-1), b.argmax(-1))
    tok = a.argmax(-1).int()
  torch.cuda.synchronize()
