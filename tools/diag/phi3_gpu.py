"""Diagnose Phi-3 GPU vs HF: fp32 HF, our CPU path (bf16 weights), our GPU path with / without graphs."""
import pathlib, sys, tempfile
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[2]))
import torch
import tests.test_hf_parity as T
from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.models.config import load_config
from xotorch_support_jetson_amd.models.weights import load_hf_weights
from xotorch_support_jetson_amd.runtime.runner import ShardRunner

torch.manual_seed(0)
for kind in sys.argv[1:] or ["phi3"]:
  hf, d = T._hf_model(kind, pathlib.Path(tempfile.mkdtemp()))
  c = load_config(d)
  L = 40
  ids = torch.randint(0, c.vocab_size, (1, L + 4))
  with torch.no_grad():
    ref = hf(ids).logits[0].float()
  s = Shard(kind, 0, c.num_layers - 1, c.num_layers)
  res = {}
  for name, dev, dt, graphs in [("cpu_bf16", "cpu", torch.bfloat16, False), ("gpu_eager", "cuda:0", torch.bfloat16, False),
                                ("gpu_graph", "cuda:0", torch.bfloat16, True)]:
    r = ShardRunner(c, s, dev, weights=load_hf_weights(d, c, s, device=dev, dtype=dt), max_batch=4, max_ctx=128,
                    use_graphs=graphs)
    got = [r.forward(["q"], [L], ids[0, :L].to(torch.int32).to(dev)).float().view(-1).cpu()]
    for t in range(L, L + 4):
      got.append(r.forward(["q"], [1], ids[0, t:t + 1].to(torch.int32).to(dev)).float().view(-1).cpu())
    res[name] = got
  for k in range(5):
    rr = ref[L - 1 + k]
    line = [f"{kind} k={k}"]
    for name, got in res.items():
      g = got[k]
      line.append(f"{name}: cos {torch.nn.functional.cosine_similarity(g, rr, dim=0).item():.5f} "
                  f"err {(g - rr).abs().max().item() / rr.abs().max().item():.4f}")
    g, cb = res["gpu_eager"][k], res["cpu_bf16"][k]
    line.append(f"gpu-vs-cpu cos {torch.nn.functional.cosine_similarity(g, cb, dim=0).item():.5f}")
    print(" | ".join(line), flush=True)
