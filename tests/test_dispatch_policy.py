"""Host-side dispatch policy (CPU): decode-attention partitioning per batch / block-table width, and the
GEMM tuner's split-K slab charge.  The kernels these choices select are covered in tests/test_kernels_gpu.py."""
import torch

from xotorch_support_jetson_amd.ops import kernels as K
from xotorch_support_jetson_amd.ops import linear as L


def test_decode_partition_defaults():
  ws = K.DecodeWorkspace(512, 64, 128, 8192, torch.device("cpu"), algo=-1)
  # few (sequence, KV head) pairs: 4-wave workgroups over 4-page partitions, merged by the reduce launch
  assert ws.partition(1, 8, 32) == (4, 8, 0)
  # many pairs: one wave per unit with page prefetch
  ppp, nparts, algo = ws.partition(512, 8, 9)
  assert algo == 3 and ppp * nparts >= 9  # one wave per unit, page prefetch, non-temporal page loads



def test_decode_partition_small_batch():
  ws = K.DecodeWorkspace(8, 32, 128, 4096, torch.device("cpu"), algo=-1)
  assert ws.partition(1, 8, 16)[2] == 0 and ws.partition(1, 8, 32)[2] == 0  # the workgroup kernel, split
  assert ws.partition(8, 8, 8)[2] == 2  # 64 pairs: the wave kernel (cache-resident pages: plain loads)
  assert K.DecodeWorkspace(64, 32, 128, 8192, torch.device("cpu"), algo=-1).partition(64, 8, 128)[2] == 3  # 2 GB: nt
  fixed = K.DecodeWorkspace(8, 32, 128, 4096, torch.device("cpu"), pages_per_part=4, algo=-1)
  assert fixed.partition(1, 8, 16)[2] == 0  # an explicit partition size is honoured


def test_slab_charge(monkeypatch):
  assert L._slab_read_ms(("big", 256, 1), 512, 8192) == 0.0
  four = L._slab_read_ms(("big", 256, 4), 512, 8192)
  assert abs(four - 4 * 512 * 8192 * 4 / (L.SLAB_TBPS * 1e9)) < 1e-12
  assert L._slab_read_ms(("big", 256, 2), 512, 8192) * 2 == four
  monkeypatch.setattr(L, "SLAB_TBPS", 0.0)
  assert L._slab_read_ms(("big", 256, 4), 512, 8192) == 0.0


def test_tuner_tie_break_prefers_ping_pong(monkeypatch):
  """Within XOT_GEMM_TIE of the fastest, a 256-row tile variant at the same K split gives way to the ping-pong
  256 x 256 tile; other kernels and other splits keep the plain minimum."""
  t = {("big", 224, 1): 0.400, ("big", 1256, 1): 0.408, ("big", 256, 1): 0.401, ("big", 1256, 2): 0.399}
  assert L._tie_break(t) == ("big", 1256, 2)  # the fastest is already a ping-pong config
  t.pop(("big", 1256, 2))
  assert L._tie_break(t) == ("big", 1256, 1)
  t[("big", 1256, 1)] = 0.500  # beyond the tie window: the next preference inside it
  assert L._tie_break(t) == ("big", 256, 1)
  assert L._tie_break({("stream", 2, 4): 0.1, ("big", 1256, 1): 0.101}) == ("stream", 2, 4)
  monkeypatch.setattr(L, "TIE", 0.0)
  assert L._tie_break({("big", 224, 1): 0.4, ("big", 1256, 1): 0.401}) == ("big", 224, 1)


def test_tuner_offers_two_phase_ping_pong(monkeypatch):
  """The two-phase ping-pong tile (2256) is a gemm_big candidate and the first choice inside the tie window."""
  codes = {c[1] for c in L.GemmPolicy._big_cands(512, 57344, 8192)}
  assert {256, 1256, 2256, 128} <= codes
  assert L._tie_break({("big", 1256, 1): 0.40, ("big", 2256, 1): 0.41}) == ("big", 2256, 1)
  # across K splits only the two-phase tile gets a (wider) window
  t = {("big", 128, 2): 0.843, ("big", 2256, 4): 0.927, ("big", 256, 4): 0.90}
  assert L._tie_break(t) == ("big", 2256, 4)
  t[("big", 2256, 4)] = 0.95
  assert L._tie_break(t) == ("big", 128, 2)
  # short row tiles: the two-phase 192-row tile is offered and preferred like the 256-row one
  assert ("big", 1922256, 1) in L.GemmPolicy._big_cands(384, 8192, 8192)
  assert L._tie_break({("big", 1920256, 2): 0.50, ("big", 1922256, 2): 0.51}) == ("big", 1922256, 2)
  monkeypatch.setattr(L, "TIE_X", 0.0)
  assert L._tie_break({("big", 128, 2): 0.843, ("big", 2256, 4): 0.85}) == ("big", 128, 2)
  monkeypatch.setattr(L, "PP2", False)
  assert 2256 not in {c[1] for c in L.GemmPolicy._big_cands(512, 57344, 8192)}


def test_cpu_reference_linear_caches_fp32_weights():
  """The CPU path widens a low-precision weight once and reuses it, re-widening after an in-place write (a
  trained weight written back) and never caching a weight that requires grad."""
  from xotorch_support_jetson_amd.ops import reference as ref
  torch.manual_seed(0)
  x = torch.randn(3, 64)
  w = torch.randn(32, 64).to(torch.bfloat16)
  y1 = ref.linear(x, w)
  assert hasattr(w, "_xot_f32")
  f32 = w._xot_f32[1]
  assert ref.linear(x, w) is not None and w._xot_f32[1] is f32  # reused
  w.mul_(2)
  y2 = ref.linear(x, w)
  assert torch.allclose(y2, 2 * y1, rtol=1e-2, atol=1e-2)
  wg = torch.randn(32, 64, requires_grad=True)
  ref.linear(x, wg.to(torch.bfloat16))
  assert not hasattr(wg, "_xot_f32")


def test_tuner_prefers_four_wave_tile_on_tall_gemms(monkeypatch):
  """The four-wave 256 x 256 tile (4256) is a candidate wherever N % 256 == 0; from W4_PREF_M rows it takes the
  ping-pong tile's place as first choice inside the tie windows, below it the ping-pong tile keeps it."""
  assert 4256 in {c[1] for c in L.GemmPolicy._big_cands(4096, 4096, 4096)}
  assert 4256 not in {c[1] for c in L.GemmPolicy._big_cands(4096, 4096 + 224, 4096)}
  t = {("big", 2256, 1): 0.40, ("big", 4256, 1): 0.41}
  assert L._tie_break(t, 4096) == ("big", 4256, 1)
  assert L._tie_break(t, 512) == ("big", 2256, 1)
  t = {("big", 2256, 2): 0.40, ("big", 4256, 1): 0.43}  # across K splits: the preferred tile's wider window
  assert L._tie_break(t, 4096) == ("big", 4256, 1)
  monkeypatch.setattr(L, "W4", False)
  assert 4256 not in {c[1] for c in L.GemmPolicy._big_cands(4096, 4096, 4096)}


def test_tall_gemms_take_the_four_wave_tile_untimed(monkeypatch):
  """M >= W4_PREF_M: ('big', 4256, 1) straight away (no cold-timing pass inside the first prefill chunk), except a
  residual epilogue into fp32 (the tile has none); XOT_GEMM_TALL_TUNE=1 times them again."""
  pol = L.GemmPolicy()
  x, w = torch.empty(4096, 1024, dtype=torch.bfloat16), torch.empty(2048, 1024, dtype=torch.bfloat16)
  assert pol.shuffled_cfg(x, w, None, None, "none", torch.bfloat16) == ("big", 4256, 1)
  assert pol.shuffled_cfg(x, w, None, None, "none", torch.float32) == ("big", 4256, 1)
  monkeypatch.setattr(L, "TALL_FIXED", False)
  monkeypatch.setattr(L.GemmPolicy, "_no_tuning", lambda self: True)  # the heuristic instead of a GPU timing
  pol2 = L.GemmPolicy()
  assert pol2.shuffled_cfg(x, w, None, None, "none", torch.bfloat16)[0] == "big"


def test_seed_table_parses_and_loads_under_the_box_table(tmp_path):
  """ops/gemm_seed_mi355x.json: comment keys skipped, the headline decode picks load, and a key the box tuned itself
  keeps the box's choice (the seed only fills gaps)."""
  import json
  from xotorch_support_jetson_amd.ops import linear as L
  pol = L.GemmPolicy()
  own = ("sh", 512, 10240, 8192, "none", False, "torch.bfloat16")
  pol.table[own] = ("big", 256, 2)  # as if the box had tuned it
  pol._load(L.SEED_TABLE)
  assert pol.table[own] == ("big", 256, 2)
  assert pol.table[("sh", 512, 57344, 8192, "silu", False, "torch.bfloat16")] == ("big", 2256, 1)
  assert not any(isinstance(k, tuple) and k and str(k[0]).startswith("_") for k in pol.table)
  assert all(k.startswith("_") or json.loads(k)[0] == "sh" for k in json.load(open(L.SEED_TABLE)))
