"""Parity of the shard model (CPU path: same fused layouts, paged KV cache, gate/up interleave and
RoPE tables as the HIP path) against HuggingFace transformers reference implementations built from
small random configs, loaded through our safetensors shard loader (reference parity target:
xotorch/inference/torch/models/llm_utils.py + general_mha.py).  Prefill + teacher-forced decode,
also split across two shards."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.models.config import load_config
from xotorch_support_jetson_amd.models.weights import load_hf_weights
from xotorch_support_jetson_amd.runtime.runner import ShardRunner


def _hf_model(kind, tmp_path):
  torch.manual_seed(0)
  common = dict(vocab_size=300, hidden_size=256, intermediate_size=384, num_hidden_layers=3, num_attention_heads=4,
                num_key_value_heads=2, max_position_embeddings=512)
  if kind == "llama":
    cfg = transformers.LlamaConfig(**common, rope_theta=500000.0, tie_word_embeddings=True,
                                   rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                                 "high_freq_factor": 4.0, "original_max_position_embeddings": 64})
    m = transformers.LlamaForCausalLM(cfg)
  elif kind == "qwen2":
    cfg = transformers.Qwen2Config(**common, rope_theta=1000000.0, tie_word_embeddings=False)
    m = transformers.Qwen2ForCausalLM(cfg)
  elif kind.startswith("phi3"):
    # partial rotary (48 of 64 dims), LongRoPE: past an 8-token window the sequence uses the long factors;
    # phi3-short stays inside a 64-token window (short factors)
    cfg = transformers.Phi3Config(**common, tie_word_embeddings=True, partial_rotary_factor=0.75, pad_token_id=0,
                                  bos_token_id=1, eos_token_id=2,
                                  original_max_position_embeddings=8 if kind == "phi3" else 64,
                                  rope_scaling={"type": "longrope", "short_factor": [1.0 + 0.1 * i for i in range(24)],
                                                "long_factor": [3.0 + 0.2 * i for i in range(24)]})
    m = transformers.Phi3ForCausalLM(cfg)
  elif kind == "deepseek_v2":
    # MLA without q_lora, dense first layer, 8 routed experts in 4 groups (group-limited greedy), 2 shared
    cfg = transformers.DeepseekV2Config(**dict(common, num_key_value_heads=4), moe_intermediate_size=256,
                                        n_routed_experts=8, n_shared_experts=2, num_experts_per_tok=2,
                                        first_k_dense_replace=1, kv_lora_rank=256, q_lora_rank=None,
                                        qk_nope_head_dim=64, qk_rope_head_dim=64, v_head_dim=64,
                                        topk_method="group_limited_greedy", n_group=4, topk_group=2,
                                        routed_scaling_factor=1.5, pad_token_id=0, bos_token_id=1, eos_token_id=2)
    m = transformers.DeepseekV2ForCausalLM(cfg)
  elif kind == "deepseek_v3":
    # MLA with q_lora, sigmoid scores + selection bias, top-2-sum groups, renormalised x 2.5, YaRN rope
    cfg = transformers.DeepseekV3Config(**dict(common, num_key_value_heads=4), moe_intermediate_size=256,
                                        n_routed_experts=16, n_shared_experts=1, num_experts_per_tok=4,
                                        first_k_dense_replace=1, kv_lora_rank=256, q_lora_rank=128,
                                        qk_nope_head_dim=64, qk_rope_head_dim=64, v_head_dim=64, n_group=4,
                                        topk_group=2, routed_scaling_factor=2.5, norm_topk_prob=True,
                                        rope_scaling={"type": "yarn", "factor": 4.0, "original_max_position_embeddings": 16,
                                                      "beta_fast": 32, "beta_slow": 1, "mscale": 0.707,
                                                      "mscale_all_dim": 1.0},
                                        pad_token_id=0, bos_token_id=1, eos_token_id=2)
    m = transformers.DeepseekV3ForCausalLM(cfg)
  else:
    cfg = transformers.MixtralConfig(**common, num_local_experts=4, num_experts_per_tok=2, rope_theta=1e6)
    m = transformers.MixtralForCausalLM(cfg)
  m = m.float().eval()
  with torch.no_grad():  # non-trivial norms so their weights matter
    for n, p in m.named_parameters():
      if "norm" in n:
        p.uniform_(0.5, 1.5)
      elif "bias" in n:
        p.normal_(0, 0.1)
      elif "q_proj" in n or "qkv_proj" in n or "q_b_proj" in n:
        p.mul_(6.0)  # peaked attention, so positions (RoPE) visibly change the logits
    for n, b in m.named_buffers():
      if "e_score_correction_bias" in n:
        b.normal_(0, 0.05)
  d = tmp_path / kind
  m.save_pretrained(str(d), safe_serialization=True)
  return m, d


@pytest.mark.parametrize("kind", ["phi3", "deepseek_v2", "deepseek_v3"])
def test_checkpoint_roundtrip(kind, tmp_path):
  """HF names survive to_hf_state_dict -> load exactly: Phi-3's fused qkv / gate_up and partial-rotary q/k
  row permutation, DeepSeek's MLA row reorders (nope | de-interleaved rope), expert and shared-expert stacks."""
  hf, d = _hf_model(kind, tmp_path)
  c = load_config(d)
  sw = load_hf_weights(d, c, Shard(kind, 0, 2, 3), dtype=torch.float32)
  sd = sw.to_hf_state_dict()
  from safetensors.torch import load_file  # the hub-format names save_pretrained wrote
  ref = {}
  for f in sorted(d.glob("*.safetensors")):
    ref.update(load_file(str(f)))
  for k, v in sd.items():
    assert k in ref, k
    torch.testing.assert_close(v, ref[k].float(), rtol=0, atol=0)
  missing = [k for k in ref if k not in sd and "rotary" not in k and "lm_head" not in k]
  assert not missing, missing
  if kind == "phi3":
    assert "model.layers.0.self_attn.qkv_proj.weight" in sd and "model.layers.0.mlp.gate_up_proj.weight" in sd


@pytest.mark.parametrize("kind", ["llama", "qwen2", "mixtral", "phi3", "phi3-short", "deepseek_v2", "deepseek_v3"])
def test_hf_parity(kind, tmp_path):
  hf, d = _hf_model(kind, tmp_path)
  c = load_config(d)
  if c.head_dim < 64:
    pytest.skip("attention kernels need head_dim >= 64")  # CPU path is generic but keep shapes kernel-legal
  L = 12
  ids = torch.randint(0, c.vocab_size, (1, L + 3))
  with torch.no_grad():
    ref = hf(ids).logits[0].float()
  shards = [Shard(kind, 0, 2, 3)], [Shard(kind, 0, 0, 3), Shard(kind, 1, 2, 3)]
  for split in shards:
    runners = [ShardRunner(c, s, "cpu", weights=load_hf_weights(d, c, s, dtype=torch.float32), max_batch=2,
                           max_ctx=64) for s in split]

    def step(x, n):
      for r in runners:
        x = r.forward(["q"], [n], x)
      return x

    out = step(ids[0, :L].to(torch.int32), L)
    got = [out.float().view(-1)]
    for t in range(L, L + 3):
      got.append(step(ids[0, t:t + 1].to(torch.int32), 1).float().view(-1))
    for k, g in enumerate(got):
      r = ref[L - 1 + k]
      # the engine keeps activations and the KV cache in bf16 (the HF reference runs fp32)
      err = (g - r).abs().max().item() / r.abs().max().item()
      cos = torch.nn.functional.cosine_similarity(g, r, dim=0).item()
      assert err < 6e-2 and cos > 0.999, (kind, len(split), k, err, cos)


def _hf_llava(tmp_path):
  torch.manual_seed(0)
  tc = transformers.LlamaConfig(vocab_size=300, hidden_size=256, intermediate_size=384, num_hidden_layers=3,
                                num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512,
                                pad_token_id=0, bos_token_id=1, eos_token_id=2)
  vc = transformers.CLIPVisionConfig(hidden_size=128, intermediate_size=256, num_hidden_layers=3, num_attention_heads=4,
                                     patch_size=14, image_size=56)
  m = transformers.LlavaForConditionalGeneration(transformers.LlavaConfig(text_config=tc, vision_config=vc,
                                                                          image_token_index=299)).float().eval()
  with torch.no_grad():
    for n, p in m.named_parameters():
      if "norm" in n and n.endswith("weight"):
        p.uniform_(0.5, 1.5)
      elif n.endswith("bias"):
        p.normal_(0, 0.05)
  d = tmp_path / "llava"
  m.save_pretrained(str(d), safe_serialization=True)
  return m, d


def test_llava_parity(tmp_path):
  """LLaVA: CLIP tower (feature layer -2, CLS dropped) + projector features spliced into the image-token
  rows, then the Llama decoder, prefill + decode, vs HF LlavaForConditionalGeneration."""
  from xotorch_support_jetson_amd.models.vision import num_image_tokens
  hf, d = _hf_llava(tmp_path)
  c = load_config(d)
  assert c.model_type == "llava" and c.image_token_id == 299 and num_image_tokens(c) == 16
  n_img = num_image_tokens(c)
  ids = torch.cat([torch.tensor([1, 5, 6]), torch.full((n_img,), 299), torch.randint(3, 298, (7,))])
  pixels = torch.randn(1, 3, 56, 56)
  L = ids.numel()
  with torch.no_grad():
    ref = hf(input_ids=ids[None], pixel_values=pixels).logits[0].float()
  for split in ([Shard("llava", 0, 2, 3)], [Shard("llava", 0, 0, 3), Shard("llava", 1, 2, 3)]):
    runners = [ShardRunner(c, s, "cpu", weights=load_hf_weights(d, c, s, dtype=torch.float32), max_batch=2,
                           max_ctx=64) for s in split]
    assert runners[0].weights.vision is not None and (len(runners) == 1 or runners[1].weights.vision is None)
    feats = runners[0].image_features(pixels)
    x = runners[0].forward(["q"], [L - 2], ids[:L - 2].to(torch.int32), image_embeds=feats)
    for r in runners[1:]:
      x = r.forward(["q"], [L - 2], x)
    got = [x.float().view(-1)]
    for t in range(L - 2, L):
      x = ids[t:t + 1].to(torch.int32)
      for r in runners:
        x = r.forward(["q"], [1], x)
      got.append(x.float().view(-1))
    for k, g in enumerate(got):
      rr = ref[L - 3 + k]
      err = (g - rr).abs().max().item() / rr.abs().max().item()
      cos = torch.nn.functional.cosine_similarity(g, rr, dim=0).item()
      assert err < 6e-2 and cos > 0.999, (len(split), k, err, cos)


def test_llava_preprocess_matches_clip_processor():
  from PIL import Image
  from xotorch_support_jetson_amd.models.vision import preprocess
  g = torch.Generator().manual_seed(0)
  arr = torch.randint(0, 256, (45, 70, 3), generator=g, dtype=torch.uint8).numpy()
  img = Image.fromarray(arr)
  proc = transformers.CLIPImageProcessor(size={"shortest_edge": 56}, crop_size={"height": 56, "width": 56})
  ref = torch.as_tensor(proc(images=img, return_tensors="np")["pixel_values"][0])
  got = preprocess(img, 56)
  assert got.shape == ref.shape
  assert (got - ref).abs().max().item() < 0.05  # resampling implementations differ by a few grey levels


def test_checkpoint_roundtrip_llava(tmp_path):
  hf, d = _hf_llava(tmp_path)
  c = load_config(d)
  sw = load_hf_weights(d, c, Shard("llava", 0, 2, 3), dtype=torch.float32)
  sd = sw.to_hf_state_dict()
  from safetensors.torch import load_file
  from xotorch_support_jetson_amd.models.weights import canonical_name
  ref = {}
  for f in sorted(d.glob("*.safetensors")):
    ref.update({canonical_name(k): v for k, v in load_file(str(f)).items()})
  for k, v in sd.items():
    torch.testing.assert_close(v, ref[k].float(), rtol=0, atol=0)
  assert not [k for k in ref if k not in sd], [k for k in ref if k not in sd]
