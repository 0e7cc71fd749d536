"""LLaVA-1.5 vision path: CLIP ViT-L/14-336 tower + 2-layer GELU projector, run on the first pipeline
shard, whose image features replace the `<image>` token rows of the prompt's embeddings.

Reference parity: the reference lists `llava-1.5-7b-hf` (xotorch/models.py) and keeps the last image of a
chat as an image part (chatgpt_api.py:97-128), but its torchtune engine has no vision path; the semantics
here follow HF LlavaForConditionalGeneration (vision_feature_layer -2, "default" select = drop CLS,
linear_1 -> GELU -> linear_2) and CLIPImageProcessor (shortest edge 336 bicubic, center crop, CLIP mean /
std).  The tower runs once per image at prefill: its GEMMs go through the kernel library's `linear`
(weights shuffled once into the stream / big-tile layout), attention through the flash-style MFMA kernel
with the causal mask off (577 tokens, ops.kernels.attention_bidir), LayerNorm in torch.

Images travel inside the prompt string as `<|xot_image:URL|>` markers (URL = data: base64 or a file inside
image_dir(); there is no network), so a prompt forwarded to the first shard over gRPC keeps its image; the first
shard's engine turns each marker into `num_image_tokens` copies of the image token id.
"""
from __future__ import annotations

import base64
import io
import re
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F
from torch.utils.weak import WeakIdKeyDictionary

from ..ops import kernels as K

IMAGE_MARK = "<|xot_image:{}|>"
_MARK_RE = re.compile(r"<\|xot_image:(.*?)\|>", re.S)
CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def split_image_marks(prompt: str) -> Tuple[List[str], List[str]]:
  """prompt -> (text pieces, image urls) with len(pieces) == len(urls) + 1."""
  pieces, urls, pos = [], [], 0
  for m in _MARK_RE.finditer(prompt):
    pieces.append(prompt[pos:m.start()])
    urls.append(m.group(1))
    pos = m.end()
  pieces.append(prompt[pos:])
  return pieces, urls


def encode_with_images(tokenizer, c, prompt: str) -> Tuple[List[int], List[str]]:
  """Token ids of a prompt that may carry `<|xot_image:URL|>` markers, and the image urls: for a vision model
  each marker becomes its run of image tokens (the features replace those rows on the first shard); any other
  model reads a marker as the text "[image]" (then no urls are returned)."""
  pieces, urls = split_image_marks(prompt)
  if not urls:
    return list(tokenizer.encode(prompt)), []
  if c.vision is None:
    return list(tokenizer.encode("".join(p + ("[image]" if i < len(urls) else "") for i, p in enumerate(pieces)))), []
  n_img = num_image_tokens(c)
  ids: List[int] = []
  for i, piece in enumerate(pieces):
    ids += list(tokenizer.encode(piece, add_special_tokens=(i == 0)))
    if i < len(urls):
      ids += [c.image_token_id] * n_img
  return ids, urls


def image_pixels(c, urls: List[str]) -> torch.Tensor:
  """[N, 3, S, S] preprocessed pixels of the urls (CLIP preprocessing at the tower's resolution)."""
  size = c.vision["image_size"]
  return torch.stack([preprocess(load_image(u), size) for u in urls])


def escape_marks(text: str) -> str:
  """User text must not be able to produce an image marker: only markers build_prompt writes for the
  chat's image part survive (a literal `<|xot_image:/etc/...|>` typed into a message stays text)."""
  return text.replace("<|xot_image:", "<| xot_image:")


def image_dir():
  """The one directory local image paths may point into (XOT_IMAGE_DIR, default $XOT_HOME/images)."""
  import os
  from pathlib import Path
  env = os.environ.get("XOT_IMAGE_DIR")
  if env:
    return Path(env).resolve()
  from ..helpers import get_xot_images_dir
  return get_xot_images_dir().resolve()


def load_image(url: str):
  """data: URLs, or files inside image_dir() -- never an arbitrary server path named by a client."""
  from pathlib import Path

  from PIL import Image
  if url.startswith("data:"):
    data = base64.b64decode(url.split(",", 1)[1])
    return Image.open(io.BytesIO(data)).convert("RGB")
  if url.startswith("http://") or url.startswith("https://"):
    raise ValueError("image URLs are not fetched (offline runtime): send the image as a data: URL")
  root = image_dir()
  path = (root / url).resolve() if not Path(url).is_absolute() else Path(url).resolve()
  if root != path and root not in path.parents:
    raise ValueError(f"image path outside {root} refused: send the image as a data: URL")
  return Image.open(path).convert("RGB")


def preprocess(img, size: int) -> torch.Tensor:
  """CLIPImageProcessor (llava-1.5): shortest edge -> size (bicubic), center crop size x size, /255,
  normalise with the CLIP mean / std.  Returns [3, size, size] fp32."""
  from PIL import Image
  w, h = img.size
  s = size / min(w, h)
  nw, nh = max(size, int(round(w * s))), max(size, int(round(h * s)))
  img = img.resize((nw, nh), Image.BICUBIC)
  left, top = (nw - size) // 2, (nh - size) // 2
  img = img.crop((left, top, left + size, top + size))
  x = torch.frombuffer(bytearray(img.tobytes()), dtype=torch.uint8).view(size, size, 3).permute(2, 0, 1).float()
  x = x / 255.0
  mean = torch.tensor(CLIP_MEAN).view(3, 1, 1)
  std = torch.tensor(CLIP_STD).view(3, 1, 1)
  return (x - mean) / std


# ---------------------------------------------------------------------------------- weights
def vision_names(v: dict) -> List[str]:
  """HF parameter names of the tower + projector (checkpoint keys, canonical form: the hub's
  `vision_tower.vision_model.*` is read as `vision_tower.*`, see weights.canonical_name)."""
  p = "vision_tower."
  names = [p + "embeddings.class_embedding", p + "embeddings.patch_embedding.weight",
           p + "embeddings.position_embedding.weight", p + "pre_layrnorm.weight", p + "pre_layrnorm.bias"]
  for i in range(v["num_hidden_layers"]):
    q = p + f"encoder.layers.{i}."
    for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
      names += [q + f"self_attn.{n}.weight", q + f"self_attn.{n}.bias"]
    for n in ("layer_norm1", "layer_norm2", "mlp.fc1", "mlp.fc2"):
      names += [q + f"{n}.weight", q + f"{n}.bias"]
  names += [p + "post_layernorm.weight", p + "post_layernorm.bias"]  # pooled-output norm: kept, unused by LLaVA
  names += ["multi_modal_projector.linear_1.weight", "multi_modal_projector.linear_1.bias",
            "multi_modal_projector.linear_2.weight", "multi_modal_projector.linear_2.bias"]
  return names


def random_vision(c, device, dtype=torch.bfloat16, seed: int = 0, std: float = 0.02) -> Dict[str, torch.Tensor]:
  v = c.vision
  Dv, Fv, P, C = v["hidden_size"], v["intermediate_size"], v["patch_size"], v.get("num_channels", 3)
  n_pos = (v["image_size"] // P) ** 2 + 1
  g = torch.Generator(device=device)
  g.manual_seed(seed * 1_000_003 + 7)
  out = {}
  for name in vision_names(v):
    if name.endswith("class_embedding"):
      shape = (Dv,)
    elif "patch_embedding" in name:
      shape = (Dv, C, P, P)
    elif "position_embedding" in name:
      shape = (n_pos, Dv)
    elif "linear_1" in name:
      shape = (c.hidden_size, Dv) if name.endswith("weight") else (c.hidden_size,)
    elif "linear_2" in name:
      shape = (c.hidden_size, c.hidden_size) if name.endswith("weight") else (c.hidden_size,)
    elif "fc1" in name:
      shape = (Fv, Dv) if name.endswith("weight") else (Fv,)
    elif "fc2" in name:
      shape = (Dv, Fv) if name.endswith("weight") else (Dv,)
    elif "_proj" in name:
      shape = (Dv, Dv) if name.endswith("weight") else (Dv,)
    else:  # layer norms
      shape = (Dv,)
    if ("norm" in name or "layrnorm" in name) and name.endswith("weight"):
      t = 1.0 + torch.empty(shape, device=device, dtype=torch.float32).normal_(0, 0.05, generator=g)
    elif name.endswith("bias"):
      t = torch.empty(shape, device=device, dtype=torch.float32).normal_(0, 0.01, generator=g)
    else:
      t = torch.empty(shape, device=device, dtype=torch.float32).normal_(0, std, generator=g)
    out[name] = t.to(dtype)
  return out


# ---------------------------------------------------------------------------------- forward
# GPU copies of the tower's projection weights in the kernel library's pre-shuffled layout (made once per weight
# tensor, on first use), so the tower runs on the same stream / big-tile GEMMs as the language model; the
# checkpoint-facing dict keeps the HF row-major tensors
# keyed by tensor identity: a WeakKeyDictionary would compare tensors with the elementwise __eq__ on a hash clash
_SHUF = WeakIdKeyDictionary()


def _stream_weight(w: torch.Tensor) -> torch.Tensor:
  got = _SHUF.get(w)
  if got is None:
    from ..ops.weights_layout import shuffle_for_stream
    N, K = w.shape
    wp = w if K % 128 == 0 else F.pad(w, (0, -K % 128))  # zero columns: the patch embedding's K = 3 * 14 * 14
    got = shuffle_for_stream(wp.contiguous())
    got.xot_layout = "stream"
    _SHUF[w] = got
  return got


def _lin(x, w, b):
  from ..ops.linear import linear
  x = x.contiguous()
  if x.is_cuda and w.dim() == 2 and w.shape[0] % 16 == 0 and w.dtype == torch.bfloat16 == x.dtype:
    ws = _stream_weight(w)
    if ws.shape[1] != x.shape[1]:
      x = F.pad(x, (0, ws.shape[1] - x.shape[1]))
    y = linear(x, ws, bias=b.to(x.dtype) if b is not None else None)
    return y
  y = linear(x, w)
  return y + b.to(y.dtype) if b is not None else y


def image_features(c, vw: Dict[str, torch.Tensor], pixels: torch.Tensor) -> torch.Tensor:
  """pixels [N, 3, S, S] -> projected features [N * num_image_tokens, hidden] (the LM's dtype)."""
  v = c.vision
  p = "vision_tower."
  Dv, P, nh = v["hidden_size"], v["patch_size"], v["num_attention_heads"]
  eps = float(v.get("layer_norm_eps", 1e-5))
  dt = vw[p + "embeddings.patch_embedding.weight"].dtype
  N = pixels.shape[0]
  g = v["image_size"] // P
  # patch embedding as one GEMM over unfolded 14x14 patches (conv stride = kernel, no bias)
  x = pixels.to(dt)
  patches = x.unfold(2, P, P).unfold(3, P, P)  # [N, C, g, g, P, P]
  patches = patches.permute(0, 2, 3, 1, 4, 5).reshape(N * g * g, -1)
  wpe = vw[p + "embeddings.patch_embedding.weight"].reshape(Dv, -1)
  emb = _lin(patches, wpe, None).view(N, g * g, Dv)
  cls = vw[p + "embeddings.class_embedding"].to(emb.dtype).view(1, 1, Dv).expand(N, 1, Dv)
  h = torch.cat([cls, emb], 1) + vw[p + "embeddings.position_embedding.weight"].to(emb.dtype)[None]
  h = F.layer_norm(h.float(), (Dv,), vw[p + "pre_layrnorm.weight"].float(), vw[p + "pre_layrnorm.bias"].float(),
                   eps).to(dt)
  L = v["num_hidden_layers"]
  fl = c.vision_feature_layer
  n_run = L + 1 + fl if fl < 0 else fl  # hidden_states[k] = output of layer k (k = 0: embeddings)
  T = h.shape[1]
  for i in range(n_run):
    q = p + f"encoder.layers.{i}."
    r = h
    y = F.layer_norm(h.float(), (Dv,), vw[q + "layer_norm1.weight"].float(), vw[q + "layer_norm1.bias"].float(),
                     eps).to(dt).view(N * T, Dv)
    qkv = [_lin(y, vw[q + f"self_attn.{n}.weight"], vw[q + f"self_attn.{n}.bias"]) for n in ("q_proj", "k_proj", "v_proj")]
    a = K.attention_bidir(*qkv, N, T, nh, Dv // nh, (Dv // nh) ** -0.5)  # [N*T, Dv]
    h = r + _lin(a, vw[q + "self_attn.out_proj.weight"], vw[q + "self_attn.out_proj.bias"]).view(N, T, Dv).to(dt)
    r = h
    y = F.layer_norm(h.float(), (Dv,), vw[q + "layer_norm2.weight"].float(), vw[q + "layer_norm2.bias"].float(),
                     eps).to(dt).view(N * T, Dv)
    y = _lin(y, vw[q + "mlp.fc1.weight"], vw[q + "mlp.fc1.bias"])
    act = v.get("hidden_act", "quick_gelu")
    y = (y.float() * torch.sigmoid(1.702 * y.float())).to(dt) if act == "quick_gelu" else F.gelu(y.float()).to(dt)
    h = r + _lin(y, vw[q + "mlp.fc2.weight"], vw[q + "mlp.fc2.bias"]).view(N, T, Dv).to(dt)
  feats = h[:, 1:] if c.vision_select == "default" else h
  feats = feats.reshape(-1, Dv)
  y = _lin(feats, vw["multi_modal_projector.linear_1.weight"], vw["multi_modal_projector.linear_1.bias"])
  y = F.gelu(y.float()).to(dt) if c.projector_act == "gelu" else y
  return _lin(y, vw["multi_modal_projector.linear_2.weight"], vw["multi_modal_projector.linear_2.bias"])


def num_image_tokens(c) -> int:
  v = c.vision
  n = (v["image_size"] // v["patch_size"]) ** 2
  return n if c.vision_select == "default" else n + 1
