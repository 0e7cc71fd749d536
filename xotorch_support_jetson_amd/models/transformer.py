"""Forward pass of one pipeline shard of a dense (Llama/Qwen2/Mistral) or MoE (Mixtral) decoder.

Per layer, all on the kernel library (ops.*), with the residual stream `h` carried in place:
  xn  = rmsnorm(h, ln1)
  qkv = xn @ qkv_w.T (+b)                          fused QKV GEMM
  q   = rope(qkv.q); cache <- rope(qkv.k), qkv.v   one kernel, paged write (slot mapping)
  a   = attention(q, paged cache)                  decode: split-KV GQA; prefill: causal varlen
  h   = h + a @ o_w.T                              residual add in the GEMM epilogue
  xn  = rmsnorm(h, ln2)
  act = silu(xn @ gate.T) * (xn @ up.T)            one GEMM (interleaved gate/up), SiLU in the epilogue
  h   = h + act @ down.T                           residual add in the GEMM epilogue
Last shard: rmsnorm + LM head on each sequence's LAST row only (the reference computes the head over
every prompt row and keeps [:, -1], sharded_inference_engine.py:366), fp32 logits for the sampler.

Hidden-state contract between shards: the output of this shard's end_layer (fixing the reference's
off-by-one that returns the *input* of the last layer and IndexErrors on middle shards,
llm_utils.py:404-440 / general_mha.py:209).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch

from ..inference.shard import Shard
from ..ops import kernels as K
from ..ops._ext import require
from ..ops.linear import FUSE_MERGE, FUSE_NORM, PendingNorm, layout_of, linear, linear_resid_norm, linear_rope_kv, scratch
from ..ops.rope import longrope_window, rope_shift, rope_table
from .config import ModelConfig
from .weights import ShardWeights, expert

# average rows per expert above which the grouped expert GEMMs run on gemm_big tiles
MOE_BIG_MIN_ROWS = float(os.environ.get("XOT_MOE_BIG_MIN_ROWS", "24"))
# K splits of the grouped gate/up GEMM for decode-sized batches (1: fused SiLU epilogue, no slabs)
MOE_GU_SPLITS = int(os.environ.get("XOT_MOE_GU_SPLITS", "4"))
MOE_BM = int(os.environ.get("XOT_MOE_BM", "0"))  # force the grouped gemm_big tile code (tests, A/B)
MOE_DN_SPLITS = int(os.environ.get("XOT_MOE_DN_SPLITS", "0"))  # force the grouped down GEMM's K split on gemm_big tiles
MOE_PP2 = os.environ.get("XOT_MOE_PP2", "1") == "1"  # 256-row expert tiles on the two-phase ping-pong schedule
PAGE = 64


def moe_tiles(rows: float, E: int) -> Tuple[int, int, int]:
  """(gate/up tile code, down tile code, down K split) of the grouped expert GEMMs on gemm_big tiles at `rows`
  average rows per expert.  Tile code = row tile + 1000 for the deeper LDS pipeline (three 64-deep stages for
  128 rows: more expert-weight bytes in flight, which is what the HBM-bound small groups need).  Measured at
  Mixtral shapes (tools/bench_moe.py, profiles/r3/moe_tiles/): ~32 rows gate/up 315 us (1128) vs 356 (128),
  down 144 (1128, S 2) vs 166; ~64 rows gate/up 441 (1128) vs 566 (128), down 178 (256, S 2) vs 288 (128, S 2);
  ~128 rows 192-row tiles (gate/up 439 us, down 254 at S 4).  Many small experts (DeepSeek-V2-Lite, 64 x ~24
  rows) keep 256-row tiles (11.0 vs 12.6 ms per step with 128)."""
  if rows <= 96 and E > 16:
    return 256, 256, 2
  if rows <= 48:
    return 1128, 1128, 2
  if rows <= 96:
    return 1128, 256, 2
  if rows <= 160:
    return 192, 192, 4
  return 256, 256, 2


@dataclass
class StepInputs:
  """Device-side description of one forward step over a batch of sequences (all int tensors)."""
  positions: torch.Tensor  # [T] int32 absolute position of each new token
  slots: torch.Tensor  # [T] int64 global KV slot of each new token (-1: do not write)
  block_tables: torch.Tensor  # [B, max_blocks] int32
  ctx_lens: torch.Tensor  # [B] int32 context length INCLUDING the new tokens
  cu_q: torch.Tensor  # [B+1] int32 offsets of each sequence's new tokens in T
  last_idx: torch.Tensor  # [B] int64 row of each sequence's last new token
  max_qlen: int
  decode: bool  # every sequence has exactly one new token
  image_embeds: Optional[torch.Tensor] = None  # LLaVA: [n image-token rows, D], in token order (first shard)

  @property
  def num_tokens(self) -> int:
    return int(self.positions.numel())

  @property
  def batch(self) -> int:
    return int(self.ctx_lens.numel())


class KVCache:
  """Per-shard paged KV pool: K [L, pages, Hkv, 64, Dh] and V [L, pages, Hkv, Dh, 64] (V storage: each page chunk-major,
  [8 chunks][Dh][8 keys], ops/reference.py v_chunks).
  MLA models (DeepSeek) keep one latent row per token instead: k = C [L, pages, 64, kv_lora + rope], v None."""

  def __init__(self, c: ModelConfig, n_layers: int, num_pages: int, device, dtype=torch.bfloat16):
    self.num_pages = num_pages
    if c.is_mla:
      self.k = torch.zeros(n_layers, num_pages, PAGE, c.mla_dim, device=device, dtype=dtype)
      self.v = None
      return
    self.k = torch.zeros(n_layers, num_pages, c.num_kv_heads, PAGE, c.head_dim, device=device, dtype=dtype)
    self.v = torch.zeros(n_layers, num_pages, c.num_kv_heads, c.head_dim, PAGE, device=device, dtype=dtype)

  @staticmethod
  def bytes_per_page(c: ModelConfig, n_layers: int) -> int:
    if c.is_mla:
      return n_layers * PAGE * c.mla_dim * 2
    return 2 * n_layers * c.num_kv_heads * PAGE * c.head_dim * 2

  def nbytes(self) -> int:
    return sum(t.numel() * t.element_size() for t in (self.k, self.v) if t is not None)


class ShardModel:
  def __init__(self, weights: ShardWeights, kv: KVCache, max_batch: int = 256, max_ctx: int = 8192):
    self.w = weights
    self.c: ModelConfig = weights.config
    self.shard: Shard = weights.shard
    self.kv = kv
    self.device = kv.k.device
    c = self.c
    self.scale = 1.0 / math.sqrt(c.head_dim)
    max_pos = max(max_ctx, 16)
    self.cos_sin = rope_table(c, max_pos, self.device)
    self.rope_rows, self.rope_window = max_pos, longrope_window(c)
    self.layer_ids: List[int] = list(self.shard.layers())
    self.max_batch = max_batch
    self.max_ctx = max_ctx
    self.ws = None
    if self.device.type == "cuda":
      if c.is_mla:
        self.ws = K.MLAWorkspace(max_batch, c.num_heads, c.kv_lora_rank, max_ctx, self.device)
      else:
        self.ws = K.DecodeWorkspace(max_batch, c.num_heads, c.head_dim, max_ctx, self.device)
    if c.is_mla:
      self.scale = c.attn_scale()
    # last shard with the LM head split across two ring stages: logits of vocab rows [0, head_rows) only,
    # and forward returns (logits, normed hidden)
    self.head_rows: Optional[int] = None
    self._head_cache = None

  def rope_pos(self, start: int, n: int) -> range:
    """RoPE table rows of a step's n new tokens at positions start.. (LongRoPE: the long-factor half
    once the sequence outgrows the pretraining window; positions only feed the RoPE kernels)."""
    o = rope_shift(self.rope_window, self.rope_rows, start + n)
    return range(start + o, start + n + o)

  # ------------------------------------------------------------------ helpers
  def _attention(self, q: torch.Tensor, li: int, inp: StepInputs, ws=None, defer_merge: bool = False):
    kc, vc = self.kv.k[li], self.kv.v[li]
    if inp.decode:
      return K.attn_decode(q, kc, vc, inp.block_tables, inp.ctx_lens, self.scale, ws or self.ws,
                           defer_merge=defer_merge)
    return K.attn_prefill(q, kc, vc, inp.block_tables, inp.cu_q, inp.ctx_lens, inp.max_qlen, self.scale)

  def _mla(self, xn: torch.Tensor, lw, li: int, inp: StepInputs) -> torch.Tensor:
    """DeepSeek multi-head latent attention -> [T, H * v_head_dim] (before o_proj).
    A = xn @ [q_a | kv_a]^T; q = rmsnorm(q_a) @ q_b^T (or A's q part); latent norm + rope + cache write;
    absorbed query q_lat = q_nope . W_UK per head; attention over the latent cache (csrc/mla.hip);
    o = o_lat . W_UV^T per head."""
    c = self.c
    T = xn.shape[0]
    H, dn, dr, dv, L = c.num_heads, c.qk_nope_head_dim, c.qk_rope_head_dim, c.v_head_dim, c.kv_lora_rank
    A = linear(xn, lw.qkv_w)
    nq = c.q_lora_rank or H * (dn + dr)
    if c.q_lora_rank:
      qa, _ = K.rmsnorm(A[:, :nq].contiguous(), lw.q_ln, c.rms_norm_eps)
      q = linear(qa, lw.qb_w)  # [T, H dn | H dr]
    else:
      q = A  # q = A[:, :nq], rows of stride A.shape[1]
    ckv = A[:, nq:]
    cache = self.kv.k[li]
    K.mla_prep(ckv, lw.kv_ln, q, H * dn, H, inp.positions, self.cos_sin, inp.slots, cache, c.rms_norm_eps)
    dt = q.dtype
    q_pe = q[:, H * dn:]
    if getattr(lw.wuk, "xot_layout", "rowmajor") == "stream_t":
      # absorbed projections on the batched stream GEMM (pre-shuffled per head, csrc/gemm.hip MOE==3 mode):
      # head h reads q[:, h dn:(h+1) dn] in place and writes q_lat[h]; o_lat[h] . W_UV[h]^T lands in o[:, h dv:]
      KC = require()
      q_lat = torch.empty(H, T, L, device=q.device, dtype=dt)
      KC.gemm_batched(q[:, :H * dn], dn, dn, lw.wuk, q_lat, T * L, L, T)
      o_lat = K.mla_attn(q_lat, q_pe, cache, inp.block_tables, inp.cu_q, inp.ctx_lens, self.scale, self.ws)
      o = torch.empty(T, H * dv, device=q.device, dtype=dt)
      KC.gemm_batched(o_lat.view(H * T, L), T * L, L, lw.wuv, o, dv, H * dv, T)
      return o
    q_nope = q[:, :H * dn].view(T, H, dn).transpose(0, 1)  # [H, T, dn]
    if xn.is_cuda:
      q_lat = torch.bmm(q_nope, lw.wuk)  # [H, T, L] (row-major weights: shapes gemm_batched does not tile)
    else:  # CPU reference path: fp32 math whatever the shard's storage dtypes
      q_lat = torch.bmm(q_nope.float(), lw.wuk.float()).to(dt)
    o_lat = K.mla_attn(q_lat, q_pe, cache, inp.block_tables, inp.cu_q, inp.ctx_lens, self.scale, self.ws)
    if xn.is_cuda:
      o = torch.bmm(o_lat, lw.wuv.transpose(1, 2))  # [H, T, dv]
    else:
      o = torch.bmm(o_lat.float(), lw.wuv.float().transpose(1, 2)).to(dt)
    return o.transpose(0, 1).reshape(T, H * dv)

  def _mlp(self, xn: torch.Tensor, lw, h: torch.Tensor, next_norm: Optional[torch.Tensor], li: int = -1,
           defer_to: Optional[torch.Tensor] = None):
    """h += MLP(xn) in place; returns rmsnorm(h) * next_norm (None if there is no following norm), or a
    PendingNorm whose residual continues in defer_to (see linear_resid_norm)."""
    c = self.c
    if lw.router is None:
      act = linear(xn, lw.gu_w, epi="silu")
      if next_norm is not None:
        return linear_resid_norm(act, lw.down_w, h, next_norm, c.rms_norm_eps, defer_to=defer_to)
      linear(act, lw.down_w, residual=h, epi="resid", out=h)
      return None
    if isinstance(xn, PendingNorm):
      xn = xn.materialize()
    out = self._moe(xn, lw, h, next_norm)
    if out is not None:  # the combine kernel also applied the following RMSNorm
      return out
    return K.rmsnorm(h, next_norm, c.rms_norm_eps)[0] if next_norm is not None else None

  @property
  def _ds_route(self) -> bool:
    """DeepSeekMoE routing (groups / sigmoid / bias / unnormalised scaled weights) vs Mixtral's."""
    c = self.c
    return not (c.topk_method == "greedy" and c.scoring_func == "softmax" and c.norm_topk_prob
                and c.routed_scaling_factor == 1.0)

  def _route_args(self):
    c = self.c
    method = {"greedy": 0, "group_limited_greedy": 1, "noaux_tc": 2}[c.topk_method]
    return (c.num_experts_per_tok, c.n_group if method else 1, c.topk_group if method else 1, method,
            c.scoring_func == "sigmoid", c.norm_topk_prob, c.routed_scaling_factor)

  def _moe(self, xn: torch.Tensor, lw, h: torch.Tensor, next_norm: Optional[torch.Tensor] = None):
    """Sparse MoE: top-k routing (Mixtral softmax, or DeepSeek's grouped / sigmoid-with-bias rules), shared
    experts (DeepSeek) added as a dense SwiGLU, tokens grouped per expert, expert GEMMs on the kernel library
    (gate/up with fused SiLU epilogue), weighted scatter-add back into h."""
    c = self.c
    if lw.sh_gu_w is not None:  # shared experts: h += down(silu(gate) * up) of every token
      linear(linear(xn, lw.sh_gu_w, epi="silu"), lw.sh_down_w, residual=h, epi="resid", out=h)
    if xn.is_cuda and (c.num_experts in (4, 8, 16) or (c.num_experts in (32, 64, 128, 160, 256)
                                                       and c.hidden_size % 512 == 0)) and layout_of(lw.router) == "rowmajor":
      # fp32 router logits, one small kernel (instead of a bf16 library GEMM + cast)
      logits = torch.empty(xn.shape[0], c.num_experts, dtype=torch.float32, device=xn.device)
      require().router_logits(xn.contiguous(), lw.router.contiguous(), logits)
    else:
      logits = linear(xn, lw.router, out_dtype=torch.float32)  # [T, E]
    if xn.is_cuda:
      return self._moe_gpu(xn, lw, h, logits, next_norm)
    if self._ds_route:
      topw, topi = K.moe_route_ds(logits, lw.router_bias, *self._route_args())
    else:
      probs = torch.softmax(logits, dim=-1)
      topw, topi = torch.topk(probs, c.num_experts_per_tok, dim=-1)
      topw = topw / topw.sum(-1, keepdim=True)
    T = xn.shape[0]
    flat_e = topi.reshape(-1)
    order = torch.argsort(flat_e, stable=True)
    tok = order // c.num_experts_per_tok
    counts = torch.bincount(flat_e, minlength=c.num_experts).tolist()
    out = torch.zeros(T, c.hidden_size, device=xn.device, dtype=torch.float32)
    start = 0
    wflat = topw.reshape(-1)[order]
    for e, n in enumerate(counts):
      if n == 0:
        continue
      idx = tok[start:start + n]
      xe = xn.index_select(0, idx)  # (expert weights of Fe = c.expert_dim rows)
      act = linear(xe, expert(lw.gu_w, e), epi="silu")
      ye = linear(act, expert(lw.down_w, e), out_dtype=torch.float32)
      out.index_add_(0, idx, ye * wflat[start:start + n, None])
      start += n
    h += out.to(h.dtype)
    return None

  def _moe_gpu(self, xn: torch.Tensor, lw, h: torch.Tensor, logits: torch.Tensor,
               next_norm: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Device-only MoE (graph-capturable): routing kernel (softmax top-k, per-expert slot order),
    grouped gate/up GEMM gathering token rows with the SiLU*mul epilogue, grouped down GEMM into fp32
    slots, combine kernel adding sum_j w_j * y_slot(j) into the residual stream."""
    c = self.c
    T, D = xn.shape
    k, E, F = c.num_experts_per_tok, c.num_experts, c.expert_dim
    dev = xn.device
    C = require()
    topw = torch.empty(T * k, dtype=torch.float32, device=dev)
    topi = torch.empty(T * k, dtype=torch.int32, device=dev)
    slot_of = torch.empty(T * k, dtype=torch.int32, device=dev)
    sorted_tok = torch.empty(T * k, dtype=torch.int32, device=dev)
    off = torch.empty(E + 1, dtype=torch.int32, device=dev)
    if self._ds_route:
      K.moe_route_ds(logits, lw.router_bias, *self._route_args(), outs=(topw, topi, slot_of, sorted_tok, off))
    else:
      C.moe_route(logits.contiguous(), k, topw, topi, slot_of, sorted_tok, off)
    shuffled = layout_of(lw.gu_w) == "stream" and layout_of(lw.down_w) == "stream"
    # rows per expert decide the kernel: the weight-streaming GEMM for decode-sized groups, gemm_big
    # tiles (128 or 256 rows) once the groups are compute-bound
    rows = T * k / E
    bm, bm_dn, S_dn = (0, 0, 0) if not shuffled or rows < MOE_BIG_MIN_ROWS else moe_tiles(rows, E)
    if MOE_PP2:  # 256- / 192-row expert tiles on the two-phase ping-pong schedule (csrc/gemm_big.hip 2256 / 2192)
      bm, bm_dn = ({256: 2256, 192: 2192}.get(b, b) for b in (bm, bm_dn))
    if MOE_BM and bm:
      bm = bm_dn = MOE_BM
    if MOE_DN_SPLITS and bm:
      S_dn = MOE_DN_SPLITS
    act = torch.empty(T * k, F, dtype=torch.bfloat16, device=dev)
    Sg = MOE_GU_SPLITS if (bm == 0 and T * k <= 32 and D % (256 * MOE_GU_SPLITS) == 0) else 1
    if Sg > 1:
      # decode-sized groups: the weight-streaming gate/up split over K into fp32 slabs (k experts x N/128
      # column blocks alone leave the last wave of workgroups short, e.g. 448 on 512 slots at batch 1),
      # SiLU*mul applied by the slab reduce
      ys = torch.empty(Sg * T * k, 2 * F, dtype=torch.float32, device=dev)
      C.gemm_moe(xn, lw.gu_w, ys, off, sorted_tok, K.EPI["none"], T, layout_of(lw.gu_w) == "stream", Sg, 0)
      C.splitk_silu(ys, Sg, act)
    else:
      C.gemm_moe(xn, lw.gu_w, act, off, sorted_tok, K.EPI["silu"], T, layout_of(lw.gu_w) == "stream", 1, bm)
    # down projection split over K (fp32 partial slabs summed by the combine): the grouped GEMM only has
    # (experts hit) x N/tile workgroups with work, too few to stream the expert weights at full HBM rate
    S = (4 if T * k <= 64 else 2) if bm == 0 else S_dn
    if F % (256 * S):
      S = 1
    y = torch.empty(S * T * k, D, dtype=torch.float32, device=dev)
    C.gemm_moe(act, lw.down_w, y, off, None, K.EPI["none"], T, layout_of(lw.down_w) == "stream", S, bm_dn)
    if next_norm is not None:  # combine + the following RMSNorm in one kernel
      out = torch.empty_like(h)
      C.moe_combine_norm(y, slot_of, topw, h, S, next_norm, out, float(c.rms_norm_eps))
      return out
    C.moe_combine(y, slot_of, topw, h, S)
    return None

  # ------------------------------------------------------------------ forward
  @torch.inference_mode()
  def forward(self, x: torch.Tensor, inp: StepInputs) -> torch.Tensor:
    """x: token ids [T] (first shard) or hidden [T, D] bf16.  Returns hidden [T, D] (non-last shard)
    or fp32 logits [B, V] of each sequence's last token (last shard)."""
    c, w = self.c, self.w
    if self.shard.is_first_layer():
      h = K.embedding(x, w.embed)
      if inp.image_embeds is not None:  # LLaVA: projected image features replace the image-token rows
        rows = (x.view(-1) == c.image_token_id).nonzero().view(-1)
        if rows.numel() != inp.image_embeds.shape[0]:
          raise ValueError(f"{rows.numel()} image tokens but {inp.image_embeds.shape[0]} image feature rows")
        h.index_copy_(0, rows, inp.image_embeds.to(h.dtype))
    else:
      h = x.contiguous().clone() if x.dtype == torch.bfloat16 else x.to(torch.bfloat16).contiguous()
    last = self.shard.is_last_layer()
    n = len(self.layer_ids)
    xn, _ = K.rmsnorm(h, w.layers[self.layer_ids[0]].ln1, c.rms_norm_eps) if n else (None, None)
    # batch-1 decode: the split-K reduce + residual + RMSNorm after o_proj / down_proj is deferred into the next
    # GEMM's prologue (ops.linear.PendingNorm); the residual stream then alternates between two row buffers
    fuse = FUSE_NORM and h.is_cuda and h.shape[0] == 1 and not c.is_mla and n > 0
    hb = (h, torch.empty_like(h)) if fuse else None
    other = (lambda t: hb[1] if t is hb[0] else hb[0]) if fuse else (lambda t: None)
    for j, li in enumerate(self.layer_ids):
      lw = w.layers[li]
      if c.is_mla:
        a = self._mla(xn, lw, j, inp)
      else:
        # QKV projection + RoPE + paged KV write (split-K slabs reduced inside the RoPE kernel)
        q = linear_rope_kv(xn, lw.qkv_w, lw.qkv_b, inp.positions, self.cos_sin, inp.slots, self.kv.k[j],
                           self.kv.v[j], c.num_heads, c.num_kv_heads)
        if isinstance(xn, PendingNorm):
          h = xn.dst
        a = self._attention(q, j, inp, defer_merge=fuse and FUSE_MERGE and lw.router is None)
        if not isinstance(a, K.PendingMerge):  # (a pending merge is finished inside o_proj's prologue)
          a = a.view(h.shape[0], c.num_heads * c.head_dim)
      # o_proj + residual + post-attention norm (one fused pass when the projection runs split-K)
      xn = linear_resid_norm(a, lw.o_w, h, lw.ln2, c.rms_norm_eps,
                             defer_to=other(h) if lw.router is None else None)
      if isinstance(xn, PendingNorm):
        h = xn.dst  # gate/up's prologue stores the summed residual there
      # the norm that follows this layer: the next layer's input norm, or the final norm (decode: every row
      # is a sequence's last token) -- fused into the down projection's reduce the same way
      nxt = w.layers[self.layer_ids[j + 1]].ln1 if j + 1 < n else (w.norm if last and inp.decode else None)
      xn = self._mlp(xn, lw, h, nxt, li, defer_to=other(h) if j + 1 < n else None)
    if not last:
      return h
    if not inp.decode or n == 0:
      hl = h.index_select(0, inp.last_idx) if not inp.decode else h
      xn, _ = K.rmsnorm(hl, w.norm, c.rms_norm_eps)
    if self.head_rows is None:
      return linear(xn, w.lm_head, out_dtype=torch.float32)
    # LM head split with another stage (parallel/pipeline.py): logits of vocab rows [0, head_rows) and
    # the normed hidden state the other stage applies the remaining rows to
    return linear(xn, self._head_slice(), out_dtype=torch.float32), xn

  def _head_slice(self) -> torch.Tensor:
    w = self.w.lm_head
    if self._head_cache is None or self._head_cache[0] != self.head_rows:
      # rows [0, r) of the pre-shuffled layout (16-row groups) are a storage prefix: a view, no copy
      hs = w[: self.head_rows]
      if layout_of(w) != "rowmajor":
        hs.xot_layout = layout_of(w)
      self._head_cache = (self.head_rows, hs)
    return self._head_cache[1]


def make_step_inputs(seqs: List[tuple], device, block_width: Optional[int] = None) -> StepInputs:
  """Host helper: seqs = [(positions list, slots list, block_table list, ctx_len)] -> StepInputs."""
  pos, slots, cu, last = [], [], [0], []
  width = block_width or max(1, max(len(s[2]) for s in seqs))
  tables = torch.zeros(len(seqs), width, dtype=torch.int32)
  ctx = torch.zeros(len(seqs), dtype=torch.int32)
  for b, (p, s, bt, n) in enumerate(seqs):
    pos += list(p)
    slots += list(s)
    cu.append(cu[-1] + len(p))
    last.append(cu[-1] - 1)
    tables[b, :len(bt)] = torch.tensor(bt, dtype=torch.int32)
    ctx[b] = n
  qlens = [cu[i + 1] - cu[i] for i in range(len(seqs))]
  return StepInputs(
    positions=torch.tensor(pos, dtype=torch.int32, device=device),
    slots=torch.tensor(slots, dtype=torch.int64, device=device),
    block_tables=tables.to(device),
    ctx_lens=ctx.to(device),
    cu_q=torch.tensor(cu, dtype=torch.int32, device=device),
    last_idx=torch.tensor(last, dtype=torch.int64, device=device),
    max_qlen=max(qlens),
    decode=all(q == 1 for q in qlens),
  )
