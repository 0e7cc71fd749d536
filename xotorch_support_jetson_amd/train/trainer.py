"""Pipeline-stage trainer: the engine.train / engine.evaluate the reference's Node calls but never
implements (xotorch/orchestration/node.py:299-345, inference_engine.py:34-35).

Protocol (one micro-batch, synchronous, like the reference's SendExample recursion):
  non-last stage:  out = train_forward(x)  -> next stage ... -> grad wrt out comes back
                   step(x, grad_out, loss="back_gradient")  -> backward + AdamW, returns grad wrt x
  last stage:      step(x, y, lengths)     -> length-masked CE, backward + AdamW, returns (loss, grad wrt x)
The stage recomputes its forward inside `step` (activation checkpointing at stage granularity), so
no activations are kept between the hops.

Numerics: bf16 working weights (leaf tensors with grads), fp32 master weights + fp32 AdamW moments
updated by the fused HIP AdamW kernel, which also refreshes the bf16 copy.  RMSNorm, SiLU*mul, RoPE,
the causal GQA attention (flash-style fwd / dQ / dK-dV kernels), the projections (OwnLinearFn: forward, dX and
dW on the MFMA tiles, ragged token counts zero-padded to 128 rows) and the LM head + cross-entropy (LmHeadCEFn,
chunked, no [T, V] logits) run on the kernel library; torch GEMMs remain only on the CPU and for shapes the
tiles do not cover.  Updated weights are written back into the inference shard lazily
(`sync_to_inference`) so `xot run` after `xot train` uses the trained model.
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from ..models.config import ModelConfig
from ..models.weights import ShardWeights, _rowmajor, interleave_gate_up, split_gate_up
from ..ops._ext import require
from ..ops.rope import longrope_window, rope_shift, rope_table
from . import autograd_ops as A


# XOT_TRAIN_OWN_GEMM=0: projections on torch.matmul (hipBLASLt) instead of the MFMA kernels (A/B, debugging)
OWN_GEMM = os.environ.get("XOT_TRAIN_OWN_GEMM", "1") == "1"
# XOT_FUSED_CE=0: materialise [T, V] logits and run the separate cross-entropy (A/B, debugging)
FUSED_CE = os.environ.get("XOT_FUSED_CE", "1") == "1"
# rows per fused LM-head + CE chunk: 4096 (one [4096, V] fp32 logits block, 2.1 GB at V = 128256) ran the
# Llama-3-8B step 1.1 % faster than 1024 (profiles/r5/train/knobs_r5s/)
CE_CHUNK = int(os.environ.get("XOT_CE_CHUNK", "4096"))


def _resid_mm(h: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
  """h + x @ w.T; on the GPU the residual add rides in the hipBLASLt epilogue (addmm, beta = 1)."""
  return torch.addmm(h, x, w.t()) if h.is_cuda else h + x @ w.t()


class ShardTrainer:
  def __init__(self, weights: ShardWeights, device, lr: float = 1e-5, betas=(0.9, 0.95), eps: float = 1e-8,
               weight_decay: float = 0.0, max_seq: int = 4096, grad_clip: float = 1.0):
    self.w = weights
    self.c: ModelConfig = weights.config
    self.shard = weights.shard
    self.device = torch.device(device)
    self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
    self.grad_clip = grad_clip
    self.step_count = 0
    self.dirty = False
    self.cos_sin = rope_table(self.c, max_seq, self.device)
    self.max_seq = max_seq
    # training parameters (row-major, gate|up halves), bf16 leaves + fp32 master + moments
    self.params: Dict[str, torch.Tensor] = {}
    self.router_bias: Dict[int, torch.Tensor] = {}  # DeepSeek-V3 selection bias: a buffer, not trained
    c = self.c
    for i, lw in weights.layers.items():
      g, u = split_gate_up(_rowmajor(lw.gu_w))  # [F, D] each, or [E, F, D] expert stacks
      self._add(f"{i}.qkv", _rowmajor(lw.qkv_w))  # MLA: the fused A projection [q_a | kv latent | rope key]
      if lw.qkv_b is not None:
        self._add(f"{i}.qkv_b", lw.qkv_b)
      self._add(f"{i}.o", _rowmajor(lw.o_w))
      if c.is_mla:
        if c.q_lora_rank:
          self._add(f"{i}.q_ln", lw.q_ln)
          self._add(f"{i}.qb", _rowmajor(lw.qb_w))
        self._add(f"{i}.kv_ln", lw.kv_ln)
        # kv_b_proj as one [H (dn + dv), kv_lora] projection (HF layout; the serving path splits it)
        self._add(f"{i}.kvb", torch.cat([_rowmajor(lw.wuk), _rowmajor(lw.wuv)], 1).reshape(-1, c.kv_lora_rank))
      if lw.router is not None:  # MoE: router [E, D], experts' gate|up [E, 2F, D], down [E, D, F]
        self._add(f"{i}.router", _rowmajor(lw.router))
        self._add(f"{i}.egu", torch.cat([g, u], 1))
        self._add(f"{i}.edown", _rowmajor(lw.down_w))
        if lw.router_bias is not None:
          self.router_bias[i] = lw.router_bias.detach().to(self.device, torch.float32)
        if lw.sh_gu_w is not None:  # DeepSeek shared experts: a dense SwiGLU
          sg, su = split_gate_up(_rowmajor(lw.sh_gu_w))
          self._add(f"{i}.sh_gu", torch.cat([sg, su], 0))
          self._add(f"{i}.sh_down", _rowmajor(lw.sh_down_w))
      else:
        self._add(f"{i}.gu", torch.cat([g, u], 0))
        self._add(f"{i}.down", _rowmajor(lw.down_w))
      self._add(f"{i}.ln1", lw.ln1)
      self._add(f"{i}.ln2", lw.ln2)
    if weights.embed is not None and self.shard.is_first_layer():
      self._add("embed", weights.embed)
    if self.shard.is_last_layer():
      self._add("norm", weights.norm)
      if not self.c.tie_word_embeddings or "embed" not in self.params:
        self._add("lm_head", _rowmajor(weights.lm_head))
    # projection weights accumulate their gradients inside the backward GEMM (A.LinearFn) on the GPU
    self.acc: Dict[str, A.GradAcc] = {}
    if self.device.type == "cuda":
      for k in self.params:
        if k.split(".")[-1] in ("qkv", "o", "gu", "down", "egu", "edown", "qb", "kvb", "sh_gu", "sh_down"):
          self.acc[k] = A.GradAcc(k, self.params[k])
    # own-GEMM operand layouts of the 2-D projections and expert stacks (refreshed after each optimizer step)
    self.tw: Dict[str, object] = {}
    if self.device.type == "cuda" and OWN_GEMM:
      for k in self.acc:
        t = A.TrainWeight(self.params[k]) if self.params[k].dim() == 2 else A.StackWeight(self.params[k])
        if t.ok:
          self.tw[k] = t
    # fused LM head + chunked CE on the last stage (A.LmHeadCEFn): forward_train hands back the final normed
    # hidden state and backward_accumulate computes the loss from it without [T, V] logits
    self.head_name = None
    if self.shard.is_last_layer():
      self.head_name = "lm_head" if "lm_head" in self.params else "embed"
    if self.device.type == "cuda" and OWN_GEMM and FUSED_CE and self.head_name in self.params:
      t = A.TrainWeight(self.params[self.head_name])
      if t.ok:
        self.tw[self.head_name] = t
        if self.head_name == "lm_head":  # untied: the fused CE accumulates dHead into a GradAcc (A.LmHeadCEFn)
          self.acc["lm_head"] = A.GradAcc("lm_head", self.params["lm_head"])
    # RMSNorm weights: the backward kernel's dw reduce adds into an fp32 GradAcc across micro-batches (no zeroed
    # vector, bf16 copy and autograd accumulation add per norm and micro-batch)
    if self.device.type == "cuda":
      for k in self.params:
        if k == "norm" or k.split(".")[-1] in ("ln1", "ln2"):
          a = A.GradAcc(k, self.params[k])
          a.buf = torch.empty(self.params[k].shape, dtype=torch.float32, device=self.device)
          self.acc[k] = a
    # untied input embedding: its gradient accumulates into an fp32 GradAcc (A.EmbedAccFn), not a dense autograd
    # gradient per micro-batch (after the TrainWeight loop above: the table has no operand images)
    if self.device.type == "cuda" and "embed" in self.params and self.head_name != "embed":
      a = A.GradAcc("embed", self.params["embed"])
      a.buf = torch.empty(self.params["embed"].shape, dtype=torch.float32, device=self.device)
      self.acc["embed"] = a
    self.master = {k: p.detach().float().clone() for k, p in self.params.items()}
    self._pb_stale: set = set()  # bf16 params the fused AdamW did not rewrite (refresh_params)
    self.m = {k: torch.zeros_like(v) for k, v in self.master.items()}
    self.v = {k: torch.zeros_like(v) for k, v in self.master.items()}

  def _add(self, name: str, t: torch.Tensor):
    self.params[name] = t.detach().to(self.device, torch.bfloat16).clone().requires_grad_(True)

  # ------------------------------------------------------------------ model
  def fused_head(self) -> bool:
    return self.head_name is not None and self.head_name in self.tw

  def forward(self, x: torch.Tensor, logits: bool = True) -> torch.Tensor:
    """x: ids [B, L] (first stage) or hidden [B, L, D].  Returns hidden [B, L, D] or logits [B, L, V]
    (logits=False on the last stage: the final normed hidden state [B, L, D], for the fused head + CE)."""
    c, P = self.c, self.params
    H, Hkv, Dh, D = c.num_heads, c.num_kv_heads, c.head_dim, c.hidden_size
    if self.shard.is_first_layer():
      ids = x.long().clamp(0, c.vocab_size - 1)
      acc = self.acc.get("embed")
      h = A.embed_acc(ids, P["embed"], acc) if acc is not None and torch.is_grad_enabled() else F.embedding(ids, P["embed"])
    else:
      h = x.to(torch.bfloat16)
    B, L = h.shape[0], h.shape[1]
    # (LongRoPE: a training sequence longer than the pretraining window rotates with the long factors, as HF)
    shift = rope_shift(longrope_window(self.c), self.max_seq, L)
    pos = (torch.arange(L, device=self.device, dtype=torch.int32) + shift).repeat(B)
    h = h.reshape(B * L, D)
    for i in self.shard.layers():
      h, xn = A.res_rmsnorm(h, P[f"{i}.ln1"], c.rms_norm_eps, self.acc.get(f"{i}.ln1"))
      if c.is_mla:
        a = self._mla(xn, i, pos, B, L)
      else:
        qkv = self._mm(xn, f"{i}.qkv")
        if f"{i}.qkv_b" in P:
          qkv = qkv + P[f"{i}.qkv_b"]
        a = A.qkv_attention(qkv, pos, self.cos_sin, B, L, H, Hkv, Dh)  # RoPE + flash-style HIP kernels
      h = self._mm(a, f"{i}.o", h)
      h, xn = A.res_rmsnorm(h, P[f"{i}.ln2"], c.rms_norm_eps, self.acc.get(f"{i}.ln2"))
      if f"{i}.router" in P:
        h = h + self._moe(xn, i)
      else:
        h = self._ffn(xn, f"{i}.gu", f"{i}.down", h)
    if not self.shard.is_last_layer():
      return h.view(B, L, D)
    xn = A.rmsnorm(h, P["norm"], c.rms_norm_eps, self.acc.get("norm"))
    if not logits:
      return xn.view(B, L, D)
    head = P["lm_head"] if "lm_head" in P else P["embed"]
    tw = self.tw.get(self.head_name)
    if tw is not None and not torch.is_grad_enabled():
      from ..ops.linear import linear
      return linear(xn.contiguous(), tw.ws).view(B, L, -1)
    return (xn @ head.t()).view(B, L, -1)

  def _mla(self, xn: torch.Tensor, i: int, pos: torch.Tensor, B: int, L: int) -> torch.Tensor:
    """DeepSeek multi-head latent attention with autograd, in HF's expanded form (training sees whole
    sequences, so the key / value up-projection runs once per token): A = xn . [q_a | kv_a]^T,
    q = rmsnorm(q_a) . q_b^T, latent c = rmsnorm(kv_a), k_pe = rope(shared key), [k_nope | v] = c . kv_b^T,
    causal attention over [q_nope | q_pe] . [k_nope | k_pe] (192-wide q/k, 128-wide v; on the GPU the MFMA
    flash kernels with v zero-padded to 192)."""
    c, P = self.c, self.params
    T = xn.shape[0]
    H, dn, dr, dv, Lr = c.num_heads, c.qk_nope_head_dim, c.qk_rope_head_dim, c.v_head_dim, c.kv_lora_rank
    nq = c.q_lora_rank or H * (dn + dr)
    a = self._mm(xn, f"{i}.qkv")
    if c.q_lora_rank:
      q = self._mm(A.rmsnorm(a[:, :nq].contiguous(), P[f"{i}.q_ln"], c.rms_norm_eps), f"{i}.qb")
    else:
      q = a[:, :nq]
    cn = A.rmsnorm(a[:, nq:nq + Lr].contiguous(), P[f"{i}.kv_ln"], c.rms_norm_eps)
    kpe = A.rope(a[:, nq + Lr:].contiguous(), pos, self.cos_sin, 1, dr)
    qpe = A.rope(q[:, H * dn:].contiguous(), pos, self.cos_sin, H, dr)
    kv = self._mm(cn, f"{i}.kvb").view(T, H, dn + dv)
    qf = torch.cat([q[:, :H * dn].reshape(T, H, dn), qpe.view(T, H, dr)], -1)
    kf = torch.cat([kv[..., :dn], kpe.view(T, 1, dr).expand(T, H, dr)], -1)
    vf = kv[..., dn:]

    if xn.is_cuda and dn + dr in A.ATTN_DH and dv <= dn + dr:  # the MFMA flash kernels (v padded to 192)
      return A.attention_qk_v(qf.reshape(T, -1), kf.reshape(T, -1), vf.reshape(T, -1), B, L, H, dn + dr, dv,
                              c.attn_scale())

    def heads(t):  # CPU reference (and head sizes the kernels do not cover: the tiny test configs)
      return t.reshape(B, L, H, -1).transpose(1, 2)
    o = F.scaled_dot_product_attention(heads(qf), heads(kf), heads(vf), is_causal=True, scale=c.attn_scale())
    return o.transpose(1, 2).reshape(T, H * dv)

  def _route(self, logits: torch.Tensor, i: int):
    """(weights [T, k] with autograd to the router, expert ids [T, k]): Mixtral softmax top-k renormalised,
    or DeepSeek's rule (ops.reference.moe_route_ds: groups, sigmoid scores + selection bias, scale)."""
    c = self.c
    ds = not (c.topk_method == "greedy" and c.scoring_func == "softmax" and c.norm_topk_prob
              and c.routed_scaling_factor == 1.0)
    if not ds:
      topw, topi = torch.topk(torch.softmax(logits, dim=-1), c.num_experts_per_tok, dim=-1)
      return topw / topw.sum(-1, keepdim=True), topi
    from ..ops.reference import moe_route_ds
    method = {"greedy": 0, "group_limited_greedy": 1, "noaux_tc": 2}[c.topk_method]
    with torch.no_grad():  # the selection itself is not differentiable
      _, topi = moe_route_ds(logits.detach(), self.router_bias.get(i), c.num_experts_per_tok,
                             c.n_group if method else 1, c.topk_group if method else 1, method,
                             c.scoring_func == "sigmoid", c.norm_topk_prob, c.routed_scaling_factor)
    scores = torch.sigmoid(logits) if c.scoring_func == "sigmoid" else torch.softmax(logits, dim=-1)
    topw = scores.gather(1, topi)
    if c.norm_topk_prob:
      topw = topw / (topw.sum(-1, keepdim=True) + 1e-20)
    return topw * c.routed_scaling_factor, topi

  def _moe(self, xn: torch.Tensor, i: int) -> torch.Tensor:
    """Sparse MLP with autograd: fp32 router scores, top-k weights (the router learns through them; Mixtral
    renormalised softmax or DeepSeek's routing), each expert's gate/up -> SiLU*mul -> down on the rows
    routed to it, weighted fp32 scatter-add, plus DeepSeek's shared experts.  Same routing as the
    inference path (models/transformer.py `_moe`)."""
    c, P = self.c, self.params
    logits = A.router_logits(xn, P[f"{i}.router"])  # [T, E] fp32
    topw, topi = self._route(logits, i)
    sgu, sdown = self.tw.get(f"{i}.egu"), self.tw.get(f"{i}.edown")
    if sgu is not None and sdown is not None and f"{i}.egu" in self.acc and f"{i}.edown" in self.acc:
      out = self._moe_grouped(xn, i, topw, topi, sgu, sdown)
      if f"{i}.sh_gu" in P:
        out = out + self._mm(A.silu_mul(self._mm(xn, f"{i}.sh_gu").contiguous()), f"{i}.sh_down").float()
      return out.to(xn.dtype)
    # per-expert views, taken once per layer: indexing egu[e] per expert would zero-fill and add a full
    # [E, 2F, D] gradient for every expert; on the GPU the routed experts' grads go straight into the
    # stack's accumulation buffer (A.StackAccFn)
    ea, da = self.acc.get(f"{i}.egu"), self.acc.get(f"{i}.edown")
    if ea is not None and torch.is_grad_enabled():
      egu, edown = A.unbind_acc(P[f"{i}.egu"], ea), A.unbind_acc(P[f"{i}.edown"], da)
    else:
      egu, edown = P[f"{i}.egu"].unbind(0), P[f"{i}.edown"].unbind(0)
    # group the (token, slot) pairs by expert: one gather, one host sync for the group sizes
    flat = topi.reshape(-1)
    order = torch.argsort(flat, stable=True)
    tok = order // c.num_experts_per_tok
    counts = torch.bincount(flat, minlength=c.num_experts).tolist()
    xs = xn.index_select(0, tok)
    ys, start = [], 0
    for e, n in enumerate(counts):
      if n:
        ys.append(A.silu_mul((xs[start:start + n] @ egu[e].t()).contiguous()) @ edown[e].t())
      start += n
    y = torch.cat(ys).float() * topw.reshape(-1)[order].unsqueeze(1)
    out = torch.zeros(xn.shape[0], c.hidden_size, device=xn.device, dtype=torch.float32).index_add(0, tok, y)
    if f"{i}.sh_gu" in P:
      out = out + self._mm(A.silu_mul(self._mm(xn, f"{i}.sh_gu").contiguous()), f"{i}.sh_down").float()
    return out.to(xn.dtype)

  def _moe_grouped(self, xn: torch.Tensor, i: int, topw: torch.Tensor, topi: torch.Tensor, sgu, sdown) -> torch.Tensor:
    """Routed experts on the grouped kernels with no host sync (A.GroupedExpertsFn): the (token, choice)
    rows are scattered into a slot array where expert e's rows start at poff[e], a multiple of 64 (zero
    rows pad each segment; the array is sized for the worst case T k + 63 E, so no count leaves the
    device), and the weighted expert outputs are gathered back and summed per token in fp32."""
    c = self.c
    T, D = xn.shape
    k, E = c.num_experts_per_tok, c.num_experts
    dev = xn.device
    flat = topi.reshape(-1)
    counts = torch.bincount(flat, minlength=E)
    start = torch.cumsum(counts, 0) - counts  # first sorted slot of each expert
    pad = (counts + 63) // 64 * 64
    poff = torch.zeros(E + 1, dtype=torch.int32, device=dev)
    poff[1:] = torch.cumsum(pad, 0).to(torch.int32)
    order = torch.argsort(flat, stable=True)
    se = flat[order]
    dest = poff[se].long() + torch.arange(T * k, device=dev) - start[se]
    tok = order // k
    P = -(-(T * k + 63 * E) // 128) * 128
    xs = torch.zeros(P, D, dtype=xn.dtype, device=dev).index_copy(0, dest, xn.index_select(0, tok))
    y = A.grouped_experts(xs, poff, -(-T // 64) * 64, sgu, sdown, self.acc[f"{i}.egu"], self.acc[f"{i}.edown"])
    y = y.index_select(0, dest).float() * topw.reshape(-1)[order].unsqueeze(1)
    return torch.zeros(T, D, device=dev, dtype=torch.float32).index_add(0, tok, y)

  def _ffn(self, xn: torch.Tensor, gu: str, down: str, h: torch.Tensor) -> torch.Tensor:
    """h + down(silu(gate) * up) of the gated MLP; while training on the own GEMMs as one A.SiluDownFn (the SiLU
    backward runs in the down projection's input-gradient GEMM epilogue)."""
    g = self._mm(xn, gu)
    tw, acc = self.tw.get(down), self.acc.get(down)
    if torch.is_grad_enabled() and isinstance(tw, A.TrainWeight) and acc is not None:
      return A.silu_down_own(g, self.params[down], tw, acc, h)
    return self._mm(A.silu_mul(g.contiguous()), down, h)

  def _mm(self, x: torch.Tensor, name: str, h: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x @ W.T (+ h) for projection `name`: fused gradient accumulation on the GPU while training."""
    w = self.params[name]
    acc = self.acc.get(name)
    tw = self.tw.get(name)
    if tw is not None and (acc is not None or not torch.is_grad_enabled()):
      if torch.is_grad_enabled():
        return A.linear_own(x, w, tw, acc, h)
      from ..ops.linear import linear
      x = x if (x.stride(1) == 1 and x.stride(0) % 8 == 0) else x.contiguous()
      return linear(x, tw.ws, residual=h.contiguous(), epi="resid") if h is not None else linear(x, tw.ws)
    if acc is not None and torch.is_grad_enabled():
      return A.linear_acc(x, w, acc, h)
    return _resid_mm(h, x, w) if h is not None else x @ w.t()

  def grads(self) -> Dict[str, torch.Tensor]:
    """The accumulated gradients of this step: fused buffers and .grad of the other parameters."""
    A.join_dw_stream()
    out = {k: a.buf for k, a in self.acc.items() if not a.fresh}
    for k, p in self.params.items():
      if k not in out and p.grad is not None:
        out[k] = p.grad
    return out

  # ------------------------------------------------------------------ steps
  def _to(self, a, dtype=None):
    t = a if isinstance(a, torch.Tensor) else torch.as_tensor(np.asarray(a))
    return t.to(self.device, dtype) if dtype is not None else t.to(self.device)

  @torch.no_grad()
  def train_forward(self, example) -> torch.Tensor:
    x = self._to(example)
    return self.forward(x).detach().cpu()

  def loss_of(self, logits: torch.Tensor, target, lengths, denom: Optional[float] = None) -> Tuple[torch.Tensor, int]:
    """Length-masked CE summed over valid tokens / denom (default: this batch's valid-token count)."""
    B, L, V = logits.shape
    y = self._to(target, torch.int64)
    ln = self._to(lengths, torch.int64).view(-1)
    mask = torch.arange(L, device=self.device)[None, :] < ln[:, None]
    tgt = torch.where(mask, y, torch.full_like(y, -100)).view(-1).to(torch.int32)
    if denom is None:
      n = int(mask.sum().item())
      denom = float(max(n, 1))
    else:
      n = -1  # not computed (no host sync)
    w = torch.full((B * L,), 1.0 / denom, device=self.device, dtype=torch.float32)
    return A.cross_entropy(logits.reshape(B * L, V), tgt, w), n

  def head_loss(self, xn: torch.Tensor, target, lengths, denom: float) -> torch.Tensor:
    """The fused LM head + chunked CE of loss_of, from the final normed hidden state [B, L, D]."""
    B, L, D = xn.shape
    y = self._to(target, torch.int64)
    ln = self._to(lengths, torch.int64).view(-1)
    mask = torch.arange(L, device=self.device)[None, :] < ln[:, None]
    tgt = torch.where(mask, y, torch.full_like(y, -100)).view(-1).to(torch.int32)
    w = torch.full((B * L,), 1.0 / denom, device=self.device, dtype=torch.float32)
    name = self.head_name
    return A.lm_head_ce(xn.reshape(B * L, D), self.params[name], self.tw[name], tgt, w, CE_CHUNK, self.acc.get(name))

  # ------------------------------------------------------------------ accumulate / apply
  # (pipeline schedules: forward every micro-batch, backward every micro-batch, then one optimizer
  # step; see parallel/pipeline_train.py)
  def zero_grad(self) -> None:
    for p in self.params.values():
      p.grad = None
    for a in self.acc.values():
      a.fresh = True

  def forward_train(self, x) -> Tuple[Optional[torch.Tensor], torch.Tensor]:
    """Forward with autograd: returns (input leaf or None for token ids, output)."""
    x = self._to(x)
    leaf = None
    if not self.shard.is_first_layer():
      leaf = x.to(torch.bfloat16).detach().requires_grad_(True)
      x = leaf
    return leaf, self.forward(x, logits=not self.fused_head())

  def backward_accumulate(self, leaf, out, grad_out=None, target=None, length=None,
                          denom: Optional[float] = None) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """Accumulate parameter grads of one micro-batch.  Last stage: CE(out, target) / denom (returned
    as a device scalar, no sync); other stages: out.backward(grad_out).  Returns (loss, grad wrt input)."""
    loss = None
    if grad_out is None:
      if self.fused_head():  # forward_train returned the final normed hidden state
        if denom is None:
          denom = float(max(int((self._to(length, torch.int64)).sum().item()), 1))
        loss = self.head_loss(out, target, length, denom)
      else:
        loss, _ = self.loss_of(out, target, length, denom)
      loss.backward()
      loss = loss.detach()
    else:
      out.backward(grad_out.to(out.dtype).view_as(out))
    return loss, (leaf.grad if leaf is not None else None)

  def apply(self, grad_norm_sq_reduce=None, norm_exclude=(), grads: Optional[Dict[str, torch.Tensor]] = None) -> None:
    """One AdamW step on the accumulated grads.  `grad_norm_sq_reduce(t)` (e.g. an all-reduce over
    the pipeline stages) turns the local squared grad norm into the global one for clipping;
    `norm_exclude` names parameters counted by another stage (a tied head copy); `grads` overrides
    the parameters' .grad (e.g. fp32 all-reduced buckets of data parallelism)."""
    self._optimizer_step(grad_norm_sq_reduce, norm_exclude, grads)

  def step(self, request_id, example, target, length, train: bool = True, evaluate: bool = False,
           loss: str = "length_masked_ce"):
    x = self._to(example)
    need_in_grad = not self.shard.is_first_layer()
    if need_in_grad:
      x = x.to(torch.bfloat16).detach().requires_grad_(train)
    if not train:
      with torch.no_grad():
        out = self.forward(x)
        if self.shard.is_last_layer():
          l, _ = self.loss_of(out, target, length)
          return float(l)
        return 0.0
    self.zero_grad()
    head_loss = self.shard.is_last_layer() and loss != "back_gradient"
    fused = head_loss and self.fused_head()
    out = self.forward(x, logits=not fused)
    if fused:  # the LM head + CE on own GEMMs, chunked: no [T, V] logits (A.LmHeadCEFn)
      L = out.shape[1]
      denom = float(max(int(self._to(length, torch.int64).clamp(max=L).sum()), 1))
      lval = self.head_loss(out, target, length, denom)
      lval.backward()
      loss_out = float(lval.detach())
    elif head_loss:
      lval, _ = self.loss_of(out, target, length)
      lval.backward()
      loss_out = float(lval.detach())
    else:
      g = self._to(target).to(out.dtype)
      out.backward(g.view_as(out))
      loss_out = 0.0
    self._optimizer_step()
    grad_in = x.grad.detach().cpu() if need_in_grad and x.grad is not None else None
    return loss_out, grad_in

  def _optimizer_step(self, grad_norm_sq_reduce=None, norm_exclude=(), grads=None):
    self.step_count += 1
    if grads is None:
      grads = self.grads()
    counted = [g for k, g in grads.items() if k not in norm_exclude]
    # GPU: one multi-tensor sum-of-squares pass (csrc/train_ops.hip multi_sumsq) over every gradient, no fp32
    # copies; CPU: an fp32-accumulating norm per tensor
    if counted and all(g.is_cuda and g.is_contiguous() and g.dtype in (torch.bfloat16, torch.float32)
                       for g in counted):
      sq = require().multi_sumsq(counted).reshape(())
    else:
      sq = (torch.stack([torch.linalg.vector_norm(g, dtype=torch.float32) for g in counted]).square().sum()
            if counted else torch.zeros((), device=self.device))
    if grad_norm_sq_reduce is not None:
      sq = grad_norm_sq_reduce(sq.reshape(1).float()).reshape(())
    gnorm = torch.sqrt(sq)
    scale = float(min(1.0, self.grad_clip / (float(gnorm) + 1e-6))) if self.grad_clip else 1.0
    b1, b2 = self.betas
    fused = set()
    for k, g in grads.items():
      p, m, v, pb = self.master[k], self.m[k], self.v[k], self.params[k]
      tw = self.tw.get(k)
      if p.is_cuda and isinstance(tw, A.TrainWeight) and p.dim() == 2:
        # the update writes the own-GEMM operand images directly (no bf16 copy + two relayouts); the plain bf16
        # copy only where something may still read it: a projection without a GradAcc runs torch's matmul on it,
        # the LM head / tied embedding is read by the embedding lookup and the unfused logits path.  Projections
        # with a GradAcc read only the images while training; refresh_params() catches their copies up on demand.
        keep = k not in self.acc or k == self.head_name
        require().adamw_tiled(p, g.contiguous(), m, v, pb.data if keep else None, tw.ws, tw.wts, self.lr, b1, b2,
                              self.eps, self.wd, self.step_count, scale)
        fused.add(k)
        if not keep:
          self._pb_stale.add(k)
      elif p.is_cuda:
        require().adamw(p, g.contiguous(), m, v, pb.data, self.lr, b1, b2, self.eps, self.wd, self.step_count, scale)
      else:
        gf = g.float() * scale
        m.mul_(b1).add_(gf, alpha=1 - b1)
        v.mul_(b2).addcmul_(gf, gf, value=1 - b2)
        bc1, bc2 = 1 - b1 ** self.step_count, 1 - b2 ** self.step_count
        p.mul_(1 - self.lr * self.wd).addcdiv_(m / bc1, (v / bc2).sqrt_().add_(self.eps), value=-self.lr)
        pb.data.copy_(p.to(pb.dtype))
    for k, t in self.tw.items():
      if k not in fused:
        t.refresh()
    self.dirty = True

  @torch.no_grad()
  def refresh_params(self) -> None:
    """Bring the plain bf16 parameters the fused AdamW left stale back in line with the fp32 masters."""
    for k in self._pb_stale:
      self.params[k].data.copy_(self.master[k].to(torch.bfloat16))
    self._pb_stale.clear()

  # ------------------------------------------------------------------ write-back
  @torch.no_grad()
  def sync_to_inference(self) -> None:
    """Copy the trained weights into the inference shard (re-interleave gate/up, re-shuffle on GPU)."""
    if not self.dirty:
      return
    self.refresh_params()
    from ..models.weights import assign_weight
    P = self.params
    c = self.c
    Fd = c.intermediate_size
    for i, lw in self.w.layers.items():
      assign_weight(lw.qkv_w, P[f"{i}.qkv"].detach())
      if f"{i}.qkv_b" in P:
        assign_weight(lw.qkv_b, P[f"{i}.qkv_b"].detach())
      assign_weight(lw.o_w, P[f"{i}.o"].detach())
      if c.is_mla:
        if c.q_lora_rank:
          assign_weight(lw.q_ln, P[f"{i}.q_ln"].detach())
          assign_weight(lw.qb_w, P[f"{i}.qb"].detach())
        assign_weight(lw.kv_ln, P[f"{i}.kv_ln"].detach())
        kvb = P[f"{i}.kvb"].detach().view(c.num_heads, c.qk_nope_head_dim + c.v_head_dim, c.kv_lora_rank)
        assign_weight(lw.wuk, kvb[:, :c.qk_nope_head_dim].contiguous())
        assign_weight(lw.wuv, kvb[:, c.qk_nope_head_dim:].contiguous())
      if f"{i}.router" in P:
        Fe = c.expert_dim
        egu = P[f"{i}.egu"].detach()
        assign_weight(lw.gu_w, torch.stack([interleave_gate_up(egu[e, :Fe].contiguous(), egu[e, Fe:].contiguous())
                                            for e in range(egu.shape[0])]))
        assign_weight(lw.down_w, P[f"{i}.edown"].detach())
        assign_weight(lw.router, P[f"{i}.router"].detach())
        if f"{i}.sh_gu" in P:
          sgu = P[f"{i}.sh_gu"].detach()
          Fs = sgu.shape[0] // 2
          assign_weight(lw.sh_gu_w, interleave_gate_up(sgu[:Fs].contiguous(), sgu[Fs:].contiguous()))
          assign_weight(lw.sh_down_w, P[f"{i}.sh_down"].detach())
      else:
        gu = P[f"{i}.gu"].detach()
        assign_weight(lw.gu_w, interleave_gate_up(gu[:Fd].contiguous(), gu[Fd:].contiguous()))
        assign_weight(lw.down_w, P[f"{i}.down"].detach())
      assign_weight(lw.ln1, P[f"{i}.ln1"].detach())
      assign_weight(lw.ln2, P[f"{i}.ln2"].detach())
    if "embed" in P:
      assign_weight(self.w.embed, P["embed"].detach())
    if "norm" in P:
      assign_weight(self.w.norm, P["norm"].detach())
    head = P["lm_head"] if "lm_head" in P else P.get("embed")
    if head is not None and self.w.lm_head is not None and self.w.lm_head is not self.w.embed:
      assign_weight(self.w.lm_head, head.detach())
    self.dirty = False

  def state_dict(self) -> Dict[str, torch.Tensor]:
    out = {}
    for k in self.master:
      out[f"master.{k}"] = self.master[k]
      out[f"m.{k}"] = self.m[k]
      out[f"v.{k}"] = self.v[k]
    out["step"] = torch.tensor([self.step_count], dtype=torch.int64)
    return out

  def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
    for k in self.master:
      if f"master.{k}" in sd:
        self.master[k].copy_(sd[f"master.{k}"])
        self.m[k].copy_(sd[f"m.{k}"])
        self.v[k].copy_(sd[f"v.{k}"])
        self.params[k].data.copy_(self.master[k].to(torch.bfloat16))
    for t in self.tw.values():
      t.refresh()
    if "step" in sd:
      self.step_count = int(sd["step"][0])
