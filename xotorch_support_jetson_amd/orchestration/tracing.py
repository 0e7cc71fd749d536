"""Request tracing (reference: xotorch/orchestration/tracing.py — an OpenTelemetry tracer nothing imports).

Live here, dependency-free:
  * `tracer.span(name, **attrs)`: timed spans kept in a bounded in-memory ring (exported as JSON by
    the API at /v1/traces) and fed to the Prometheus histograms in utils.metrics;
  * per-request contexts with W3C `traceparent` propagation and token-group spans (10 tokens per
    span, like the reference);
  * roctx ranges around each span when XOT_ROCTX=1 so rocprofv3 --marker-trace timelines line up
    host phases (prompt / hop / decode step) with kernels.
"""
from __future__ import annotations

import contextlib
import os
import secrets
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional

_ROCTX = os.environ.get("XOT_ROCTX", "0") == "1"


def _roctx_push(name: str):
  if not _ROCTX:
    return False
  try:
    import torch
    torch.cuda.nvtx.range_push(name)  # maps to roctx on ROCm builds
    return True
  except Exception:
    return False


def _roctx_pop():
  try:
    import torch
    torch.cuda.nvtx.range_pop()
  except Exception:
    pass


@dataclass
class Span:
  name: str
  trace_id: str
  span_id: str
  parent_id: Optional[str]
  start_ns: int
  end_ns: int = 0
  attrs: Dict[str, object] = field(default_factory=dict)
  status: str = "ok"

  def to_dict(self) -> dict:
    return {"name": self.name, "trace_id": self.trace_id, "span_id": self.span_id, "parent_id": self.parent_id,
            "start_ns": self.start_ns, "duration_ms": (self.end_ns - self.start_ns) / 1e6, "attrs": self.attrs,
            "status": self.status}


@dataclass
class TraceContext:
  request_id: str
  trace_id: str = field(default_factory=lambda: secrets.token_hex(16))
  root_span_id: str = field(default_factory=lambda: secrets.token_hex(8))
  token_count: int = 0
  token_group_start: int = 0

  def traceparent(self) -> str:
    return f"00-{self.trace_id}-{self.root_span_id}-01"

  @staticmethod
  def from_traceparent(request_id: str, header: str) -> "TraceContext":
    parts = header.split("-")
    if len(parts) == 4 and len(parts[1]) == 32:
      return TraceContext(request_id, trace_id=parts[1], root_span_id=parts[2])
    return TraceContext(request_id)


class Tracer:
  TOKEN_GROUP = 10

  def __init__(self, capacity: int = 4096):
    self.spans: Deque[Span] = deque(maxlen=capacity)
    self.contexts: Dict[str, TraceContext] = {}
    self._lock = threading.Lock()

  def context(self, request_id: Optional[str]) -> Optional[TraceContext]:
    if request_id is None:
      return None
    with self._lock:
      ctx = self.contexts.get(request_id)
      if ctx is None:
        ctx = self.contexts[request_id] = TraceContext(request_id)
        if len(self.contexts) > 10000:
          self.contexts.pop(next(iter(self.contexts)))
      return ctx

  def inject(self, request_id: str) -> Dict[str, str]:
    return {"traceparent": self.context(request_id).traceparent()}

  def extract(self, request_id: str, headers: Dict[str, str]) -> TraceContext:
    tp = headers.get("traceparent")
    ctx = TraceContext.from_traceparent(request_id, tp) if tp else TraceContext(request_id)
    with self._lock:
      self.contexts[request_id] = ctx
    return ctx

  @contextlib.contextmanager
  def span(self, name: str, request_id: Optional[str] = None, **attrs):
    ctx = self.context(request_id)
    sp = Span(name, ctx.trace_id if ctx else secrets.token_hex(16), secrets.token_hex(8),
              ctx.root_span_id if ctx else None, time.perf_counter_ns(), attrs=dict(attrs))
    if request_id:
      sp.attrs["request_id"] = request_id
    pushed = _roctx_push(name)
    try:
      yield sp
    except BaseException as e:
      sp.status = f"error: {type(e).__name__}"
      raise
    finally:
      if pushed:
        _roctx_pop()
      sp.end_ns = time.perf_counter_ns()
      with self._lock:
        self.spans.append(sp)
      try:
        from ..utils.metrics import observe_span
        observe_span(name, (sp.end_ns - sp.start_ns) / 1e9)
      except Exception:
        pass

  def on_token(self, request_id: str, n: int = 1) -> None:
    """Close a `token_group_k` span every TOKEN_GROUP tokens of a request."""
    ctx = self.context(request_id)
    now = time.perf_counter_ns()
    if ctx.token_count == 0:
      ctx.token_group_start = now
    ctx.token_count += n
    if ctx.token_count % self.TOKEN_GROUP == 0:
      g = ctx.token_count // self.TOKEN_GROUP - 1
      sp = Span(f"token_group_{g}", ctx.trace_id, secrets.token_hex(8), ctx.root_span_id, ctx.token_group_start, now,
                {"request_id": request_id, "tokens": self.TOKEN_GROUP})
      with self._lock:
        self.spans.append(sp)
      ctx.token_group_start = now

  def finish(self, request_id: str) -> None:
    with self._lock:
      self.contexts.pop(request_id, None)

  def export(self, limit: int = 1000) -> List[dict]:
    with self._lock:
      return [s.to_dict() for s in list(self.spans)[-limit:]]


tracer = Tracer()
