"""Prometheus metrics (the reference lists prometheus-client as a dependency but never uses it).

Exposed by the API at GET /metrics: generated tokens, time-to-first-token, per-span latency (hop,
process_prompt, decode step), outstanding requests, KV-page occupancy and HBM use per GPU peer.
Falls back to no-ops when prometheus_client is missing.
"""
from __future__ import annotations

try:
  from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest
  REGISTRY = CollectorRegistry()
  TOKENS = Counter("xot_generated_tokens_total", "Generated tokens", ["model"], registry=REGISTRY)
  REQUESTS = Counter("xot_requests_total", "Chat completion requests", ["model", "stream"], registry=REGISTRY)
  TTFT = Histogram("xot_time_to_first_token_seconds", "Time to first token", ["model"], registry=REGISTRY,
                   buckets=(0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30))
  SPAN = Histogram("xot_span_seconds", "Traced span durations", ["span"], registry=REGISTRY,
                   buckets=(1e-4, 5e-4, 1e-3, 5e-3, 0.01, 0.05, 0.1, 0.5, 1, 5, 30))
  OUTSTANDING = Gauge("xot_outstanding_requests", "Requests in flight on this node", registry=REGISTRY)
  KV_USED = Gauge("xot_kv_pages_used", "KV cache pages in use", ["device"], registry=REGISTRY)
  KV_TOTAL = Gauge("xot_kv_pages_total", "KV cache pages", ["device"], registry=REGISTRY)
  HBM_USED = Gauge("xot_hbm_bytes_used", "GPU memory allocated by this process", ["device"], registry=REGISTRY)
  AVAILABLE = True
except Exception:  # pragma: no cover
  AVAILABLE = False


def observe_span(name: str, seconds: float) -> None:
  if AVAILABLE:
    SPAN.labels(name).observe(seconds)


def render(node=None) -> bytes:
  if not AVAILABLE:
    return b"# prometheus_client not installed\n"
  if node is not None:
    OUTSTANDING.set(len(getattr(node, "outstanding_requests", {})))
    eng = getattr(node, "inference_engine", None)
    runner = getattr(eng, "runner", None)
    if runner is not None:
      dev = str(runner.device)
      KV_TOTAL.labels(dev).set(runner.bm.num_blocks)
      KV_USED.labels(dev).set(runner.bm.num_blocks - runner.bm.num_free)
      try:
        import torch
        if runner.device.type == "cuda":
          HBM_USED.labels(dev).set(torch.cuda.memory_allocated(runner.device))
      except Exception:
        pass
  return generate_latest(REGISTRY)
