#!/usr/bin/env python3
"""End-to-end serving benchmark through the ChatGPT-compatible HTTP API on one peer (one GPU):
Node + ShardedInferenceEngine (continuous batching, HIP-graph decode) behind the aiohttp app, N concurrent
streaming chat completions.  Reports what the reference's clients measure (tinychat index.js:330-340:
time to first token and output tokens/s), aggregated over the requests.

  python tools/bench_serve.py --model llama-3-8b --concurrency 64 --max-tokens 128 --prompt-words 200

Random-init weights (no checkpoint on the GPU box) and the offline byte tokenizer: the prompt is
--prompt-words synthetic words; generation runs to --max-tokens unless an EOS id is sampled.
"""
import argparse
import asyncio
import json
import os
import socket
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


async def main(a):
  import torch
  from aiohttp import ClientSession
  from aiohttp.test_utils import TestServer

  from xotorch_support_jetson_amd.api.chatgpt_api import ChatGPTAPI
  from xotorch_support_jetson_amd.download.shard_download import NoopShardDownloader
  from xotorch_support_jetson_amd.inference.sharded_engine import ShardedInferenceEngine
  from xotorch_support_jetson_amd.networking.grpc.grpc_peer_handle import GRPCPeerHandle
  from xotorch_support_jetson_amd.networking.grpc.grpc_server import GRPCServer
  from xotorch_support_jetson_amd.networking.manual.manual_discovery import ManualDiscovery
  from xotorch_support_jetson_amd.orchestration.node import Node
  from xotorch_support_jetson_amd.topology.device_capabilities import device_capabilities
  from xotorch_support_jetson_amd.topology.ring_memory_weighted_partitioning_strategy import \
    RingMemoryWeightedPartitioningStrategy

  os.environ.setdefault("XOT_MAX_BATCH", str(max(a.concurrency, 1)))
  caps = device_capabilities()
  port = free_port()
  cfg = {"peers": {"bench": {"address": "127.0.0.1", "port": port, "device_capabilities": caps.to_dict()}}}
  topo = os.path.join(tempfile.mkdtemp(), "topology.json")
  with open(topo, "w") as f:
    json.dump(cfg, f)
  eng = ShardedInferenceEngine(NoopShardDownloader())
  disc = ManualDiscovery(topo, "bench", create_peer_handle=lambda pid, addr, desc, c: GRPCPeerHandle(pid, addr, desc, c))
  node = Node("bench", None, eng, disc, NoopShardDownloader(), RingMemoryWeightedPartitioningStrategy(),
              max_generate_tokens=a.max_tokens, device_caps=caps)
  node.server = GRPCServer(node, "127.0.0.1", port)
  await node.server.start()
  await node.start(wait_for_peers=0)
  api = ChatGPTAPI(node, "ShardedInferenceEngine", response_timeout=3600, default_model=a.model)
  server = TestServer(api.app, host="127.0.0.1", port=free_port())
  await server.start_server()
  url = f"http://127.0.0.1:{server.port}/v1/chat/completions"
  words = " ".join(f"w{i % 97}" for i in range(a.prompt_words))

  async def one(session, i, max_tokens):
    text = f"{words} (request {i})" if a.shared_prefix else f"request {i}: {words}"
    body = {"model": a.model, "stream": True, "max_tokens": max_tokens, "temperature": a.temperature,
            "messages": [{"role": "user", "content": text}]}
    t0 = time.perf_counter()
    ttft, n = None, 0
    async with session.post(url, json=body) as r:
      assert r.status == 200, await r.text()
      async for raw in r.content:
        line = raw.decode().strip()
        if not line.startswith("data: ") or line == "data: [DONE]":
          continue
        d = json.loads(line[6:])
        if d["choices"][0].get("delta", {}).get("content") is not None:
          n += 1
          if ttft is None:
            ttft = time.perf_counter() - t0
    return ttft or 0.0, n, time.perf_counter() - t0

  async with ClientSession() as session:
    t0 = time.perf_counter()
    await one(session, -1, 4)  # warm-up: shard load, prefill / decode graph capture, GEMM policy
    for b in (a.concurrency,):  # second warm-up at the measured concurrency (its batch bucket's graph)
      await asyncio.gather(*(one(session, -2 - j, 4) for j in range(b)))
    warm = time.perf_counter() - t0
    t0 = time.perf_counter()
    s0 = dict(eng.stats)
    res = await asyncio.gather(*(one(session, i, a.max_tokens) for i in range(a.concurrency)))
    wall = time.perf_counter() - t0
    steps = eng.stats["steps"] - s0["steps"]
    reqs = eng.stats["requests"] - s0["requests"]
  toks = sum(r[1] for r in res)
  ttfts = sorted(r[0] for r in res)
  out = {"metric": "API streaming output tokens/sec (one peer)", "model": a.model, "concurrency": a.concurrency,
         "prompt_words": a.prompt_words, "max_tokens": a.max_tokens, "output_tokens": toks,
         "value": round(toks / wall, 2), "unit": "tokens/s", "wall_s": round(wall, 2), "warmup_s": round(warm, 1),
         "ttft_s": {"p50": round(ttfts[len(ttfts) // 2], 3), "max": round(ttfts[-1], 3)},
         "per_request_tok_s_p50": round(sorted(r[1] / r[2] for r in res)[len(res) // 2], 2),
         "engine_steps": steps, "mean_requests_per_step": round(reqs / max(steps, 1), 1),
         "ms_per_step": round(wall * 1e3 / max(steps, 1), 2),
         "presampled_tokens": eng.stats.get("presampled", 0) - s0.get("presampled", 0),
         "shared_prefix": a.shared_prefix,
         "prefix_cache": dict(eng.prefix_cache.stats) if eng.prefix_cache is not None else None,
         "data": "random-init weights, byte tokenizer, synthetic prompts", "dtype": "bf16",
         "device": caps.chip}
  print(json.dumps(out), flush=True)
  if os.environ.get("XOT_PROFILE"):
    import pstats
    PROF.disable()
    pstats.Stats(PROF).sort_stats("tottime").print_stats(25)
  await server.close()
  await node.stop()
  sys.stdout.flush()
  os._exit(0)  # engine executor threads / gRPC server: leave without waiting on them


if __name__ == "__main__":
  ap = argparse.ArgumentParser()
  ap.add_argument("--model", default="llama-3-8b")
  ap.add_argument("--concurrency", type=int, default=64)
  ap.add_argument("--max-tokens", type=int, default=128)
  ap.add_argument("--prompt-words", type=int, default=200)
  ap.add_argument("--temperature", type=float, default=0.6)
  ap.add_argument("--shared-prefix", action="store_true",
                  help="every prompt starts with the same words (a system prompt / earlier turns) and ends with "
                       "the request index, so prompt-prefix KV reuse applies")
  if os.environ.get("XOT_PROFILE"):  # host-side hot spots of the serving loop
    import cProfile
    PROF = cProfile.Profile()
    PROF.enable()
  asyncio.run(main(ap.parse_args()))
