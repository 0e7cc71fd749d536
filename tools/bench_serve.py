#!/usr/bin/env python3
"""End-to-end serving benchmark through the ChatGPT-compatible HTTP API on one peer (one GPU):
Node + ShardedInferenceEngine (continuous batching, HIP-graph decode) behind the aiohttp app, N concurrent
streaming chat completions.  Reports what the reference's clients measure (tinychat index.js:330-340:
time to first token and output tokens/s), aggregated over the requests.

  python tools/bench_serve.py --model llama-3-8b --concurrency 64 --max-tokens 128 --prompt-words 200
  python tools/bench_serve.py --ring 2 ...     the same load against `xot --gpus 2` (RingServer: the layers
                                               split over 2 ranks, RCCL hand-off; XOT_DIST_BACKEND=gloo
                                               rehearses 2 ranks on one GPU)

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


PROF = None


def free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


async def one(session, url, a, i, max_tokens, base=None):
  """One streaming request: (TTFT, tokens, seconds, [first, last] token times relative to `base`, token times)."""
  words = " ".join(f"w{j % 97}" for j in range(a.prompt_words))
  text = f"{words} (request {i})" if a.shared_prefix else f"request {i}: {words}"
  body = {"model": a.model, "stream": True, "max_tokens": max_tokens, "temperature": a.temperature,
          "messages": [{"role": "user", "content": text}]}
  t0 = time.perf_counter()
  base = t0 if base is None else base
  ttft, n, stamps = None, 0, []
  async with session.post(url, json=body) as r:
    assert r.status == 200, await r.text()
    async for raw in r.content:
      line = raw.decode().strip()
      if not line.startswith("data: ") or line == "data: [DONE]":
        continue
      d = json.loads(line[6:])
      if d["choices"][0].get("delta", {}).get("content") is not None:
        n += 1
        now = time.perf_counter()
        stamps.append(now - base)
        if ttft is None:
          ttft = now - t0
  return ttft or 0.0, n, time.perf_counter() - t0, stamps


def decode_window(res):
  """Aggregate output tokens/s while EVERY stream is decoding: from the last first token to the first last
  token (prefill of the later arrivals and the tail of the early finishers excluded) -- the serving
  counterpart of bench.py's decode-step rate.  None when the window is empty."""
  starts = [r[3][0] for r in res if r[3]]
  ends = [r[3][-1] for r in res if r[3]]
  if not starts:
    return None
  lo, hi = max(starts), min(ends)
  if hi <= lo:
    return None
  n = sum(1 for r in res for t in r[3] if lo < t <= hi)
  return {"tok_s": round(n / (hi - lo), 2), "window_s": round(hi - lo, 3), "tokens": n}


async def client_warmup(session, url, a):
  await one(session, url, a, -1, 4)  # shard load, prefill / decode graph capture, GEMM policy
  # the measured concurrency once (its batch bucket's graph)
  await asyncio.gather(*(one(session, url, a, -2 - j, 4) for j in range(a.concurrency)))


async def client_main(a):
  """--client URL: the load generator in its own process (see main)."""
  from aiohttp import ClientSession, TCPConnector
  loop = asyncio.get_running_loop()
  # limit=0: aiohttp's default connector caps a session at 100 open connections, which silently
  # turned every concurrency above 100 into 100 streams
  async with ClientSession(connector=TCPConnector(limit=0)) as session:
    t0 = time.perf_counter()
    await client_warmup(session, a.client, a)
    print("READY", flush=True)
    print(json.dumps({"warmup_s": time.perf_counter() - t0}), flush=True)
    await loop.run_in_executor(None, sys.stdin.readline)
    t0 = time.perf_counter()
    res = await asyncio.gather(*(one(session, a.client, a, i, a.max_tokens, t0) for i in range(a.concurrency)))
    wall = time.perf_counter() - t0
  print(json.dumps({"results": res, "wall_s": wall}), flush=True)


async def ring_main(a):
  """--ring N: start `xot --gpus N` (the RCCL ring server with the API on rank 0) as a child process group,
  wait for its API, run the same warmup + measured load with in-process clients, stop the group."""
  import signal
  import subprocess
  from aiohttp import ClientSession, TCPConnector
  port = free_port()
  env = dict(os.environ, XOT_MAX_BATCH=str(max(a.concurrency, 1)))
  # --ring always: `xot --gpus 1` alone is the single-process Node path (main.run sets args.ring only for N > 1)
  cmd = [sys.executable, "-m", "xotorch_support_jetson_amd.main", "--gpus", str(a.ring), "--ring", "--default-model",
         a.model, "--chatgpt-api-port", str(port), "--disable-tui", "--max-generate-tokens", str(a.max_tokens)]
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  log_path = a.server_log or os.path.join(tempfile.gettempdir(), f"xot_ring_{port}.log")
  log_f = open(log_path, "w")
  proc = subprocess.Popen(cmd, cwd=root, env=env, start_new_session=True, stdout=log_f, stderr=subprocess.STDOUT)
  base = f"http://127.0.0.1:{port}"
  try:
    async with ClientSession(connector=TCPConnector(limit=0)) as session:
      t0 = time.perf_counter()
      while True:  # the ranks load their shards and start the API on rank 0
        if proc.poll() is not None:
          raise SystemExit(f"ring server exited with {proc.returncode} before its API came up")
        try:
          async with session.get(base + "/healthcheck") as r:
            if r.status == 200:
              break
        except OSError:
          pass
        if time.perf_counter() - t0 > 600:
          raise SystemExit("ring server API did not come up within 600 s")
        await asyncio.sleep(1.0)
      url = base + "/v1/chat/completions"
      await client_warmup(session, url, a)
      warm = time.perf_counter() - t0
      t0 = time.perf_counter()
      res = await asyncio.gather(*(one(session, url, a, i, a.max_tokens, t0) for i in range(a.concurrency)))
      wall = time.perf_counter() - t0
  finally:
    try:
      os.killpg(proc.pid, signal.SIGTERM)  # the group this call started (ranks are its children)
      proc.wait(timeout=60)
    except (ProcessLookupError, subprocess.TimeoutExpired):
      os.killpg(proc.pid, signal.SIGKILL)
    log_f.close()
  # which server answered: RingServer's rank 0 announces its API as "[ring 0] ChatGPT API on ..."
  with open(log_path) as f:
    server = "RingServer" if "[ring 0] ChatGPT API" in f.read() else "Node (single-process)"
  toks = sum(r[1] for r in res)
  ttfts = sorted(r[0] for r in res)
  print(json.dumps({"metric": f"API streaming output tokens/sec (ring of {a.ring} ranks)", "model": a.model,
                    "ring": a.ring, "server": server, "server_log": log_path,
                    "dist_backend": os.environ.get("XOT_DIST_BACKEND", "nccl"),
                    "concurrency": a.concurrency, "prompt_words": a.prompt_words, "max_tokens": a.max_tokens,
                    "output_tokens": toks, "value": round(toks / wall, 2), "unit": "tokens/s",
                    "wall_s": round(wall, 2), "warmup_s": round(warm, 1),
                    "ttft_s": {"p50": round(ttfts[len(ttfts) // 2], 3), "max": round(ttfts[-1], 3)},
                    "per_request_tok_s_p50": round(sorted(r[1] / r[2] for r in res)[len(res) // 2], 2),
                    "decode_window": decode_window(res),
                    "data": "random-init weights, byte tokenizer, synthetic prompts", "dtype": "bf16"}), flush=True)


async def main(a):
  import torch
  from aiohttp import ClientSession, TCPConnector  # noqa: F401  (in-process clients)
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
  if a.client_proc:
    # the clients run in a child process, as real ones would: parsing 64 SSE streams is no part of the
    # server's host time.  The child warms up, says READY, waits for GO, runs the measured phase.
    child = await asyncio.create_subprocess_exec(
      sys.executable, os.path.abspath(__file__), "--client", url, "--model", a.model, "--concurrency",
      str(a.concurrency), "--max-tokens", str(a.max_tokens), "--prompt-words", str(a.prompt_words),
      "--temperature", str(a.temperature), *(["--shared-prefix"] if a.shared_prefix else []),
      stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE)
    line = await child.stdout.readline()
    assert line.strip() == b"READY", line
    warm = float(json.loads((await child.stdout.readline()).decode())["warmup_s"])
    s0 = dict(eng.stats)
    if PROF is not None:
      PROF.enable()
    child.stdin.write(b"GO\n")
    await child.stdin.drain()
    d = json.loads((await child.stdout.readline()).decode())
    if PROF is not None:
      PROF.disable()
    await child.wait()
    res, wall = [tuple(r) for r in d["results"]], d["wall_s"]
  else:
    async with ClientSession(connector=TCPConnector(limit=0)) as session:
      t0 = time.perf_counter()
      await client_warmup(session, url, a)
      warm = time.perf_counter() - t0
      s0 = dict(eng.stats)
      if PROF is not None:  # host-side profile of the measured phase only
        PROF.enable()
      t0 = time.perf_counter()
      res = await asyncio.gather(*(one(session, url, a, i, a.max_tokens, t0) for i in range(a.concurrency)))
      wall = time.perf_counter() - t0
      if PROF is not None:
        PROF.disable()
  steps = eng.stats["steps"] - s0["steps"]
  reqs = eng.stats["requests"] - s0["requests"]
  toks = sum(r[1] for r in res)
  ttfts = sorted(r[0] for r in res)
  out = {"metric": "API streaming output tokens/sec (one peer)", "model": a.model, "concurrency": a.concurrency,
         "prompt_words": a.prompt_words, "max_tokens": a.max_tokens, "output_tokens": toks,
         "value": round(toks / wall, 2), "unit": "tokens/s", "wall_s": round(wall, 2), "warmup_s": round(warm, 1),
         "ttft_s": {"p50": round(ttfts[len(ttfts) // 2], 3), "max": round(ttfts[-1], 3)},
         "per_request_tok_s_p50": round(sorted(r[1] / r[2] for r in res)[len(res) // 2], 2),
         "decode_window": decode_window(res),
         "engine_steps": steps, "mean_requests_per_step": round(reqs / max(steps, 1), 1),
         "ms_per_step": round(wall * 1e3 / max(steps, 1), 2),
         # time inside the engine's step call (host prep + GPU + token copy), vs. ms_per_step of wall time
         "engine_ms_per_step": round((eng.stats.get("step_s", 0.0) - s0.get("step_s", 0.0)) * 1e3 / max(steps, 1), 2),
         **{f"engine_{k}_ms_per_step": round((eng.stats.get(f"{k}_s", 0.0) - s0.get(f"{k}_s", 0.0)) * 1e3 / max(steps, 1), 2)
            for k in ("launch", "wait", "gpu_step")},
         "gpu_gap_ms_mean": round((eng.stats.get("gpu_gap_s", 0.0) - s0.get("gpu_gap_s", 0.0)) * 1e3
                                  / max(eng.stats.get("gpu_gaps", 0) - s0.get("gpu_gaps", 0), 1), 3),
         "presampled_tokens": eng.stats.get("presampled", 0) - s0.get("presampled", 0),
         "engine_loop_tokens": eng.stats.get("loop_tokens", 0) - s0.get("loop_tokens", 0),
         "shared_prefix": a.shared_prefix,
         "prefix_cache": dict(eng.prefix_cache.stats) if eng.prefix_cache is not None else None,
         "data": "random-init weights, byte tokenizer, synthetic prompts", "dtype": "bf16",
         "device": caps.chip}
  print(json.dumps(out), flush=True)
  if PROF is not None:
    import pstats
    pstats.Stats(PROF).sort_stats("tottime").print_stats(30)
    pstats.Stats(PROF).sort_stats("cumulative").print_stats(40)
  await server.close()
  await node.stop()
  sys.stdout.flush()
  if os.environ.get("XOT_BENCH_CLEAN_EXIT") == "1":  # under a profiler: let its exit handlers flush the trace
    return
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
  ap.add_argument("--in-process-clients", dest="client_proc", action="store_false",
                  help="run the HTTP clients on the server's event loop (their SSE parsing then counts as server time)")
  ap.add_argument("--client", default=None, help=argparse.SUPPRESS)  # internal: load-generator child mode
  ap.add_argument("--ring", type=int, default=0, help="serve from `xot --gpus N --ring` (the RCCL ring server) instead")
  ap.add_argument("--server-log", default=None, help="--ring: where the server's output goes (default: a temp file)")
  if os.environ.get("XOT_PROFILE"):  # host-side hot spots of the serving loop (main thread)
    import cProfile
    PROF = cProfile.Profile()
  args = ap.parse_args()
  if os.environ.get("XOT_SWITCH_INTERVAL_US"):  # diagnostic: CPython's GIL hand-off interval (default 5000 us)
    sys.setswitchinterval(float(os.environ["XOT_SWITCH_INTERVAL_US"]) * 1e-6)
  asyncio.run(client_main(args) if args.client else (ring_main(args) if args.ring else main(args)))
