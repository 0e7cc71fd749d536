"""`xot` command line (reference: xotorch/main.py:73-402; same flags and commands).

  xot                                   start a peer: gRPC server + discovery + ChatGPT API (+ TUI)
  xot run <model> [--prompt ...]        one prompt through the ring, print the answer
  xot eval <model> [--data DIR]         one pass over test.jsonl, print the length-weighted loss
  xot train <model> [--iters N ...]     pipeline training over the ring, checkpoint every --save-every
  xot --gpus N ...                      one process per local GPU as ONE RCCL ring (parallel/ring_serve.py:
                                        continuous batching, activations over xGMI, rank 0 serves the API;
                                        train / eval: parallel/pipeline_train.py)
  xot --gpus N --grpc-peers ...         the reference's topology instead: one gRPC peer process per GPU,
                                        connected by a generated manual-discovery file (cross-host rings
                                        always use gRPC + discovery)
  xot --gpus N --federate ...           the local RCCL ring as ONE peer of the discovered cluster: rank 0 runs
                                        the Node, the range the cluster assigns it is split over the GPUs
                                        (parallel/ring_federation.py)
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import subprocess
import sys
import tempfile
import time
import traceback
import uuid
from pathlib import Path

import numpy as np

os.environ.setdefault("GRPC_VERBOSITY", "error")
os.environ.setdefault("TRANSFORMERS_VERBOSITY", "error")
os.environ.setdefault("TOKENIZERS_PARALLELISM", "true")

from .helpers import DEBUG, VERSION, find_available_port, get_or_create_node_id, print_banner, xot_home  # noqa: E402


def build_parser() -> argparse.ArgumentParser:
  p = argparse.ArgumentParser(description="xot: MI355X-native peer-partitioned LLM inference/training")
  p.add_argument("command", nargs="?", choices=["run", "eval", "train"], help="Command to run")
  p.add_argument("model_name", nargs="?", help="Model name to run")
  p.add_argument("--default-model", type=str, default=None, help="Default model")
  p.add_argument("--iters", type=int, default=100, help="Training iterations")
  p.add_argument("--save-every", type=int, default=5, help="Save the model every N iterations")
  p.add_argument("--data", type=str, default=None, help="Directory with train/valid/test.jsonl")
  p.add_argument("--batch-size", type=int, default=1, help="Minibatch size")
  p.add_argument("--resume-checkpoint", type=str, default=None, help="Checkpoint directory to resume from")
  p.add_argument("--save-checkpoint-dir", type=str, default="checkpoints", help="Where to save checkpoints")
  p.add_argument("--lr", type=float, default=1e-5, help="AdamW learning rate")
  p.add_argument("--node-id", type=str, default=None, help="Node ID")
  p.add_argument("--node-host", type=str, default="0.0.0.0", help="Node host")
  p.add_argument("--node-port", type=int, default=None, help="Node port")
  p.add_argument("--models-seed-dir", type=str, default=None, help="Model seed directory")
  p.add_argument("--listen-port", type=int, default=5678, help="Listening port for discovery")
  p.add_argument("--download-quick-check", action="store_true", help="Quick check local path for model shards")
  p.add_argument("--max-parallel-downloads", type=int, default=8, help="Max parallel downloads")
  p.add_argument("--broadcast-port", type=int, default=5678, help="Broadcast port for discovery")
  p.add_argument("--discovery-module", type=str, choices=["udp", "manual"], default="udp")
  p.add_argument("--discovery-timeout", type=int, default=30, help="Discovery timeout in seconds")
  p.add_argument("--discovery-config-path", type=str, default=None, help="Manual discovery topology JSON")
  p.add_argument("--wait-for-peers", type=int, default=0, help="Number of peers to wait for before starting")
  p.add_argument("--chatgpt-api-port", type=int, default=52415, help="ChatGPT API port")
  p.add_argument("--chatgpt-api-response-timeout", type=int, default=900, help="ChatGPT API response timeout (s)")
  p.add_argument("--max-generate-tokens", type=int, default=1024, help="Max tokens to generate per request")
  p.add_argument("--inference-engine", type=str, default="mi355x", choices=["mi355x", "torch", "dummy"])
  p.add_argument("--disable-tui", action=argparse.BooleanOptionalAction, help="Disable the topology TUI")
  p.add_argument("--chat-tui", action="store_true", help="Interactive chat in the terminal")
  p.add_argument("--run-model", type=str, help="Specify a model to run directly")
  p.add_argument("--prompt", type=str, default="Who are you?", help="Prompt for --run-model / run")
  p.add_argument("--default-temp", type=float, default=0.0, help="Default token sampling temperature")
  p.add_argument("--tailnet-name", type=str, default=None, help="(accepted for compatibility)")
  p.add_argument("--node-id-filter", type=str, default=None, help="Comma separated node ids to allow")
  p.add_argument("--interface-type-filter", type=str, default=None, help="Comma separated interface types to allow")
  p.add_argument("--system-prompt", type=str, default=None, help="System prompt for the ChatGPT API")
  p.add_argument("--gpus", type=int, default=0,
                 help="Serve/run/train/eval over N local GPUs as one RCCL ring, one process per GPU (0 = single process)")
  p.add_argument("--ring", action="store_true",
                 help="(default with --gpus N > 1) the local GPUs as one RCCL ring; with --gpus 0/1: every visible GPU")
  p.add_argument("--grpc-peers", action="store_true",
                 help="--gpus N: one gRPC peer process per GPU (the reference's per-hop RPC) instead of the RCCL ring")
  p.add_argument("--federate", action="store_true",
                 help="--gpus N: join discovery as ONE cluster peer whose assigned layer range is split over the "
                      "local GPUs over RCCL (parallel/ring_federation.py)")
  p.add_argument("--micro-batch", type=int, default=1, help="--ring: sequences per pipeline micro-batch")
  p.add_argument("--parallel", choices=("pp", "dp"), default="pp",
                 help="--ring: pp = layer pipeline over the GPUs; dp = a full replica per GPU, gradients all-reduced")
  p.add_argument("--schedule", choices=("gpipe", "1f1b"), default="gpipe",
                 help="--ring --parallel pp: micro-batch order (1f1b keeps at most N - rank activations alive)")
  p.add_argument("--no-api", action="store_true", help="Do not start the ChatGPT API on this peer")
  p.add_argument("--max-batch", type=int, default=None,
                 help="Serving: most sequences per batched decode step on a peer (XOT_MAX_BATCH, default 64)")
  p.add_argument("--max-ctx", type=int, default=None,
                 help="Serving: longest context (prompt + generated tokens) per request (XOT_MAX_CTX, default 8192)")
  p.add_argument("--weight-dtype", choices=("bf16", "fp8"), default=None,
                 help="fp8: weight-only e4m3 dense projections (half the weight bytes per decode step)")
  return p


# ------------------------------------------------------------------ multi-GPU spawner
def spawn_gpu_peers(args, argv) -> int:
  """One child process per GPU; LOCAL_RANK selects the device.  Peers find each other through a
  generated manual-discovery file; rank 0 keeps the API port, others run without API/TUI."""
  n = args.gpus
  base_port = args.node_port or find_available_port("127.0.0.1")
  base_id = args.node_id or get_or_create_node_id()
  from .topology.device_capabilities import gpu_capabilities, cpu_capabilities
  caps = gpu_capabilities() or [cpu_capabilities()] * n
  peers = {f"{base_id}-gpu{i}": {"address": "127.0.0.1", "port": base_port + i,
                                 "device_capabilities": caps[i % len(caps)].to_dict()} for i in range(n)}
  cfg = Path(tempfile.gettempdir()) / f"xot_local_peers_{base_id}.json"
  cfg.write_text(json.dumps({"peers": peers}, indent=1))
  strip = {"--gpus", "--node-id", "--node-port", "--discovery-module", "--discovery-config-path", "--wait-for-peers"}
  rank0, skip = [], False
  for a in argv:
    if skip:
      skip = False
      continue
    if a.split("=")[0] in strip:
      skip = "=" not in a
      continue
    rank0.append(a)
  # serving-only peers: same engine settings, no command, no API/TUI
  serve = ["--inference-engine", args.inference_engine, "--max-generate-tokens", str(args.max_generate_tokens),
           "--default-temp", str(args.default_temp), "--no-api", "--disable-tui"]
  procs = []
  for i in range(n):
    env = dict(os.environ, LOCAL_RANK=str(i), XOT_PEER_RANK=str(i), XOT_NUM_PEERS=str(n))
    common = ["--node-id", f"{base_id}-gpu{i}", "--node-port", str(base_port + i), "--discovery-module", "manual",
              "--discovery-config-path", str(cfg), "--wait-for-peers", str(n - 1)]
    cmd = (rank0 if i == 0 else serve) + common
    procs.append(subprocess.Popen([sys.executable, "-m", "xotorch_support_jetson_amd.main"] + cmd, env=env))
  try:
    rc = procs[0].wait()
  except KeyboardInterrupt:
    rc = 130
  for p in procs[1:]:
    p.terminate()
  for p in procs[1:]:
    try:
      p.wait(timeout=10)
    except subprocess.TimeoutExpired:
      p.kill()
  return rc


# ------------------------------------------------------------------ commands
async def run_model_cli(node, model_name: str, prompt: str, topology_viz=None):
  from .inference.tokenizers import resolve_tokenizer
  from .models.registry import build_base_shard, get_repo
  cls = type(node.inference_engine).__name__
  shard = build_base_shard(model_name, cls)
  if not shard:
    print(f"Error: Unsupported model '{model_name}' for inference engine {cls}")
    return
  tok = getattr(node.inference_engine, "tokenizer", None)
  if tok is None or getattr(node.inference_engine, "shard", None) is None or node.inference_engine.shard.model_id != model_name:
    vocab = None
    try:
      from .models.config import preset
      vocab = preset(model_name).vocab_size
    except KeyError:
      pass
    tok = await resolve_tokenizer(get_repo(shard.model_id, cls) or model_name, vocab)
  request_id = str(uuid.uuid4())
  cb_id = f"cli-wait-response-{request_id}"
  cb = node.on_token.register(cb_id)
  if topology_viz:
    topology_viz.update_prompt(request_id, prompt)
  templ = tok.apply_chat_template([{"role": "user", "content": prompt}], tokenize=False, add_generation_prompt=True)
  try:
    print(f"Processing prompt: {prompt}")
    t0 = time.perf_counter()
    await node.process_prompt(shard, templ, request_id=request_id)
    tokens, first = [], []

    def on_token(_rid, _tokens, _finished):
      if _rid == request_id:
        if _tokens and not first:
          first.append(time.perf_counter())
        tokens.extend(_tokens)
      return _rid == request_id and _finished

    await cb.wait(on_token, timeout=300)
    t1 = time.perf_counter()
    dt = t1 - t0
    print("\nGenerated response:")
    print(tok.decode(tokens))
    # time to the first token includes loading / initialising the shard on a cold start
    ttft = (first[0] - t0) if first else dt
    decode = (len(tokens) - 1) / max(t1 - first[0], 1e-9) if first and len(tokens) > 1 else 0.0
    print(f"\n[{len(tokens)} tokens in {dt:.2f}s: first token {ttft:.2f}s, then {decode:.1f} tok/s]")
  except Exception as e:
    print(f"Error processing prompt: {e}")
    traceback.print_exc()
  finally:
    node.on_token.deregister(cb_id)


async def hold_outstanding(node):
  while node.outstanding_requests:
    await asyncio.sleep(0.5)


async def run_iter(node, shard, train: bool, data, batch_size: int = 1):
  from .train.dataset import iterate_batches
  losses, tokens = [], []
  for x, y, lengths in iterate_batches(data, batch_size, train=False):
    loss = await node.enqueue_example(shard, x, y, lengths, train=train)
    loss = float(loss if not isinstance(loss, tuple) else loss[0]) if loss is not None else float("nan")
    losses.append(np.sum(lengths) * loss)
    tokens.append(np.sum(lengths))
  total = float(np.sum(tokens))
  return float(np.sum(losses)) / max(total, 1.0), total


async def _dataset_for(node, model_name: str, data_dir):
  from .inference.tokenizers import resolve_tokenizer
  from .models.registry import build_base_shard, get_repo
  from .train.dataset import DEFAULT_DATA, load_dataset
  cls = type(node.inference_engine).__name__
  shard = build_base_shard(model_name, cls)
  if not shard:
    print(f"Error: Unsupported model '{model_name}' for inference engine {cls}")
    return None, None
  vocab = None
  try:
    from .models.config import preset
    vocab = preset(model_name).vocab_size
  except KeyError:
    pass
  tok = await resolve_tokenizer(get_repo(shard.model_id, cls) or model_name, vocab)
  return shard, load_dataset(data_dir or DEFAULT_DATA, lambda s: tok.encode(s))


async def eval_model_cli(node, model_name: str, data_dir, batch_size: int):
  shard, ds = await _dataset_for(node, model_name, data_dir)
  if shard is None:
    return
  _, _, test = ds
  print(f"Evaluating {len(test)} examples with batch_size {batch_size}")
  loss, tokens = await run_iter(node, shard, False, test, batch_size)
  print(f"total | loss={loss}, tokens={tokens}")
  await hold_outstanding(node)


async def train_model_cli(node, model_name: str, data_dir, batch_size: int, iters: int, save_every: int = 0,
                          checkpoint_dir=None, resume=None):
  shard, ds = await _dataset_for(node, model_name, data_dir)
  if shard is None:
    return
  train, _, _ = ds
  if resume:
    await node.inference_engine.load_checkpoint(node.get_current_shard(shard), resume)
    print(f"Resumed from {resume}")
  print(f"Training on {len(train)} examples with batch_size {batch_size} for {iters} epochs")
  for epoch in range(iters):
    loss, tokens = await run_iter(node, shard, True, train, batch_size)
    print(f"epoch {epoch + 1}/{iters}\t| loss: {loss}, tokens: {tokens}")
    if save_every > 0 and epoch > 0 and epoch % save_every == 0 and checkpoint_dir is not None:
      await node.coordinate_save(shard, epoch, checkpoint_dir)
      await hold_outstanding(node)
  await hold_outstanding(node)


# ------------------------------------------------------------------ assembly
def build_node(args, engine=None, device_caps=None):
  from .api.chatgpt_api import ChatGPTAPI
  from .download.new_shard_download import new_shard_downloader
  from .download.shard_download import NoopShardDownloader
  from .inference.inference_engine import get_inference_engine, inference_engine_classes
  from .networking.grpc.grpc_peer_handle import GRPCPeerHandle
  from .networking.grpc.grpc_server import GRPCServer
  from .networking.manual.manual_discovery import ManualDiscovery
  from .networking.udp.udp_discovery import UDPDiscovery
  from .orchestration.node import Node
  from .topology.ring_memory_weighted_partitioning_strategy import RingMemoryWeightedPartitioningStrategy

  engine_name = args.inference_engine
  downloader = NoopShardDownloader() if engine_name == "dummy" else new_shard_downloader(args.max_parallel_downloads)
  if engine is None:
    engine = get_inference_engine(engine_name, downloader)
  else:  # --federate: the local RCCL ring's engine (its sub-ranges download through each rank's own engine)
    engine_name = "ShardedInferenceEngine"
  if hasattr(engine, "lr"):
    engine.lr = args.lr
  print(f"Using inference engine: {type(engine).__name__} with shard downloader: {type(downloader).__name__}")
  port = args.node_port or find_available_port(args.node_host)
  node_id = args.node_id or get_or_create_node_id()
  make_peer = lambda pid, addr, desc, caps: GRPCPeerHandle(pid, addr, desc, caps)  # noqa: E731
  if args.discovery_module == "manual":
    if not args.discovery_config_path:
      raise ValueError("--discovery-module manual requires --discovery-config-path")
    discovery = ManualDiscovery(args.discovery_config_path, node_id, create_peer_handle=make_peer)
  else:
    discovery = UDPDiscovery(node_id, port, args.listen_port, args.broadcast_port, make_peer,
                             discovery_timeout=args.discovery_timeout,
                             allowed_node_ids=args.node_id_filter.split(",") if args.node_id_filter else None,
                             allowed_interface_types=(args.interface_type_filter.split(",")
                                                      if args.interface_type_filter else None))
  viz = None
  if not args.disable_tui and not args.chat_tui and sys.stdout.isatty():
    try:
      from .viz.topology_viz import TopologyViz
      viz = TopologyViz(chatgpt_api_endpoints=[f"http://localhost:{args.chatgpt_api_port}/v1/chat/completions"],
                        web_chat_urls=[f"http://localhost:{args.chatgpt_api_port}"])
    except Exception:
      viz = None
  node = Node(node_id, None, engine, discovery, downloader, RingMemoryWeightedPartitioningStrategy(),
              max_generate_tokens=args.max_generate_tokens, default_sample_temperature=args.default_temp,
              topology_viz=viz, device_caps=device_caps)
  node.server = GRPCServer(node, args.node_host, port)
  api = None
  if not args.no_api:
    api = ChatGPTAPI(node, type(engine).__name__, response_timeout=args.chatgpt_api_response_timeout,
                     on_chat_completion_request=(lambda rid, req, prompt: viz.update_prompt(rid, prompt)) if viz else None,
                     default_model=args.default_model, system_prompt=args.system_prompt)

  # preemptively load the shard on every peer when a prompt starts anywhere in the ring
  def preload(request_id, opaque_status):
    try:
      st = json.loads(opaque_status)
      if st.get("type") == "node_status" and st.get("status") == "start_process_prompt":
        from .inference.shard import Shard
        cur = node.get_current_shard(Shard.from_dict(st["base_shard"]))
        asyncio.get_running_loop().create_task(engine.ensure_shard(cur))
    except Exception:
      if DEBUG >= 2:
        traceback.print_exc()

  node.on_opaque_status.register("preemptively_load_shard").on_next(preload)
  last = [0.0]

  def progress(shard, event):
    if time.time() - last[0] < 0.1:
      return
    last[0] = time.time()
    asyncio.get_running_loop().create_task(node.broadcast_opaque_status("", json.dumps({
      "type": "download_progress", "node_id": node.id, "progress": event.to_dict()})))

  downloader.on_progress.register("broadcast").on_next(progress)
  if viz is not None:
    node.on_token.register("update_topology_viz").on_next(
      lambda rid, toks, fin: viz.update_prompt_output(rid, getattr(engine, "tokenizer", None).decode(toks))
      if getattr(engine, "tokenizer", None) is not None and hasattr(viz, "update_prompt_output") else None)
  return node, api, engine, viz


async def async_main(args, engine=None, device_caps=None):
  if args.models_seed_dir:
    from .download.new_shard_download import seed_models
    seed_models(args.models_seed_dir)
  node, api, engine, viz = build_node(args, engine=engine, device_caps=device_caps)
  loop = asyncio.get_running_loop()
  # SIGINT / SIGTERM end the command, then the node shuts down in order (tasks, discovery, gRPC server, API)
  # before the loop closes -- cancelling every task from the handler instead (the reference's helpers.shutdown,
  # xotorch/helpers.py:318-326) left the gRPC server's own shutdown to run on a closed loop
  stop = asyncio.Event()

  def on_signal(s):
    print(f"Received exit signal {s.name}...")
    stop.set()

  for s in (signal.SIGINT, signal.SIGTERM):
    try:
      loop.add_signal_handler(s, on_signal, s)
    except NotImplementedError:  # pragma: no cover
      pass
  halt = asyncio.ensure_future(stop.wait())
  start = work = None
  rc = 0
  try:
    start = asyncio.ensure_future(node.start(wait_for_peers=args.wait_for_peers))
    await asyncio.wait({start, halt}, return_when=asyncio.FIRST_COMPLETED)
    if start.done():
      start.result()
      work = asyncio.ensure_future(_command(args, node, api, viz))  # the command once the node is up
      done, _ = await asyncio.wait({work, halt}, return_when=asyncio.FIRST_COMPLETED)
      if work in done:
        rc = work.result() or 0
  finally:
    pending = [t for t in (start, work, halt) if t is not None]
    for t in pending:
      t.cancel()
    await asyncio.gather(*pending, return_exceptions=True)
    await node.stop()
    if api is not None:
      await api.stop()
  return rc


async def _command(args, node, api, viz) -> int:
  model_name = args.model_name or args.run_model
  if args.command == "run" or args.run_model:
    if not model_name:
      print("Error: model name is required")
      return 1
    await run_model_cli(node, model_name, args.prompt, viz)
  elif args.command == "eval":
    await eval_model_cli(node, model_name, args.data, args.batch_size)
  elif args.command == "train":
    await train_model_cli(node, model_name, args.data, args.batch_size, args.iters, args.save_every,
                          args.save_checkpoint_dir, args.resume_checkpoint)
  else:
    if api is not None:
      await api.run(port=args.chatgpt_api_port)
      print(f"ChatGPT API listening on http://localhost:{args.chatgpt_api_port}")
      if args.chat_tui:
        from .viz.chat_tui import run_chat_tui
        await run_chat_tui(args, api, node)
    await asyncio.Event().wait()
  if args.wait_for_peers > 0:
    await asyncio.sleep(5)  # let peers finish their side of the last request
  return 0


def run(argv=None):
  argv = list(sys.argv[1:] if argv is None else argv)
  args = build_parser().parse_args(argv)
  if args.weight_dtype:  # read by every ShardRunner this process (and its spawned peers) builds
    os.environ["XOT_WEIGHT_DTYPE"] = args.weight_dtype
  if args.max_batch:
    os.environ["XOT_MAX_BATCH"] = str(args.max_batch)
  if args.max_ctx:
    os.environ["XOT_MAX_CTX"] = str(args.max_ctx)
  if args.federate and args.gpus and args.gpus > 1 and "XOT_PEER_RANK" not in os.environ:
    from .parallel.ring_federation import federate_ring  # the local RCCL ring as one discovered peer
    sys.exit(federate_ring(args, argv))
  if args.gpus and args.gpus > 1 and not args.grpc_peers and "XOT_PEER_RANK" not in os.environ:
    args.ring = True  # local GPUs are ring peers over RCCL unless the gRPC topology is asked for
  if args.ring and args.command in ("train", "eval"):
    from .train.ring_train import run_ring
    sys.exit(run_ring(args))
  if args.ring:  # serve / run over the local GPU ring: continuous batching, RCCL activation hand-off
    from .parallel.ring_serve import serve_ring
    sys.exit(serve_ring(args))
  if args.gpus and args.gpus > 1 and "XOT_PEER_RANK" not in os.environ:
    sys.exit(spawn_gpu_peers(args, argv))
  if DEBUG >= 0 and not args.no_api and os.environ.get("XOT_PEER_RANK", "0") == "0":
    print_banner()
  try:
    rc = asyncio.run(async_main(args))
  except (KeyboardInterrupt, asyncio.CancelledError):
    rc = 0
  sys.exit(rc or 0)


if __name__ == "__main__":
  run()
