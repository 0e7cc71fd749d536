"""Terminal chat REPL (`xot --chat-tui`; reference: xotorch/viz/chat_tui.py:11-166).

Each line is sent through `node.process_prompt`; `model <name>` switches model, `quit` exits.
Prints time-to-first-token and decode tokens/s separately (the reference folds prefill into tok/s).
"""
from __future__ import annotations

import asyncio
import sys
import time
import uuid

from ..inference.tokenizers import resolve_tokenizer
from ..models.registry import build_base_shard, get_repo


async def _ainput(prompt: str) -> str:
  return await asyncio.get_running_loop().run_in_executor(None, lambda: input(prompt))


async def run_chat_tui(args, api, node):
  model = args.default_model or args.model_name or "llama-3.2-1b"
  cls = type(node.inference_engine).__name__
  print(f"xot chat — model {model}.  Commands: 'model <name>', 'quit'.")
  while True:
    try:
      line = (await _ainput("> ")).strip()
    except (EOFError, KeyboardInterrupt):
      break
    if not line:
      continue
    if line in ("quit", "exit"):
      break
    if line.startswith("model "):
      model = line.split(None, 1)[1].strip()
      print(f"switched to {model}")
      continue
    shard = build_base_shard(model, cls)
    if shard is None:
      print(f"unsupported model {model}")
      continue
    tok = await resolve_tokenizer(get_repo(model, cls) or model)
    prompt = tok.apply_chat_template([{"role": "user", "content": line}], tokenize=False, add_generation_prompt=True)
    rid = str(uuid.uuid4())
    done = asyncio.Event()
    tokens = []
    first = [None]
    t0 = time.perf_counter()

    def on_token(req, toks, fin):
      if req != rid:
        return
      if first[0] is None and toks:
        first[0] = time.perf_counter()
      tokens.extend(toks)
      sys.stdout.write(tok.decode(toks))
      sys.stdout.flush()
      if fin:
        done.set()

    node.on_token.register(f"chat-tui-{rid}").on_next(on_token)
    try:
      await node.process_prompt(shard, prompt, request_id=rid)
      await asyncio.wait_for(done.wait(), timeout=args.chatgpt_api_response_timeout)
    except asyncio.TimeoutError:
      print("\n[timed out]")
    finally:
      node.on_token.deregister(f"chat-tui-{rid}")
    t1 = time.perf_counter()
    ttft = (first[0] - t0) if first[0] else float("nan")
    dec = len(tokens) / (t1 - first[0]) if first[0] and t1 > first[0] else 0.0
    print(f"\n[{len(tokens)} tokens, TTFT {ttft * 1000:.0f} ms, {dec:.1f} tok/s decode]")
