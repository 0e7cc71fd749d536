"""ChatGPT-compatible HTTP API (reference: xotorch/api/chatgpt_api.py, routes :208-234).

Same routes and JSON shapes: /v1/models, /v1/chat/token/encode,
/v1/chat/completions (stream + non-stream), /v1/download/progress, /modelpool (SSE),
/initial_models, /download, DELETE /models/{name}, /v1/topology, /healthcheck, /quit, tinychat at /.
Additions: `temperature`, `top_k` and `max_tokens` are honoured per request (the reference parses
temperature and drops it), streams end with `data: [DONE]`, GET /metrics (Prometheus) and
GET /v1/traces (recent spans).
"""
from __future__ import annotations

import asyncio
import json
import os
import time
import traceback
import uuid
from pathlib import Path
from typing import Dict, List, Literal, Optional, Union

from aiohttp import web

from ..helpers import DEBUG, VERSION, shutdown
from ..inference.tokenizers import resolve_tokenizer
from ..models import registry
from ..models.registry import (build_base_shard, build_full_shard, get_pretty_name, get_repo, get_supported_models,
                               is_vision_model)
from ..models.vision import IMAGE_MARK, escape_marks
from ..orchestration.tracing import tracer
from ..utils import metrics

ENGINE_CLASS = {"ShardedInferenceEngine": "ShardedInferenceEngine", "DummyInferenceEngine": "DummyInferenceEngine"}


class Message:
  def __init__(self, role: str, content: Union[str, List[dict]], tools: Optional[List[dict]] = None):
    self.role = role
    self.content = content
    self.tools = tools

  def to_dict(self) -> dict:
    d = {"role": self.role, "content": self.content}
    if self.tools:
      d["tools"] = self.tools
    return d


class ChatCompletionRequest:
  def __init__(self, model: str, messages: List[Message], temperature: Optional[float], tools=None,
               max_tokens: Optional[int] = None, top_k: Optional[int] = None, stream: bool = False):
    self.model = model
    self.messages = messages
    self.temperature = temperature
    self.tools = tools
    self.max_tokens = max_tokens
    self.top_k = top_k
    self.stream = stream

  def to_dict(self) -> dict:
    return {"model": self.model, "messages": [m.to_dict() for m in self.messages], "temperature": self.temperature,
            "tools": self.tools, "max_tokens": self.max_tokens}


def parse_message(d: dict) -> Message:
  if "role" not in d or "content" not in d:
    raise ValueError(f"Invalid message: {d}. Must have 'role' and 'content'")
  return Message(d["role"], d["content"], d.get("tools"))


def parse_chat_request(d: dict, default_model: str) -> ChatCompletionRequest:
  return ChatCompletionRequest(d.get("model", default_model), [parse_message(m) for m in d["messages"]],
                               d.get("temperature"), d.get("tools"), d.get("max_tokens") or d.get("max_completion_tokens"),
                               d.get("top_k"), bool(d.get("stream", False)))


IMAGE_PLACEHOLDER = "[An image was uploaded but is not displayed here]"


def remap_messages(messages: List[Message]) -> List[Message]:
  """Images become text placeholders except the LAST one, which stays an image part."""
  out: List[Message] = []
  last_image = None
  for m in messages:
    if not isinstance(m.content, list):
      out.append(m)
      continue
    parts = []
    for c in m.content:
      if isinstance(c, dict) and c.get("type") in ("image_url", "image"):
        url = (c.get("image_url") or {}).get("url") if isinstance(c.get("image_url"), dict) else c.get("image")
        if url:
          last_image = {"type": "image", "image": url}
          parts.append({"type": "text", "text": IMAGE_PLACEHOLDER})
      else:
        parts.append(c)
    out.append(Message(m.role, parts))
  if last_image:
    for m in reversed(out):
      if isinstance(m.content, list):
        for i, c in enumerate(m.content):
          if isinstance(c, dict) and c.get("type") == "text" and c.get("text") == IMAGE_PLACEHOLDER:
            m.content[i] = last_image
            return out
  return out


def build_prompt(tokenizer, messages: List[Message], tools: Optional[List[dict]] = None, vision: bool = False) -> str:
  """Chat-template prompt.  For a vision model (LLaVA) the kept image becomes an in-prompt
  `<|xot_image:URL|>` marker that the first shard's engine expands into image tokens (models/vision.py),
  so the image travels with the prompt to whichever peer holds the first shard."""
  msgs = [m.to_dict() for m in remap_messages(messages)]
  for m in msgs:  # user text cannot forge an image marker (only the kept image part below becomes one)
    if isinstance(m["content"], str):
      m["content"] = escape_marks(m["content"])
    elif isinstance(m["content"], list):
      m["content"] = [dict(c, text=escape_marks(c["text"]))
                      if isinstance(c, dict) and c.get("type") == "text" and isinstance(c.get("text"), str) else c
                      for c in m["content"]]
  for m in msgs:
    if isinstance(m["content"], list):
      for i, c in enumerate(m["content"]):
        if isinstance(c, dict) and c.get("type") == "image":
          m["content"][i] = {"type": "text", "text": IMAGE_MARK.format(c["image"]) if vision else IMAGE_PLACEHOLDER}
      if all(isinstance(c, dict) and c.get("type") == "text" for c in m["content"]):
        m["content"] = "".join(c["text"] for c in m["content"])
  kw = {"tokenize": False, "add_generation_prompt": True}
  if tools:
    kw["tools"] = tools
  try:
    return tokenizer.apply_chat_template(msgs, **kw)
  except Exception:
    # tokenizers without a chat template: plain role-prefixed transcript
    text = "".join(f"{m['role']}: {m['content'] if isinstance(m['content'], str) else json.dumps(m['content'])}\n"
                   for m in msgs)
    return text + "assistant: "


def generate_completion(req: ChatCompletionRequest, tokenizer, prompt: str, request_id: str, tokens: List[int],
                        stream: bool, finish_reason: Optional[Literal["length", "stop"]],
                        object_type: str = "chat.completion") -> dict:
  text = tokenizer.decode(tokens)
  comp = {
    "id": f"chatcmpl-{request_id}",
    "object": object_type,
    "created": int(time.time()),
    "model": req.model,
    "system_fingerprint": f"xot_{VERSION}",
    "choices": [{"index": 0, "logprobs": None, "finish_reason": finish_reason}],
  }
  choice = comp["choices"][0]
  if object_type.startswith("chat.completion"):
    choice["delta" if stream else "message"] = {"role": "assistant", "content": text}
  else:
    choice["text"] = text
  if not stream:
    n_prompt = len(tokenizer.encode(prompt))
    comp["usage"] = {"prompt_tokens": n_prompt, "completion_tokens": len(tokens), "total_tokens": n_prompt + len(tokens)}
  return comp


class StreamChunks:
  """SSE `data:` lines of one streaming chat completion, byte-identical to json.dumps of
  generate_completion(..., stream=True, object_type="chat.completion.chunk"): the request's constant JSON is
  encoded once and only the token text (and finish reason) is escaped per chunk -- this runs once per
  generated token per stream."""

  def __init__(self, req: ChatCompletionRequest, tokenizer, request_id: str):
    self.tokenizer = tokenizer
    self.head = '{"id": ' + json.dumps(f"chatcmpl-{request_id}") + ', "object": "chat.completion.chunk", "created": '
    self.mid = (', "model": ' + json.dumps(req.model) + ', "system_fingerprint": ' + json.dumps(f"xot_{VERSION}")
                + ', "choices": [{"index": 0, "logprobs": null, "finish_reason": ')

  def line(self, tokens: List[int], finish_reason: Optional[str]) -> bytes:
    text = self.tokenizer.decode(tokens)
    fr = "null" if finish_reason is None else json.dumps(finish_reason)
    return ("data: " + self.head + str(int(time.time())) + self.mid + fr
            + ', "delta": {"role": "assistant", "content": ' + json.dumps(text) + "}}]}\n\n").encode()


# XOT_DIRECT_SSE=0: every streamed token goes through the request's queue and wakes its handler task
DIRECT_SSE = os.environ.get("XOT_DIRECT_SSE", "1") == "1"
# above this many bytes waiting in a stream's socket buffer (a slow reader) its tokens go back to the queue path
DIRECT_SSE_MAX_BUFFER = 1 << 20


class _DirectStream:
  """One streaming response fed straight from the token callback: each token's SSE chunk is framed (HTTP/1.1
  chunked encoding, which the response was prepared with) and handed to the connection's transport inside
  the emitter's call -- no queue hop and no handler-task wake-up per token, which at hundreds of streams was
  the serving loop's largest host cost.  The handler task only waits for `done`."""

  def __init__(self, transport, chunks: "StreamChunks", eos: set, counter, on_first):
    self.transport, self.chunks, self.eos, self.counter, self.on_first = transport, chunks, eos, counter, on_first
    self.done = asyncio.get_running_loop().create_future()
    self.first = True
    self.fallback = False  # set when the stream went back to the queue path

  def usable(self) -> bool:
    t = self.transport
    return not t.is_closing() and t.get_write_buffer_size() <= DIRECT_SSE_MAX_BUFFER

  def feed(self, tokens: List[int], finished: bool) -> None:
    if self.first and tokens:
      self.first = False
      self.on_first()
    if self.counter is not None:
      self.counter.inc(len(tokens))
    eos_hit = finished and tokens and tokens[-1] in self.eos
    emit = tokens[:-1] if eos_hit else tokens
    line = self.chunks.line(list(emit), ("stop" if eos_hit else "length") if finished else None)
    self.transport.write(b"%x\r\n%s\r\n" % (len(line), line))
    if finished and not self.done.done():
      self.done.set_result(None)


class ChatGPTAPI:
  def __init__(self, node, inference_engine_classname: str, response_timeout: int = 900,
               on_chat_completion_request=None, default_model: Optional[str] = None,
               system_prompt: Optional[str] = None):
    self.node = node
    self.inference_engine_classname = inference_engine_classname
    self.response_timeout = response_timeout
    self.on_chat_completion_request = on_chat_completion_request
    self.default_model = default_model or "llama-3.2-1b"
    self.system_prompt = system_prompt
    self.token_queues: Dict[str, asyncio.Queue] = {}
    self._direct: Dict[str, _DirectStream] = {}  # streaming requests fed straight from the token callback
    self.prompts: Dict[str, dict] = {}
    self.app = web.Application(client_max_size=100 * 1024 * 1024, middlewares=[self.timeout_middleware,
                                                                               self.log_request, self.cors_middleware])
    r = self.app.router
    r.add_get("/models", self.handle_get_models)
    r.add_get("/v1/models", self.handle_get_models)
    r.add_post("/chat/token/encode", self.handle_post_chat_token_encode)
    r.add_post("/v1/chat/token/encode", self.handle_post_chat_token_encode)
    r.add_post("/chat/completions", self.handle_post_chat_completions)
    r.add_post("/v1/chat/completions", self.handle_post_chat_completions)
    r.add_post("/v1/image/generations", self.handle_post_image_generations)
    r.add_get("/v1/download/progress", self.handle_get_download_progress)
    r.add_get("/modelpool", self.handle_model_support)
    r.add_get("/healthcheck", self.handle_healthcheck)
    r.add_post("/quit", self.handle_quit)
    r.add_delete("/models/{model_name}", self.handle_delete_model)
    r.add_get("/initial_models", self.handle_get_initial_models)
    r.add_post("/download", self.handle_post_download)
    r.add_get("/topology", self.handle_get_topology)
    r.add_get("/v1/topology", self.handle_get_topology)
    r.add_get("/metrics", self.handle_metrics)
    r.add_get("/v1/traces", self.handle_traces)
    r.add_route("OPTIONS", "/{tail:.*}", self.handle_options)
    static = Path(__file__).resolve().parent.parent / "tinychat"
    if static.exists():
      r.add_get("/", self.handle_root)
      r.add_static("/", static, name="static")
    node.on_token.register("chatgpt-api-token-handler").on_next(self.handle_tokens)

  # ------------------------------------------------------------------ middleware
  @web.middleware
  async def cors_middleware(self, request, handler):
    resp = await handler(request)
    if isinstance(resp, web.StreamResponse) and not resp.prepared:
      resp.headers.setdefault("Access-Control-Allow-Origin", "*")
      resp.headers.setdefault("Access-Control-Allow-Methods", "*")
      resp.headers.setdefault("Access-Control-Allow-Headers", "*")
    return resp

  async def handle_options(self, request):
    return web.Response(headers={"Access-Control-Allow-Origin": "*", "Access-Control-Allow-Methods": "*",
                                 "Access-Control-Allow-Headers": "*"})

  @web.middleware
  async def timeout_middleware(self, request, handler):
    try:
      return await asyncio.wait_for(handler(request), timeout=self.response_timeout)
    except asyncio.TimeoutError:
      return web.json_response({"detail": "Request timed out"}, status=408)

  @web.middleware
  async def log_request(self, request, handler):
    if DEBUG >= 2:
      print(f"Received request: {request.method} {request.path}")
    return await handler(request)

  # ------------------------------------------------------------------ helpers
  def _resolve_model(self, model: Optional[str]) -> str:
    if not model or model.startswith("gpt-") or model not in registry.model_cards:
      return self.default_model
    return model

  async def _tokenizer(self, model: str):
    eng = self.node.inference_engine
    shard = getattr(eng, "shard", None)
    if shard is not None and shard.model_id == model and getattr(eng, "tokenizer", None) is not None:
      return eng.tokenizer
    repo = get_repo(model, self.inference_engine_classname)
    vocab = None
    try:
      from ..models.config import preset
      vocab = preset(model).vocab_size
    except KeyError:
      pass
    return await resolve_tokenizer(repo or model, vocab)

  # ------------------------------------------------------------------ handlers
  async def handle_root(self, request):
    return web.FileResponse(Path(__file__).resolve().parent.parent / "tinychat" / "index.html")

  async def handle_healthcheck(self, request):
    return web.json_response({"status": "ok"})

  async def handle_quit(self, request):
    if DEBUG >= 1:
      print("Received quit signal")
    resp = web.json_response({"detail": "Quit signal received"}, status=200)
    await resp.prepare(request)
    await resp.write_eof()
    import signal
    asyncio.get_running_loop().call_later(0.1, lambda: asyncio.ensure_future(
      shutdown(signal.SIGINT, asyncio.get_running_loop(), self.node.server)))
    return resp

  async def handle_get_models(self, request):
    owner = os.environ.get("XOT_UUID", "self")
    return web.json_response({"object": "list", "data": [{"id": m, "object": "model", "owned_by": owner, "ready": True}
                                                         for m in registry.model_cards]})

  async def handle_get_initial_models(self, request):
    return web.json_response({m: {"name": get_pretty_name(m) or m, "downloaded": None, "download_percentage": None,
                                  "total_size": None, "total_downloaded": None, "loading": True}
                              for m in get_supported_models([[self.inference_engine_classname]])})

  async def handle_model_support(self, request):
    resp = web.StreamResponse(status=200, headers={"Content-Type": "text/event-stream", "Cache-Control": "no-cache",
                                                   "Connection": "keep-alive", "Access-Control-Allow-Origin": "*"})
    await resp.prepare(request)
    dl = getattr(self.node, "shard_downloader", None)
    if dl is not None:
      async for path, s in dl.get_shard_download_status(self.inference_engine_classname):
        model_id = s.shard.model_id
        pct = 100.0 * s.downloaded_bytes / s.total_bytes if s.total_bytes else 0.0
        payload = {model_id: {"name": get_pretty_name(model_id) or model_id, "downloaded": s.status == "complete",
                              "download_percentage": pct, "total_size": s.total_bytes,
                              "total_downloaded": s.downloaded_bytes}}
        await resp.write(f"data: {json.dumps(payload)}\n\n".encode())
    await resp.write(b"data: [DONE]\n\n")
    return resp

  async def handle_post_chat_token_encode(self, request):
    data = await request.json()
    model = self._resolve_model(data.get("model"))
    tok = await self._tokenizer(model)
    messages = [parse_message(m) for m in data.get("messages", [])]
    prompt = build_prompt(tok, messages, data.get("tools"), vision=is_vision_model(model))
    ids = tok.encode(prompt)
    return web.json_response({"length": len(prompt), "num_tokens": len(ids), "encoded_tokens": list(map(int, ids)),
                              "encoded_prompt": prompt})

  async def handle_get_download_progress(self, request):
    out = {}
    for node_id, prog in self.node.node_download_progress.items():
      if isinstance(prog, dict) and prog.get("status") == "in_progress":
        out[node_id] = prog
      elif hasattr(prog, "status") and prog.status == "in_progress":
        out[node_id] = prog.to_dict()
    return web.json_response(out)

  async def handle_post_chat_completions(self, request):
    data = await request.json()
    stream = bool(data.get("stream", False))
    try:
      req = parse_chat_request(data, self.default_model)
    except (KeyError, ValueError) as e:
      return web.json_response({"detail": str(e)}, status=400)
    req.model = self._resolve_model(req.model)
    shard = build_base_shard(req.model, self.inference_engine_classname)
    if shard is None:
      supported = get_supported_models([[self.inference_engine_classname]])
      return web.json_response({"detail": f"Unsupported model: {req.model} with inference engine "
                                          f"{self.inference_engine_classname}. Supported models: {supported}"}, status=400)
    tok = await self._tokenizer(req.model)
    if self.system_prompt and not any(m.role == "system" for m in req.messages):
      req.messages.insert(0, Message("system", self.system_prompt))
    prompt = build_prompt(tok, req.messages, req.tools, vision=is_vision_model(req.model))
    request_id = str(uuid.uuid4())
    tracer.extract(request_id, dict(request.headers))
    if self.on_chat_completion_request:
      try:
        self.on_chat_completion_request(request_id, req, prompt)
      except Exception:
        traceback.print_exc()
    metrics.AVAILABLE and metrics.REQUESTS.labels(req.model, str(stream)).inc()
    self.token_queues[request_id] = asyncio.Queue()
    state = {"temperature": req.temperature, "top_k": req.top_k, "max_tokens": req.max_tokens}
    t_start = time.perf_counter()
    try:
      await asyncio.wait_for(asyncio.shield(asyncio.create_task(
        self.node.process_prompt(shard, prompt, request_id=request_id, inference_state=state))),
        timeout=self.response_timeout)
      eos = set(getattr(self.node.inference_engine, "eos_token_ids", ()) or ())
      if getattr(tok, "eos_token_id", None) is not None:
        eos.add(int(tok.eos_token_id))
      if stream:
        resp = web.StreamResponse(status=200, reason="OK", headers={"Content-Type": "text/event-stream",
                                                                   "Cache-Control": "no-cache",
                                                                   "Access-Control-Allow-Origin": "*"})
        resp.enable_chunked_encoding()
        await resp.prepare(request)
        first = True
        chunks = StreamChunks(req, tok, request_id)
        counter = metrics.TOKENS.labels(req.model) if metrics.AVAILABLE else None
        q = self.token_queues[request_id]
        transport = request.transport
        if DIRECT_SSE and transport is not None and getattr(resp, "chunked", False):
          def on_first():
            metrics.AVAILABLE and metrics.TTFT.labels(req.model).observe(time.perf_counter() - t_start)
          d = _DirectStream(transport, chunks, eos, counter, on_first)
          finished = False
          while not q.empty() and not finished:  # tokens that arrived before this point, in order
            toks, finished = q.get_nowait()
            d.feed(toks, finished)
          if not finished:
            self._direct[request_id] = d
            try:
              await d.done
            finally:
              self._direct.pop(request_id, None)
            finished = not d.fallback
          first = d.first
          if finished:
            await resp.write(b"data: [DONE]\n\n")
            await resp.write_eof()
            return resp
        try:  # queue path (also where a direct stream continues after a fallback)
          while True:
            tokens, finished = await self._next_tokens(q)
            if first and tokens:
              first = False
              metrics.AVAILABLE and metrics.TTFT.labels(req.model).observe(time.perf_counter() - t_start)
            if counter is not None:
              counter.inc(len(tokens))
            eos_hit = finished and tokens and tokens[-1] in eos
            emit = tokens[:-1] if eos_hit else tokens
            finish_reason = ("stop" if eos_hit else "length") if finished else None
            await resp.write(chunks.line(list(emit), finish_reason))
            if finished:
              break
          await resp.write(b"data: [DONE]\n\n")
          await resp.write_eof()
          return resp
        except asyncio.TimeoutError:
          return web.json_response({"detail": "Response generation timed out"}, status=408)
      tokens: List[int] = []
      while True:
        new, finished = await self._next_tokens(self.token_queues[request_id])
        tokens.extend(new)
        if finished:
          break
      finish_reason = "length"
      if tokens and tokens[-1] in eos:
        tokens = tokens[:-1]
        finish_reason = "stop"
      metrics.AVAILABLE and metrics.TOKENS.labels(req.model).inc(len(tokens))
      return web.json_response(generate_completion(req, tok, prompt, request_id, tokens, False, finish_reason))
    except asyncio.TimeoutError:
      return web.json_response({"detail": "Response generation timed out"}, status=408)
    except Exception as e:
      if DEBUG >= 2:
        traceback.print_exc()
      return web.json_response({"detail": f"Error processing prompt: {e}"}, status=500)
    finally:
      self.token_queues.pop(request_id, None)
      tracer.finish(request_id)

  async def handle_post_image_generations(self, request):
    return web.json_response({"detail": "image generation is not supported by this build"}, status=400)

  async def handle_delete_model(self, request):
    from ..download.new_shard_download import delete_model
    name = request.match_info.get("model_name")
    try:
      if delete_model(name, self.inference_engine_classname):
        return web.json_response({"status": "success", "message": f"Model {name} deleted successfully"})
      return web.json_response({"detail": f"Model {name} files not found"}, status=404)
    except Exception as e:
      return web.json_response({"detail": f"Error deleting model: {e}"}, status=500)

  async def handle_post_download(self, request):
    try:
      data = await request.json()
      model = data.get("model")
      if not model:
        return web.json_response({"error": "model parameter is required"}, status=400)
      if model not in registry.model_cards:
        return web.json_response({"error": f"Invalid model: {model}. Available models: {list(registry.model_cards)}"},
                                 status=400)
      shard = build_full_shard(model, self.inference_engine_classname)
      if not shard:
        return web.json_response({"error": f"Could not build shard for model {model}"}, status=400)
      asyncio.create_task(self.node.inference_engine.shard_downloader.ensure_shard(shard,
                                                                                 self.inference_engine_classname))
      return web.json_response({"status": "success", "message": f"Download started for model: {model}"})
    except Exception as e:
      return web.json_response({"error": str(e)}, status=500)

  async def handle_get_topology(self, request):
    try:
      topo = self.node.current_topology
      d = topo.to_json() if topo else {}
      ranges = getattr(self.node, "layer_ranges", None)
      if topo and callable(ranges):  # which layers each peer serves (extra key; the reference shape is unchanged)
        d["partitions"] = [{"node_id": nid, "start_layer": a, "end_layer": b} for nid, a, b in ranges()]
      return web.json_response(d)
    except Exception as e:
      return web.json_response({"detail": f"Error getting topology: {e}"}, status=500)

  async def handle_metrics(self, request):
    return web.Response(body=metrics.render(self.node), content_type="text/plain")

  async def handle_traces(self, request):
    return web.json_response(tracer.export(int(request.query.get("limit", 1000))))

  # ------------------------------------------------------------------ token fan-in
  def handle_tokens(self, request_id: str, tokens: List[int], is_finished: bool):
    """Token callback (plain function: runs inside the emitter's call, no task per token)."""
    d = self._direct.get(request_id)
    if d is not None:
      tracer.on_token(request_id, len(tokens))
      if d.usable():
        d.feed(tokens, is_finished)
        return
      # slow reader or closing connection: back to the queue path (the handler's direct wait ends)
      self._direct.pop(request_id, None)
      d.fallback = True
      if not d.done.done():
        d.done.set_result(None)
    q = self.token_queues.get(request_id)
    if q is not None:
      if d is None:
        tracer.on_token(request_id, len(tokens))
      q.put_nowait((list(tokens), is_finished))

  async def _next_tokens(self, q: asyncio.Queue):
    """Every token chunk queued for a request, merged: (tokens, finished), so a stream that fell behind
    catches up in one write.  No per-token wait_for (a task per token): timeout_middleware already bounds
    the whole request by the response timeout."""
    try:
      toks, fin = q.get_nowait()
    except asyncio.QueueEmpty:
      toks, fin = await q.get()
    toks = list(toks)
    while not fin and not q.empty():
      more, fin = q.get_nowait()
      toks.extend(more)
    return toks, fin

  async def run(self, host: str = "0.0.0.0", port: int = 52415):
    runner = web.AppRunner(self.app)
    await runner.setup()
    site = web.TCPSite(runner, host, port)
    await site.start()
    self._runner = runner

  async def stop(self) -> None:
    """Close the HTTP listener (its open connections get the server's shutdown)."""
    runner = getattr(self, "_runner", None)
    self._runner = None
    if runner is not None:
      await runner.cleanup()
