"""Shard downloader against a local fake HF hub (aiohttp on 127.0.0.1): per-shard allow patterns,
resumable Range downloads, sha256 verification, progress events, offline mode, delete
(reference: xotorch/download/new_shard_download.py; its own test needs the real hub)."""
import asyncio
import hashlib
import json
import os

import pytest
from aiohttp import web

from xotorch_support_jetson_amd.download.new_shard_download import (HFRepoClient, delete_model, download_shard,
                                                                    repo_dir)
from xotorch_support_jetson_amd.helpers import AsyncCallbackSystem
from xotorch_support_jetson_amd.inference.shard import Shard

REPO = "unsloth/Llama-3.2-1B-Instruct"  # card of llama-3.2-1b (16 layers)
ENGINE = "ShardedInferenceEngine"


def _files():
  wm = {}
  for l in range(16):
    wm[f"model.layers.{l}.mlp.down_proj.weight"] = "model-00001-of-00002.safetensors" if l < 8 else \
      "model-00002-of-00002.safetensors"
  wm["model.embed_tokens.weight"] = "model-00001-of-00002.safetensors"
  wm["model.norm.weight"] = "model-00002-of-00002.safetensors"
  return {
    "config.json": json.dumps({"num_hidden_layers": 16}).encode(),
    "tokenizer.json": b"{}",
    "model.safetensors.index.json": json.dumps({"weight_map": wm}).encode(),
    "model-00001-of-00002.safetensors": os.urandom(300_000),
    "model-00002-of-00002.safetensors": os.urandom(200_000),
    "original/consolidated.pth": os.urandom(1000),  # never wanted
  }


async def _hub(files, log):
  app = web.Application()

  async def tree(req):
    return web.json_response([{"type": "file", "path": p, "size": len(b)} for p, b in files.items()
                              if "/" not in p] + [{"type": "directory", "path": "original"}]) \
      if not req.match_info.get("path") else web.json_response(
        [{"type": "file", "path": p, "size": len(b)} for p, b in files.items() if p.startswith("original/")])

  async def resolve(req):
    path = req.match_info["path"]
    if path not in files:
      return web.Response(status=404)
    body = files[path]
    etag = hashlib.sha256(body).hexdigest()
    hdr = {"ETag": f'"{etag}"', "Content-Length": str(len(body))}
    if req.method == "HEAD":
      return web.Response(headers=hdr)
    rng = req.headers.get("Range")
    log.append((path, rng))
    if rng:
      start = int(rng.split("=")[1].split("-")[0])
      return web.Response(status=206, body=body[start:], headers={"ETag": f'"{etag}"'})
    return web.Response(body=body, headers={"ETag": f'"{etag}"'})

  app.router.add_get("/api/models/{org}/{name}/tree/{rev}", tree)
  app.router.add_get("/api/models/{org}/{name}/tree/{rev}/{path:.*}", tree)
  app.router.add_route("*", "/{org}/{name}/resolve/{rev}/{path:.*}", resolve)
  runner = web.AppRunner(app)
  await runner.setup()
  site = web.TCPSite(runner, "127.0.0.1", 0)
  await site.start()
  port = site._server.sockets[0].getsockname()[1]
  return runner, f"http://127.0.0.1:{port}"


def test_download_shard_with_resume(tmp_path, monkeypatch):
  monkeypatch.setenv("XOT_HOME", str(tmp_path / "home"))
  files = _files()

  async def main():
    log = []
    runner, url = await _hub(files, log)
    try:
      client = HFRepoClient(endpoint=url, attempts=2)
      target = repo_dir(REPO)
      target.mkdir(parents=True)
      # half-downloaded first weight file: must resume with a Range request
      part = target / "model-00001-of-00002.safetensors.partial"
      part.write_bytes(files["model-00001-of-00002.safetensors"][:100_000])
      events = []
      cbs = AsyncCallbackSystem()
      cbs.register("t").on_next(lambda shard, ev: events.append(ev))
      path, final = await download_shard(Shard("llama-3.2-1b", 0, 7, 16), ENGINE, cbs, client=client)
      assert path == target
      got = sorted(p.name for p in path.iterdir())
      assert got == ["config.json", "model-00001-of-00002.safetensors", "model.safetensors.index.json",
                     "tokenizer.json"], got
      assert (path / "model-00001-of-00002.safetensors").read_bytes() == files["model-00001-of-00002.safetensors"]
      assert ("model-00001-of-00002.safetensors", "bytes=100000-") in log
      assert final.status == "complete" and events
      # second shard pulls the other weight file only
      _, fin2 = await download_shard(Shard("llama-3.2-1b", 8, 15, 16), ENGINE, cbs, client=client)
      assert (path / "model-00002-of-00002.safetensors").exists()
      assert not (path / "original").exists()
      # offline mode serves what is on disk
      os.environ["XOT_OFFLINE"] = "1"
      try:
        p2, _ = await download_shard(Shard("llama-3.2-1b", 0, 15, 16), ENGINE, cbs, client=client)
        assert p2 == path
      finally:
        del os.environ["XOT_OFFLINE"]
      assert delete_model("llama-3.2-1b", ENGINE)
      assert not path.exists()
    finally:
      await runner.cleanup()

  asyncio.run(asyncio.wait_for(main(), 60))


def test_corrupt_download_rejected(tmp_path, monkeypatch):
  monkeypatch.setenv("XOT_HOME", str(tmp_path / "home"))
  files = _files()

  async def main():
    log = []
    runner, url = await _hub(files, log)
    try:
      client = HFRepoClient(endpoint=url, attempts=1)
      target = tmp_path / "t"
      target.mkdir()
      # a wrong partial prefix makes the final hash mismatch -> rejected, partial removed
      (target / "tokenizer.json.partial").write_bytes(b"X")
      with pytest.raises(IOError):
        await client.download(REPO, "main", "tokenizer.json", target)
      assert not (target / "tokenizer.json").exists()
      assert not (target / "tokenizer.json.partial").exists()
    finally:
      await runner.cleanup()

  asyncio.run(asyncio.wait_for(main(), 60))


def test_unreachable_hub_fails_fast(monkeypatch):
  """Connection-level failures (no route / DNS / refused) stop the retries after `unreachable_after` attempts and
  mark the hub unreachable for the process, so later calls fail at once; transient errors keep their retries."""
  import socket
  import aiohttp
  import xotorch_support_jetson_amd.download.new_shard_download as nsd
  monkeypatch.setattr(nsd, "_retry_delay", lambda attempt: 0.0)
  monkeypatch.setattr(nsd.HFRepoClient, "unreachable", False)
  calls = []

  async def refused():
    calls.append(1)
    raise ConnectionRefusedError("no route")

  async def flaky():
    calls.append(1)
    if len(calls) < 5:
      raise IOError("HTTP 500")
    return "ok"

  async def main():
    c = nsd.HFRepoClient(endpoint="http://127.0.0.1:9", attempts=30)
    assert await c._with_retry(flaky) == "ok" and len(calls) == 5  # transient: retried
    for transient in (aiohttp.SocketTimeoutError("read"), ConnectionResetError("reset"), asyncio.TimeoutError(),
                      aiohttp.ServerDisconnectedError()):
      calls.clear()

      async def slow(exc=transient):
        calls.append(1)
        if len(calls) < 4:
          raise exc
        return "ok"
      assert await c._with_retry(slow) == "ok" and len(calls) == 4 and not nsd.HFRepoClient.unreachable
    assert nsd._unreachable_error(aiohttp.ConnectionTimeoutError()) and nsd._unreachable_error(socket.gaierror(-2, "x"))
    calls.clear()
    with pytest.raises(ConnectionError):
      await c._with_retry(refused)
    assert len(calls) == 2 and nsd.HFRepoClient.unreachable
    calls.clear()
    with pytest.raises(ConnectionError):
      await c._with_retry(flaky)
    assert calls == []  # not even tried

  asyncio.run(main())
