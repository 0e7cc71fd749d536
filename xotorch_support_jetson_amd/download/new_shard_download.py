"""HF-compatible shard downloader (reference: xotorch/download/new_shard_download.py:24-308).

  * lists repo files via {HF_ENDPOINT}/api/models/{repo}/tree/{rev} (recursive, cached under XOT_HOME/tmp)
  * reads model.safetensors.index.json and fetches only the files that hold this shard's tensors
    plus configs/tokenizers (hf_helpers.get_allow_patterns)
  * resumable downloads into `<file>.partial` with HTTP Range, verified against the sha1 git-blob or
    sha256 LFS hash from the ETag before the atomic rename
  * retries with exponential backoff (<= 8 s), at most `max_parallel_downloads` files in flight
  * progress events through an AsyncCallbackSystem; Singleton (dedupe concurrent calls) ->
    Cached (memoise the path) -> New wrappers.
Offline behaviour: with XOT_OFFLINE=1 (or when the hub is unreachable) a shard already present in
XOT_HOME/downloads is used as is and a missing one raises, letting the engine fall back to random
weights of the same architecture.
"""
from __future__ import annotations

import asyncio
import errno
import hashlib
import json
import os
import shutil
import socket
import time
import traceback
from datetime import timedelta
from pathlib import Path
from typing import Callable, Dict, List, Optional, Tuple
from urllib.parse import urljoin

from ..helpers import DEBUG, AsyncCallbackSystem, xot_home
from ..inference.shard import Shard
from ..models.registry import get_repo, get_supported_models, build_full_shard
from .download_progress import RepoFileProgressEvent, RepoProgressEvent
from .hf_helpers import filter_repo_objects, get_allow_patterns, get_auth_headers, get_hf_endpoint
from .shard_download import ShardDownloader


def downloads_dir() -> Path:
  d = xot_home() / "downloads"
  d.mkdir(parents=True, exist_ok=True)
  return d


def tmp_dir() -> Path:
  d = xot_home() / "tmp"
  d.mkdir(parents=True, exist_ok=True)
  return d


def repo_dir(repo_id: str) -> Path:
  return downloads_dir() / repo_id.replace("/", "--")


def delete_model(model_id: str, engine_classname: str) -> bool:
  repo = get_repo(model_id, engine_classname)
  if repo is None:
    raise ValueError(f"no repo for {model_id}")
  d = repo_dir(repo)
  if not d.exists():
    return False
  shutil.rmtree(d)
  return True


def seed_models(seed_dir: str) -> None:
  """Move pre-downloaded `models--org--name` / `org--name` directories into XOT_HOME/downloads."""
  src = Path(seed_dir)
  for p in src.iterdir():
    if not p.is_dir():
      continue
    name = p.name[len("models--"):] if p.name.startswith("models--") else p.name
    dest = downloads_dir() / name
    if dest.exists():
      print(f"Skipping {p}: {dest} exists")
      continue
    try:
      p.rename(dest)
    except OSError:
      traceback.print_exc()


def _retry_delay(attempt: int) -> float:
  return min(8.0, 0.1 * (2 ** attempt))


def _unreachable_error(e: BaseException) -> bool:
  """A CONNECT-phase failure: the hub cannot be reached at all (no DNS, no route, refused, connect timeout).
  Failures after a connection was made -- socket read timeouts, resets mid-transfer, HTTP errors -- are transient
  and keep the normal backoff retries (a slow large file must not mark the hub unreachable for the process)."""
  try:
    import aiohttp
    # (ConnectionTimeoutError exists from aiohttp 3.10; older releases raise ServerTimeoutError for connect timeouts)
    connect_timeout = getattr(aiohttp, "ConnectionTimeoutError", aiohttp.ServerTimeoutError)
    if isinstance(e, (aiohttp.ClientConnectorError, connect_timeout)):
      return True
    if isinstance(e, aiohttp.ClientError):
      return False  # ServerDisconnectedError, SocketTimeoutError (read), ClientPayloadError, ...
  except ImportError:
    pass
  if isinstance(e, (ConnectionRefusedError, socket.gaierror)):
    return True
  return isinstance(e, OSError) and e.errno in (errno.ENETUNREACH, errno.EHOSTUNREACH)


class HFRepoClient:
  """Minimal async client for the HF hub file API.

  Transient failures are retried with backoff (`attempts`).  Connection-level failures (no DNS, no route,
  refused, connect timeout) are retried only `unreachable_after` times; then the hub is marked unreachable for
  the rest of the process and every later call fails at once -- without that, a host with no network spent the
  whole backoff budget (minutes) on each file before falling back to local / random weights."""

  unreachable = False  # process-wide: set after repeated connection-level failures

  def __init__(self, endpoint: Optional[str] = None, attempts: int = 30, unreachable_after: int = 2):
    self.endpoint = endpoint or get_hf_endpoint()
    self.attempts = attempts
    self.unreachable_after = unreachable_after

  def _session(self, total: float = 1800):
    import aiohttp
    return aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=total, connect=30, sock_read=total))

  async def _with_retry(self, fn, *args):
    if HFRepoClient.unreachable:
      raise ConnectionError(f"{self.endpoint} unreachable (an earlier connection attempt failed)")
    conn_failures = 0
    for attempt in range(self.attempts):
      try:
        return await fn(*args)
      except FileNotFoundError:
        raise
      except Exception as e:
        if _unreachable_error(e):
          conn_failures += 1
          if conn_failures >= self.unreachable_after:
            HFRepoClient.unreachable = True
            raise
        if attempt == self.attempts - 1:
          raise
        await asyncio.sleep(_retry_delay(attempt))

  async def list_files(self, repo_id: str, revision: str = "main") -> List[dict]:
    cache = tmp_dir() / f"{repo_id.replace('/', '--')}--{revision}--file_list.json"
    if cache.exists():
      return json.loads(cache.read_text())
    files = await self._with_retry(self._list, repo_id, revision, "")
    cache.write_text(json.dumps(files))
    return files

  async def _list(self, repo_id: str, revision: str, path: str) -> List[dict]:
    url = f"{self.endpoint}/api/models/{repo_id}/tree/{revision}" + (f"/{path}" if path else "")
    async with self._session(30) as s:
      async with s.get(url, headers=get_auth_headers()) as r:
        if r.status != 200:
          raise IOError(f"file list {url}: HTTP {r.status}")
        items = await r.json()
    out: List[dict] = []
    for it in items:
      if it["type"] == "file":
        out.append({"path": it["path"], "size": it["size"]})
      elif it["type"] == "directory":
        out += await self._list(repo_id, revision, it["path"])
    return out

  async def file_meta(self, repo_id: str, revision: str, path: str) -> Tuple[int, str]:
    url = urljoin(f"{self.endpoint}/{repo_id}/resolve/{revision}/", path)
    async with self._session(120) as s:
      async with s.head(url, headers=get_auth_headers(), allow_redirects=True) as r:
        if r.status == 404:
          raise FileNotFoundError(url)
        size = int(r.headers.get("x-linked-size") or r.headers.get("content-length") or 0)
        etag = r.headers.get("X-Linked-ETag") or r.headers.get("ETag") or r.headers.get("Etag")
    if size <= 0 or not etag:
      raise IOError(f"no size/etag for {url}")
    return size, etag.strip("\"'")

  async def download(self, repo_id: str, revision: str, path: str, target: Path,
                     on_progress: Callable[[int, int], None] = lambda a, b: None) -> Path:
    return await self._with_retry(self._download, repo_id, revision, path, target, on_progress)

  async def _download(self, repo_id, revision, path, target: Path, on_progress) -> Path:
    final = target / path
    if final.exists():
      return final
    final.parent.mkdir(parents=True, exist_ok=True)
    size, etag = await self.file_meta(repo_id, revision, path)
    remote_hash = etag[:-5] if etag.endswith("-gzip") else etag
    partial = target / f"{path}.partial"
    have = partial.stat().st_size if partial.exists() else 0
    if have != size:
      url = urljoin(f"{self.endpoint}/{repo_id}/resolve/{revision}/", path)
      headers = get_auth_headers()
      if have:
        headers["Range"] = f"bytes={have}-"
      async with self._session() as s:
        async with s.get(url, headers=headers) as r:
          if r.status == 404:
            raise FileNotFoundError(url)
          if r.status not in (200, 206):
            raise IOError(f"download {url}: HTTP {r.status}")
          if r.status == 200:
            have = 0  # server ignored the range: start over
          with open(partial, "ab" if have else "wb") as f:
            async for chunk in r.content.iter_chunked(8 << 20):
              f.write(chunk)
              have += len(chunk)
              on_progress(have, size)
    digest = await asyncio.to_thread(_file_hash, partial, "sha256" if len(remote_hash) == 64 else "sha1")
    if digest != remote_hash:
      partial.unlink(missing_ok=True)
      raise IOError(f"{final}: hash {digest} != remote {remote_hash}")
    partial.rename(final)
    return final


def _file_hash(path: Path, kind: str) -> str:
  h = hashlib.sha1() if kind == "sha1" else hashlib.sha256()
  if kind == "sha1":
    h.update(f"blob {path.stat().st_size}\0".encode())
  with open(path, "rb") as f:
    while chunk := f.read(8 << 20):
      h.update(chunk)
  return h.hexdigest()


def _repo_progress(shard: Shard, repo_id: str, revision: str, files: Dict[str, RepoFileProgressEvent],
                   t0: float) -> RepoProgressEvent:
  total = sum(p.total for p in files.values())
  done = sum(p.downloaded for p in files.values())
  session = sum(p.downloaded_this_session for p in files.values())
  dt = time.time() - t0
  speed = session / dt if dt > 0 else 0.0
  eta = timedelta(seconds=(total - done) / speed) if speed > 0 else timedelta(0)
  if files and all(p.status == "complete" for p in files.values()):
    status = "complete"
  elif any(p.status == "in_progress" for p in files.values()):
    status = "in_progress"
  else:
    status = "not_started"
  completed = sum(1 for p in files.values() if p.downloaded == p.total)
  return RepoProgressEvent(shard, repo_id, revision, completed, len(files), done, session, total, speed, eta, files,
                           status)


async def download_shard(shard: Shard, engine_classname: str,
                         on_progress: AsyncCallbackSystem[str, Tuple[Shard, RepoProgressEvent]],
                         max_parallel_downloads: int = 8, skip_download: bool = False,
                         client: Optional[HFRepoClient] = None) -> Tuple[Path, RepoProgressEvent]:
  repo_id = get_repo(shard.model_id, engine_classname)
  if repo_id is None:
    raise ValueError(f"No repo found for {shard.model_id=} and inference engine {engine_classname}")
  revision = "main"
  target = repo_dir(repo_id)
  client = client or HFRepoClient()
  offline = os.environ.get("XOT_OFFLINE", "0") == "1"
  if offline:
    if (target / "config.json").exists():
      return target, RepoProgressEvent(shard, repo_id, revision, 0, 0, 0, 0, 0, 0, timedelta(0), {}, "complete")
    raise FileNotFoundError(f"offline and {target} is not present")
  try:
    idx = await client.download(repo_id, revision, "model.safetensors.index.json", tmp_dir() / repo_id.replace("/", "--"))
    allow = get_allow_patterns(json.loads(idx.read_text())["weight_map"], shard)
  except Exception:
    if DEBUG >= 1:
      print(f"no weight map for {repo_id}; downloading every file")
    allow = ["*"]
  t0 = time.time()
  listing = await client.list_files(repo_id, revision)
  wanted = list(filter_repo_objects(listing, allow_patterns=allow, key=lambda x: x["path"]))
  files: Dict[str, RepoFileProgressEvent] = {}
  for f in wanted:
    p = target / f["path"]
    have = p.stat().st_size if p.exists() else ((target / f"{f['path']}.partial").stat().st_size
                                                if (target / f"{f['path']}.partial").exists() else 0)
    files[f["path"]] = RepoFileProgressEvent(repo_id, revision, f["path"], have, 0, f["size"], 0, timedelta(0),
                                             "complete" if have == f["size"] else "not_started", time.time())

  def progress(f: dict, cur: int, tot: int):
    prev = files[f["path"]]
    sess = prev.downloaded_this_session + (cur - prev.downloaded)
    dt = time.time() - prev.start_time
    spd = sess / dt if dt > 0 else 0.0
    files[f["path"]] = RepoFileProgressEvent(repo_id, revision, f["path"], cur, sess, tot, spd,
                                             timedelta(seconds=(tot - cur) / spd) if spd > 0 else timedelta(0),
                                             "complete" if cur == tot else "in_progress", prev.start_time)
    on_progress.trigger_all(shard, _repo_progress(shard, repo_id, revision, files, t0))

  if not skip_download:
    target.mkdir(parents=True, exist_ok=True)
    sem = asyncio.Semaphore(max_parallel_downloads)

    async def one(f):
      async with sem:
        await client.download(repo_id, revision, f["path"], target, lambda c, t: progress(f, c, t))

    await asyncio.gather(*(one(f) for f in wanted))
  final = _repo_progress(shard, repo_id, revision, files, t0)
  on_progress.trigger_all(shard, final)
  return target, final


class NewShardDownloader(ShardDownloader):
  def __init__(self, max_parallel_downloads: int = 8, client: Optional[HFRepoClient] = None):
    self.max_parallel_downloads = max_parallel_downloads
    self.client = client
    self._on_progress = AsyncCallbackSystem[str, Tuple[Shard, RepoProgressEvent]]()

  @property
  def on_progress(self):
    return self._on_progress

  async def ensure_shard(self, shard: Shard, inference_engine_name: str) -> Path:
    path, _ = await download_shard(shard, inference_engine_name, self._on_progress, self.max_parallel_downloads,
                                   client=self.client)
    return path

  async def get_shard_download_status(self, inference_engine_name: str):
    for model_id in get_supported_models([[inference_engine_name]]):
      shard = build_full_shard(model_id, inference_engine_name)
      if shard is None:
        continue
      try:
        path, prog = await download_shard(shard, inference_engine_name, self._on_progress, skip_download=True,
                                          client=self.client)
        yield path, prog
      except Exception as e:
        if DEBUG >= 2:
          print(f"status of {model_id} unavailable: {e}")


class CachedShardDownloader(ShardDownloader):
  def __init__(self, inner: ShardDownloader):
    self.inner = inner
    self.cache: Dict[Tuple[str, Shard], Path] = {}

  @property
  def on_progress(self):
    return self.inner.on_progress

  async def ensure_shard(self, shard: Shard, inference_engine_name: str) -> Path:
    key = (inference_engine_name, shard)
    if key not in self.cache:
      self.cache[key] = await self.inner.ensure_shard(shard, inference_engine_name)
    return self.cache[key]

  async def get_shard_download_status(self, inference_engine_name: str):
    async for item in self.inner.get_shard_download_status(inference_engine_name):
      yield item


class SingletonShardDownloader(ShardDownloader):
  """Concurrent ensure_shard calls for the same shard share one download task."""

  def __init__(self, inner: ShardDownloader):
    self.inner = inner
    self.active: Dict[Shard, asyncio.Task] = {}

  @property
  def on_progress(self):
    return self.inner.on_progress

  async def ensure_shard(self, shard: Shard, inference_engine_name: str) -> Path:
    task = self.active.get(shard)
    if task is None:
      task = self.active[shard] = asyncio.create_task(self.inner.ensure_shard(shard, inference_engine_name))
    try:
      return await task
    finally:
      if self.active.get(shard) is task and task.done():
        self.active.pop(shard, None)

  async def get_shard_download_status(self, inference_engine_name: str):
    async for item in self.inner.get_shard_download_status(inference_engine_name):
      yield item


def new_shard_downloader(max_parallel_downloads: int = 8) -> ShardDownloader:
  return SingletonShardDownloader(CachedShardDownloader(NewShardDownloader(max_parallel_downloads)))
