"""tinychat (the web UI) against the API: the UI's own helpers run under node -- markdown rendering with escaped
model output and highlighted fenced code, and the exact request body it builds for a message with an attached
image -- and that body, posted to the ChatGPT API serving tiny-LLaVA, reaches the vision path and is answered."""
import asyncio
import json
import os
import shutil
import subprocess
import threading

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(ROOT, "xotorch_support_jetson_amd", "tinychat", "index.js")
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def _js(expr: str):
  """Evaluate `expr` with the UI module bound to `t`; returns the JSON-decoded result."""
  code = f"const t = require({json.dumps(JS)}); process.stdout.write(JSON.stringify({expr}));"
  r = subprocess.run([NODE, "-e", code], capture_output=True, text=True, timeout=60)
  assert r.returncode == 0, r.stderr
  return json.loads(r.stdout)


def test_markdown_rendering_escapes_and_highlights():
  md = "# Title\n**bold** `x<y`\n<img src=x onerror=alert(1)>\n1. one\n2. two\n```python\nimport os  # hi\n```\n[a](javascript:alert(1))"
  html = _js(f"t.renderMarkdown({json.dumps(md)})")
  assert "<h1>Title</h1>" in html and "<strong>bold</strong>" in html and "<code>x&lt;y</code>" in html
  assert "<img" not in html and "&lt;img src=x" in html  # model output never becomes markup
  assert "<ol><li>one</li><li>two</li></ol>" in html
  assert '<span class="hl-keyword">import</span>' in html and '<span class="hl-comment"># hi</span>' in html
  assert "href" not in html  # only http(s) links become anchors


def test_ui_image_message_body_is_answered_by_llava(tmp_path):
  from tests.test_vision import _png_data_url
  from xotorch_support_jetson_amd.api.chatgpt_api import ChatGPTAPI
  from xotorch_support_jetson_amd.inference.shard import Shard
  from xotorch_support_jetson_amd.inference.tokenizers import _resolve_tokenizer
  from xotorch_support_jetson_amd.models.config import PRESETS
  from xotorch_support_jetson_amd.parallel.comm import P2PTransport
  from xotorch_support_jetson_amd.parallel.ring_serve import RingNode, RingServer
  from xotorch_support_jetson_amd.runtime.runner import ShardRunner
  from tests.test_ring_serve import _free_port

  url = _png_data_url(7)
  conv = [{"role": "user", "content": "what is in this picture?", "image": url}]
  body = _js(f"t.requestBody('tiny-llava', {json.dumps(conv)}, 0.0, 4)")
  assert body["messages"][0]["content"][0] == {"type": "image_url", "image_url": {"url": url}}
  assert body["stream"] is True

  model = "tiny-llava"
  c = PRESETS[model]
  shard = Shard(model, 0, c.num_layers - 1, c.num_layers)
  srv = RingServer(ShardRunner(c, shard, "cpu", max_batch=4, max_ctx=1024), 0, 1, P2PTransport(0, 1))
  seen = []
  submit = srv.submit
  srv.submit = lambda rid, ids, temp, mt, pixels=None: (seen.append((len(ids), pixels)), submit(rid, ids, temp, mt, pixels))
  tok = _resolve_tokenizer("byte", c.vocab_size)
  port = _free_port()

  async def main():
    import aiohttp
    node = RingNode(srv, shard, tok, (), 0.0, 16, loop=asyncio.get_running_loop(), config=c)
    th = threading.Thread(target=srv.serve_forever, kwargs=dict(idle_wait=0.05), daemon=True)
    th.start()
    api = ChatGPTAPI(node, "ShardedInferenceEngine", response_timeout=60, default_model=model)
    await api.run(host="127.0.0.1", port=port)
    async with aiohttp.ClientSession() as s:
      async with s.get(f"http://127.0.0.1:{port}/") as r:
        page = await r.text()
      async with s.post(f"http://127.0.0.1:{port}/v1/chat/completions", json=body) as r:
        status, text = r.status, await r.text()
    srv.stop()
    th.join(10)
    await api._runner.cleanup()
    return page, status, text

  page, status, text = asyncio.run(asyncio.wait_for(main(), 120))
  assert 'id="image-input"' in page and 'id="attach"' in page
  assert status == 200, text
  chunks = [ln for ln in text.splitlines() if ln.startswith("data: ")]
  assert chunks[-1] == "data: [DONE]" and len(chunks) >= 2
  from xotorch_support_jetson_amd.models.vision import num_image_tokens
  (n_ids, pixels), = seen
  assert isinstance(pixels, torch.Tensor) and pixels.shape[0] == 1 and n_ids > num_image_tokens(c)


def test_failed_send_resumes_only_after_a_download_completes():
  """A failed send is re-sent only after a download was seen in progress and then finished -- never on an empty
  progress map (a plain server error would otherwise be re-sent every second) -- and at most 3 times."""
  got = _js("""(() => {
    const w = {failed: true, sawDownload: false, tries: 0}, out = [];
    const busy = [["n", {status: "in_progress", total_bytes: 10, downloaded_bytes: 3}]];
    const done = [["n", {status: "complete", total_bytes: 10, downloaded_bytes: 10}]];
    out.push(t.resumeAfterDownload(w, []));        // error with no download at all: no resume
    out.push(t.resumeAfterDownload(w, []));
    out.push(t.resumeAfterDownload(w, busy));      // the model starts downloading
    out.push(t.resumeAfterDownload(w, done));      // ... and finishes: resume once
    out.push(t.resumeAfterDownload(w, done));      // not again without a new failure
    for (let i = 0; i < 5; i++) { w.failed = true; t.resumeAfterDownload(w, busy); out.push(t.resumeAfterDownload(w, [])); }
    return out; })()""")
  assert got == [False, False, False, True, False, True, True, False, False, False]
