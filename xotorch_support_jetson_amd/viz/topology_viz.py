"""Terminal topology view (reference: xotorch/viz/topology_viz.py:20-379).

A rich Live layout of three panels:
  * cluster   -- "N Node Cluster": a ring of peers drawn on a character canvas (red = the active node, green =
                 this node, blue = others) with each peer's device / memory / fp16 TFLOPS / partition
                 fraction and layer range, the link description of every ring edge in both directions, the
                 API / web-chat endpoints and a "GPU poor ... GPU rich" gauge of the summed fp16 TFLOPS;
  * chat      -- the three most recent prompts and responses, word-wrapped into a fixed height (shown
                 only once there is a request);
  * downloads -- this node's repo download (files done / total, bytes, speed, ETA, a bar per unfinished
                 file) and one summary row per other node with its device and partition (shown only while
                 some download is in progress).
Progress entries may be RepoProgressEvent objects or their to_dict() form (what /v1/download/progress and
the gRPC opaque status carry).
"""
from __future__ import annotations

import math
import textwrap
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

from ..helpers import VERSION
from ..topology.partitioning_strategy import Partition
from ..topology.topology import Topology

try:
  from rich.console import Console, Group
  from rich.layout import Layout
  from rich.live import Live
  from rich.panel import Panel
  from rich.table import Table
  from rich.text import Text
  HAVE_RICH = True
except Exception:  # pragma: no cover
  HAVE_RICH = False

CANVAS_W, CANVAS_H = 100, 30
CHAT_HEIGHT = 15


def _fmt_bytes(n: float) -> str:
  for unit in ("B", "KB", "MB", "GB", "TB"):
    if abs(n) < 1024 or unit == "TB":
      return f"{n:.0f} {unit}" if unit == "B" else f"{n:.2f} {unit}"
    n /= 1024.0
  return f"{n:.2f} TB"


def _fmt_eta(v) -> str:
  s = v.total_seconds() if hasattr(v, "total_seconds") else float(v or 0)
  s = int(max(0, s))
  return f"{s // 3600}:{s // 60 % 60:02d}:{s % 60:02d}"


def _prog(p) -> dict:
  """A RepoProgressEvent or its dict form -> a plain dict with defaults for the fields the view reads."""
  d = p if isinstance(p, dict) else p.to_dict()
  out = {"repo_id": "?", "repo_revision": "main", "completed_files": 0, "total_files": 0, "downloaded_bytes": 0,
         "total_bytes": 0, "overall_speed": 0.0, "overall_eta": 0, "status": "not_started", "file_progress": {}}
  out.update({k: v for k, v in d.items() if v is not None})
  fp = {}
  for name, f in (out.get("file_progress") or {}).items():
    fp[name] = f if isinstance(f, dict) else f.to_dict()
  out["file_progress"] = fp
  return out


def _bar(frac: float, width: int = 30) -> str:
  n = max(0, min(width, int(round(frac * width))))
  return "[" + "=" * n + " " * (width - n) + "]"


class _Canvas:
  """A fixed character grid with a style per cell; rendered to one rich Text."""

  def __init__(self, w: int, h: int):
    self.w, self.h = w, h
    self.cells = [[(" ", None) for _ in range(w)] for _ in range(h)]

  def put(self, x: int, y: int, s: str, style: Optional[str] = None, keep: Sequence[Tuple[int, int]] = ()):
    for i, ch in enumerate(s):
      if 0 <= x + i < self.w and 0 <= y < self.h and (x + i, y) not in keep:
        self.cells[y][x + i] = (ch, style)

  def line(self, x0: int, y0: int, x1: int, y1: int, style: Optional[str] = None):
    n = max(abs(x1 - x0), abs(y1 - y0))
    for k in range(1, n):
      x = round(x0 + (x1 - x0) * k / n)
      y = round(y0 + (y1 - y0) * k / n)
      ch = "─" if abs(x1 - x0) >= 2 * abs(y1 - y0) else ("│" if abs(y1 - y0) >= 2 * abs(x1 - x0) else "·")
      if 0 <= x < self.w and 0 <= y < self.h and self.cells[y][x][0] == " ":
        self.cells[y][x] = (ch, style)

  def text(self) -> "Text":
    t = Text()
    last = max((y for y in range(self.h) if any(c[0] != " " for c in self.cells[y])), default=0)
    for y in range(last + 1):
      for ch, st in self.cells[y]:
        t.append(ch, style=st)
      t.append("\n")
    return t


class TopologyViz:
  def __init__(self, chatgpt_api_endpoints: List[str] = (), web_chat_urls: List[str] = (), start: bool = True,
               num_layers: Optional[int] = None):
    self.chatgpt_api_endpoints = list(chatgpt_api_endpoints)
    self.web_chat_urls = list(web_chat_urls)
    self.topology = Topology()
    self.partitions: List[Partition] = []
    self.node_id: Optional[str] = None
    self.num_layers = num_layers  # when known, each peer's partition is also shown as a layer range
    self.node_download_progress: Dict[str, dict] = {}
    self.requests: "OrderedDict[str, list]" = OrderedDict()
    self.live = None
    self.console = None
    if HAVE_RICH and start:
      self.console = Console()
      self.live = Live(self.render(), console=self.console, refresh_per_second=4, auto_refresh=False)
      self.live.start()

  # ---------------------------------------------------------------- updates
  def update_visualization(self, topology: Topology, partitions: List[Partition], node_id: Optional[str] = None,
                           node_download_progress: Optional[Dict[str, dict]] = None,
                           num_layers: Optional[int] = None):
    self.topology = topology
    self.partitions = list(partitions)
    self.node_id = node_id
    if num_layers:
      self.num_layers = num_layers
    if node_download_progress:
      self.node_download_progress = dict(node_download_progress)
    self.refresh()

  def update_prompt(self, request_id: str, prompt: Optional[str] = None):
    self.requests.setdefault(request_id, ["", ""])
    if prompt is not None:
      self.requests[request_id][0] = prompt
    self.requests.move_to_end(request_id)
    while len(self.requests) > 3:
      self.requests.popitem(last=False)
    self.refresh()

  def update_prompt_output(self, request_id: str, output: Optional[str] = None):
    if request_id not in self.requests:
      self.update_prompt(request_id)
    if output:
      self.requests[request_id][1] += output
    self.refresh()

  def refresh(self):
    if self.live is not None:
      self.live.update(self.render(), refresh=True)

  # ---------------------------------------------------------------- cluster panel
  def total_tflops(self) -> float:
    ids = [p.node_id for p in self.partitions] or [nid for nid, _ in self.topology.all_nodes()]
    return sum(c.flops.fp16 for c in (self.topology.get_node(i) for i in ids) if c is not None)

  def _layers(self, i: int) -> str:
    if not self.num_layers:
      return ""
    from ..topology.partitioning_strategy import map_partitions_to_shards
    shards = {id(p): s for p, s in zip(self.partitions, map_partitions_to_shards(self.partitions, self.num_layers, "m"))}
    s = shards.get(id(self.partitions[i]))
    return f" layers {s.start_layer}-{s.end_layer}" if s is not None else " (no layers)"

  def _link(self, a: str, b: str) -> str:
    d1 = next((c.description for c in self.topology.peer_graph.get(a, ()) if c.to_id == b), None)
    d2 = next((c.description for c in self.topology.peer_graph.get(b, ()) if c.to_id == a), None)
    if not d1 and not d2:
      return ""
    return f"{d1 or '?'}/{d2 or '?'}"

  def gauge(self) -> "Text":
    """GPU poor ... GPU rich: log-scaled position of the summed fp16 TFLOPS (one MI355X ~ 2.5 PFLOPS sits
    a little past the middle, an 8-GPU node near the rich end)."""
    tf = self.total_tflops()
    width = 40
    frac = 0.0 if tf <= 0 else max(0.0, min(1.0, math.log10(tf) / 5.0))  # 1 TFLOPS .. 100 PFLOPS
    pos = min(width - 1, int(frac * width))
    colours = ["red", "dark_orange", "yellow", "green"]
    t = Text("GPU poor ", style="bold red")
    for i in range(width):
      t.append("▼" if i == pos else "█", style=colours[min(len(colours) - 1, i * len(colours) // width)])
    t.append(" GPU rich", style="bold green")
    t.append(f"\n{' ' * (9 + max(0, pos - 6))}{tf:,.1f} TFLOPS (fp16)")
    return t

  def ring_canvas(self) -> "_Canvas":
    cv = _Canvas(CANVAS_W, CANVAS_H)
    n = len(self.partitions)
    if n == 0:
      cv.put(2, 1, "(no peers yet)", "dim")
      return cv
    cx, cy, rx, ry = CANVAS_W // 2, CANVAS_H // 2, 26, 9
    pts = []
    for i in range(n):
      a = 2 * math.pi * i / n - math.pi / 2  # first peer at the top, clockwise
      pts.append((int(round(cx + rx * math.cos(a))), int(round(cy + ry * math.sin(a))), a))
    marks = [(x, y) for x, y, _ in pts]
    for i, (x, y, a) in enumerate(pts):  # edges first, so labels and markers draw over them
      nx, ny, _ = pts[(i + 1) % n]
      if n > 1:
        cv.line(x, y, nx, ny, "grey50")
        desc = self._link(self.partitions[i].node_id, self.partitions[(i + 1) % n].node_id)
        if desc:
          cv.put((x + nx) // 2 - len(desc) // 2, (y + ny) // 2, desc, "magenta", keep=marks)
    for i, (x, y, a) in enumerate(pts):
      p = self.partitions[i]
      caps = self.topology.get_node(p.node_id)
      if p.node_id == self.topology.active_node_id:
        style = "bold red"
      elif p.node_id == self.node_id:
        style = "bold green"
      else:
        style = "bold blue"
      cv.put(x, y, "●", style)
      info = [f"{p.node_id[:18]}",
              f"{(caps.model if caps else '?')[:22]} {(caps.memory // 1024) if caps else '?'}GB",
              f"{caps.flops.fp16 if caps else 0:.1f} TFLOPS",
              f"[{p.start:.2f}-{p.end:.2f}]{self._layers(i)}"]
      wid = max(len(s) for s in info)
      # label outside the ring: right of right-half nodes, left of left-half ones, centred at top / bottom
      c = math.cos(a)
      if c > 0.3:
        lx = x + 2
      elif c < -0.3:
        lx = x - wid - 1
      else:
        lx = x - wid // 2
      s = math.sin(a)
      ly = y - len(info) if s < -0.7 else (y + 1 if s > 0.7 else y - len(info) // 2)
      for j, line in enumerate(info):
        cv.put(max(0, min(CANVAS_W - len(line), lx)), ly + j, line, style if j == 0 else None, keep=marks)
    return cv

  def cluster_text(self) -> "Text":
    t = Text()
    t.append(f"xot v{VERSION} — MI355X\n", style="bold red")
    for url in self.web_chat_urls[:1]:
      t.append(f"Web chat (tinychat): {url}\n")
    for url in self.chatgpt_api_endpoints[:1]:
      t.append(f"ChatGPT API endpoint: {url}\n")
    t.append("\n")
    t.append_text(self.gauge())
    t.append("\n\n")
    t.append_text(self.ring_canvas().text())
    return t

  # ---------------------------------------------------------------- chat panel
  def chat_text(self, width: int = 100) -> "Text":
    reqs = list(self.requests.values())[-3:]
    t = Text()
    if not reqs:
      return t
    per = max(2, (CHAT_HEIGHT - 2) // len(reqs))
    p_lines, o_lines = max(1, per // 2 - 1), max(1, per - per // 2 - 2)

    def clip(s: str, k: int) -> str:
      out = []
      for para in (s or "").split("\n"):
        out += textwrap.wrap(para, width) or [""]
      if len(out) > k:
        out = out[:k]
        out[-1] = out[-1][:max(0, width - 4)] + " ..."
      return "\n".join(out)

    for prompt, output in reversed(reqs):  # newest first
      t.append("[Prompt]\n", style="bold grey70")
      t.append(clip(prompt, p_lines) + "\n", style="deep_sky_blue1")
      if output:
        t.append("[Response]\n", style="bold grey70")
        t.append(clip(output, o_lines) + "\n", style="white")
      t.append("\n")
    return t

  # ---------------------------------------------------------------- downloads panel
  def downloads_table(self) -> "Table":
    tab = Table(show_header=False, box=None, padding=(0, 1), expand=True)
    tab.add_column("what", style="cyan", no_wrap=True, ratio=50)
    tab.add_column("progress", style="cyan", no_wrap=True, ratio=40)
    tab.add_column("pct", style="cyan", no_wrap=True, ratio=10)
    mine = self.node_download_progress.get(self.node_id) if self.node_id else None
    if mine is not None:
      d = _prog(mine)
      tab.add_row(Text(f"Downloading {d['repo_id']}@{d['repo_revision']} ({d['completed_files']}/{d['total_files']} files)",
                       style="bold"))
      tab.add_row(f"{_fmt_bytes(d['downloaded_bytes'])} / {_fmt_bytes(d['total_bytes'])} "
                  f"({_fmt_bytes(d['overall_speed'])}/s)", f"ETA {_fmt_eta(d['overall_eta'])}")
      for name, f in d["file_progress"].items():
        if f.get("status") != "complete" and f.get("total"):
          frac = f.get("downloaded", 0) / f["total"]
          tab.add_row(Text(name[-40:], style="cyan"), _bar(frac), f"{100 * frac:.0f}%")
      tab.add_row("")
    others = [(nid, p) for nid, p in self.node_download_progress.items() if nid != self.node_id]
    if others:
      tab.add_row(Text("Other nodes:", style="bold"))
    for nid, p in others:
      d = _prog(p)
      caps = self.topology.get_node(nid)
      part = next((q for q in self.partitions if q.node_id == nid), None)
      dev = f"{nid[:16]} {caps.model if caps else 'unknown device'} {(caps.memory // 1024) if caps else '?'}GB"
      if part is not None:
        dev += f" [{part.start:.2f}-{part.end:.2f}]"
      tot = d["total_bytes"] or 0
      pct = 100.0 * d["downloaded_bytes"] / tot if tot else 0.0
      tab.add_row(dev, f"{d['repo_id']}@{d['repo_revision']} ({_fmt_bytes(d['overall_speed'])}/s, {d['status']})",
                  f"{pct:.1f}%")
      tab.add_row("", _bar(pct / 100.0), f"ETA {_fmt_eta(d['overall_eta'])}")
    return tab

  def _downloading(self) -> bool:
    return any(_prog(p)["status"] == "in_progress" for p in self.node_download_progress.values())

  # ---------------------------------------------------------------- layout
  def render(self):
    if not HAVE_RICH:
      return None
    width = (self.console.width if self.console is not None else 120) - 6
    n = len(self.topology.nodes) if hasattr(self.topology, "nodes") else len(list(self.topology.all_nodes()))
    panels = [Panel(self.cluster_text(), title=f"{n} Node Cluster", border_style="red1")]
    if any(p or o for p, o in self.requests.values()):
      panels.append(Panel(self.chat_text(max(20, width)), title="Chat", border_style="orange1"))
    if self._downloading():
      panels.append(Panel(self.downloads_table(), title="Download Progress", border_style="bright_white"))
    if self.live is None:
      return Group(*panels)
    lay = Layout()
    parts = [Layout(panels[0], name="main")]
    for p in panels[1:]:
      parts.append(Layout(p, size=CHAT_HEIGHT if p.title == "Chat" else 25))
    lay.split(*parts)
    return lay
