"""Terminal topology view (reference: xotorch/viz/topology_viz.py:20-379).

rich Live layout: the ring of peers (red = active, green = this node, blue = others) with model /
memory / TFLOPS / layer range per peer, a "GPU poor <-> GPU rich" bar from the summed fp16 TFLOPS,
recent prompts and answers, and a download-progress table.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Optional

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


class TopologyViz:
  def __init__(self, chatgpt_api_endpoints: List[str] = (), web_chat_urls: List[str] = (), start: bool = True):
    self.chatgpt_api_endpoints = list(chatgpt_api_endpoints)
    self.web_chat_urls = list(web_chat_urls)
    self.topology = Topology()
    self.partitions: List[Partition] = []
    self.node_id: Optional[str] = None
    self.node_download_progress: Dict[str, dict] = {}
    self.requests: "OrderedDict[str, list]" = OrderedDict()
    self.live = None
    if HAVE_RICH and start:
      self.console = Console()
      self.live = Live(self.render(), console=self.console, refresh_per_second=4, auto_refresh=False)
      self.live.start()

  # ---------------------------------------------------------------- updates
  def update_visualization(self, topology: Topology, partitions: List[Partition], node_id: Optional[str] = None,
                           node_download_progress: Optional[Dict[str, dict]] = None):
    self.topology = topology
    self.partitions = partitions
    self.node_id = node_id
    if node_download_progress:
      self.node_download_progress = node_download_progress
    self.refresh()

  def update_prompt(self, request_id: str, prompt: Optional[str] = None):
    self.requests.setdefault(request_id, [prompt or "", ""])
    if prompt is not None:
      self.requests[request_id][0] = prompt
    while len(self.requests) > 3:
      self.requests.popitem(last=False)
    self.refresh()

  def update_prompt_output(self, request_id: str, output: Optional[str] = None):
    if request_id in self.requests and output:
      self.requests[request_id][1] += output
      self.refresh()

  def refresh(self):
    if self.live is not None:
      self.live.update(self.render(), refresh=True)

  # ---------------------------------------------------------------- rendering
  def total_tflops(self) -> float:
    return sum(c.flops.fp16 for _, c in self.topology.all_nodes())

  def ring_text(self) -> "Text":
    t = Text()
    t.append(f"xot v{VERSION} — MI355X ring\n", style="bold")
    tf = self.total_tflops()
    frac = math.tanh(tf / 4000.0)
    width = 30
    fill = int(frac * width)
    t.append("GPU poor ", style="red")
    t.append("█" * fill, style="yellow")
    t.append("░" * (width - fill))
    t.append(f" GPU rich  ({tf:.0f} fp16 TFLOPS)\n\n")
    for i, p in enumerate(self.partitions):
      caps = self.topology.get_node(p.node_id)
      style = "red" if p.node_id == self.topology.active_node_id else ("green" if p.node_id == self.node_id else "blue")
      mem = f"{caps.memory / 1024:.0f}GB" if caps else "?"
      chip = caps.chip if caps else "?"
      t.append(f"  [{i}] ", style=style)
      t.append(f"{p.node_id[:24]:24s} {chip:22s} {mem:>7s} [{p.start:.3f}, {p.end:.3f})\n", style=style)
      if i < len(self.partitions) - 1:
        t.append("       │\n")
    if self.partitions:
      t.append("       └──► back to [0]\n")
    for url in self.web_chat_urls:
      t.append(f"\nWeb chat: {url}")
    for url in self.chatgpt_api_endpoints:
      t.append(f"\nChatGPT API: {url}")
    return t

  def prompts_table(self) -> "Table":
    tab = Table(title="Recent requests", expand=True)
    tab.add_column("prompt")
    tab.add_column("response")
    for rid, (p, o) in self.requests.items():
      tab.add_row(p[-200:], o[-400:])
    return tab

  def downloads_table(self) -> "Table":
    tab = Table(title="Downloads", expand=True)
    tab.add_column("node")
    tab.add_column("repo")
    tab.add_column("progress")
    for nid, prog in self.node_download_progress.items():
      if not isinstance(prog, dict):
        prog = prog.to_dict()
      tot = prog.get("total_bytes") or 0
      done = prog.get("downloaded_bytes") or 0
      pct = 100 * done / tot if tot else 0
      tab.add_row(nid[:16], str(prog.get("repo_id")), f"{pct:5.1f}% ({prog.get('status')})")
    return tab

  def render(self):
    if not HAVE_RICH:
      return None
    parts = [Panel(self.ring_text(), title="Topology")]
    if self.requests:
      parts.append(self.prompts_table())
    if self.node_download_progress:
      parts.append(self.downloads_table())
    return Group(*parts)
