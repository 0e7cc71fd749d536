"""Download progress events (reference: xotorch/download/download_progress.py); same dict shapes, which
the API's /v1/download/progress and the topology TUI consume."""
from __future__ import annotations

from dataclasses import dataclass, field
from datetime import timedelta
from typing import Dict, Literal

from ..inference.shard import Shard

Status = Literal["not_started", "in_progress", "complete"]


@dataclass
class RepoFileProgressEvent:
  repo_id: str
  repo_revision: str
  file_path: str
  downloaded: int
  downloaded_this_session: int
  total: int
  speed: float
  eta: timedelta
  status: Status
  start_time: float

  def to_dict(self) -> dict:
    d = dict(self.__dict__)
    d["eta"] = self.eta.total_seconds()
    return d

  @classmethod
  def from_dict(cls, d: dict) -> "RepoFileProgressEvent":
    d = dict(d)
    d["eta"] = timedelta(seconds=d.get("eta", 0))
    return cls(**d)


@dataclass
class RepoProgressEvent:
  shard: Shard
  repo_id: str
  repo_revision: str
  completed_files: int
  total_files: int
  downloaded_bytes: int
  downloaded_bytes_this_session: int
  total_bytes: int
  overall_speed: float
  overall_eta: timedelta
  file_progress: Dict[str, RepoFileProgressEvent] = field(default_factory=dict)
  status: Status = "not_started"

  def to_dict(self) -> dict:
    return {"shard": self.shard.to_dict(), "repo_id": self.repo_id, "repo_revision": self.repo_revision,
            "completed_files": self.completed_files, "total_files": self.total_files,
            "downloaded_bytes": self.downloaded_bytes, "downloaded_bytes_this_session": self.downloaded_bytes_this_session,
            "total_bytes": self.total_bytes, "overall_speed": self.overall_speed,
            "overall_eta": self.overall_eta.total_seconds(),
            "file_progress": {k: v.to_dict() for k, v in self.file_progress.items()}, "status": self.status}

  @classmethod
  def from_dict(cls, d: dict) -> "RepoProgressEvent":
    d = dict(d)
    d["overall_eta"] = timedelta(seconds=d.get("overall_eta", 0))
    d["file_progress"] = {k: RepoFileProgressEvent.from_dict(v) for k, v in d.get("file_progress", {}).items()}
    d["shard"] = Shard.from_dict(d["shard"])
    return cls(**d)
