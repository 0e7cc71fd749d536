"""Server contract (reference: xotorch/networking/server.py:4-11)."""
from abc import ABC, abstractmethod


class Server(ABC):
  @abstractmethod
  async def start(self) -> None: ...

  @abstractmethod
  async def stop(self) -> None: ...
