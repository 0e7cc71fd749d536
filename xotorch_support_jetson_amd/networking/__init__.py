from .discovery import Discovery
from .peer_handle import PeerHandle
from .server import Server

__all__ = ["Discovery", "PeerHandle", "Server"]
