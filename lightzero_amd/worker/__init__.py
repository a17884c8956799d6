"""lzero.worker drop-ins: MuZeroCollector over the GPU search (lightzero_amd.worker.muzero_collector)."""
from .muzero_collector import MuZeroCollector

__all__ = ["MuZeroCollector"]
