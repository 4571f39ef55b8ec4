"""Domain decomposition, in-process ranks and torch.distributed/RCCL transports."""
from .decomposition import PyDecomposition, split_range
from .inprocess import InProcessGroup

__all__ = ["PyDecomposition", "split_range", "InProcessGroup"]
