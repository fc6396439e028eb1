from .ddp import DDP, DistributedDataParallel
from .buckets import assign_buckets
from . import dist

__all__ = ["DDP", "DistributedDataParallel", "assign_buckets", "dist"]
