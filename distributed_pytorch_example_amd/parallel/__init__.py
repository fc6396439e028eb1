from .ddp import DDP, DistributedDataParallel
from .buckets import assign_buckets
from . import dist
from . import hooks

__all__ = ["DDP", "DistributedDataParallel", "assign_buckets", "dist", "hooks"]
