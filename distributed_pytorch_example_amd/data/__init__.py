from .sampler import DistributedSampler
from .synthetic import SyntheticDataset, SyntheticTokens, DeviceLoader
from .loader import create_data_loader

__all__ = ["DistributedSampler", "SyntheticDataset", "SyntheticTokens", "DeviceLoader", "create_data_loader"]
