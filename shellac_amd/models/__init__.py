"""Cache "models": the sharded HBM cache served over torch.distributed + workloads."""
from .sharded_cache import GetResult, SetBatch, ShardedCache

__all__ = ["GetResult", "SetBatch", "ShardedCache"]
