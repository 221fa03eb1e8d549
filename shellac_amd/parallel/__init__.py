"""Sharding (consistent-hash rings) and collectives (RCCL/gloo) for the cache."""
from .ring import ShardRing
from .exchange import all_to_all_rows, allreduce_stats, dist_info, exchange_counts

__all__ = ["ShardRing", "all_to_all_rows", "allreduce_stats", "dist_info", "exchange_counts"]
