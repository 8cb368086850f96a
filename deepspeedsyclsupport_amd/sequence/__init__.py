from .layer import DistributedAttention, UlyssesAttention, single_all_to_all, shard_sequence  # noqa: F401
