"""Distribution: RCCL data parallelism, row-sharded embeddings, input shard policy, launcher."""
