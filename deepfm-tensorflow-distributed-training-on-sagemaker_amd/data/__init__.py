"""Input pipeline: TFRecord / tf.train.Example / libsvm I/O, shard policy, synthetic data."""
