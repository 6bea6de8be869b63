"""DeepFM model family: golden PyTorch reference and the native MI355X executor."""
