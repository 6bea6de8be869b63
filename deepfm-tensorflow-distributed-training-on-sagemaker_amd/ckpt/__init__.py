"""Checkpointing: native per-rank checkpoints with auto-resume, TF tensor_bundle interop,
servable export."""
