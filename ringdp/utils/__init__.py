"""ringdp.utils - hipGraph step capture, timing, tracing, checkpointing helpers."""
