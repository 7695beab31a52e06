"""Process entrypoints: ``harness`` (trial container), ``worker_process`` (one per slot),
``gc_checkpoints`` (checkpoint GC job)."""
