"""Profiling: flops profiler (module-level MACs/flops/latency) and the custom-op flop hook."""
