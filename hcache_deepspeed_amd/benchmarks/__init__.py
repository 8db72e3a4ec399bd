"""Benchmarks shipped with the framework (``ds_bench``)."""
