"""Launcher CLI (``bin/hds`` / ``bin/deepspeed``): runner.py -> launch.py (per node) -> one process per GPU."""
