"""NVMe / file-tier I/O benchmarking and tuning (reference deepspeed/nvme: ds_io, ds_nvme_tune)."""
from .ds_io import main as ds_io_main, run_io  # noqa: F401
from .tune import main as ds_nvme_tune_main, sweep  # noqa: F401
