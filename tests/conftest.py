import os
import sys

# the GPU tests spill activations: the blit workgroup limit must reach the HIP runtime, i.e. be in the environment
# before any test module imports torch (hcache_deepspeed_amd.offload.activation_cache.check_blit_limit)
os.environ.setdefault("DEBUG_CLR_LIMIT_BLIT_WG", "16")

import pytest  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels, RCCL)")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "world_size(n): distributed test world size")


@pytest.fixture
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
