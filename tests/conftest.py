import os
import sys

# the GPU tests spill activations: the blit workgroup limit must reach the HIP runtime, i.e. be in the environment
# before any test module imports torch (hcache_deepspeed_amd.offload.activation_cache.check_blit_limit)
os.environ.setdefault("DEBUG_CLR_LIMIT_BLIT_WG", "16")

import pytest  # noqa: E402

if "MASTER_PORT" not in os.environ or (os.environ.get("PYTEST_XDIST_WORKER")
                                       and os.environ.get("HDS_TEST_PORT_OWNER") != os.environ["PYTEST_XDIST_WORKER"]):
    # tests that initialise torch.distributed in-process (ds.initialize on one rank) would all take the default
    # port 29500 -- or the port the xdist controller picked and its workers inherited -- and collide across
    # pytest-xdist workers: every worker process gets a free port of its own
    import socket

    os.environ["HDS_TEST_PORT_OWNER"] = os.environ.get("PYTEST_XDIST_WORKER", "")

    with socket.socket() as _s:
        _s.bind(("127.0.0.1", 0))
        os.environ["MASTER_PORT"] = str(_s.getsockname()[1])

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
