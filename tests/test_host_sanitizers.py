"""Host C++ runtime under AddressSanitizer + UndefinedBehaviorSanitizer (the reference has no
sanitizer integration; the plan asks for ASAN builds of the host libraries). Builds tests/native/host_selftest.cpp
together with csrc/host/{cpu_optim,aio,shm_comm}.cpp with g++ -fsanitize=address,undefined and runs it (CPU only)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "hcache_deepspeed_amd", "csrc", "host")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_runtime_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_selftest")
    srcs = [os.path.join(ROOT, "tests", "native", "host_selftest.cpp")] + \
        [os.path.join(HOST, f) for f in ("cpu_optim.cpp", "aio.cpp", "shm_comm.cpp")]
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fopenmp", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=undefined", *srcs, "-o", exe, "-lpthread", "-lrt"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1", OMP_NUM_THREADS="4")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "host selftest ok" in r.stdout
