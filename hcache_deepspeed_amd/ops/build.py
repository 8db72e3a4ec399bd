"""Ahead-of-time build of the native libraries (gfx950 HIP kernels + host C++ runtime).

Replaces the reference's JIT ``OpBuilder`` matrix (op_builder/builder.py:523-606, which hipifies
CUDA sources on ROCm, :745-757). Here there is one target (gfx950), sources are HIP written for
CDNA4, and everything is built in-tree into ``hcache_deepspeed_amd/_lib``:

* ``libhds_kernels.so`` -- every ``csrc/kernels/*.hip`` compiled by ``hipcc --offload-arch=gfx950``.
  The exported entry points are plain ``extern "C"`` launchers taking raw pointers and a
  ``hipStream_t``; python binds them with ctypes (ops/native.py), so no torch headers are in the
  device compile and a kernel rebuild takes seconds.
* ``libhds_host.so`` -- ``csrc/host/*.cpp`` (pinned ring buffers, CPU Adam/Lion/Adagrad with
  AVX-512/AVX2 clones, async file I/O thread pool) built with g++ against the HIP runtime.

Rebuilds are content-hash driven (sources + headers + flags), so ``build()`` is cheap when
nothing changed.
"""
import concurrent.futures as _cf
import hashlib
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_DIR = os.path.join(PKG_DIR, "_lib")
BUILD_DIR = os.path.join(os.path.dirname(PKG_DIR), "build", "hds")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("HDS_OFFLOAD_ARCH", "gfx950")

KERNEL_LIB = os.path.join(LIB_DIR, "libhds_kernels.so")
HOST_LIB = os.path.join(LIB_DIR, "libhds_host.so")

HIPCC_FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=fast",
               "-fno-gpu-rdc", "-Wno-unused-result"]
# per-source extra flags (part of the content hash). FlashAttention without SLP vectorization: hipcc otherwise packs
# adjacent scalar f32 muls / adds of the softmax into v_pk_mul_f32 / v_pk_add_f32, which cost MORE issue cycles than
# two scalar ops beside the MFMAs (MI355X_MICROARCH "price of one filler"): backward 4.10 -> 3.84 ms, headline
# 24,121 -> 24,440 tok/s on the same box (profiles/r3/fa_noslp_ab_r3p.txt)
FILE_FLAGS = {"flash_attn.hip": ["-fno-slp-vectorize"],
              # the one-wave-per-SIMD forward keeps S in VGPRs (builtin MFMAs, schedulable) and O in AGPRs (asm)
              "flash_attn_w64.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"],
              "flash_attn_bwd_w64.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"]}
HOST_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-fopenmp", "-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include",
              "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def _sources(sub, exts):
    d = os.path.join(CSRC, sub)
    if not os.path.isdir(d):
        return []
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(exts))


def _digest(paths, extra):
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    h.update(" ".join(extra).encode())
    return h.hexdigest()


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _stamp_ok(lib, digest):
    st = lib + ".sha256"
    return os.path.exists(lib) and os.path.exists(st) and open(st).read().strip() == digest


def build_kernels(force=False, jobs=None, verbose=False, file_flags=None, out=None):
    """``file_flags`` / ``out``: an A/B build with different per-source flags into another path (loaded with
    HDS_KERNEL_LIB=<out>); the default build uses FILE_FLAGS into _lib/libhds_kernels.so."""
    file_flags = FILE_FLAGS if file_flags is None else file_flags
    lib_path = out or KERNEL_LIB
    srcs = _sources("kernels", (".hip",))
    hdrs = _sources("kernels", (".h",))
    digest = _digest(srcs + hdrs, HIPCC_FLAGS + sorted(f"{k}:{' '.join(v)}" for k, v in file_flags.items()))
    if not force and _stamp_ok(lib_path, digest):
        return lib_path
    bdir = BUILD_DIR if out is None else BUILD_DIR + "_ab"
    os.makedirs(bdir, exist_ok=True)
    os.makedirs(os.path.dirname(lib_path), exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    objs = []

    def one(src):
        obj = os.path.join(bdir, os.path.basename(src) + ".o")
        extra = file_flags.get(os.path.basename(src), [])
        _run([hipcc, *HIPCC_FLAGS, *extra, "-I", os.path.join(CSRC, "kernels"), "-c", src, "-o", obj])
        return obj

    jobs = jobs or min(8, max(1, (os.cpu_count() or 4)))
    with _cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(one, srcs))
    tmp = lib_path + ".tmp"
    _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp,
          f"-Wl,-rpath,{ROCM}/lib"])
    # a kernel the host pass rejects silently (a device-only type held by a host-device lambda) leaves its launch
    # stub undefined: the shared object still links and only fails at dlopen on the GPU box -- refuse it here
    nm = subprocess.run(["nm", "-u", tmp], capture_output=True, text=True)
    missing = [ln.split()[-1] for ln in nm.stdout.splitlines() if "__device_stub__" in ln]
    if missing:
        os.remove(tmp)
        raise RuntimeError(f"kernel library leaves launch stubs undefined: {missing[:4]}")
    os.replace(tmp, lib_path)
    with open(lib_path + ".sha256", "w") as f:
        f.write(digest)
    if verbose:
        print(f"[hds build] {lib_path} ({len(srcs)} kernel sources)", file=sys.stderr)
    return lib_path


DIAG_LIB = os.path.join(os.path.dirname(KERNEL_LIB), "libhds_kernels_diag.so")


def build_kernels_diag(force=False, jobs=None, verbose=False):
    """The A/B experiment library: the FlashAttention units built with -DHDS_FA_DIAG=1 (earlier forward schedules,
    cycle-stamp builds, timing-only diagnostics with WRONG results) into ``_lib/libhds_kernels_diag.so``. Never the
    library the package loads by default; tools load it with HDS_KERNEL_LIB=<path> (tools/fa_stamps.py)."""
    flags = {k: list(v) for k, v in FILE_FLAGS.items()}
    for f in ("flash_attn.hip", "flash_attn_w64.hip", "flash_attn_bwd_w64.hip"):
        flags[f] = flags.get(f, []) + ["-DHDS_FA_DIAG=1"]
    return build_kernels(force=force, jobs=jobs, verbose=verbose, file_flags=flags, out=DIAG_LIB)


def build_host(force=False, verbose=False):
    srcs = _sources("host", (".cpp",))
    hdrs = _sources("host", (".h",))
    if not srcs:
        return None
    digest = _digest(srcs + hdrs, HOST_FLAGS)
    if not force and _stamp_ok(HOST_LIB, digest):
        return HOST_LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = HOST_LIB + ".tmp"
    _run(["g++", *HOST_FLAGS, "-shared", *srcs, "-o", tmp, f"-L{ROCM}/lib", "-lamdhip64",
          f"-Wl,-rpath,{ROCM}/lib", "-lpthread", "-ldl"])
    os.replace(tmp, HOST_LIB)
    with open(HOST_LIB + ".sha256", "w") as f:
        f.write(digest)
    if verbose:
        print(f"[hds build] {HOST_LIB}", file=sys.stderr)
    return HOST_LIB


def build_all(force=False, verbose=True):
    k = build_kernels(force=force, verbose=verbose)
    h = build_host(force=force, verbose=verbose)
    return k, h


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
