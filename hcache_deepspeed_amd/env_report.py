"""``ds_report``: environment and native-op status.

Reference parity: deepspeed/env_report.py (``op_report`` :30, ``debug_report``, ``cli_main``). The
reference lists every JIT op builder and whether it is compatible/installed; here every native library
and each exported kernel symbol group is listed with its build state (in-tree ``_lib/*.so``, gfx950),
plus the ROCm / HIP / RCCL / torch stack and the visible MI355X devices.
"""
import argparse
import os
import shutil
import subprocess

GREEN, RED, YELLOW, END = "\033[92m", "\033[91m", "\033[93m", "\033[0m"
OKAY, FAIL, WARN = f"{GREEN}[OKAY]{END}", f"{RED}[FAIL]{END}", f"{YELLOW}[WARNING]{END}"

# op name -> (library, representative exported symbol)
OPS = {
    "fused_adam": ("kernels", "hds_adam_multi"),
    "fused_lion": ("kernels", "hds_lion_flat"),
    "fused_lamb": ("kernels", "hds_lamb_multi"),
    "fused_adagrad": ("kernels", "hds_adagrad_flat"),
    "rms_norm / layer_norm": ("kernels", "hds_norm_fwd"),
    "rotary_embedding": ("kernels", "hds_rope"),
    "gated_activations": ("kernels", "hds_glu_fwd"),
    "bias_activations": ("kernels", "hds_bias_act_fwd"),
    "flash_attention (fwd/bwd)": ("kernels", "hds_attn_fwd"),
    "cross_entropy": ("kernels", "hds_xent"),
    "paged_attention (ragged)": ("kernels", "hds_paged_attn"),
    "kv_rotary_scatter (HCache restore)": ("kernels", "hds_kv_rope_scatter"),
    "moe_scatter / moe_gather": ("kernels", "hds_moe_dispatch"),
    "quantizer (int8/int4)": ("kernels", "hds_quant_int"),
    "fp_quantizer (fp8)": ("kernels", "hds_quant_fp8"),
    "cpu_adam / cpu_lion / cpu_adagrad": ("host", "hds_cpu_adam"),
    "async_io": ("host", "hds_aio_create"),
    "pinned_host_ring": ("host", "hds_ring_create"),
}


def _lib_status():
    from .ops import native
    out = {}
    for name, loader in (("kernels", native.load_kernels), ("host", native.host_lib)):
        try:
            out[name] = loader()
        except Exception as e:  # noqa: BLE001
            out[name] = e
    return out


def op_report(verbose=True):
    libs = _lib_status()
    width = max(len(k) for k in OPS) + 2
    print("-" * 70)
    print("Native ops (hand-written HIP for gfx950 / host C++), built in-tree by __graft_entry__.build()")
    print("-" * 70)
    print(f"{'op name':<{width}} {'library':<10} built")
    for op, (lib, sym) in OPS.items():
        h = libs.get(lib)
        ok = h is not None and not isinstance(h, Exception) and hasattr(h, sym)
        print(f"{op:<{width}} {lib:<10} {OKAY if ok else FAIL}")
    for lib, h in libs.items():
        if isinstance(h, Exception) or h is None:
            print(f"{WARN} lib{lib}: {h}")


def _cmd(args):
    try:
        return subprocess.check_output(args, stderr=subprocess.STDOUT, timeout=20).decode().strip()
    except Exception:  # noqa: BLE001
        return None


def debug_report():
    import torch
    from .version import __version__
    rows = [("torch install path", os.path.dirname(torch.__file__)), ("torch version", torch.__version__),
            ("hcache_deepspeed_amd version", __version__),
            ("hcache_deepspeed_amd install path", os.path.dirname(os.path.abspath(__file__))),
            ("torch hip version", getattr(torch.version, "hip", None)),
            ("rocm path", os.environ.get("ROCM_PATH", "/opt/rocm")),
            ("hipcc", shutil.which("hipcc") or "not found")]
    rocm_ver = None
    for p in ("/opt/rocm/.info/version", "/opt/rocm/.info/version-dev"):
        if os.path.isfile(p):
            rocm_ver = open(p).read().strip()
            break
    rows.append(("rocm version", rocm_ver))
    try:
        import torch.distributed as tdist
        rows.append(("rccl (nccl backend) available", tdist.is_nccl_available()))
        if tdist.is_nccl_available():
            rows.append(("rccl version", ".".join(str(v) for v in torch.cuda.nccl.version())))
    except Exception:  # noqa: BLE001
        pass
    rows.append(("HSA_ENABLE_IPC_MODE_LEGACY", os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")))
    try:
        n = torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        n = 0
    rows.append(("visible GPUs", n))
    if n and torch.cuda.is_available():
        p = torch.cuda.get_device_properties(0)
        rows.append(("device 0", f"{p.name} {getattr(p, 'gcnArchName', '')} {p.total_memory / 2**30:.0f} GiB "
                                 f"{p.multi_processor_count} CUs"))
    print("-" * 70)
    print("General environment info:")
    for k, v in rows:
        print(f"{k:<38} {v}")


def cli_main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--hide_operator_status", action="store_true")
    ap.add_argument("--hide_errors_and_warnings", action="store_true")
    a = ap.parse_args(argv)
    if not a.hide_operator_status:
        op_report(verbose=not a.hide_errors_and_warnings)
    debug_report()


def main():
    cli_main()


if __name__ == "__main__":
    main()
