"""Device -> pinned-host copies for the activation spills (csrc/kernels/hostcopy.hip).

``d2h_(dst_host, src_dev)`` copies on the CURRENT stream. Default (``HDS_D2H_WG=0``): ``copy_``, i.e. the runtime's
blit kernel, with its workgroup count limited by ``DEBUG_CLR_LIMIT_BLIT_WG`` (in the environment before torch loads
HIP: bench.py, the launcher; package ``__init__``).
``HDS_D2H_WG=n`` runs the own n-workgroup kernel instead (csrc/kernels/hostcopy.hip). Measured in situ (32k plan,
profiles/r4/copy_engine_ab_r4f.txt) the own kernel cost the overlapped forward ~14 ms per spilled GB against
~0.01-0.06 for the limited runtime blit at 8-32 workgroups, so it is not the default.
"""
import os

from . import native

D2H_WG = int(os.environ.get("HDS_D2H_WG", "0"))


def d2h_(dst, src, n_wg=None):
    """dst (pinned host, contiguous) <- src (device, contiguous), asynchronous on the current stream."""
    wg = D2H_WG if n_wg is None else int(n_wg)
    nbytes = src.numel() * src.element_size()
    if (wg <= 0 or not src.is_cuda or dst.is_cuda or not src.is_contiguous() or not dst.is_contiguous()
            or dst.numel() * dst.element_size() < nbytes or src.data_ptr() % 16 or dst.data_ptr() % 16):
        dst.view(-1)[:src.numel()].copy_(src.view(-1), non_blocking=True) if dst.dtype == src.dtype else \
            dst.copy_(src, non_blocking=True)
        return dst
    native.check(native.kernels().hds_copy_d2h(dst.data_ptr(), src.data_ptr(), nbytes, wg, native.stream()),
                 "copy_d2h")
    return dst
