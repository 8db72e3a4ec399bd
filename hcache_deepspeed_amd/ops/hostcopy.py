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


def latent_slot_store(src, ring, slot, layer):
    """ring[slot, layer] <- src rows (inside a captured decode graph: ``slot`` is a device int32 read by the kernel, so
    every replay stores into the slot the ring has advanced to). ``src``: [rows, W] with contiguous rows (any row
    stride); ``ring``: [S, L, rows, W] contiguous, same dtype. CPU tensors: a plain indexed copy."""
    rows, W = src.shape
    assert ring.dim() == 4 and ring.shape[2] == rows and ring.shape[3] == W and ring.dtype == src.dtype
    assert src.stride(1) == 1 and ring.is_contiguous()
    if not src.is_cuda:
        ring[int(slot.item()), layer].copy_(src)
        return
    es = src.element_size()
    dst = ring[0, layer]
    native.check(native.kernels().hds_latent_slot_store(src.data_ptr(), src.stride(0) * es, dst.data_ptr(),
                                                        slot.data_ptr(), ring.stride(0) * es, rows, W * es,
                                                        native.stream()), "latent_slot_store")


def slot_advance(slot, mod):
    """slot <- (slot + 1) % mod on the device (the last kernel of a captured decode step)."""
    if not slot.is_cuda:
        slot.fill_((int(slot.item()) + 1) % mod)
        return
    native.check(native.kernels().hds_slot_advance(slot.data_ptr(), int(mod), native.stream()), "slot_advance")
