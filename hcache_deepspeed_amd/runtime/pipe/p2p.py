"""Point-to-point transfers between adjacent pipeline stages.

Reference parity: runtime/pipe/p2p.py (``send``/``recv`` :46-85 with a 2-rank broadcast fallback) and
pipe/engine.py ``_send_tensor_meta``/``_recv_tensor_meta`` (:929-1040). Here every step's transfers go
out as ONE ``batch_isend_irecv`` (an RCCL group: the send to stage s+1 and the receive from stage s+1
use the two directions of the same xGMI link concurrently). Tensor metadata (count, dtypes, shapes) is
exchanged once per (direction, shape-change) as a fixed 64-int header so receivers can pre-allocate.
"""
import torch
import torch.distributed as tdist

_DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.bool, torch.uint8,
           torch.float64, torch.int8]
_META_LEN = 64


def _encode_meta(tensors):
    meta = [len(tensors)]
    for t in tensors:
        meta += [_DTYPES.index(t.dtype), int(t.requires_grad or t.is_floating_point()), t.dim()] + list(t.shape)
    assert len(meta) <= _META_LEN, "too many / too high-rank tensors for the pipeline meta header"
    return torch.tensor(meta + [0] * (_META_LEN - len(meta)), dtype=torch.int64)


def _decode_meta(buf):
    m = buf.tolist()
    n, i, out = m[0], 1, []
    for _ in range(n):
        dt, grad, nd = m[i], m[i + 1], m[i + 2]
        shape = tuple(m[i + 3:i + 3 + nd])
        out.append((_DTYPES[dt], bool(grad), shape))
        i += 3 + nd
    return out


def _meta_device(device):
    # RCCL needs device tensors; gloo takes host tensors
    return device if tdist.get_backend() == "nccl" else torch.device("cpu")


def send_meta(tensors, dst, device):
    buf = _encode_meta(tensors).to(_meta_device(device))
    tdist.send(buf, dst)


def recv_meta(src, device):
    buf = torch.empty(_META_LEN, dtype=torch.int64, device=_meta_device(device))
    tdist.recv(buf, src)
    return _decode_meta(buf.cpu())


def alloc_from_meta(meta, device):
    return [torch.empty(shape, dtype=dt, device=device) for dt, _, shape in meta]


def batch_p2p(ops):
    """ops: list of ("send"|"recv", tensor, peer). Issues them as one group and waits."""
    if not ops:
        return
    if tdist.get_backend() == "gloo":
        # gloo: plain async isend/irecv (no coalescing manager needed)
        works = [(tdist.isend if kind == "send" else tdist.irecv)(t.contiguous() if kind == "send" else t, peer)
                 for kind, t, peer in ops]
        for w in works:
            w.wait()
        return
    p2p = [tdist.P2POp(tdist.isend if kind == "send" else tdist.irecv, t, peer) for kind, t, peer in ops]
    for w in tdist.batch_isend_irecv(p2p):
        w.wait()


def can_send_recv():
    return True
