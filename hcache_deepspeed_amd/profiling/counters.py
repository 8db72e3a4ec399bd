"""Flop reporting hook for ops whose work is invisible to the aten dispatcher (hand-written HIP kernels
called through ctypes: flash attention, fused norms, gated activations, fused cross-entropy).

Ops call ``add(flops, macs)``; it is a no-op unless a FlopsProfiler is running."""
_ACTIVE = []


def active():
    return bool(_ACTIVE)


def push(prof):
    _ACTIVE.append(prof)


def pop(prof):
    if prof in _ACTIVE:
        _ACTIVE.remove(prof)


def add(flops, macs=0, name=None):
    for prof in _ACTIVE:
        prof._add(int(flops), int(macs), name)
