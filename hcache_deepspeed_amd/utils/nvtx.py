"""Range markers for profilers (reference utils/nvtx.py ``instrument_w_nvtx`` :12-25).

On ROCm ``torch.cuda.nvtx.range_push/pop`` emit roctx ranges, which ``rocprofv3 --marker-trace`` records next to
the kernel trace. Ranges are skipped while torch.compile is tracing (as in the reference).
"""
import functools

import torch

enable_nvtx = True


def _push(name):
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)
            return True
        except Exception:  # roctx not available in this build
            return False
    return False


def _pop():
    try:
        torch.cuda.nvtx.range_pop()
    except Exception:
        pass


def _compiling():
    try:
        return torch.compiler.is_compiling()
    except Exception:
        return False


def instrument_w_nvtx(func):
    """Decorator: wrap ``func`` in a roctx range named after its qualified name."""

    @functools.wraps(func)
    def wrapped(*args, **kwargs):
        if not enable_nvtx or _compiling():
            return func(*args, **kwargs)
        pushed = _push(func.__qualname__)
        try:
            return func(*args, **kwargs)
        finally:
            if pushed:
                _pop()

    return wrapped


class range_ctx:
    """``with range_ctx("name"):`` -- context-manager form of the same marker."""

    def __init__(self, name):
        self.name = name
        self.pushed = False

    def __enter__(self):
        self.pushed = enable_nvtx and not _compiling() and _push(self.name)
        return self

    def __exit__(self, *exc):
        if self.pushed:
            _pop()
        return False
