"""``deepspeed.runtime.compiler`` (reference runtime/compiler.py): torch.compile availability checks.

The MI355X hot path does not depend on a tracing compiler (HIP kernels + HIP graphs); these helpers only
report whether a user model can additionally be wrapped by ``engine.compile()``."""
import torch


def is_compile_supported():
    return hasattr(torch, "compile") and hasattr(torch, "compiler")


def disable(func):
    return torch.compiler.disable(func) if is_compile_supported() else func


def is_compiling():
    return bool(is_compile_supported() and torch.compiler.is_compiling())
