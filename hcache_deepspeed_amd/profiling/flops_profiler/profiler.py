"""Flops profiler: per-module parameters, MACs, flops and forward latency.

Reference parity: profiling/flops_profiler/profiler.py (``FlopsProfiler`` :30-510 with
``start_profile``/``stop_profile``/``reset_profile``/``end_profile``, ``get_total_flops/macs/duration/
params``, ``print_model_profile`` :286, ``print_model_aggregated_profile`` :452, ``get_model_profile``
:1195, the number formatters). The reference monkey-patches ~34 ``torch.nn.functional`` / tensor
methods; here GEMM/conv/SDPA flops are counted at the aten dispatch level (``TorchDispatchMode`` with
torch's own flop formulas, so every matmul path is seen, including the ones inside autograd Functions),
and the framework's HIP kernels report their flops through :mod:`hcache_deepspeed_amd.profiling.counters`.
"""
import sys
import time
from collections import OrderedDict

import torch
import torch.nn as nn
from torch.utils._python_dispatch import TorchDispatchMode
from torch.utils.flop_counter import flop_registry

from .. import counters

DEFAULT_PRECISION = 2
aten = torch.ops.aten

# pointwise / normalisation ops counted as numel (x k) flops, no MACs
_POINTWISE = {
    aten.add: 1, aten.sub: 1, aten.mul: 1, aten.div: 1, aten.relu: 1, aten.gelu: 8, aten.silu: 5, aten.sigmoid: 4,
    aten.tanh: 4, aten.exp: 1, aten._softmax: 5, aten.native_layer_norm: 5, aten.native_dropout: 1,
    aten.rsqrt: 1, aten.pow: 1,
}


class _DispatchCounter(TorchDispatchMode):

    def __init__(self, prof):
        super().__init__()
        self.prof = prof

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        pkt = func._overloadpacket
        try:
            if pkt in flop_registry:
                f = flop_registry[pkt](*args, **kwargs, out_val=out)
                self.prof._add(f, f // 2, pkt.__name__)
            elif pkt in _POINTWISE and isinstance(out, torch.Tensor):
                self.prof._add(_POINTWISE[pkt] * out.numel(), 0, pkt.__name__)
        except Exception:  # noqa: BLE001  (a formula that cannot handle an exotic call never breaks the run)
            pass
        return out


class FlopsProfiler:
    """Measures the forward pass of ``model`` between ``start_profile()`` and ``stop_profile()``."""

    def __init__(self, model, ds_engine=None, recompute_fwd_factor=0.0):
        self.model = model
        self.ds_engine = ds_engine
        self.recompute_fwd_factor = recompute_fwd_factor
        self.started = False
        self.func_patched = False
        self._hooks = []
        self._stack = []
        self._mode = None
        self._t0 = None

    # ---------------------------------------------------------------------------------
    def _add(self, flops, macs, name=None):
        for m in self._stack:
            m.__flops__ += flops
            m.__macs__ += macs
        if not self._stack:
            self.model.__flops__ += flops
            self.model.__macs__ += macs

    def _sync(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def start_profile(self, ignore_list=None):
        self.reset_profile()
        ignore = tuple(ignore_list or ())

        def pre(mod, inp):
            self._stack.append(mod)
            self._sync()
            mod.__start_time__ = time.perf_counter()

        def post(mod, inp, out):
            self._sync()
            mod.__duration__ += time.perf_counter() - mod.__start_time__
            if self._stack and self._stack[-1] is mod:
                self._stack.pop()

        for m in self.model.modules():
            if ignore and isinstance(m, ignore):
                continue
            self._hooks.append(m.register_forward_pre_hook(pre))
            self._hooks.append(m.register_forward_hook(post))
        self._mode = _DispatchCounter(self)
        self._mode.__enter__()
        counters.push(self)
        self.started = True
        self.func_patched = True

    def stop_profile(self):
        if self.started and self._mode is not None:
            self._mode.__exit__(None, None, None)
            self._mode = None
            counters.pop(self)
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.started = False
        self.func_patched = False

    def reset_profile(self):
        for m in self.model.modules():
            m.__flops__ = 0
            m.__macs__ = 0
            m.__duration__ = 0.0
            m.__params__ = sum(p.numel() if p.numel() else getattr(p, "ds_numel", 0)
                               for p in m.parameters(recurse=False))
            m.__start_time__ = 0.0

    def end_profile(self):
        self.stop_profile()
        for m in self.model.modules():
            for a in ("__flops__", "__macs__", "__duration__", "__params__", "__start_time__"):
                if hasattr(m, a):
                    delattr(m, a)

    # ---------------------------------------------------------------------------------
    def _tree_params(self, m):
        return sum(getattr(c, "__params__", 0) for c in m.modules())

    def get_total_flops(self, as_string=False):
        f = self.model.__flops__
        return flops_to_string(f) if as_string else f

    def get_total_macs(self, as_string=False):
        m = self.model.__macs__
        return macs_to_string(m) if as_string else m

    def get_total_duration(self, as_string=False):
        d = self.model.__duration__
        return duration_to_string(d) if as_string else d

    def get_total_params(self, as_string=False):
        p = self._tree_params(self.model)
        return params_to_string(p) if as_string else p

    def is_expert_tensor_parallelism_enabled(self):
        return False

    # ---------------------------------------------------------------------------------
    def print_model_profile(self, profile_step=1, module_depth=-1, top_modules=1, detailed=True, output_file=None):
        out = open(output_file, "w") if output_file else sys.stdout
        try:
            total_flops, total_macs = self.get_total_flops(), self.get_total_macs()
            total_dur, total_params = self.get_total_duration(), self.get_total_params()
            fwd_factor = 3 + self.recompute_fwd_factor  # fwd + 2x bwd (+ recompute)
            lines = ["", "-------------------------- Flops Profiler --------------------------",
                     f"Profile Summary at step {profile_step}:"]
            if self.ds_engine is not None:
                e = self.ds_engine
                lines += [f"{'world size:':<60}{getattr(e, 'dp_world_size', 1)}",
                          f"{'batch size per GPU:':<60}{e.train_micro_batch_size_per_gpu()}"]
            lines += [f"{'params per GPU:':<60}{params_to_string(total_params)}",
                      f"{'fwd MACs per GPU:':<60}{macs_to_string(total_macs)}",
                      f"{'fwd flops per GPU:':<60}{number_to_string(total_flops)}",
                      f"{'fwd+bwd flops per GPU (x{}):'.format(fwd_factor):<60}"
                      f"{number_to_string(total_flops * fwd_factor)}",
                      f"{'fwd latency:':<60}{duration_to_string(total_dur)}",
                      f"{'fwd FLOPS per GPU = fwd flops per GPU / fwd latency:':<60}"
                      f"{flops_to_string(total_flops / total_dur if total_dur else 0)}"]
            print("\n".join(lines), file=out)
            self.print_model_aggregated_profile(module_depth, top_modules, file=out)
            if detailed:
                print("\n------------------------------ Detailed Profile per module "
                      "------------------------------", file=out)
                print("Each module: params, MACs, fwd latency, percentage of total", file=out)
                self._print_tree(self.model, "", 0, module_depth, total_flops, total_dur, out)
            print("-" * 68, file=out)
        finally:
            if output_file:
                out.close()

    def _print_tree(self, m, name, depth, max_depth, total_flops, total_dur, out):
        if max_depth >= 0 and depth > max_depth:
            return
        pct = 100.0 * m.__flops__ / total_flops if total_flops else 0.0
        print(f"{'  ' * depth}{name or type(m).__name__} ({type(m).__name__}): "
              f"{params_to_string(self._tree_params(m))} params, {macs_to_string(m.__macs__)}, "
              f"{duration_to_string(m.__duration__)}, {pct:.2f}% flops", file=out)
        for cname, c in m.named_children():
            self._print_tree(c, cname, depth + 1, max_depth, total_flops, total_dur, out)

    def print_model_aggregated_profile(self, module_depth=-1, top_modules=1, file=None):
        out = file or sys.stdout
        info = OrderedDict()

        def walk(m, d):
            info.setdefault(d, {})
            key = type(m).__name__
            agg = info[d].setdefault(key, [0, 0, 0.0])
            agg[0] += m.__macs__
            agg[1] += self._tree_params(m)
            agg[2] += m.__duration__
            for c in m.children():
                walk(c, d + 1)

        walk(self.model, 0)
        depth = max(info) if module_depth == -1 else min(module_depth, max(info))
        print(f"\n----------------------------- Aggregated Profile per GPU -----------------------------", file=out)
        print(f"Top {top_modules} modules in terms of params, MACs or fwd latency at different model depths:",
              file=out)
        for d in range(depth + 1):
            items = info[d]
            by_macs = sorted(items.items(), key=lambda kv: kv[1][0], reverse=True)[:top_modules]
            by_params = sorted(items.items(), key=lambda kv: kv[1][1], reverse=True)[:top_modules]
            by_lat = sorted(items.items(), key=lambda kv: kv[1][2], reverse=True)[:top_modules]
            print(f"depth {d}:", file=out)
            print(f"    params      - {{{', '.join(f'{k!r}: {params_to_string(v[1])!r}' for k, v in by_params)}}}",
                  file=out)
            print(f"    MACs        - {{{', '.join(f'{k!r}: {macs_to_string(v[0])!r}' for k, v in by_macs)}}}",
                  file=out)
            print(f"    fwd latency - {{{', '.join(f'{k!r}: {duration_to_string(v[2])!r}' for k, v in by_lat)}}}",
                  file=out)


def _fmt(num, units, precision, table):
    if units is None:
        for suffix, scale in table:
            if abs(num) >= scale:
                return f"{round(num / scale, precision):g} {suffix}"
        return f"{round(num, precision):g}"
    return f"{round(num / dict(table)[units], precision):g} {units}"


_TABLE = [("T", 1e12), ("G", 1e9), ("M", 1e6), ("K", 1e3)]


def number_to_string(num, units=None, precision=DEFAULT_PRECISION):
    return _fmt(num, units, precision, _TABLE)


def macs_to_string(macs, units=None, precision=DEFAULT_PRECISION):
    return f"{number_to_string(macs, units, precision)}MACs"


def flops_to_string(flops, units=None, precision=DEFAULT_PRECISION):
    return f"{number_to_string(flops, units, precision)}FLOPS"


def bytes_to_string(b, units=None, precision=DEFAULT_PRECISION):
    return f"{number_to_string(b, units, precision)}B"


def params_to_string(params_num, units=None, precision=DEFAULT_PRECISION):
    return number_to_string(params_num, units, precision).replace("G", "B")


def duration_to_string(duration, units=None, precision=DEFAULT_PRECISION):
    if units is None:
        if duration >= 1:
            return f"{round(duration, precision):g} s"
        if duration >= 1e-3:
            return f"{round(duration * 1e3, precision):g} ms"
        return f"{round(duration * 1e6, precision):g} us"
    scale = {"s": 1, "ms": 1e3, "us": 1e6}[units]
    return f"{round(duration * scale, precision):g} {units}"


def get_module_flops(module):
    return module.__flops__


def get_module_macs(module):
    return module.__macs__


def get_module_duration(module):
    return module.__duration__


def get_model_profile(model, input_shape=None, args=None, kwargs=None, print_profile=True, detailed=True,
                      module_depth=-1, top_modules=1, warm_up=1, as_string=True, output_file=None,
                      ignore_modules=None, mode="forward"):
    """Profile one forward of ``model``; returns (flops, macs, params)."""
    args = list(args or [])
    kwargs = dict(kwargs or {})
    if input_shape is not None:
        dev = next(model.parameters()).device
        args = [torch.ones(input_shape, device=dev)] + args
    prof = FlopsProfiler(model)
    model.eval()
    with torch.no_grad():
        for _ in range(warm_up):
            model(*args, **kwargs)
        prof.start_profile(ignore_list=ignore_modules)
        model(*args, **kwargs)
        flops, macs, params = prof.get_total_flops(), prof.get_total_macs(), prof.get_total_params()
        if print_profile:
            prof.print_model_profile(profile_step=warm_up, module_depth=module_depth, top_modules=top_modules,
                                     detailed=detailed, output_file=output_file)
        prof.end_profile()
    if as_string:
        return number_to_string(flops), macs_to_string(macs), params_to_string(params)
    return flops, macs, params
