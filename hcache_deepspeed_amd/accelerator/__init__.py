"""``get_accelerator()``: the device interface user scripts import (reference accelerator/real_accelerator.py:51,
abstract_accelerator.py).

The reference dispatches over eight vendors; this framework runs on exactly one device family, so there is
one concrete class. On an MI355X host it is backed by PyTorch-ROCm's HIP device module (``torch.cuda`` IS
HIP on ROCm: streams, events, graphs, memory stats), collectives report ``"nccl"`` (= RCCL over xGMI), and
ranges go to roctx. Without a GPU (CPU tests, ``ds_report`` on a login node) the same object answers for
the host so scripts written against ``get_accelerator()`` still run.
"""
import functools

import torch


class MI355XAccelerator:
    """Device abstraction for AMD Instinct MI355X (gfx950, CDNA4) under PyTorch-ROCm."""

    def __init__(self):
        self._name = "cuda" if torch.cuda.is_available() else "cpu"
        self._communication_backend_name = "nccl" if self._name == "cuda" else "gloo"
        self._compile_backend = "inductor"

    # --- identity ----------------------------------------------------------------------
    def is_synchronized_device(self):
        return self._name == "cpu"

    def use_host_timers(self):
        return self.is_synchronized_device()

    def resolves_data_dependency(self):
        return self.is_synchronized_device()

    def handles_memory_backpressure(self):
        return self.is_synchronized_device()

    def device_name(self, device_index=None):
        if device_index is None or self._name == "cpu":
            return self._name
        return f"{self._name}:{device_index}"

    def device(self, device_index=None):
        return torch.device(self.device_name(device_index))

    def set_device(self, device_index):
        if self._name == "cuda":
            torch.cuda.set_device(device_index)

    def current_device(self):
        return torch.cuda.current_device() if self._name == "cuda" else 0

    def current_device_name(self):
        return f"cuda:{torch.cuda.current_device()}" if self._name == "cuda" else "cpu"

    def device_count(self):
        return torch.cuda.device_count() if self._name == "cuda" else 1

    def synchronize(self, device_index=None):
        if self._name == "cuda":
            torch.cuda.synchronize(device_index)

    def is_available(self):
        return self._name == "cuda"

    def arch(self):
        """gfx target of the current device (``gfx950`` on MI355X)."""
        if self._name != "cuda":
            return "cpu"
        return getattr(torch.cuda.get_device_properties(self.current_device()), "gcnArchName", "gfx950").split(":")[0]

    # --- RNG ---------------------------------------------------------------------------
    def random(self):
        return torch.random

    def set_rng_state(self, new_state, device_index=None):
        if self._name == "cuda":
            return torch.cuda.set_rng_state(new_state) if device_index is None else \
                torch.cuda.set_rng_state(new_state, device_index)
        return torch.set_rng_state(new_state)

    def get_rng_state(self, device_index=None):
        if self._name == "cuda":
            return torch.cuda.get_rng_state() if device_index is None else torch.cuda.get_rng_state(device_index)
        return torch.get_rng_state()

    def manual_seed(self, seed):
        return torch.cuda.manual_seed(seed) if self._name == "cuda" else torch.manual_seed(seed)

    def manual_seed_all(self, seed):
        return torch.cuda.manual_seed_all(seed) if self._name == "cuda" else torch.manual_seed(seed)

    def initial_seed(self):
        return torch.cuda.initial_seed() if self._name == "cuda" else torch.initial_seed()

    def default_generator(self, device_index):
        return torch.cuda.default_generators[device_index] if self._name == "cuda" else torch.default_generator

    # --- streams / events / graphs -------------------------------------------------------
    @property
    def Stream(self):
        return torch.cuda.Stream if self._name == "cuda" else _NullStream

    def stream(self, stream):
        return torch.cuda.stream(stream) if self._name == "cuda" else _NullContext()

    def current_stream(self, device_index=None):
        return torch.cuda.current_stream(device_index) if self._name == "cuda" else _NullStream()

    def default_stream(self, device_index=None):
        return torch.cuda.default_stream(device_index) if self._name == "cuda" else _NullStream()

    @property
    def Event(self):
        return torch.cuda.Event if self._name == "cuda" else _NullEvent

    def create_graph(self):
        return torch.cuda.CUDAGraph() if self._name == "cuda" else None

    def capture_to_graph(self, graph, pool=None, stream=None):
        if self._name != "cuda":
            return _NullContext()
        return torch.cuda.graph(graph, pool=pool, stream=stream)

    def replay_graph(self, graph):
        if graph is not None:
            graph.replay()

    # --- memory ------------------------------------------------------------------------
    def empty_cache(self):
        if self._name == "cuda":
            torch.cuda.empty_cache()

    def _mem(self, fn, device_index=None, default=0):
        return getattr(torch.cuda, fn)(device_index) if self._name == "cuda" else default

    def memory_allocated(self, device_index=None):
        return self._mem("memory_allocated", device_index)

    def max_memory_allocated(self, device_index=None):
        return self._mem("max_memory_allocated", device_index)

    def reset_max_memory_allocated(self, device_index=None):
        if self._name == "cuda":
            torch.cuda.reset_peak_memory_stats(device_index)

    def memory_cached(self, device_index=None):
        return self._mem("memory_reserved", device_index)

    def max_memory_cached(self, device_index=None):
        return self._mem("max_memory_reserved", device_index)

    def reset_max_memory_cached(self, device_index=None):
        self.reset_max_memory_allocated(device_index)

    def memory_stats(self, device_index=None):
        return torch.cuda.memory_stats(device_index) if self._name == "cuda" else {}

    def reset_peak_memory_stats(self, device_index=None):
        self.reset_max_memory_allocated(device_index)

    def memory_reserved(self, device_index=None):
        return self._mem("memory_reserved", device_index)

    def max_memory_reserved(self, device_index=None):
        return self._mem("max_memory_reserved", device_index)

    def total_memory(self, device_index=None):
        if self._name != "cuda":
            import psutil
            return psutil.virtual_memory().total
        return torch.cuda.get_device_properties(device_index or self.current_device()).total_memory

    def available_memory(self, device_index=None):
        if self._name != "cuda":
            import psutil
            return psutil.virtual_memory().available
        free, _ = torch.cuda.mem_get_info(device_index)
        return free

    # --- dtypes ------------------------------------------------------------------------
    def is_bf16_supported(self):
        return True

    def is_fp16_supported(self):
        return True

    def supported_dtypes(self):
        return [torch.float, torch.half, torch.bfloat16]

    def amp(self):
        return torch.amp

    # --- tracing -----------------------------------------------------------------------
    def range_push(self, msg):
        from ..utils.nvtx import _push
        _push(msg)

    def range_pop(self):
        from ..utils.nvtx import _pop
        _pop()

    def lazy_call(self, callback):
        if self._name == "cuda":
            return torch.cuda._lazy_call(callback)
        return callback()

    # --- communication / compile -------------------------------------------------------
    def communication_backend_name(self):
        return self._communication_backend_name

    def is_triton_supported(self):
        return False  # no Triton: hot ops are hand-written HIP kernels

    def get_compile_backend(self):
        return self._compile_backend

    def set_compile_backend(self, backend):
        self._compile_backend = backend

    # --- tensor types ------------------------------------------------------------------
    def _tt(self, dtype):
        return functools.partial(torch.tensor, dtype=dtype, device=self._name)

    @property
    def BFloat16Tensor(self):
        return self._tt(torch.bfloat16)

    @property
    def ByteTensor(self):
        return self._tt(torch.uint8)

    @property
    def DoubleTensor(self):
        return self._tt(torch.double)

    @property
    def FloatTensor(self):
        return self._tt(torch.float)

    @property
    def HalfTensor(self):
        return self._tt(torch.half)

    @property
    def IntTensor(self):
        return self._tt(torch.int)

    @property
    def LongTensor(self):
        return self._tt(torch.long)

    # --- host memory -------------------------------------------------------------------
    def pin_memory(self, tensor, align_bytes=1):
        return tensor.pin_memory() if self._name == "cuda" else tensor

    def is_pinned(self, tensor):
        return tensor.is_pinned() if self._name == "cuda" else False

    def on_accelerator(self, tensor):
        return tensor.device.type == self._name

    # --- native ops --------------------------------------------------------------------
    def op_builder_dir(self):
        return "hcache_deepspeed_amd.ops"

    def create_op_builder(self, class_name):
        return _OpBuilder(class_name)

    def get_op_builder(self, class_name):
        return _OpBuilder

    def build_extension(self):
        from ..ops import build
        return build

    def export_envs(self):
        return ["NCCL", "RCCL", "HIP", "HSA", "ROCR", "GPU_MAX_HW_QUEUES"]

    def visible_devices_envs(self):
        return ["HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"]

    def set_visible_devices_envs(self, current_env, local_accelerator_ids):
        for env in self.visible_devices_envs()[:1]:
            current_env[env] = ",".join(map(str, local_accelerator_ids))


class _OpBuilder:
    """Stand-in for the reference's JIT op builders: every native op here is compiled ahead of time for gfx950
    (ops/build.py) into two in-tree libraries; ``load()`` returns the loaded kernel library."""

    def __init__(self, name="HDSKernels"):
        self.name = name

    def is_compatible(self, verbose=False):
        return True

    def load(self, verbose=False):
        from ..ops import native
        return native.kernels() if "CPU" not in self.name and "AIO" not in self.name else native.host_lib()


class _NullContext:

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class _NullStream:

    def __init__(self, *a, **k):
        pass

    def synchronize(self):
        pass

    def wait_stream(self, other):
        pass

    def wait_event(self, event):
        pass

    def record_event(self, event=None):
        return event or _NullEvent()


class _NullEvent:

    def __init__(self, *a, **k):
        pass

    def record(self, stream=None):
        pass

    def synchronize(self):
        pass

    def wait(self, stream=None):
        pass

    def query(self):
        return True

    def elapsed_time(self, other):
        return 0.0


_ACCELERATOR = None


def get_accelerator():
    global _ACCELERATOR
    if _ACCELERATOR is None:
        _ACCELERATOR = MI355XAccelerator()
    return _ACCELERATOR


def set_accelerator(accel_obj):
    global _ACCELERATOR
    _ACCELERATOR = accel_obj


def is_current_accelerator_supported():
    return True


