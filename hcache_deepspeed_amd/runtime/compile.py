"""``engine.compile()``: the DeepCompile entry point, realised by this framework's native runtime passes.

Reference parity: compile/config.py (``CompileConfig``: deepcompile, free_activation, offload_activation,
offload_opt_states, double_buffer, symmetric_memory, offload_parameters, sync_* switches), runtime/engine.py
``compile`` :3876-3941 (``init_z1`` / ``init_z3`` graph passes, ``register_compile_pass``, ``get_compile_time``,
``is_compiled``) and compile/passes/* (zero3 gather/release insertion, prefetch scheduling, selective gather,
Adam-state offload, activation / parameter offload).

MI355X design: the reference gets its schedule by tracing the model with torch.compile (Inductor, which emits
Triton) and rewriting the FX graph. This framework has no tracing compiler; every pass the reference inserts is
already a runtime mechanism of the engine, driven by the module-execution trace it records on the first step:

  * zero3 gather/release + prefetch scheduling  -> ZeRO-3 trace-driven prefetch (``zero3_prefetch_depth``) with
    all-gathers on RCCL's stream and release on last use (runtime/zero/optimizer.py);
  * selective gather                            -> persistent small units (``stage3_param_persistence_threshold``);
  * offload_activation                          -> HCache host activation cache (offload/activation_cache.py):
    saved activations go D2H into pinned rings on a side stream, prefetched back in backward;
  * offload_opt_states                          -> optimizer states (and the fp32 master) move to pinned host
    right after ``step()`` on a copy stream and come back during the late backward, at the trace position the
    ``plan_state_reload`` pass picks from the profiled step (runtime/zero/state_offload.py); compile_kwargs
    ``offload_states_ratio`` (the byte fraction moved: each state's tail), ``offload_states_chunk_mb`` and
    ``offload_states_host_step`` (the tails stay on the host and step there with the host Adam -- Llama-3-8B mb10:
    +21.6 % over ZeRO-Offload, where the reload form is 2-5 % behind it);
  * offload_parameters                          -> parameter shards on pinned host (ZeRO-Infinity at init, or
    switched on here for a GPU-optimizer ZeRO-3 engine): fetches are H2D + all-gather at the planned prefetch
    positions; the ``plan_param_offload`` pass keeps the most-fetched shards on the device within the HBM budget;
  * double_buffer                               -> RCCL reduce-scatter buckets are already double-buffered per
    unit;
  * symmetric_memory                            -> the ZeRO unit all-gathers / reduce-scatters of intra-node groups
    run as one-kernel direct-read collectives over IPC-mapped uncached buffers (comm/symmetric.py,
    csrc/kernels/symm_comm.hip; reference csrc/compile/z3.cpp:91-110).

The gather schedule itself is compiled (hcache_deepspeed_amd/compile/): with ``deepcompile`` at ZeRO-3 a
``DeepCompileBackend`` profiles one step of the unit trace (HIP-event timestamps, live HBM bytes), measures an
RCCL all-gather cost model, and runs the selective-gather and prefetch passes; the resulting
``CompiledSchedule`` replaces the depth-bounded prefetch from the next step on.

``compile()`` therefore validates the configuration, switches those mechanisms on and records per-pass setup
times (``get_compile_time``). User passes registered with ``register_compile_pass`` are called once with the
engine (they may adjust knobs such as the prefetch depth).
"""
import time

from ..utils.logging import log_dist, logger

_FIELDS = {
    "deepcompile": False, "free_activation": False, "offload_activation": False, "offload_opt_states": False,
    "double_buffer": True, "symmetric_memory": False, "debug_log": False, "offload_parameters": False,
    "sync_before_reduce": False, "sync_after_reduce": False, "sync_before_allgather": False,
    "sync_after_allgather": False, "native_comm": False
}

_user_passes = {}


class CompileConfig:

    def __init__(self, d=None):
        d = dict(d or {})
        unknown = set(d) - set(_FIELDS)
        if unknown:
            raise ValueError(f"unknown compile config keys: {sorted(unknown)}")
        for k, v in _FIELDS.items():
            setattr(self, k, bool(d.get(k, v)))

    def to_dict(self):
        return {k: getattr(self, k) for k in _FIELDS}


def register_compile_pass(name, fn):
    _user_passes[name] = fn


def compile_engine(engine, backend="native", compile_kwargs=None, schedule=None):
    """Apply the DeepCompile configuration to ``engine`` (see module docstring). Returns per-pass setup times."""
    cfg = CompileConfig(engine._config.raw.get("compile", {}))
    times = {}
    if backend not in ("native", "eager", "inductor", "hip_graph"):
        raise ValueError(f"backend {backend} is not supported")
    if backend == "inductor":
        logger.warning("compile(backend='inductor'): Inductor emits Triton, which this framework does not use; "
                       "running the native runtime passes instead")
    if cfg.deepcompile:
        stage = engine.zero_optimization_stage()
        assert stage in (1, 3), "DeepCompile supports ZeRO stage 1 or 3 only"
        assert engine.optimizer is not None, "DeepCompile needs an optimizer"
    t0 = time.perf_counter()
    if cfg.offload_activation and engine._activation_cache is None:
        from ..offload.activation_cache import build_activation_cache
        hc = engine._config.mi355x.host_act_cache
        engine._activation_cache = build_activation_cache(hc, engine.device).attach(engine.module)
    times["offload_activation"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    if cfg.offload_opt_states:
        assert engine.optimizer is not None and hasattr(engine.optimizer, "enable_state_offload"), \
            "offload_opt_states needs the ZeRO optimizer"
        kw = compile_kwargs or {}
        engine.optimizer.enable_state_offload(include_master=bool(kw.get("offload_master", True)),
                                              ratio=(kw.get("offload_states_ratio", 1.0)
                                                     if str(kw.get("offload_states_ratio", 1.0)) == "auto"
                                                     else float(kw.get("offload_states_ratio", 1.0))),
                                              chunk_mb=float(kw.get("offload_states_chunk_mb", 1024)),
                                              host_step=bool(kw.get("offload_states_host_step", False)))
    times["offload_adam_states"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    if cfg.offload_parameters and not engine._config.zero_config.offload_param.enabled:
        # parameter shards to pinned host, fetched by the (compiled) prefetch schedule; the GPU optimizer step writes
        # them back per unit (runtime/zero/optimizer.py enable_param_offload, compile/passes.py plan_param_offload)
        opt = engine.optimizer
        if opt is None or not hasattr(opt, "enable_param_offload") or not opt.enable_param_offload():
            logger.warning("compile: offload_parameters needs a ZeRO-3 engine with a fused optimizer and a "
                           "bf16/fp16 compute dtype; parameters stay on device")
    times["offload_parameters"] = time.perf_counter() - t0
    if cfg.deepcompile and engine.zero_optimization_stage() == 3:
        # profile-guided gather schedule (compile/backend.py): profiled on a later step, then installed
        from ..compile import DeepCompileBackend
        t0 = time.perf_counter()
        kw = dict(compile_kwargs or {})
        engine._dc_backend = DeepCompileBackend(
            engine, profile_step=kw.get("profile_step", 1), margin=kw.get("mem_margin", 0.1),
            mem_budget_bytes=kw.get("mem_budget_bytes"), max_buffered_bytes=kw.get("max_buffered_bytes"),
            selective_gather=kw.get("selective_gather", True), comm_sizes=kw.get("comm_sizes"))
        times["zero3_compile"] = time.perf_counter() - t0
    elif cfg.deepcompile:
        times["zero1_compile"] = 0.0
    t0 = time.perf_counter()
    if cfg.native_comm and engine.optimizer is not None and hasattr(engine.optimizer, "enable_native_comm"):
        # DeepCompile's private-communicator path (reference csrc/compile/deepcompile.cpp): ZeRO all-gathers and
        # reduce-scatters go through the C++ RCCL executor (comm/native_rccl.py) on its own priority stream
        engine.optimizer.enable_native_comm()
    times["native_comm"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    if cfg.symmetric_memory and engine.optimizer is not None and hasattr(engine.optimizer, "enable_symmetric_comm"):
        # one-kernel direct-read unit collectives over IPC-mapped symmetric buffers (comm/symmetric.py)
        engine.optimizer.enable_symmetric_comm()
    times["symmetric_memory"] = time.perf_counter() - t0
    for name, fn in _user_passes.items():
        t0 = time.perf_counter()
        fn(engine)
        times[name] = time.perf_counter() - t0
    for step, passes in (schedule or []):
        for p in passes:
            if callable(p):
                t0 = time.perf_counter()
                p(engine)
                times[getattr(p, "__name__", str(p))] = time.perf_counter() - t0
    engine._compile_config = cfg
    log_dist(f"compile: backend={backend} deepcompile={cfg.deepcompile} passes={sorted(times)}", ranks=[0])
    return times
