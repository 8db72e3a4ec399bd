"""Headline benchmark: Llama-3-8B ZeRO-3 bf16 training throughput (tokens/s for the whole job).

BASELINE.json metric: "tokens/sec (node) Llama-3-8B ZeRO-3 at 1/2/4/8 MI355X". The reference publishes
no number for it (``published: {}``), so ``vs_baseline`` is null.

    python bench.py --gpus 1 --steps 10 --warmup 3
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus 8 --steps 10 --warmup 3

Every step is a full training step of the real 8.03B-parameter architecture (32 layers, GQA 32/8,
vocab 128256) through ``hcache_deepspeed_amd.initialize``: forward, backward (ZeRO-3 all-gather /
reduce-scatter), fused AdamW on the fp32 master shard. Weights are random (zero.Init, per-unit
seeded), data is synthetic uniform token ids. Weak scaling: per-GPU micro-batch fixed as N grows.
"""
import argparse
import json
import os
import sys
import time

# device->host copies (activation spills) as blit kernels of at most 16 workgroups -- set before torch loads the HIP
# runtime (hcache_deepspeed_amd/__init__.py)
os.environ.setdefault("DEBUG_CLR_LIMIT_BLIT_WG", "16")

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _use_tuned_gemms():
    """Read the committed hipBLASLt/rocBLAS solution table (PyTorch TunableOp, tuned on MI355X for the bench's
    GEMM shapes: tools/r6/gpu_tunableop_ab.sh; +0.5 % in an interleaved A/B, profiles/r6/tunableop_ab). TunableOp
    reads one file per device ordinal (%d); the eight copies are identical. Tuning is off: shapes missing from the
    table keep the library heuristic. Must run before torch initialises its BLAS handles; HDS_TUNABLEOP=0 disables
    it."""
    table = os.path.join(ROOT, "tuning", "tunableop_results%d.csv")
    if os.environ.get("HDS_TUNABLEOP", "1") != "1" or not os.path.exists(table % 0):
        return False
    os.environ.setdefault("PYTORCH_TUNABLEOP_ENABLED", "1")
    os.environ.setdefault("PYTORCH_TUNABLEOP_TUNING", "0")
    os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", table)
    return True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=7)  # 244.5 GiB peak at N=1 (mb8: 261.6 GiB, +0.5%)
    ap.add_argument("--gas", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--zero", type=int, default=3)
    ap.add_argument("--layers", type=int, default=0, help="debug only: override layer count (result is marked invalid)")
    ap.add_argument("--prefetch", type=int, default=2)
    ap.add_argument("--ckpt", action="store_true", help="activation checkpointing")
    ap.add_argument("--act-cache-policy", default="budget", choices=["budget", "recompute", "all", "ckpt_offload", "auto", "plan"],
                    help="host activation cache: spill the over-budget layers (budget), recompute them (recompute), "
                         "spill every eligible layer (all), or checkpoint every block and spill its inputs "
                         "(ckpt_offload, long context), or recompute then spill what PCIe can hide (auto), or "
                         "keep / spill / recompute per tensor class (plan)")
    ap.add_argument("--act-cache-spill-cost", type=float, default=0.6,
                    help="host activation cache policy plan: modelled cost of a hidden spill, ms per GB")
    ap.add_argument("--act-cache-spill-overlap", type=float, default=0.5,
                    help="host activation cache policy auto: fraction of the forward the spilled blocks' D2H may take")
    ap.add_argument("--act-cache-budget-gib", type=float, default=0.0,
                    help="host activation cache: HBM budget the planner keeps activations under (0: 92%% of HBM)")
    ap.add_argument("--act-cache-host-gib", type=float, default=0.0,
                    help="host activation cache: pinned-host budget (0: 40%% of RAM shared by the node's ranks, <= 160)")
    ap.add_argument("--no-attn-stash", action="store_true",
                    help="host activation cache policy ckpt_offload: recompute attention instead of replaying its output")
    ap.add_argument("--host-act-cache", action="store_true",
                    help="HCache host activation cache (saved activations spill to pinned host memory)")
    ap.add_argument("--offload", choices=["none", "cpu", "nvme"], default="none",
                    help="ZeRO-Offload/Infinity of optimizer states (+ params with --offload-param)")
    ap.add_argument("--offload-param", action="store_true")
    ap.add_argument("--sub-group-size", type=int, default=None,
                    help="zero_optimization.sub_group_size (ZeRO-Offload's host-step piece, elements)")
    ap.add_argument("--offload-ratio", type=float, default=1.0,
                    help="with --offload cpu/nvme: fraction of the optimizer partition updated on the host (Twin-Flow / "
                         "ZeRO-Offload++); the rest keeps the on-device fused Adam")
    ap.add_argument("--nvme-path", default="/tmp/hds_nvme", help="swap folder of the NVMe tier (--offload nvme)")
    ap.add_argument("--ep", type=int, default=1, help="expert-parallel size (MoE models)")
    ap.add_argument("--moe-dropless", action="store_true",
                    help="MoE models: no token dropping (capacity = the largest expert load of the step; the expert "
                         "GEMMs run over the occupied slots only)")
    ap.add_argument("--sp", type=int, default=1,
                    help="Ulysses sequence-parallel size: each rank holds seq/sp tokens of every sequence (ZeRO shards "
                         "over the dp x sp ranks; tokens/s counts each sequence once)")
    ap.add_argument("--fpdt-chunk", type=int, default=0,
                    help="FPDT (Ulysses-Offload) attention with this global segment length (mi355x.fpdt): chunked "
                         "attention, segments in pinned host memory between forward and backward")
    ap.add_argument("--fpdt-no-offload", action="store_true", help="FPDT: keep the segments on the device")
    ap.add_argument("--fpdt-ffn-chunks", type=int, default=0, help="FPDT: also run the MLPs in this many chunks")
    ap.add_argument("--offload-opt-states", action="store_true",
                    help="DeepCompile offload_adam_states: Adam moments + fp32 master on pinned host between steps")
    ap.add_argument("--offload-states-ratio", type=lambda v: v if v == "auto" else float(v), default=1.0,
                    help="with --offload-opt-states: fraction of every moved state (its tail) kept on the host between "
                         "steps; 'auto': everything on the host for the first step, then the ratio that the first "
                         "step's measured peak leaves room for")
    ap.add_argument("--offload-states-host-step", action="store_true",
                    help="with --offload-opt-states: the host tails stay on the host and step there (host Adam)")
    ap.add_argument("--offload-params-compile", type=float, default=None, metavar="BUDGET_GIB",
                    help="DeepCompile offload_parameters on the GPU-optimizer engine; the pass keeps shards on the "
                         "device within BUDGET_GIB of HBM (0: every shard on the host)")
    ap.add_argument("--reuse-distance", default="auto",
                    help="ZeRO-3 stage3_max_reuse_distance in elements; 'auto' = every parameter at N > 1 (units stay "
                         "gathered from their forward to their backward: one all-gather per unit per step instead of "
                         "two; HBM allows it at every dp for Llama-3-8B), 0 = release after the forward")
    ap.add_argument("--comm-timing", action="store_true",
                    help="N>1: TORCH_NCCL_ENABLE_TIMING=1 for the whole run (in-step RCCL busbw in extra.comm; adds two "
                         "events per collective to the timed steps too)")
    ap.add_argument("--deepcompile", action="store_true",
                    help="engine.compile() with DeepCompile: profiled ZeRO-3 gather schedule (selective gather + prefetch)")
    args = ap.parse_args()
    if os.environ.get("HDS_HANG_DUMP"):
        # diagnosis of a stuck run: every N seconds print the Python stacks of all threads to stderr
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["HDS_HANG_DUMP"]), repeat=True)
    tuned = _use_tuned_gemms()

    import torch
    import torch.distributed as tdist

    import hcache_deepspeed_amd as hds
    from hcache_deepspeed_amd.models import gpt2, llama, mixtral

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and args.comm_timing:
        # opt-in: RCCL records start/end events per collective (every step, timed ones included) so the instrumented
        # step after the timed region can report in-step AG/RS busbw
        os.environ.setdefault("TORCH_NCCL_ENABLE_TIMING", "1")
    if world > 1 or "RANK" in os.environ:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    else:
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=os.environ.get("MASTER_PORT", "29533"))
    on_gpu = torch.cuda.is_available()
    # no GPU: a CPU/gloo dry run of the same multi-rank code path (timing/all-reduce/JSON), never a result
    hds.init_distributed(dist_backend=None if on_gpu else "gloo", verbose=False)
    rank = tdist.get_rank()
    if on_gpu:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    overrides = {}
    if args.model.startswith("gpt2"):
        if args.layers:
            overrides["n_layer"] = args.layers
        cfg_model = {"gpt2-small": gpt2.gpt2_small, "gpt2-medium": gpt2.gpt2_medium}[args.model](**overrides)
        build = gpt2.GPT2LMHeadModel
    elif args.model in ("mixtral-8x7b", "tiny-moe"):
        if args.layers:
            overrides["num_hidden_layers"] = args.layers
        if args.moe_dropless:
            overrides["drop_tokens"] = False
        cfg_model = {"mixtral-8x7b": mixtral.mixtral_8x7b, "tiny-moe": mixtral.tiny_moe}[args.model](
            ep_size=args.ep, **overrides)
        build = mixtral.MixtralForCausalLM
    else:
        if args.layers:
            overrides["num_hidden_layers"] = args.layers
        cfg_model = llama.PRESETS[args.model](**overrides)
        build = llama.LlamaForCausalLM
    ds_config = {
        "train_micro_batch_size_per_gpu": args.micro_batch,
        "gradient_accumulation_steps": args.gas,
        "bf16": {"enabled": True},
        "optimizer": {"type": "AdamW", "params": {"lr": 1e-4, "betas": [0.9, 0.95], "eps": 1e-8,
                                                   "weight_decay": 0.1}},
        "gradient_clipping": 1.0,
        "zero_optimization": {"stage": args.zero},
        "mi355x": {"zero3_prefetch_depth": args.prefetch, "comm_stats": False, "host_act_cache": {"enabled": bool(args.host_act_cache), "policy": args.act_cache_policy,
                                                                        "spill_overlap": args.act_cache_spill_overlap,
                                                                        "gpu_budget_gib": args.act_cache_budget_gib,
                                                                        "host_budget_gib": args.act_cache_host_gib,
                                                                        "stash_attention": not args.no_attn_stash,
                                                                        "spill_cost_ms_per_gb": args.act_cache_spill_cost}},
        "steps_per_print": 1000000,
    }
    if args.sp > 1:
        assert world % args.sp == 0 and args.seq % args.sp == 0, "--sp must divide the world size and --seq"
        ds_config["sequence_parallel_size"] = args.sp
    if args.fpdt_chunk:
        ds_config["mi355x"]["fpdt"] = {"enabled": True, "chunk_size": args.fpdt_chunk,
                                       "offload": not args.fpdt_no_offload, "ffn_chunks": args.fpdt_ffn_chunks}
    if args.zero == 3:
        rd = args.reuse_distance
        if rd == "auto":
            npar = (cfg_model.num_params() if hasattr(cfg_model, "num_params") else
                    cfg_model.active_params() if hasattr(cfg_model, "active_params") else 0)
            rd = int(4 * npar) if world > 1 else 0
        if int(rd) > 0:
            ds_config["zero_optimization"]["stage3_max_reuse_distance"] = int(rd)
    dc_on = args.deepcompile or args.offload_opt_states or args.offload_params_compile is not None
    if dc_on:
        ds_config["compile"] = {"deepcompile": bool(args.deepcompile or args.offload_params_compile is not None),
                                "offload_opt_states": bool(args.offload_opt_states),
                                "offload_parameters": args.offload_params_compile is not None}
    if args.offload != "none":
        ds_config["zero_optimization"]["offload_optimizer"] = {"device": args.offload, "pin_memory": True,
                                                               "ratio": float(args.offload_ratio)}
        if args.sub_group_size:
            ds_config["zero_optimization"]["sub_group_size"] = int(args.sub_group_size)
        if args.offload_param:
            ds_config["zero_optimization"]["offload_param"] = {"device": args.offload, "pin_memory": True}
        if args.offload == "nvme":
            for k in ("offload_optimizer", "offload_param"):
                if k in ds_config["zero_optimization"]:
                    ds_config["zero_optimization"][k]["nvme_path"] = args.nvme_path
            ds_config["aio"] = {"block_size": 1 << 20, "queue_depth": 64, "intra_op_parallelism": 8}
    t_init = time.time()
    with hds.zero.Init(enabled=args.zero == 3):
        model = build(cfg_model)
    if args.ckpt:
        model.gradient_checkpointing_enable()
    engine, _, _, _ = hds.initialize(model=model, config=ds_config)
    if dc_on:
        kw = {} if args.offload_params_compile is None else {"mem_budget_bytes": args.offload_params_compile * 2**30}
        if args.offload_opt_states:
            kw["offload_states_ratio"] = args.offload_states_ratio
            kw["offload_states_host_step"] = bool(args.offload_states_host_step)
        engine.compile(compile_kwargs=kw)  # schedule compiled after the profiled warmup step (compile/backend.py)
    t_init = time.time() - t_init
    dev = engine.device
    S, mb = args.seq, args.micro_batch
    gen = torch.Generator(device=dev)
    sp = args.sp
    if sp > 1:
        # the ranks of one sequence-parallel group draw the SAME sequences and each feeds its own token positions
        from hcache_deepspeed_amd.utils import groups as _groups
        sp_ranks = tdist.get_process_group_ranks(_groups._get_sequence_parallel_group())
        gen.manual_seed(1234 + min(sp_ranks))
        shard = engine.sequence_shard_indices(S).to(dev)
    else:
        gen.manual_seed(1234 + rank)
        shard = None

    def train_step(i):
        loss = None
        for g in range(args.gas):
            # a fresh synthetic batch every micro-step (no fixed batches to memorise)
            if shard is None:
                x = torch.randint(0, cfg_model.vocab_size, (mb, S), device=dev, generator=gen)
                loss = engine(x, labels=x)
            else:
                full = torch.randint(0, cfg_model.vocab_size, (mb, S + 1), device=dev, generator=gen)
                x, t = full[:, :-1][:, shard].contiguous(), full[:, 1:][:, shard].contiguous()
                loss = engine(x, targets=t)
            engine.backward(loss)
            engine.step()
        return loss

    progress = os.environ.get("HDS_BENCH_PROGRESS") == "1"  # long-context sweeps: a line per step on stderr
    if progress and rank == 0:
        # steps of minutes (>= 256k tokens): a line every 8 blocks entered -- forward AND backward recomputes -- so a
        # supervisor that kills silent commands sees the run move
        t_run = time.perf_counter()
        blocks = [b for m in model.modules() if isinstance(m, torch.nn.ModuleList) for b in m]

        def _block_progress(i):
            def pre(mod, args):
                if i % 8 == 0:
                    print(f"[bench] t={time.perf_counter() - t_run:.0f}s block {i} "
                          f"({'grad' if torch.is_grad_enabled() else 'no-grad'})", file=sys.stderr, flush=True)
            return pre

        for i, b in enumerate(blocks):
            b.register_forward_pre_hook(_block_progress(i))
        ac0 = getattr(engine, "_activation_cache", None)
        if ac0 is not None:
            # a checkpointed block's recompute calls its forward directly (no module hooks): report the backward's
            # position from the cache, and only when it MOVED -- a hung step still goes silent
            import threading

            ac0.track_progress = True

            def _gpu_block():  # the latest backward block whose first kernels the GPU has reached
                done = None
                for layer, ev in list(getattr(ac0, "bwd_events", [])):
                    if ev.query():
                        done = layer
                return done

            def _heartbeat():
                last = None
                while True:
                    time.sleep(20)
                    st = (ac0.bwd_layer_seen, _gpu_block(), ac0.cur_layer)
                    if st != last:
                        last = st
                        print(f"[bench] t={time.perf_counter() - t_run:.0f}s backward: host at block {st[0]}, GPU at "
                              f"block {st[1]}; forward block {st[2]}", file=sys.stderr, flush=True)

            threading.Thread(target=_heartbeat, daemon=True).start()

    def step_progress(tag, i, t_start):
        if progress and rank == 0:
            sync()
            print(f"[bench] {tag} step {i} done at {time.perf_counter() - t_start:.1f}s "
                  f"peak {torch.cuda.max_memory_allocated(dev) / 2**30 if on_gpu else 0:.1f} GiB", file=sys.stderr,
                  flush=True)

    loss = None
    tw = time.perf_counter()
    for i in range(args.warmup):
        loss = train_step(i)
        step_progress("warmup", i, tw)
    sync()
    tdist.barrier()
    sync()
    retries0 = torch.cuda.memory_stats(dev).get("num_alloc_retries", 0) if on_gpu else 0
    zopt = engine.optimizer
    timed_events = getattr(zopt, "comm_stats", None)  # None: the timed steps record no comm accounting events
    ac_t = getattr(engine, "_activation_cache", None)
    n_peaks0 = len(ac_t.step_peak_history) if ac_t is not None else 0
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = train_step(args.warmup + i)
        step_progress("timed", i, t0)
    sync()
    tdist.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], device=dev, dtype=torch.float64)
    tdist.all_reduce(dt_t, op=tdist.ReduceOp.MAX)
    dt = float(dt_t.item())
    tokens = world // sp * mb * args.gas * S * args.steps  # every sequence once (its sp ranks share it)
    value = tokens / dt
    ms_per_step = dt / args.steps * 1e3
    flops = (cfg_model.flops_per_token(S) if hasattr(cfg_model, "flops_per_token") else
             6 * cfg_model.active_params() + 12 * cfg_model.num_hidden_layers * S * cfg_model.hidden_size) * tokens
    mfu = flops / dt / (2.5e15 * world)
    # the same with causal attention FLOPs (what the causal kernels execute; matters at long context)
    flops_c = cfg_model.flops_per_token_causal(S) * tokens if hasattr(cfg_model, "flops_per_token_causal") else flops
    mfu_c = flops_c / dt / (2.5e15 * world)
    mem = torch.cuda.max_memory_allocated(dev) / 2**30 if on_gpu else 0.0
    timed_peak = None
    if ac_t is not None and on_gpu:
        # the cache resets the allocator's peak counter per forward (and per backward block): the timed steps' peaks
        # are the history entries of their forwards after the first (which closes the last warm-up step) plus the
        # running max of the last timed step
        timed_peak = max(ac_t.step_peak_history[n_peaks0 + 1:] + [ac_t.step_peak()]) / 2**30
    # caching-allocator retries in the timed steps: each one frees cached blocks after a device-wide synchronize
    retries = (torch.cuda.memory_stats(dev).get("num_alloc_retries", 0) - retries0) if on_gpu else 0
    comm = None
    if world > 1:
        # communication evidence, measured OUTSIDE the timed region: one extra instrumented step (exposed compute-
        # stream wait on every AG / RS, per-collective traffic; RCCL busbw with --comm-timing), then the unit
        # all-gather / reduce-scatter alone at the largest unit size over the data-parallel group
        from hcache_deepspeed_amd.runtime.zero.comm_stats import ZeroCommStats
        cs = None
        if hasattr(zopt, "comm_stats"):
            cs = zopt.comm_stats = ZeroCommStats(dev)
            sync()
            train_step(args.warmup + args.steps)
            sync()
            zopt.comm_stats = None
        mine = {"rank": rank, "peak_mem_gib": round(mem, 1), "timed_steps_instrumented": timed_events is not None,
                "host_threads": getattr(engine, "host_threads", None)}
        ue = getattr(zopt, "unit_events", None)
        if ue is not None:  # ZeRO-3 fetch / wait / prefetch events of the last micro-step (counts, numel, host ms)
            mine["unit_events"] = ue.summary()
        if getattr(zopt, "comm_selection", None) is not None:  # startup transport measurement + routing
            mine["transport_selection"] = zopt.comm_selection
        if cs is not None:
            summ = cs.summary()
            mine["exposed_comm_ms_per_step"] = round(summ["exposed_ms"] / args.gas, 2)
            mine["collectives"] = summ["collectives"]
        unit_bytes = max((u.shard * u.world * 2 for u in getattr(zopt, "units", []) if u.world > 1), default=0)
        if unit_bytes:
            from hcache_deepspeed_amd.compile.profiler import profile_allgather, profile_reduce_scatter
            dpg = getattr(zopt, "dp_group", None)
            ag = profile_allgather(dpg, dev, sizes_bytes=[unit_bytes // 8, unit_bytes], iters=3)
            rs = profile_reduce_scatter(dpg, dev, sizes_bytes=[unit_bytes // 8, unit_bytes], iters=3)
            mine["unit_collectives_isolated"] = {
                "unit_mib": round(unit_bytes / 2**20, 1),
                "all_gather": ag.to_dict(), "all_gather_busbw_GBps": round(ag.busbw(unit_bytes, world) / 1e9, 1),
                "reduce_scatter": rs.to_dict(),
                "reduce_scatter_busbw_GBps": round(rs.busbw(unit_bytes, world) / 1e9, 1)}
        fit = getattr(zopt, "auto_bucket_fit", None)
        if fit is not None:
            mine["auto_bucket_fit"] = fit
            mine["xgmi_bucket_mb"] = getattr(zopt.mi, "xgmi_bucket_mb", None)
            mine["zero3_unit_bucket_mb"] = getattr(zopt.mi, "zero3_unit_bucket_mb", None)
        per_rank = [None] * world
        tdist.all_gather_object(per_rank, mine)
        comm = {"backend": tdist.get_backend(), "ranks": world, "measured": "instrumented step after the timed region",
                "timed_steps_instrumented": any(r["timed_steps_instrumented"] for r in per_rank),
                "exposed_comm_ms_per_step_max": max(r.get("exposed_comm_ms_per_step", 0.0) for r in per_rank),
                "peak_mem_gib_per_rank": [r["peak_mem_gib"] for r in per_rank],
                "host_threads_per_rank": [(r.get("host_threads") or {}).get("threads") for r in per_rank],
                "rank0": per_rank[0],
                "unit_events_rank0": per_rank[0].get("unit_events"),
                "transport_selection": per_rank[0].get("transport_selection")}
        for kind in ("all_gather", "reduce_scatter"):
            bws = [r.get("collectives", {}).get(kind, {}).get("busbw_GBps") for r in per_rank]
            bws = [b for b in bws if b]
            comm[f"{kind}_busbw_GBps_min_over_ranks"] = min(bws) if bws else None
    if rank == 0:
        out = {
            "metric": ("tokens/sec (node) Llama-3-8B ZeRO-3 at 1/2/4/8 MI355X" if args.model == "llama3-8b" else
                       f"tokens/sec (node) {args.model} ZeRO-{args.zero}"),
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (uniform random token ids), random-init weights",
            "config": {"model": "Llama-3-8B" if args.model == "llama3-8b" and not args.layers else
                       f"{args.model}{'-L' + str(args.layers) if args.layers else ''}",
                       "host_act_cache": bool(args.host_act_cache), "offload": args.offload,
                       **({"offload_ratio": float(args.offload_ratio)} if args.offload != "none" and
                          args.offload_ratio < 1.0 else {}),
                       "global_batch": world // sp * mb * args.gas, "seq_len": S,
                       "parallelism": f"zero{args.zero}-dp{world // sp}" + (f"-sp{sp}" if sp > 1 else ""),
                       "micro_batch_per_gpu": mb, "gas": args.gas,
                       **({"sequence_parallel_size": sp} if sp > 1 else {}),
                       **({"fpdt": engine.fpdt_config} if getattr(engine, "fpdt_config", None) else {}),
                       "stage3_max_reuse_distance": ds_config["zero_optimization"].get("stage3_max_reuse_distance"),
                       "activation_checkpointing": bool(args.ckpt), "deepcompile": bool(args.deepcompile),
                       **({"moe_dropless": True} if args.moe_dropless else {})},
            "extra": {"mfu_bf16_dense_2.5PF": round(mfu, 4), "tflops_per_gpu": round(flops / dt / world / 1e12, 1),
                      "mfu_causal": round(mfu_c, 4), "tflops_causal_per_gpu": round(flops_c / dt / world / 1e12, 1),
                      "host_threads": getattr(engine, "host_threads", None),
                      "final_loss": round(float(loss.item()), 4), "peak_mem_gib": round(mem, 1),
                      "init_s": round(t_init, 1), "valid": on_gpu and not bool(args.layers),
                      "tuned_gemm_table": tuned, "device": "mi355x" if on_gpu else "cpu-dry-run",
                      "alloc_retries_timed": int(retries)},
        }
        if comm is not None:
            out["extra"]["comm"] = comm
        so = getattr(engine.optimizer, "state_offload", None)
        if so is not None:
            out["extra"]["offload_opt_states"] = so.stats()
            out["config"]["offload_opt_states"] = True
        sched = getattr(engine.optimizer, "dc_schedule", None)
        if sched is not None and "offload_parameters" in sched.meta:
            out["extra"]["offload_parameters"] = {k: v for k, v in sched.meta["offload_parameters"].items()
                                                  if k != "resident"}
            out["config"]["offload_parameters"] = True
        ac = getattr(engine, "_activation_cache", None)
        if ac is not None:
            out["extra"]["act_cache"] = ac.stats()
            if ac.peak_seen:  # the cache resets the peak counter every forward: report the max over all steps
                out["extra"]["peak_mem_gib"] = round(max(mem, ac.peak_seen / 2**30), 1)
            if timed_peak is not None:
                out["extra"]["peak_gib_timed_steps"] = round(timed_peak, 1)
                if ac.budget is not None:
                    out["extra"]["act_cache_budget_gib"] = round(ac.budget / 2**30, 1)
        zo = engine.optimizer
        sw = getattr(zo, "opt_swapper", None)
        if sw is not None:  # ZeRO-Infinity NVMe tier: how much of the optimizer's swap I/O hid behind CPU Adam
            out["extra"]["nvme_opt"] = {"read_gib": round(sw.bytes_read / 2**30, 2),
                                        "written_gib": round(sw.bytes_written / 2**30, 2),
                                        "step_io_wait_s": round(sw.wait_s, 2), "step_pipeline_s": round(sw.step_s, 2),
                                        "engine": zo.nvme.engine}
        ps = getattr(zo, "param_swapper", None)
        if ps is not None:
            out["extra"]["nvme_param"] = {"read_gib": round(ps.bytes_read / 2**30, 2),
                                          "written_gib": round(ps.bytes_written / 2**30, 2)}
        print(json.dumps(out), flush=True)
    tdist.barrier()
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
