"""ZeRO stages 0-3 on gloo (world_size 1 and 2): training trajectories must match a plain torch AdamW baseline.

Model: tiny Llama (CPU reference op paths). Each rank feeds its own micro-batch; the baseline sees the
concatenated global batch with mean loss, which is what data-parallel averaging computes.
"""
import pytest
import torch

from tests.dist_utils import run_distributed

TINY = dict(head_dim=16, hidden_size=64, intermediate_size=128, vocab_size=97, num_attention_heads=4,
            num_key_value_heads=2, num_hidden_layers=3)


def _models():
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**TINY))
    ref = LlamaForCausalLM(tiny(**TINY))
    ref.load_state_dict(m.state_dict())
    return m, ref


def _batches(world, n, mb=2, S=12):
    g = torch.Generator().manual_seed(42)
    return [torch.randint(0, 97, (world * mb, S), generator=g) for _ in range(n)]


def _zero_vs_torch(rank, world, stage, gas, zero_init):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    m, ref = _models()
    if zero_init:
        with ds.zero.Init():
            m = LlamaForCausalLM(tiny(**TINY))
    cfg = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": gas,
           "optimizer": {"type": "AdamW", "params": {"lr": 5e-3, "weight_decay": 0.01}},
           "zero_optimization": {"stage": stage}, "gradient_clipping": 0.5}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    if zero_init:
        # copy the materialised zero.Init weights into the reference
        full = eng.optimizer.full_fp32_state_dict(eng._param_names)
        ref.load_state_dict({k: v for k, v in full.items()}, strict=False)
    ropt = torch.optim.AdamW(ref.parameters(), lr=5e-3, weight_decay=0.01)
    batches = _batches(world, 3 * gas)
    for step in range(3):
        rl_total = 0.0
        for g in range(gas):
            b = batches[step * gas + g]
            mine = b[rank * 2:(rank + 1) * 2]
            loss = eng(mine, labels=mine)
            eng.backward(loss)
            eng.step()
            rl = ref(b, labels=b) / gas
            rl.backward()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 0.5)
        ropt.step()
        ropt.zero_grad()
    full = eng.optimizer.full_fp32_state_dict(eng._param_names)
    for n, p in ref.named_parameters():
        assert torch.allclose(full[n], p.detach(), atol=3e-4, rtol=1e-3), (stage, n, (full[n] - p).abs().max())


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
def test_zero_single_process(stage):
    run_distributed(_zero_vs_torch, 1, stage, 1, False)


@pytest.mark.parametrize("stage,gas", [(0, 1), (1, 2), (2, 1), (2, 2), (3, 1), (3, 2)])
def test_zero_world2(stage, gas):
    run_distributed(_zero_vs_torch, 2, stage, gas, False)


def test_zero3_init_world2():
    run_distributed(_zero_vs_torch, 2, 3, 1, True)


def _gathered_params(rank, world):
    import hcache_deepspeed_amd as ds
    m, _ = _models()
    eng, _, _, _ = ds.initialize(model=m, config={"train_micro_batch_size_per_gpu": 1, "optimizer": {
        "type": "AdamW", "params": {"lr": 1e-3}}, "zero_optimization": {"stage": 3}})
    w = m.model.layers[1].mlp.down_proj.weight
    assert w.numel() == 0  # partitioned
    with ds.zero.GatheredParameters([w], modifier_rank=0):
        assert w.shape == (64, 128)
        if rank == 0:
            w.data.fill_(0.5)
    with ds.zero.GatheredParameters([w]):
        assert torch.all(w == 0.5)
    full = eng.optimizer.full_fp32_state_dict(eng._param_names)
    assert torch.all(full["model.layers.1.mlp.down_proj.weight"] == 0.5)


def test_gathered_parameters_modifier():
    run_distributed(_gathered_params, 2)


def test_offload_reload_states_roundtrip():
    """engine.offload_states()/reload_states() (reference tests/unit/runtime/zero/test_offload_states.py):
    training continues bit-identically after a full offload/reload cycle."""
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny

    def run(cycle):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(**TINY))
        cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
               "zero_optimization": {"stage": 3}}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        g = torch.Generator().manual_seed(1)
        out = []
        for i in range(4):
            x = torch.randint(0, 97, (2, 12), generator=g)
            loss = eng(x, labels=x)
            eng.backward(loss)
            eng.step()
            out.append(float(loss))
            if cycle and i == 1:
                eng.offload_states()
                assert eng.optimizer.store.master.numel() == 0 and eng.optimizer.store.lp.numel() == 0
                eng.reload_states()
        return out

    import os
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=os.environ.get("MASTER_PORT", "29611"))
    assert run(True) == run(False)


def test_flops_profiler_counts_gemms_and_attention():
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.profiling.flops_profiler import FlopsProfiler, get_model_profile
    torch.manual_seed(0)
    cfg = tiny(**TINY)
    m = LlamaForCausalLM(cfg).eval()  # get_model_profile below profiles in eval mode too
    x = torch.randint(0, 97, (2, 12))
    with torch.no_grad():
        m(x)  # warm-up: the first forward also builds the RoPE tables (get_model_profile warms up too)
    prof = FlopsProfiler(m)
    prof.start_profile()
    with torch.no_grad():
        m(x)
    flops = prof.get_total_flops()
    prof.stop_profile()
    T, H, L = 24, cfg.hidden_size, cfg.num_hidden_layers
    per_layer_gemm = 2 * T * H * ((cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * cfg.head_dim +
                                  cfg.num_attention_heads * cfg.head_dim + 3 * cfg.intermediate_size)
    lm_head = 2 * T * H * cfg.vocab_size
    assert flops >= L * per_layer_gemm + lm_head
    assert m.model.layers[0].__flops__ >= per_layer_gemm
    assert prof.get_total_params() == sum(p.numel() for p in m.parameters())
    prof.print_model_profile(module_depth=2)
    prof.end_profile()
    f, macs, params = get_model_profile(m, args=[x], print_profile=False, as_string=False)
    assert f == flops


def _fragments(rank, world):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.utils import (safe_get_full_fp32_param, safe_get_full_grad, safe_get_full_optimizer_state,
                                            safe_get_local_fp32_param, safe_set_full_fp32_param)
    m, ref = _models()
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
           "zero_optimization": {"stage": 3}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    x = torch.randint(0, 97, (world * 2, 12), generator=torch.Generator().manual_seed(0))
    loss = eng(x[rank * 2:(rank + 1) * 2], labels=x[rank * 2:(rank + 1) * 2])
    eng.backward(loss)
    rl = ref(x, labels=x)
    rl.backward()
    rp = dict(ref.named_parameters())
    for name, p in m.named_parameters():
        g = safe_get_full_grad(p)
        assert torch.allclose(g, rp[name].grad, atol=1e-5, rtol=1e-4), name
        assert torch.allclose(safe_get_full_fp32_param(p), rp[name].detach(), atol=1e-6), name
    eng.step()
    name, p = next(iter(m.named_parameters()))
    ea = safe_get_full_optimizer_state(p, "exp_avg")
    assert ea.shape == p.ds_shape and ea.abs().sum() > 0
    new = torch.full(p.ds_shape, 0.25)
    safe_set_full_fp32_param(p, new)
    assert torch.allclose(safe_get_full_fp32_param(p), new)
    loc = safe_get_local_fp32_param(p)
    assert loc is None or torch.allclose(loc, torch.full_like(loc, 0.25))


def test_safe_get_set_tensor_fragments_world2():
    run_distributed(_fragments, 2)


def _released_memory(rank, world):
    """ZeRO-3 with memory-efficient linears: a layer's gathered weights are actually freed after its forward
    (the autograd graph must not pin them), and training still matches the non-partitioned trajectory."""
    import gc
    import weakref
    import hcache_deepspeed_amd as ds
    m, ref = _models()
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
           "zero_optimization": {"stage": 3}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    z = eng.optimizer
    refs = []
    orig = z._release

    def spy(u):
        if u.full is not None and not z.in_backward:
            refs.append(weakref.ref(u.full))
        orig(u)

    z._release = spy
    x = torch.randint(0, 97, (2, 12), generator=torch.Generator().manual_seed(rank))
    loss = eng(x, labels=x)
    gc.collect()
    assert refs, "no unit was released during forward"
    alive = sum(r() is not None for r in refs)
    assert alive == 0, f"{alive}/{len(refs)} released unit buffers are still referenced"
    eng.backward(loss)
    eng.step()


def test_zero3_releases_gathered_weights_world2():
    run_distributed(_released_memory, 2)


@pytest.mark.parametrize("world,stage,zinit", [(4, 3, False), (3, 3, True), (4, 1, False)])
def test_zero_world3_4(world, stage, zinit):
    """More ranks than the default harness (uneven shard padding at world 3, 4-way reduce-scatter / all-gather):
    the flat-shard collectives used at 8 GPUs, rehearsed on gloo."""
    run_distributed(_zero_vs_torch, world, stage, 1, zinit)


class _WgradToy(torch.nn.Module):
    """Linears used normally, one also used through F.linear outside its forward, one skipped on odd steps."""

    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(16, 32)
        self.b = torch.nn.Linear(32, 32, bias=False)
        self.skip = torch.nn.Linear(32, 32)
        self.out = torch.nn.Linear(32, 4)
        self.odd = False

    def forward(self, x, y):
        h = torch.tanh(self.a(x))
        h = torch.tanh(self.b(h)) + 0.5 * torch.nn.functional.linear(h, self.b.weight)  # shared use
        if not self.odd:
            h = h + self.skip(h)
        return torch.nn.functional.mse_loss(self.out(h), y)


def _direct_wgrad_equiv(rank, world, stage, gas):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.runtime.zero import linear as zl
    finals, writes = [], []
    for direct in (True, False):
        torch.manual_seed(0)
        m = _WgradToy()
        cfg = {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": gas,
               "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
               "zero_optimization": {"stage": stage}, "mi355x": {"direct_wgrad": direct}}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        n = [0]
        orig = zl.write_weight_grad

        def counting(w, compute):
            ok = orig(w, compute)
            n[0] += ok
            return ok

        zl.write_weight_grad = counting
        try:
            g = torch.Generator().manual_seed(7 + rank)
            for it in range(4 * gas):
                m.odd = bool((it // gas) % 2)
                x, y = torch.randn(4, 16, generator=g), torch.randn(4, 4, generator=g)
                eng.backward(eng(x, y))
                eng.step()
        finally:
            zl.write_weight_grad = orig
        finals.append(eng.optimizer.full_fp32_state_dict(eng._param_names))
        writes.append(n[0])
    assert writes[0] > 0 and writes[1] == 0, writes
    for k in finals[0]:
        assert torch.allclose(finals[0][k], finals[1][k], atol=1e-6, rtol=1e-5), (stage, k)


@pytest.mark.parametrize("stage,gas", [(1, 2), (2, 1), (2, 2), (3, 1), (3, 2)])
def test_direct_wgrad_matches_autograd_world2(stage, gas):
    run_distributed(_direct_wgrad_equiv, 2, stage, gas)


def test_overlapped_step_piece_plan():
    """The overlapped step's update order: root units first, then the recorded forward order, then the rest; one
    piece per (unit, parameter group) overlap; store ranges no unit covers trail. Every element exactly once."""
    from types import SimpleNamespace as NS
    from hcache_deepspeed_amd.runtime.zero.optimizer import ZeroOptimizer
    units = [NS(uid=i, store_off=off, shard=n) for i, (off, n) in enumerate([(0, 10), (10, 20), (30, 5), (40, 8)])]
    segs = [NS(store_off=0, numel=25, group=0), NS(store_off=25, numel=25, group=1)]  # [35, 40) and [48, 50): no unit
    opt = NS(units=units, root_units=[units[3]], _fwd_trace=[2, 0, 2], store=NS(segments=segs))
    pieces = ZeroOptimizer._step_pieces(opt)
    assert [(p[0], p[1], p[2]) for p in pieces] == [(3, 40, 48), (2, 30, 35), (0, 0, 10), (1, 10, 25), (1, 25, 30),
                                                   (None, 35, 40), (None, 48, 50)]
    hit = torch.zeros(50, dtype=torch.int32)
    for _, lo, hi, sg in pieces:
        assert sg.store_off <= lo < hi <= sg.store_off + sg.numel
        hit[lo:hi] += 1
    assert bool((hit == 1).all())
    assert ZeroOptimizer._step_pieces(opt) is pieces  # cached for the same forward trace
