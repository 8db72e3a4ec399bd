"""Per-shape GEMM census of one headline training step (Llama-3-8B, ZeRO-3, mb7 x 4096, bf16): torch.profiler with
input shapes, device time per (op, shapes), TFLOP/s per shape. Prints a table and writes JSON lines to argv[1]."""
import json
import os
import sys

os.environ.setdefault("DEBUG_CLR_LIMIT_BLIT_WG", "16")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import hcache_deepspeed_amd as hds  # noqa: E402
from hcache_deepspeed_amd.models import llama  # noqa: E402

out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gemm_census.jsonl"
mb, S = 7, 4096
os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29561")
hds.init_distributed(verbose=False)
cfg_model = llama.PRESETS["llama3-8b"]()
ds_config = {"train_micro_batch_size_per_gpu": mb, "bf16": {"enabled": True},
             "optimizer": {"type": "AdamW", "params": {"lr": 1e-4, "betas": [0.9, 0.95], "weight_decay": 0.1}},
             "gradient_clipping": 1.0, "zero_optimization": {"stage": 3}, "steps_per_print": 10**9}
with hds.zero.Init():
    model = llama.LlamaForCausalLM(cfg_model)
engine, _, _, _ = hds.initialize(model=model, config=ds_config)
gen = torch.Generator(device="cuda")
gen.manual_seed(0)


def step():
    x = torch.randint(0, cfg_model.vocab_size, (mb, S), device="cuda", generator=gen)
    loss = engine(x, labels=x)
    engine.backward(loss)
    engine.step()


for _ in range(2):
    step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
rows = []
for e in prof.key_averages(group_by_input_shape=True):
    name = e.key
    if not any(k in name for k in ("aten::mm", "aten::addmm", "aten::bmm", "aten::baddbmm", "aten::matmul",
                                   "aten::linear", "aten::_scaled_mm")):
        continue
    dev_us = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
    if dev_us <= 0:
        continue
    shapes = e.input_shapes
    flops = None
    try:
        a, b = shapes[0], shapes[1]
        if name in ("aten::mm",) and len(a) == 2 and len(b) == 2:
            flops = 2 * a[0] * a[1] * b[1]
        elif name == "aten::addmm" and len(shapes) >= 3:
            m1, m2 = shapes[1], shapes[2]
            flops = 2 * m1[0] * m1[1] * m2[1]
        elif name in ("aten::bmm", "aten::baddbmm"):
            x, y = (shapes[0], shapes[1]) if name == "aten::bmm" else (shapes[1], shapes[2])
            flops = 2 * x[0] * x[1] * x[2] * y[2]
    except Exception:  # noqa: BLE001
        pass
    rec = {"op": name, "shapes": shapes, "calls": e.count, "device_ms": round(dev_us / 1e3, 3)}
    if flops:
        rec["tflops"] = round(flops * e.count / (dev_us * 1e-6) / 1e12, 1)
    rows.append(rec)
rows.sort(key=lambda r: -r["device_ms"])
tot = sum(r["device_ms"] for r in rows if r["op"] in ("aten::mm", "aten::addmm", "aten::bmm", "aten::baddbmm"))
os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
with open(out_path, "w") as f:
    for r in rows:
        f.write(json.dumps(r) + "\n")
print(f"GEMM device time (mm/addmm/bmm) {tot:.1f} ms")
for r in rows[:40]:
    print(r)
# all kernels of the step, for the share table
ka = sorted(prof.key_averages(), key=lambda e: -(getattr(e, "device_self_time_total", 0) or 0))
print("top kernels by self device time:")
for e in ka[:25]:
    print(f"{(getattr(e, 'device_self_time_total', 0) or 0) / 1e3:9.2f} ms  {e.count:5d}x  {e.key[:110]}")
