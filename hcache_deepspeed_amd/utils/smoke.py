"""One tiny forward+backward+step of the flagship path (Llama architecture, ZeRO-3 engine, HIP kernels)."""
import os


def run_smoke():
    import torch
    import hcache_deepspeed_amd as hds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    cfg = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True},
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "zero_optimization": {"stage": 3},
           "gradient_clipping": 1.0}
    with hds.zero.Init():
        model = LlamaForCausalLM(tiny())
    engine, _, _, _ = hds.initialize(model=model, config=cfg)
    x = torch.randint(0, 512, (2, 256), device=engine.device)
    losses = []
    for _ in range(3):
        loss = engine(x, labels=x)
        engine.backward(loss)
        engine.step()
        losses.append(float(loss.item()))
    torch.cuda.synchronize()
    assert all(l == l for l in losses), losses
    assert losses[-1] < losses[0], losses
    print(f"smoke ok: losses {losses}")
    return losses
