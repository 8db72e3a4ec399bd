"""Which ATen ops (and with what shapes) launch the copy / fill kernels of one training step?

Runs the headline model at full width with ``--layers`` layers (2 by default) through the ZeRO-3 engine, then
records one further step under a TorchDispatchMode and prints the copy-like / fill-like ops by (op, shapes, dtypes)
with counts and the Python frame (file:line inside hcache_deepspeed_amd) that issued them."""
import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, ".")

WATCH = ("copy_", "fill_", "zero_", "clone", "cat", "_to_copy", "contiguous", "index_copy", "new_zeros", "zeros",
         "full", "fill", "add_", "add", "mul", "sum", "where", "masked_fill", "ones")


class Census(TorchDispatchMode):

    def __init__(self):
        super().__init__()
        self.rows = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__ if hasattr(func, "__name__") else str(func)
        base = str(func.overloadpacket.__name__) if hasattr(func, "overloadpacket") else name
        if any(base == w or base.startswith(w) for w in WATCH):
            shapes = tuple(tuple(a.shape) for a in args if isinstance(a, torch.Tensor))
            dts = tuple(str(a.dtype).replace("torch.", "") for a in args if isinstance(a, torch.Tensor))
            where = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if "hcache_deepspeed_amd" in fr.filename:
                    where = f"{os.path.relpath(fr.filename)}:{fr.lineno}"
                    break
            self.rows[(base, shapes, dts, where)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--mb", type=int, default=7)
    args = ap.parse_args()
    import hcache_deepspeed_amd as hds
    from hcache_deepspeed_amd.models import llama
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29561")
    hds.init_distributed(verbose=False)
    with hds.zero.Init():
        m = llama.LlamaForCausalLM(llama.llama3_8b(num_hidden_layers=args.layers))
    cfg = {"train_micro_batch_size_per_gpu": args.mb, "bf16": {"enabled": True}, "gradient_clipping": 1.0,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-4}}, "zero_optimization": {"stage": 3}}
    eng, _, _, _ = hds.initialize(model=m, config=cfg)
    dev = eng.device
    for _ in range(2):
        x = torch.randint(0, 128256, (args.mb, 4096), device=dev)
        eng.backward(eng(x, labels=x))
        eng.step()
    torch.cuda.synchronize()
    c = Census()
    x = torch.randint(0, 128256, (args.mb, 4096), device=dev)
    with c:
        eng.backward(eng(x, labels=x))
        eng.step()
    torch.cuda.synchronize()
    for (op, shp, dts, where), n in sorted(c.rows.items(), key=lambda kv: -kv[1]):
        print(f"{n:5d}  {op:14s} {where:55s} {dts} {shp}")


if __name__ == "__main__":
    main()
