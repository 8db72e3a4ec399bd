"""init_inference AutoTP = 2 with kernel injection on the HIP device path, both ranks on the one MI355X of the test
box (gloo rendezvous; RCCL refuses two ranks on one device). The row-parallel all-reduces of the injected blocks
are small and take the symmetric one-shot all-reduce (IPC-mapped buffers of the other process); the sharded
projections and the injected attention / norm / activation kernels run on the GPU. Logits must match the unsharded
HF model in bf16."""
import os

import pytest
import torch

from tests.dist_utils import run_distributed

pytestmark = pytest.mark.gpu


def _model():
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                      num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=512)
    return LlamaForCausalLM(cfg).eval()


def _run(rank, world, d):
    import hcache_deepspeed_amd as ds
    torch.cuda.set_device(0)
    ref = _model().cuda().to(torch.bfloat16)
    x = torch.randint(0, 512, (2, 128), generator=torch.Generator().manual_seed(1)).cuda()
    with torch.no_grad():
        want = ref(x).logits.float()
    del ref
    eng = ds.init_inference(_model(), dtype=torch.bfloat16, replace_with_kernel_inject=True,
                            tensor_parallel={"tp_size": world})
    with torch.no_grad():
        got = eng(x).logits.float()
    from hcache_deepspeed_amd.comm import symmetric
    assert sum(sm.calls["all_reduce"] for sm in symmetric._cache.values()) > 0, "no one-shot all-reduce ran"
    rel = float((got - want).norm() / want.norm())
    torch.save({"rel": rel}, os.path.join(d, f"r{rank}.pt"))
    assert rel < 3e-2, rel


def test_autotp_inference_kernel_inject_device_path_world2():
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        run_distributed(_run, 2, d)
        rels = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)["rel"] for r in range(2)]
    assert max(rels) < 3e-2, rels
