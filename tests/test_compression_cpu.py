"""Compression library: QAT fake-quant, sparse/row/head pruning, redundancy_clean dimension reduction, layer
reduction and the engine's compression scheduler.

Reference test analogue: tests/unit/compression/test_compression.py (init_compression on a BERT-like model,
checks module replacement, masks and redundancy_clean shapes). Parity: masked forward before clean == shrunk
forward after clean; fake-quant equals the torch group-quant reference.
"""
import os

import torch
import torch.nn as nn

from hcache_deepspeed_amd.compression import (LinearLayer_Compress, compression_scheduler, get_compression_config,
                                              init_compression, redundancy_clean)


class Attn(nn.Module):

    def __init__(self, H=16, nh=4):
        super().__init__()
        self.q = nn.Linear(H, H)
        self.k = nn.Linear(H, H)
        self.v = nn.Linear(H, H)
        self.o = nn.Linear(H, H)
        self.nh = nh

    def forward(self, x):
        B, S, H = x.shape
        d = self.q.weight.shape[0] // self.nh

        def sp(t):
            return t.view(B, S, -1, d).transpose(1, 2)

        q, k, v = sp(self.q(x)), sp(self.k(x)), sp(self.v(x))
        a = torch.softmax(q @ k.transpose(-1, -2) / d**0.5, -1) @ v
        return self.o(a.transpose(1, 2).reshape(B, S, -1))


class Block(nn.Module):

    def __init__(self, H=16):
        super().__init__()
        self.attn = Attn(H)
        self.fc1 = nn.Linear(H, 4 * H)
        self.fc2 = nn.Linear(4 * H, H)

    def forward(self, x):
        x = x + self.attn(x)
        return x + self.fc2(torch.relu(self.fc1(x)))


class Net(nn.Module):

    def __init__(self, L=2, H=16):
        super().__init__()
        self.layers = nn.ModuleList([Block(H) for _ in range(L)])
        self.head = nn.Linear(H, 8)

    def forward(self, x):
        for b in self.layers:
            x = b(x)
        return self.head(x)


def _cfg(**tech):
    return {"compression_training": tech}


def test_weight_quantization_in_forward_and_ste():
    torch.manual_seed(0)
    m = Net()
    cfg = _cfg(weight_quantization={
        "shared_parameters": {"enabled": True, "quantize_weight_in_forward": True, "schedule_offset": 0,
                              "quantize_groups": 4},
        "different_groups": {"wq1": {"params": {"start_bits": 8, "target_bits": 8}, "modules": ["fc1", "fc2"]}}})
    init_compression(m, cfg)
    assert isinstance(m.layers[0].fc1, LinearLayer_Compress) and isinstance(m.layers[0].attn.q, LinearLayer_Compress)
    sch = compression_scheduler(m, get_compression_config(cfg))
    sch.step(step_zero_check=True)
    assert m.layers[0].fc1.weight_quantization_enabled and not m.layers[0].attn.q.weight_quantization_enabled
    fc1 = m.layers[0].fc1
    w_eff = fc1.effective_weight()
    g = fc1.weight.float().reshape(4, -1)
    sc = g.abs().amax(1, keepdim=True) / 127
    ref = (torch.clamp(torch.round(g / sc), -128, 127) * sc).view_as(fc1.weight)
    assert torch.allclose(w_eff, ref, atol=1e-6)
    x = torch.randn(2, 5, 16)
    m(x).sum().backward()
    assert fc1.weight.grad is not None and fc1.weight.grad.abs().sum() > 0


def test_sparse_pruning_l1_and_clean():
    torch.manual_seed(1)
    m = Net()
    cfg = _cfg(sparse_pruning={
        "shared_parameters": {"enabled": True, "method": "l1", "schedule_offset": 2},
        "different_groups": {"sp1": {"params": {"dense_ratio": 0.25}, "modules": ["fc"]}}})
    init_compression(m, cfg)
    sch = compression_scheduler(m, get_compression_config(cfg))
    sch.step(step_zero_check=True)
    assert not m.layers[0].fc1.sparse_pruning_enabled
    sch.step()
    sch.step()
    assert m.layers[0].fc1.sparse_pruning_enabled
    x = torch.randn(2, 5, 16)
    y_mask = m(x)
    redundancy_clean(m, cfg)
    w = m.layers[0].fc1.weight
    assert abs((w != 0).float().mean().item() - 0.25) < 0.02
    assert torch.allclose(m(x), y_mask, atol=1e-5)


def test_row_pruning_with_related_modules_shrinks():
    torch.manual_seed(2)
    m = Net()
    cfg = _cfg(row_pruning={
        "shared_parameters": {"enabled": True, "method": "l1", "schedule_offset": 0},
        "different_groups": {"rp1": {"params": {"dense_ratio": 0.5}, "modules": ["fc1"],
                                     "related_modules": [["fc2"]]}}})
    init_compression(m, cfg)
    compression_scheduler(m, get_compression_config(cfg)).step(step_zero_check=True)
    x = torch.randn(2, 5, 16)
    y_mask = m(x)
    redundancy_clean(m, cfg)
    assert m.layers[0].fc1.weight.shape == (32, 16) and m.layers[0].fc2.weight.shape == (16, 32)
    assert torch.allclose(m(x), y_mask, atol=1e-5)


def test_head_pruning_with_related_qkv_shrinks():
    torch.manual_seed(3)
    m = Net()
    cfg = _cfg(head_pruning={
        "shared_parameters": {"enabled": True, "method": "topk", "schedule_offset": 0, "num_heads": 4},
        "different_groups": {"hp1": {"params": {"dense_ratio": 0.5}, "modules": [r"attn\.o"],
                                     "related_modules": [[r"attn\.q", r"attn\.k", r"attn\.v"]]}}})
    init_compression(m, cfg)
    compression_scheduler(m, get_compression_config(cfg)).step(step_zero_check=True)
    for b in m.layers:
        b.attn.nh = 4
    x = torch.randn(2, 5, 16)
    y_mask = m(x)
    # the topk head scores are trainable
    y_mask.sum().backward()
    assert m.layers[0].attn.o.head_pruning_scores.grad is not None
    redundancy_clean(m, cfg)
    a = m.layers[0].attn
    assert a.o.weight.shape == (16, 8) and a.q.weight.shape == (8, 16) and a.v.bias.shape == (8, )
    for b in m.layers:
        b.attn.nh = 2
    assert torch.allclose(m(x), y_mask, atol=1e-5)


def test_layer_reduction_student_init():
    torch.manual_seed(4)
    teacher, student = Net(L=4), Net(L=2)
    cfg = _cfg(layer_reduction={"enabled": True, "keep_number_layer": 2, "module_name_prefix": "layers",
                                "teacher_layer": [1, 3], "other_module_name": ["head"]})
    init_compression(student, cfg, teacher_model=teacher)
    assert torch.equal(student.layers[0].fc1.weight, teacher.layers[1].fc1.weight)
    assert torch.equal(student.layers[1].attn.o.weight, teacher.layers[3].attn.o.weight)
    assert torch.equal(student.head.weight, teacher.head.weight)


def test_engine_drives_compression_scheduler():
    import hcache_deepspeed_amd as ds
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=os.environ.get("MASTER_PORT", "29643"))
    torch.manual_seed(5)
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
           **_cfg(activation_quantization={
               "shared_parameters": {"enabled": True, "schedule_offset": 2},
               "different_groups": {"aq1": {"params": {"bits": 8}, "modules": ["fc1"]}}})}
    model = init_compression(Net(), cfg)

    class Wrap(nn.Module):

        def __init__(self, net):
            super().__init__()
            self.net = net

        def forward(self, x, labels=None):
            return self.net(x).float().pow(2).mean()

    eng, _, _, _ = ds.initialize(model=Wrap(model), config=cfg)
    flags = []
    for _ in range(3):
        x = torch.randn(2, 5, 16)
        loss = eng(x)
        eng.backward(loss)
        eng.step()
        flags.append(model.layers[0].fc1.activation_quantization_enabled)
    assert flags == [False, True, True]
