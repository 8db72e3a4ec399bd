"""Diffusers / Megatron-GPT(-MoE) / InternLM injection containers against the modules they replace.

The families' libraries (diffusers, Megatron-LM, InternLM remote code) are not installed here; the tests build
minimal modules with the same attribute layout and forward semantics (parity unpinned against the real libraries,
which cannot be imported in this environment) and check the injected path reproduces their outputs on the CPU
reference ops. The HIP-graph replay path is covered by the GPU test at the end."""
import math

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F


# ---------------------------------------------------------------------------------------------------------------
# Megatron GPT layer (sequence-first)
# ---------------------------------------------------------------------------------------------------------------
class _MegAttn(nn.Module):

    def __init__(self, h, nh):
        super().__init__()
        self.query_key_value = nn.Linear(h, 3 * h)
        self.dense = nn.Linear(h, h)
        self.num_attention_heads = nh


class _MegMLP(nn.Module):

    def __init__(self, h):
        super().__init__()
        self.dense_h_to_4h = nn.Linear(h, 4 * h)
        self.dense_4h_to_h = nn.Linear(4 * h, h)


class _MegLayer(nn.Module):

    def __init__(self, h=64, nh=4, post_ln_residual=False):
        super().__init__()
        self.input_layernorm = nn.LayerNorm(h)
        self.self_attention = _MegAttn(h, nh)
        self.post_attention_layernorm = nn.LayerNorm(h)
        self.mlp = _MegMLP(h)
        self.apply_residual_connection_post_layernorm = post_ln_residual

    def forward(self, x, mask=None):  # x [s, b, h]
        s, b, h = x.shape
        nh = self.self_attention.num_attention_heads
        d = h // nh
        ln = self.input_layernorm(x)
        qkv = self.self_attention.query_key_value(ln).view(s, b, nh, 3, d)
        q, k, v = (qkv[..., i, :].permute(1, 2, 0, 3) for i in range(3))
        att = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        a = self.self_attention.dense(att.permute(2, 0, 1, 3).reshape(s, b, h))
        res = ln if self.apply_residual_connection_post_layernorm else x
        li = res + a
        lo = self.post_attention_layernorm(li)
        res = lo if self.apply_residual_connection_post_layernorm else li
        return res + self.mlp.dense_4h_to_h(F.gelu(self.mlp.dense_h_to_4h(lo)))


@pytest.mark.parametrize("post_ln_residual", [False, True])
def test_megatron_gpt_block_matches_layer(post_ln_residual):
    from hcache_deepspeed_amd.inference.injection import inject
    from hcache_deepspeed_amd.inference.megatron import DSMegatronGPTBlock
    torch.manual_seed(0)
    model = nn.Sequential(_MegLayer(post_ln_residual=post_ln_residual), _MegLayer(post_ln_residual=post_ln_residual))
    x = torch.randn(10, 3, 64)
    with torch.no_grad():
        ref = model(x)
    assert inject(model) >= 2
    assert all(isinstance(m, DSMegatronGPTBlock) for m in model)
    got = model(x)
    torch.testing.assert_close(got, ref, atol=2e-4, rtol=2e-4)
    # incremental decoding with the block's KV cache equals the full forward
    for blk in model:
        blk.reset_cache()
    outs = []
    h = x[:6]
    for blk in model:
        h = blk(h, use_cache=True)
    outs.append(h)
    for t in range(6, 10):
        h = x[t:t + 1]
        for blk in model:
            h = blk(h, use_cache=True)
        outs.append(h)
    torch.testing.assert_close(torch.cat(outs, 0), ref, atol=2e-4, rtol=2e-4)
    # the cache is one preallocated buffer per layer (tokens written in place), not a concatenation per token
    blk = model[0]
    assert blk.kv_len == 10 and blk.kc.shape[2] >= 256 and blk.kv[0].shape[2] == 10


class _MoEMLP(nn.Module):
    """Megatron-DeepSpeed MoE MLP shape: ``deepspeed_moe.experts`` present, returns (out, l_aux, counts)."""

    def __init__(self, h):
        super().__init__()
        self.deepspeed_moe = nn.Module()
        self.deepspeed_moe.experts = nn.ModuleList([_MegMLP(h)])
        self.w = nn.Linear(h, h)

    def forward(self, x):
        return self.w(x), torch.zeros(()), None


def test_megatron_gpt_moe_block_keeps_expert_path():
    from hcache_deepspeed_amd.inference.megatron import DSMegatronGPTBlock, inject_megatron_layers
    torch.manual_seed(0)
    layer = _MegLayer()
    layer.mlp = _MoEMLP(64)
    x = torch.randn(5, 2, 64)
    with torch.no_grad():
        s, b, h = x.shape
        ln = layer.input_layernorm(x)
        qkv = layer.self_attention.query_key_value(ln).view(s, b, 4, 3, 16)
        q, k, v = (qkv[..., i, :].permute(1, 2, 0, 3) for i in range(3))
        a = layer.self_attention.dense(F.scaled_dot_product_attention(q, k, v, is_causal=True)
                                       .permute(2, 0, 1, 3).reshape(s, b, h))
        li = x + a
        ref = li + layer.mlp(layer.post_attention_layernorm(li))[0]
    model = nn.Sequential(layer)
    assert inject_megatron_layers(model) == 1 and isinstance(model[0], DSMegatronGPTBlock)
    assert model[0].moe is layer.mlp
    torch.testing.assert_close(model(x), ref, atol=2e-4, rtol=2e-4)


# ---------------------------------------------------------------------------------------------------------------
# InternLM attention
# ---------------------------------------------------------------------------------------------------------------
class _Rotary(nn.Module):

    def __init__(self, d, base=10000):
        super().__init__()
        self.inv = 1.0 / (base**(torch.arange(0, d, 2).float() / d))

    def forward(self, x, seq_len):
        t = torch.arange(seq_len).float()
        f = torch.outer(t, self.inv)
        emb = torch.cat([f, f], -1)
        return emb.cos()[None, None], emb.sin()[None, None]


class InternLMAttention(nn.Module):

    def __init__(self, h=64, nh=4):
        super().__init__()
        self.num_heads, self.head_dim = nh, h // nh
        self.q_proj, self.k_proj, self.v_proj = (nn.Linear(h, h) for _ in range(3))
        self.o_proj = nn.Linear(h, h)
        self.rotary_emb = _Rotary(h // nh)

    def forward(self, x, attention_mask=None, position_ids=None, past_key_value=None, output_attentions=False,
                use_cache=False):
        B, S, _ = x.shape
        nh, d = self.num_heads, self.head_dim
        q, k, v = (p(x).view(B, S, nh, d).transpose(1, 2) for p in (self.q_proj, self.k_proj, self.v_proj))
        cos, sin = self.rotary_emb(v, S)
        cos, sin = cos[0, 0][:S], sin[0, 0][:S]
        rot = lambda t: torch.cat((-t[..., d // 2:], t[..., :d // 2]), -1)  # noqa: E731
        q, k = q * cos + rot(q) * sin, k * cos + rot(k) * sin
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return self.o_proj(o.transpose(1, 2).reshape(B, S, nh * d)), None, None


def test_internlm_attention_container():
    from hcache_deepspeed_amd.inference.megatron import inject_internlm
    torch.manual_seed(0)
    m = nn.ModuleList([InternLMAttention()])
    x = torch.randn(2, 9, 64)
    with torch.no_grad():
        ref = m[0](x)[0]
        assert inject_internlm(m) == 1
        got, _, past = m[0](x, use_cache=True)
    torch.testing.assert_close(got, ref, atol=2e-4, rtol=2e-4)
    assert past[0].shape == (2, 4, 9, 16)


class InternLM2Attention(nn.Module):
    """InternLM2 remote-code layout: fused ``wqkv`` per kv head [q_per_kv query heads, k, v] x head_dim, GQA."""

    def __init__(self, h=64, nh=4, nkv=2):
        super().__init__()
        self.num_heads, self.head_dim, self.num_key_value_heads = nh, h // nh, nkv
        self.num_key_value_groups = nh // nkv
        self.wqkv = nn.Linear(h, (nh + 2 * nkv) * (h // nh), bias=False)
        self.wo = nn.Linear(h, h, bias=False)
        self.rotary_emb = _Rotary(h // nh)

    def forward(self, x, attention_mask=None, position_ids=None, past_key_value=None, output_attentions=False,
                use_cache=False):
        B, S, _ = x.shape
        nh, d, nkv, g = self.num_heads, self.head_dim, self.num_key_value_heads, self.num_key_value_groups
        qkv = self.wqkv(x).view(B, S, nkv, g + 2, d)
        q = qkv[..., :g, :].reshape(B, S, nh, d).transpose(1, 2)
        k, v = qkv[..., -2, :].transpose(1, 2), qkv[..., -1, :].transpose(1, 2)
        cos, sin = self.rotary_emb(v, S)
        cos, sin = cos[0, 0][:S], sin[0, 0][:S]
        rot = lambda t: torch.cat((-t[..., d // 2:], t[..., :d // 2]), -1)  # noqa: E731
        q, k = q * cos + rot(q) * sin, k * cos + rot(k) * sin
        k, v = k.repeat_interleave(g, 1), v.repeat_interleave(g, 1)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return self.wo(o.transpose(1, 2).reshape(B, S, nh * d)), None, None


def test_internlm2_wqkv_attention_container():
    from hcache_deepspeed_amd.inference.megatron import inject_internlm
    torch.manual_seed(0)
    m = nn.ModuleList([InternLM2Attention()])
    x = torch.randn(2, 9, 64)
    with torch.no_grad():
        ref = m[0](x)[0]
        assert inject_internlm(m) == 1
        got, _, past = m[0](x, use_cache=True)
        # incremental: 8 tokens then the 9th against the returned cache
        o8, _, p8 = m[0](x[:, :8], use_cache=True)
        o9, _, _ = m[0](x[:, 8:], past_key_value=p8, position_ids=torch.tensor([[8], [8]]), use_cache=True)
    torch.testing.assert_close(got, ref, atol=2e-4, rtol=2e-4)
    torch.testing.assert_close(o9, ref[:, 8:], atol=2e-4, rtol=2e-4)
    assert past[0].shape == (2, 2, 9, 16)  # GQA: the cache holds the 2 kv heads


# ---------------------------------------------------------------------------------------------------------------
# diffusers-style attention + UNet / VAE wrappers
# ---------------------------------------------------------------------------------------------------------------
class _RefProc:

    def __call__(self, attn, h, encoder_hidden_states=None, attention_mask=None, temb=None):
        ctx = h if encoder_hidden_states is None else encoder_hidden_states
        B, S, _ = h.shape
        q, k, v = attn.to_q(h), attn.to_k(ctx), attn.to_v(ctx)
        nh = attn.heads
        d = q.shape[-1] // nh
        sh = lambda t: t.view(B, -1, nh, d).transpose(1, 2)  # noqa: E731
        o = F.scaled_dot_product_attention(sh(q), sh(k), sh(v)).transpose(1, 2).reshape(B, S, nh * d)
        return attn.to_out[1](attn.to_out[0](o))


class Attention(nn.Module):

    def __init__(self, dim, heads, cross_dim=None):
        super().__init__()
        self.heads = heads
        self.scale = (dim // heads)**-0.5
        self.to_q = nn.Linear(dim, dim, bias=False)
        self.to_k = nn.Linear(cross_dim or dim, dim, bias=False)
        self.to_v = nn.Linear(cross_dim or dim, dim, bias=False)
        self.to_out = nn.ModuleList([nn.Linear(dim, dim), nn.Dropout(0.0)])
        self.processor = _RefProc()

    def set_processor(self, p):
        self.processor = p

    def forward(self, h, encoder_hidden_states=None, attention_mask=None):
        return self.processor(self, h, encoder_hidden_states=encoder_hidden_states, attention_mask=attention_mask)


class _TinyUNet(nn.Module):

    def __init__(self):
        super().__init__()
        self.in_channels = 4
        self.config = {"in_channels": 4}
        self.conv_in = nn.Conv2d(4, 32, 1)
        self.down_blocks = nn.ModuleList([Attention(32, 2)])
        self.up_blocks = nn.ModuleList([Attention(32, 2, cross_dim=16)])
        self.conv_out = nn.Conv2d(32, 4, 1)

    def forward(self, sample, timestep, encoder_hidden_states, return_dict=True):
        B, _, H, W = sample.shape
        x = self.conv_in(sample) * (1 + timestep.float().view(-1, 1, 1, 1) / 1000)
        t = x.flatten(2).transpose(1, 2)
        t = t + self.down_blocks[0](t)
        t = t + self.up_blocks[0](t, encoder_hidden_states=encoder_hidden_states)
        out = self.conv_out(t.transpose(1, 2).reshape(B, 32, H, W))
        return {"sample": out} if return_dict else (out, )


def test_unet_wrapper_and_attention_processor():
    from hcache_deepspeed_amd.inference.diffusers import DSUNet, HDSAttnProcessor, inject_pipeline
    torch.manual_seed(0)
    unet = _TinyUNet()
    s, t, ctx = torch.randn(2, 4, 6, 6), torch.tensor([10, 500]), torch.randn(2, 7, 16)
    with torch.no_grad():
        ref = unet(s, t, ctx)["sample"]

    class Pipe:
        pass

    pipe = Pipe()
    pipe.unet = unet
    assert inject_pipeline(pipe) == ["unet"]
    w = pipe.unet
    assert isinstance(w, DSUNet) and w.in_channels == 4 and w.n_attention == 2
    assert all(isinstance(a.processor, HDSAttnProcessor) for a in (unet.down_blocks[0], unet.up_blocks[0]))
    assert unet.down_blocks[0]._hds_qkv_w is not None and unet.up_blocks[0]._hds_qkv_w is None  # cross-attn: no fuse
    torch.testing.assert_close(w(s, t, ctx)["sample"], ref, atol=2e-5, rtol=2e-5)


@pytest.mark.gpu
def test_graphed_callable_replays_new_inputs_gpu():
    """HIP-graph wrapper: replays give the eager results for new inputs, one graph per input signature."""
    from hcache_deepspeed_amd.inference.diffusers import DSUNet
    torch.manual_seed(0)
    unet = _TinyUNet().cuda()
    w = DSUNet(unet)
    for B in (2, 2, 1, 2):
        s, t, ctx = torch.randn(B, 4, 6, 6, device="cuda"), torch.randint(0, 999, (B, ), device="cuda"), \
            torch.randn(B, 7, 16, device="cuda")
        with torch.no_grad():
            ref = unet(s, t, ctx)["sample"].clone()
        got = w(s, t, ctx)["sample"]
        torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)
    assert len(w._graph.graphs) == 2
