"""Diffusion-model injection: HIP-graph UNet / VAE / CLIP-encoder wrappers and a fused attention processor.

Reference parity: deepspeed/model_implementations/diffusers/unet.py (``DSUNet``: channels-last, frozen, the whole
denoiser forward captured in a graph and replayed with new inputs), diffusers/vae.py (``DSVAE``: separate graphs for
``encode``, ``decode`` and ``forward``), model_implementations/transformers/clip_encoder.py (``DSClipEncoder``) and
module_inject/containers/{unet,vae,clip}.py (the policies that find those modules; ``UNetPolicy.attention`` fuses
the q/k/v projections of every diffusers ``Attention``).

MI355X design:
  * the graphs are HIP graphs (torch.cuda.CUDAGraph on ROCm), one per input signature (shape / dtype / non-tensor
    arguments), so a pipeline that alternates guidance batch sizes or resolutions keeps one graph per variant
    instead of silently replaying the wrong one (the reference captures exactly once);
  * ``HDSAttnProcessor`` replaces the diffusers attention processor: self-attention runs the HIP FlashAttention
    kernel (non-causal, head dims that are multiples of 16: SD-2 / SDXL 64, 128), q|k|v come from ONE fused GEMM
    when the projections share their input (the reference's ``UNetPolicy.attention`` qkv concatenation), and
    cross-attention / masked / odd-head-dim cases run fused SDPA.
diffusers itself is not a dependency: modules are recognised by their interface (duck typing on the attributes
diffusers' classes expose), so the wrappers work with any module that has it.
"""
import torch
import torch.nn.functional as F


# ---------------------------------------------------------------------------------------------------------------
# HIP-graph capture of one callable, keyed by the input signature
# ---------------------------------------------------------------------------------------------------------------
def _sig(x):
    if isinstance(x, torch.Tensor):
        return ("T", tuple(x.shape), x.dtype, x.device.type)
    if isinstance(x, (list, tuple)):
        return ("L", tuple(_sig(v) for v in x))
    if isinstance(x, dict):
        return ("D", tuple((k, _sig(v)) for k, v in sorted(x.items())))
    return ("O", repr(x))


def _clone_tree(x):
    if isinstance(x, torch.Tensor):
        return x.clone()
    if isinstance(x, (list, tuple)):
        return type(x)(_clone_tree(v) for v in x)
    if isinstance(x, dict):
        return {k: _clone_tree(v) for k, v in x.items()}
    return x


def _copy_tree(dst, src):
    if isinstance(dst, torch.Tensor):
        dst.copy_(src)
    elif isinstance(dst, (list, tuple)):
        for d, s in zip(dst, src):
            _copy_tree(d, s)
    elif isinstance(dst, dict):
        for k in dst:
            _copy_tree(dst[k], src[k])


class GraphedCallable:
    """``fn(*args, **kwargs)`` replayed from a HIP graph captured on the first call of each input signature (three
    warm-up runs on a side stream first, as the reference does, so lazy library state is not captured)."""

    def __init__(self, fn, enabled=True, warmup=3):
        self.fn = fn
        self.enabled = enabled
        self.warmup = warmup
        self.graphs = {}
        self.pool = None

    def __call__(self, *args, **kwargs):
        if not (self.enabled and torch.cuda.is_available() and any(
                isinstance(a, torch.Tensor) and a.is_cuda for a in list(args) + list(kwargs.values()))):
            return self.fn(*args, **kwargs)
        key = _sig((args, kwargs))
        ent = self.graphs.get(key)
        if ent is None:
            s_args, s_kwargs = _clone_tree(list(args)), _clone_tree(dict(kwargs))
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(self.warmup):
                    self.fn(*s_args, **s_kwargs)
            torch.cuda.current_stream().wait_stream(side)
            if self.pool is None:
                self.pool = torch.cuda.graph_pool_handle()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self.pool):
                out = self.fn(*s_args, **s_kwargs)
            ent = self.graphs[key] = (g, s_args, s_kwargs, out)
        g, s_args, s_kwargs, out = ent
        _copy_tree(s_args, list(args))
        _copy_tree(s_kwargs, dict(kwargs))
        g.replay()
        return out


# ---------------------------------------------------------------------------------------------------------------
# attention processor
# ---------------------------------------------------------------------------------------------------------------
def _is_diffusers_attention(m):
    return all(hasattr(m, a) for a in ("to_q", "to_k", "to_v", "to_out", "heads")) and hasattr(m, "set_processor")


class HDSAttnProcessor:
    """diffusers ``Attention`` processor on this framework's kernels (see the module docstring)."""

    def _qkv(self, attn, h, ctx):
        if ctx is h and getattr(attn, "_hds_qkv_w", None) is not None:
            qkv = F.linear(h, attn._hds_qkv_w, attn._hds_qkv_b)
            return qkv.chunk(3, dim=-1)
        return attn.to_q(h), attn.to_k(ctx), attn.to_v(ctx)

    def __call__(self, attn, hidden_states, encoder_hidden_states=None, attention_mask=None, temb=None, *args,
                 **kwargs):
        from ..ops.attention import flash_attn, head_dim_supported
        residual = hidden_states
        if getattr(attn, "spatial_norm", None) is not None:
            hidden_states = attn.spatial_norm(hidden_states, temb)
        nd = hidden_states.dim()
        if nd == 4:
            B, C, Hh, Ww = hidden_states.shape
            hidden_states = hidden_states.view(B, C, Hh * Ww).transpose(1, 2)
        B, S, _ = hidden_states.shape
        if getattr(attn, "group_norm", None) is not None:
            hidden_states = attn.group_norm(hidden_states.transpose(1, 2)).transpose(1, 2)
        ctx = hidden_states if encoder_hidden_states is None else encoder_hidden_states
        if encoder_hidden_states is not None and getattr(attn, "norm_cross", None):
            ctx = attn.norm_encoder_hidden_states(ctx)
        q, k, v = self._qkv(attn, hidden_states, ctx)
        nh = attn.heads
        D = q.shape[-1] // nh
        Skv = k.shape[1]
        scale = getattr(attn, "scale", D**-0.5)
        q4, k4, v4 = q.view(B, S, nh, D), k.view(B, Skv, nh, D), v.view(B, Skv, nh, D)
        if (attention_mask is None and ctx is hidden_states and q.is_cuda and q.dtype == torch.bfloat16
                and head_dim_supported(D)):
            o = flash_attn(q4.contiguous(), k4.contiguous(), v4.contiguous(), causal=False, softmax_scale=scale)
        else:
            mask = None
            if attention_mask is not None:
                mask = attn.prepare_attention_mask(attention_mask, Skv, B) if hasattr(attn, "prepare_attention_mask") \
                    else attention_mask
                mask = mask.view(B, -1, mask.shape[-2], mask.shape[-1])
            o = F.scaled_dot_product_attention(q4.transpose(1, 2), k4.transpose(1, 2), v4.transpose(1, 2),
                                               attn_mask=mask, scale=scale).transpose(1, 2)
        o = o.reshape(B, S, nh * D).to(q.dtype)
        o = attn.to_out[0](o)
        if len(attn.to_out) > 1:
            o = attn.to_out[1](o)
        if nd == 4:
            o = o.transpose(-1, -2).reshape(B, C, Hh, Ww)
        if getattr(attn, "residual_connection", False):
            o = o + residual
        return o / getattr(attn, "rescale_output_factor", 1.0)


def fuse_attention_qkv(attn):
    """UNetPolicy.attention: one [3*inner, in] weight when to_q / to_k / to_v read the same input width."""
    qw, kw, vw = attn.to_q.weight, attn.to_k.weight, attn.to_v.weight
    if qw.shape[1] != kw.shape[1] or kw.shape != vw.shape or qw.shape != kw.shape:
        attn._hds_qkv_w = None
        return False
    attn._hds_qkv_w = torch.cat([qw, kw, vw], 0).detach()
    bs = [getattr(m, "bias", None) for m in (attn.to_q, attn.to_k, attn.to_v)]
    attn._hds_qkv_b = torch.cat(bs, 0).detach() if all(b is not None for b in bs) else None
    return True


def inject_attention_processors(module):
    """Put ``HDSAttnProcessor`` on every diffusers-style attention module under ``module``; returns the count."""
    proc = HDSAttnProcessor()
    n = 0
    for m in module.modules():
        if _is_diffusers_attention(m):
            fuse_attention_qkv(m)
            m.set_processor(proc)
            n += 1
    return n


# ---------------------------------------------------------------------------------------------------------------
# UNet / VAE / CLIP wrappers
# ---------------------------------------------------------------------------------------------------------------
class DSUNet(torch.nn.Module):
    """Frozen, channels-last denoiser whose forward replays a HIP graph (reference diffusers/unet.py ``DSUNet``)."""

    def __init__(self, unet, enable_cuda_graph=True):
        super().__init__()
        self.unet = unet
        self.in_channels = getattr(unet, "in_channels", None)  # the SD pipeline reads these
        self.config = getattr(unet, "config", None)
        self.unet.requires_grad_(False)
        self.unet.to(memory_format=torch.channels_last)
        self.n_attention = inject_attention_processors(unet)
        self._graph = GraphedCallable(self._forward, enabled=enable_cuda_graph)
        self.enable_cuda_graph = enable_cuda_graph

    @property
    def device(self):
        return next(self.unet.parameters()).device

    @property
    def dtype(self):
        return next(self.unet.parameters()).dtype

    def _forward(self, sample, timestep, encoder_hidden_states, return_dict=True, cross_attention_kwargs=None,
                 timestep_cond=None, added_cond_kwargs=None):
        kw = {}
        if cross_attention_kwargs:
            kw["cross_attention_kwargs"] = cross_attention_kwargs
        if timestep_cond is not None:
            kw["timestep_cond"] = timestep_cond
        if added_cond_kwargs is not None:
            kw["added_cond_kwargs"] = added_cond_kwargs
        return self.unet(sample, timestep, encoder_hidden_states, return_dict=return_dict, **kw)

    @torch.no_grad()
    def forward(self, *args, **kwargs):
        return self._graph(*args, **kwargs)


class DSVAE(torch.nn.Module):
    """VAE with separately captured ``encode`` / ``decode`` / ``forward`` graphs (reference diffusers/vae.py)."""

    def __init__(self, vae, enable_cuda_graph=True):
        super().__init__()
        self.vae = vae
        self.config = getattr(vae, "config", None)
        self.vae.requires_grad_(False)
        self.n_attention = inject_attention_processors(vae)
        self._enc = GraphedCallable(lambda x, return_dict=True: vae.encode(x, return_dict=return_dict),
                                    enabled=enable_cuda_graph)
        self._dec = GraphedCallable(lambda x, return_dict=True: vae.decode(x, return_dict=return_dict),
                                    enabled=enable_cuda_graph)
        self._fwd = GraphedCallable(lambda *a, **k: vae(*a, **k), enabled=enable_cuda_graph)

    @property
    def device(self):
        return next(self.vae.parameters()).device

    @property
    def dtype(self):
        return next(self.vae.parameters()).dtype

    @torch.no_grad()
    def encode(self, x, return_dict=True):
        return self._enc(x, return_dict=return_dict)

    @torch.no_grad()
    def decode(self, x, return_dict=True, generator=None):
        return self._dec(x, return_dict=return_dict)

    @torch.no_grad()
    def forward(self, *args, **kwargs):
        return self._fwd(*args, **kwargs)


class DSClipEncoder(torch.nn.Module):
    """CLIP text encoder with a graph-replayed forward (reference model_implementations/transformers/
    clip_encoder.py). Its layers go through the normal kernel injection (fused LayerNorm, attention through the
    transformers AttentionInterface)."""

    def __init__(self, enc, enable_cuda_graph=True):
        super().__init__()
        self.enc = enc
        self.config = getattr(enc, "config", None)
        self.enc.requires_grad_(False)
        self._graph = GraphedCallable(lambda *a, **k: enc(*a, **k), enabled=enable_cuda_graph)

    @property
    def device(self):
        return next(self.enc.parameters()).device

    @property
    def dtype(self):
        return next(self.enc.parameters()).dtype

    @torch.no_grad()
    def forward(self, *args, **kwargs):
        return self._graph(*args, **kwargs)


def _is_unet(m):
    return type(m).__name__ in ("UNet2DConditionModel", "UNet2DModel") or (
        hasattr(m, "in_channels") and hasattr(m, "conv_in") and hasattr(m, "down_blocks") and hasattr(m, "up_blocks"))


def _is_vae(m):
    return type(m).__name__ in ("AutoencoderKL", "AutoencoderTiny") or (
        hasattr(m, "encode") and hasattr(m, "decode") and hasattr(m, "encoder") and hasattr(m, "decoder"))


def _is_clip_text(m):
    return type(m).__name__ in ("CLIPTextModel", "CLIPTextModelWithProjection")


def wrap_diffusion_module(m, enable_cuda_graph=True):
    """The reference's UNet / VAE / CLIP policies: return the wrapped module (or ``m`` when none applies)."""
    if isinstance(m, (DSUNet, DSVAE, DSClipEncoder)):
        return m
    if _is_unet(m):
        return DSUNet(m, enable_cuda_graph)
    if _is_vae(m):
        return DSVAE(m, enable_cuda_graph)
    if _is_clip_text(m):
        return DSClipEncoder(m, enable_cuda_graph)
    return m


def inject_pipeline(pipe, enable_cuda_graph=True):
    """Wrap a diffusion pipeline's ``unet``, ``vae`` and ``text_encoder`` in place (generic_injection in the
    reference's replace_module.py); returns the names that were wrapped."""
    done = []
    for name in ("unet", "vae", "text_encoder", "text_encoder_2"):
        m = getattr(pipe, name, None)
        if m is None:
            continue
        w = wrap_diffusion_module(m, enable_cuda_graph)
        if w is not m:
            setattr(pipe, name, w)
            done.append(name)
    return done
