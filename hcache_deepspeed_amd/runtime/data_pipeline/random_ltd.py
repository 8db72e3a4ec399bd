"""Random layerwise token dropping (random-LTD).

Reference parity: runtime/data_pipeline/data_routing/basic_layer.py (``RandomLayerTokenDrop``),
scheduler.py (``RandomLTDScheduler``: reserved length grows from ``min_value`` to ``max_value`` over
``require_steps`` in ``seq_per_step`` increments), helper.py and ops/random_ltd (``gpt_sample_tokens``,
``token_gather``/``token_scatter``, K22). A wrapped layer sees only a random sorted subset of each
sequence's tokens; the untouched tokens bypass it and are scattered back, so the layer's cost scales with
the reserved length. Gather/scatter are single index_select/index_copy passes over [B*S, H] rows.
"""
import torch
import torch.nn as nn

from ...ops.random_ltd import GatherTokens, ScatterTokens, token_sort_


def gpt_sample_tokens(reserved_length, seq_length, batch_size, layers=1, device="cpu", generator=None):
    """Per (layer, batch) sorted random token indices [layers, B, reserved] (causal order preserved).

    The rows are sorted with ``token_sort_`` (LDS bitonic sort on GPU, csrc/kernels/token_ops.hip)."""
    scores = torch.rand(layers * batch_size, seq_length, device=device, generator=generator)
    idx = scores.topk(reserved_length, dim=1).indices.to(torch.int32).contiguous()
    token_sort_(idx)
    return idx.view(layers, batch_size, reserved_length)


def token_gather(x, idx):
    """x [B, S, H], idx [B, R] -> [B, R, H] (differentiable; HIP row gather on GPU)."""
    return GatherTokens.apply(x, idx, True)[1]


def token_scatter(full, part, idx):
    """Copy of full [B, S, H] with rows idx [B, R] replaced by part [B, R, H] (differentiable)."""
    return ScatterTokens.apply(full, part, idx, True)


class RandomLTDScheduler:

    def __init__(self, config):
        sch = config.get("random_ltd_schedule", config)
        self.min_value = int(sch["min_value"])
        self.max_value = int(sch["max_value"])
        sc = sch.get("schedule_config", {})
        self.require_steps = int(sc.get("require_steps", 1))
        self.seq_per_step = int(sc.get("seq_per_step", 8))
        self.current = self.min_value
        self.consumed_layer_tokens = 0

    def get_current_seq(self):
        return self.current

    def update_seq(self, global_step):
        if self.current < self.max_value:
            frac = min(1.0, global_step / max(1, self.require_steps))
            v = self.min_value + frac * (self.max_value - self.min_value)
            v = int(v) // self.seq_per_step * self.seq_per_step
            self.current = min(self.max_value, max(self.min_value, v))
        return self.current

    def state_dict(self):
        return {"current": self.current, "consumed_layer_tokens": self.consumed_layer_tokens}

    def load_state_dict(self, sd):
        self.current = sd["current"]
        self.consumed_layer_tokens = sd["consumed_layer_tokens"]


class RandomLayerTokenDrop(nn.Module):
    """Wrap a layer ``f(x [B,S,H], *args) -> [B,S,H]`` so in training it only processes ``reserved_length`` tokens."""

    def __init__(self, layer, scheduler=None):
        super().__init__()
        self.random_ltd_layer = layer
        self.scheduler = scheduler
        self.reserved_length = None

    def forward(self, x, *args, **kwargs):
        if not self.training or self.scheduler is None:
            return self.random_ltd_layer(x, *args, **kwargs)
        B, S, _ = x.shape
        R = min(S, self.scheduler.get_current_seq())
        if R >= S:
            return self.random_ltd_layer(x, *args, **kwargs)
        idx = gpt_sample_tokens(R, S, B, 1, x.device)[0]
        part = self.random_ltd_layer(token_gather(x, idx), *args, **kwargs)
        self.scheduler.consumed_layer_tokens += B * R
        return token_scatter(x, part, idx)
