"""Module interfaces + their registries (reference inference/v2/modules/interfaces/*.py)."""
from .module_registry import DSModuleBase, DSModuleRegistryBase


class DSSelfAttentionBase(DSModuleBase):
    """forward(qkv [T, nq + 2 nkv, D] (consumed: RoPE in place), kv_cache (one layer), batch, cos, sin)
    -> attention output [T, nq * D]."""


class DSLinearBase(DSModuleBase):
    """forward(x [T, in], weight (after transform_param), bias=None) -> activation(x W^T + b) [T, out or out/2]."""


class DSMoEBase(DSModuleBase):
    """forward(x [T, H], router_w [E, H], w13 [E, 2I, H], w2 [E, H, I]) -> [T, H] (top-k, dropless)."""


class DSPreNormBase(DSModuleBase):
    """forward(residual, hidden_in, gamma, beta) -> (new residual, normed); hidden_in None: norm(residual)."""


class DSPostNormBase(DSModuleBase):
    """forward(residual, hidden_in, gamma, beta) -> norm(residual + hidden_in)."""


class DSEmbeddingBase(DSModuleBase):
    """forward(batch, word_embeddings, position_embeddings=None) -> [T, H]."""


class DSUnembedBase(DSModuleBase):
    """forward(hidden, residual, batch, lm_head, lm_head_b, final_w, final_b) -> logits of each sequence's last
    token [n_seqs, V_local]."""


def _registry(base):

    class _R(DSModuleRegistryBase):
        registry = {}

        @staticmethod
        def associated_class():
            return base

    _R.__name__ = base.__name__.replace("Base", "Registry")
    return _R


DSSelfAttentionRegistry = _registry(DSSelfAttentionBase)
DSLinearRegistry = _registry(DSLinearBase)
DSMoERegistry = _registry(DSMoEBase)
DSPreNormRegistry = _registry(DSPreNormBase)
DSPostNormRegistry = _registry(DSPostNormBase)
DSEmbeddingRegistry = _registry(DSEmbeddingBase)
DSUnembedRegistry = _registry(DSUnembedBase)
