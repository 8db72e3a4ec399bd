"""Ragged serving engine with the HCache API: ``put`` -> (logits, per-sequence latents), ``restore_kv``.

Reference parity: inference/v2/engine_v2.py ``InferenceEngineV2`` (put :131-189 incl. the fork's latent
split :172-179, restore_kv :107-128, query :191, can_schedule :217, get_remaining_block_capacity :266,
flush :275, serialize :284, TP group :93-105), inference/v2/scheduling_utils.py (``SchedulingResult``),
config_v2.py (``RaggedInferenceEngineConfig``), engine_factory.py (``build_hf_engine`` :69).

Fixed relative to the fork: ``restore_kv`` only touches sequences that actually had latents (the fork
called ``post_forward`` for every uid), latents come back pinned and asynchronously copied, and every
model type returns latents.
"""
import json
import os
from dataclasses import dataclass, field
from enum import Enum
from typing import Iterable, List, Optional, Tuple

import torch

from ... import comm as dist
from ...utils.logging import log_dist
from .model import RaggedTransformer
from .ragged import BlockedKVCache, DSStateManager, DSStateManagerConfig, RaggedBatchWrapper


class SchedulingResult(Enum):
    Success = 0
    EngineSequenceLimitExceeded = 1
    BatchSequenceLimitExceeded = 2
    BatchTokenLimitExceeded = 3
    KVCacheLimitExceeded = 4
    SequenceTokenLimitExceeded = 5


class SchedulingError(RuntimeError):

    def __init__(self, result):
        self.result = result
        super().__init__(f"Batch scheduling failed with result {result}")


@dataclass
class RaggedInferenceEngineConfig:
    tensor_parallel: dict = field(default_factory=lambda: {"tp_size": 1})
    state_manager: DSStateManagerConfig = field(default_factory=DSStateManagerConfig)
    quantization: dict = field(default_factory=dict)
    latent_mode: str = "hidden"  # HCache: "hidden" (per-layer normed hidden), "hidden_fp8" (e4m3 + per-token scale) or "kv" (pre-RoPE K|V)
    dtype: str = "bf16"

    @staticmethod
    def from_dict(d):
        d = dict(d or {})
        sm = d.pop("state_manager", None)
        cfg = RaggedInferenceEngineConfig(**{k: v for k, v in d.items()
                                             if k in RaggedInferenceEngineConfig.__dataclass_fields__})
        if sm is not None:
            cfg.state_manager = sm if isinstance(sm, DSStateManagerConfig) else DSStateManagerConfig.from_dict(sm)
        return cfg


class InferenceEngineV2:

    def __init__(self, model_config, weights, engine_config: RaggedInferenceEngineConfig = None, device=None,
                 num_kv_blocks=None):
        self._config = engine_config or RaggedInferenceEngineConfig()
        self._base_mp_group = self._initialize_tp_group()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else \
                torch.device("cpu")
        self.device = device
        dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[self._config.dtype]
        from .arch import ArchSpec, convert_own_llama, spec_from_llama_config
        if not isinstance(model_config, ArchSpec):  # this framework's Llama / Mixtral training configs
            model_config = spec_from_llama_config(model_config)
            weights = convert_own_llama(weights, model_config)
        self._model = RaggedTransformer(model_config, weights, device, dtype, tp_group=self._base_mp_group,
                                        latent_mode=self._config.latent_mode, engine_config=self._config)
        sm = self._config.state_manager
        kvc = self._model.kv_cache_config()
        self._kv = BlockedKVCache(kvc["num_layers"], kvc["n_kv_heads"], kvc["head_dim"], sm.kv_block_size, dtype,
                                  device, sm.memory_config, tp_group=self._base_mp_group, num_blocks=num_kv_blocks)
        self._model.set_kv_cache(self._kv)
        self._state_manager = DSStateManager(sm, self._kv)
        self._batch = RaggedBatchWrapper(sm, device, self._state_manager.max_blocks_per_seq)
        from ...ops.paged import ROWS_PER_ATOM
        self._batch.set_attention_geometry(self._model.n_q, self._model.n_kv, ROWS_PER_ATOM)
        log_dist(f"InferenceEngineV2: {self._kv.num_blocks} KV blocks of {sm.kv_block_size} tokens "
                 f"(tp={self._model.tp}, latent_mode={self._config.latent_mode})", ranks=[0])

    def _initialize_tp_group(self):
        tp = int(self._config.tensor_parallel.get("tp_size", 1))
        if tp == 1 and not dist.is_initialized():
            return None
        dist.init_distributed(verbose=False)
        if tp == 1:
            return None
        if dist.get_rank() >= tp and dist.get_world_size() == tp:
            raise RuntimeError("Local rank is greater than TP size, ensure that the TP config is correct.")
        return dist.new_group(ranks=list(range(tp)))

    # ------------------------------------------------------------------------------------------
    @property
    def free_blocks(self):
        return self._state_manager.free_blocks

    @property
    def n_kv_cache_groups(self):
        return 1

    def model(self):
        return self._model

    @property
    def state_manager(self):
        return self._state_manager

    # ------------------------------------------------------------------------------------------
    def put(self, batch_uids: Iterable[int], batch_tokens: Iterable[torch.Tensor], do_checks: bool = True,
            capture_latents: bool = True, sync_latents: Optional[bool] = None
            ) -> Tuple[torch.Tensor, List[Optional[torch.Tensor]]]:
        """One ragged forward. Returns logits [n_seqs, V] and, per sequence, its latents [L, n_tokens, W] (host).
        ``sync_latents=False``: the host does not wait for the latent copies (no per-forward synchronize, reference
        engine_v2.py:131-189 keeps its host free the same way); call ``wait_latents()`` (or check
        ``latents_ready()``) before reading them -- ``restore_kv`` / ``evict`` wait on their own; HIP-graph decode
        steps then leave their latents in a device ring drained in bulk (inference/v2/model.py ``_LatentRing``), so a
        decode loop does not synchronize per token. The default (None) is synchronous: the returned latents are on
        the host when ``put`` returns (a graph-decode step flushes its ring first)."""
        batch_uids = list(batch_uids)
        batch_tokens = [t if isinstance(t, torch.Tensor) else torch.tensor(t) for t in batch_tokens]
        if do_checks:
            res = self.can_schedule(batch_uids, [t.numel() for t in batch_tokens])
            if res != SchedulingResult.Success:
                raise SchedulingError(res)
        sm, batch = self._state_manager, self._batch
        batch.clear()
        for uid, tokens in zip(batch_uids, batch_tokens):
            seq = sm.get_or_create_sequence(uid)
            sm.maybe_allocate_kv(seq, tokens.numel())
            seq.pre_forward(tokens.numel())
            batch.insert_sequence(seq, tokens, do_checks=do_checks)
        batch.finalize()
        if self._model.decode_graph_eligible(batch, capture_latents):
            # HIP-graph decode step (latents, if captured, land in the graph's device ring)
            logits, latents = self._model.forward_decode_graph(batch, capture_latents=capture_latents)
            if latents is not None and sync_latents is not False:
                self.wait_latents()
        else:
            logits, latents = self._model.forward(batch, capture_latents=capture_latents,
                                                  sync_latents=True if sync_latents is None else sync_latents)
            self._latent_event = getattr(self._model, "latent_event", None)
        split = []
        for (q0, n, _) in batch.seq_meta_host:
            split.append(latents[:, q0:q0 + n] if latents is not None else None)
        for uid in batch_uids:
            sm.get_sequence(uid).post_forward()
        return logits, split

    def latents_ready(self) -> bool:
        """Every latent returned so far is on the host (no synchronize; a decode-graph ring with undrained steps
        counts as not ready until ``wait_latents`` flushes it)."""
        if any(r.pending() for r in self._model.latent_rings()):
            return False
        ev = getattr(self, "_latent_event", None)
        if ev is not None and not ev.query():
            return False
        return all(r.done[h] is None or r.done[h].query() for r in self._model.latent_rings() for h in (0, 1))

    def wait_latents(self):
        """Block until every latent returned by ``put`` (eager prefill copies and the decode graphs' rings) is on
        the host."""
        ring_ev = self._model.drain_latents()
        for ev in (getattr(self, "_latent_event", None), ring_ev):
            if ev is not None:
                ev.synchronize()
        for r in self._model.latent_rings():
            for e in r.done:
                if e is not None:
                    e.synchronize()
        self._latent_event = None

    def restore_kv(self, batch_uids: Iterable[int], batch_tokens: Iterable[torch.Tensor],
                   batch_latents: Iterable[Optional[torch.Tensor]]):
        """Rebuild the KV cache of previously-evicted sequences from their host latents (HCache)."""
        self.wait_latents()
        sm, batch = self._state_manager, self._batch
        batch.clear()
        lat, restored = [], []
        for uid, tokens, latents in zip(batch_uids, batch_tokens, batch_latents):
            if latents is None:
                continue
            n = tokens.numel() if isinstance(tokens, torch.Tensor) else len(tokens)
            assert latents.shape[1] == n, "latents must cover exactly the tokens being restored"
            seq = sm.get_or_create_sequence(uid)
            sm.maybe_allocate_kv(seq, n)
            seq.pre_forward(n)
            batch.insert_sequence(seq, tokens if isinstance(tokens, torch.Tensor) else torch.tensor(tokens),
                                  do_checks=False)
            lat.append(latents)
            restored.append(uid)
        if not lat:
            return
        batch.finalize()
        self._model.restore_kv(batch, lat)  # per-sequence pinned pieces, copied straight to the device
        for uid in restored:
            sm.get_sequence(uid).post_forward()

    def evict(self, uid):
        """Free a sequence's KV blocks but keep tracking it (its tokens/latents live on the host)."""
        seq = self._state_manager.get_sequence(uid)
        self.wait_latents()
        if seq is not None:
            self._state_manager.free_kv(seq)
            seq.seen_tokens = 0

    # ------------------------------------------------------------------------------------------
    def query(self, uid: int, max_request_tokens: int, max_request_blocks: int) -> Tuple[int, int]:
        seq = self._state_manager.get_sequence(uid)
        seen = seq.seen_tokens if seq else 0
        alloc = seq.cur_allocated_blocks if seq else 0
        bs = self._kv.block_size
        room_in_alloc = alloc * bs - seen
        if max_request_tokens <= room_in_alloc:
            return max_request_tokens, 0
        extra_blocks = min(max_request_blocks, (max_request_tokens - room_in_alloc + bs - 1) // bs)
        tokens = min(max_request_tokens, room_in_alloc + extra_blocks * bs)
        return tokens, extra_blocks

    def can_schedule(self, uids: Iterable[int], lengths: Iterable[int]) -> SchedulingResult:
        sm = self._state_manager
        cfg = self._config.state_manager
        uids, lengths = list(uids), list(lengths)
        new_seqs = sum(1 for u in uids if sm.get_sequence(u) is None)
        if sm.n_tracked_sequences + new_seqs > cfg.max_tracked_sequences:
            return SchedulingResult.EngineSequenceLimitExceeded
        if len(uids) > cfg.max_ragged_sequence_count:
            return SchedulingResult.BatchSequenceLimitExceeded
        if sum(lengths) > cfg.max_ragged_batch_size:
            return SchedulingResult.BatchTokenLimitExceeded
        need = 0
        bs = self._kv.block_size
        for u, n in zip(uids, lengths):
            seq = sm.get_sequence(u)
            seen = seq.seen_tokens if seq else 0
            alloc = seq.cur_allocated_blocks if seq else 0
            if seen + n > cfg.max_context:
                return SchedulingResult.SequenceTokenLimitExceeded
            need += max(0, (seen + n + bs - 1) // bs - alloc)
        if need > sm.free_blocks:
            return SchedulingResult.KVCacheLimitExceeded
        return SchedulingResult.Success

    def get_remaining_block_capacity(self, uid: int) -> int:
        seq = self._state_manager.get_sequence(uid)
        if seq is None:
            return 0
        return seq.cur_allocated_blocks * self._kv.block_size - seq.seen_tokens

    def flush(self, uid: int) -> None:
        self._state_manager.flush_sequence(uid)

    def serialize(self, save_path: str) -> None:
        """Write this rank's canonical weight shards + the ArchSpec (reference engine_v2.py ``serialize`` :284)."""
        import dataclasses
        os.makedirs(save_path, exist_ok=True)
        m = self._model
        sd = {"embed": m.embed, "pos_embed": m.pos_embed, "final.w": m.final_w, "final.b": m.final_b,
              "lm_head.w": m.lm_head, "lm_head.b": m.lm_head_b,
              "layers": [{k: v for k, v in L.w.items() if v is not None} for L in m.layers]}

        from .modules.implementations import _PackedWeight

        def cpu(x):
            if isinstance(x, torch.Tensor):
                return x.cpu()
            if isinstance(x, _PackedWeight):  # weight-only quantized: packed codes + scales + shape
                return {"q": x.q.cpu(), "scales": x.scales.cpu(),
                        "meta": torch.tensor([x.out_features, x.in_features, x.group_size])}
            if isinstance(x, dict):
                return {k: cpu(v) for k, v in x.items() if v is not None}
            if isinstance(x, list):
                return [cpu(v) for v in x]
            return x

        torch.save(cpu(sd), os.path.join(save_path, f"params_rank_{m.tp_rank}.pt"))
        meta = dataclasses.asdict(m.spec)
        meta["tp_size"] = m.tp
        with open(os.path.join(save_path, "ds_model_config.json"), "w") as f:
            json.dump(meta, f, default=str)

    # ------------------------------------------------------------------------------------------
    def generate(self, uid, prompt, max_new_tokens=16):
        """Greedy decoding helper (prefill + decode through ``put``)."""
        logits, _ = self.put([uid], [prompt], capture_latents=False)
        out = []
        for _ in range(max_new_tokens):
            nxt = int(logits[0].argmax())
            out.append(nxt)
            logits, _ = self.put([uid], [torch.tensor([nxt])], capture_latents=False)
        return out


def build_engine_from_model(model, engine_config=None, device=None, num_kv_blocks=None):
    """Serving engine from a training ``LlamaForCausalLM`` (weights copied into the serving layout)."""
    sd = {k: v.detach() for k, v in model.state_dict().items()}
    cfg = model.config
    if isinstance(engine_config, dict):
        engine_config = RaggedInferenceEngineConfig.from_dict(engine_config)
    return InferenceEngineV2(cfg, sd, engine_config, device=device, num_kv_blocks=num_kv_blocks)


def build_hf_engine(path, engine_config=None, debug_level=None, device=None):
    """Serving engine from a HuggingFace checkpoint directory (config.json + *.safetensors / *.bin).

    Supported ``model_type``: llama, mistral, mixtral, qwen, qwen2, qwen2_moe, phi, phi3, falcon, opt
    (reference inference/v2/engine_factory.py:69-130)."""
    from .arch import convert_hf, spec_from_hf
    with open(os.path.join(path, "config.json")) as f:
        hf = json.load(f)
    spec = spec_from_hf(hf)
    sd = {}
    for fn in sorted(os.listdir(path)):
        full = os.path.join(path, fn)
        if fn.endswith(".safetensors"):
            from safetensors.torch import load_file
            sd.update(load_file(full))
        elif fn.endswith(".bin") and fn.startswith("pytorch_model"):
            sd.update(torch.load(full, map_location="cpu", weights_only=True))
    if isinstance(engine_config, dict):
        engine_config = RaggedInferenceEngineConfig.from_dict(engine_config)
    return InferenceEngineV2(spec, convert_hf(sd, spec), engine_config, device=device)


def build_engine_from_hf_model(hf_model, engine_config=None, device=None, num_kv_blocks=None):
    """Serving engine from an in-memory ``transformers`` model (any supported model_type)."""
    from .arch import convert_hf, spec_from_hf
    spec = spec_from_hf(hf_model.config.to_dict())
    sd = {k: v.detach() for k, v in hf_model.state_dict().items()}
    if isinstance(engine_config, dict):
        engine_config = RaggedInferenceEngineConfig.from_dict(engine_config)
    return InferenceEngineV2(spec, convert_hf(sd, spec), engine_config, device=device, num_kv_blocks=num_kv_blocks)


def build_engine_from_ds_checkpoint(path, engine_config=None, device=None, num_kv_blocks=None):
    """Reload a ``serialize()``d engine (same tensor-parallel size)."""
    from .arch import ArchSpec
    with open(os.path.join(path, "ds_model_config.json")) as f:
        meta = json.load(f)
    tp = meta.pop("tp_size", 1)
    spec = ArchSpec(**{k: v for k, v in meta.items() if k in ArchSpec.__dataclass_fields__})
    if isinstance(engine_config, dict):
        engine_config = RaggedInferenceEngineConfig.from_dict(engine_config)
    rank = dist.get_rank() if (tp > 1 and dist.is_initialized()) else 0
    sd = torch.load(os.path.join(path, f"params_rank_{rank}.pt"), map_location="cpu", weights_only=True)
    return InferenceEngineV2(spec, {"__presharded__": True, **sd}, engine_config, device=device,
                             num_kv_blocks=num_kv_blocks)
