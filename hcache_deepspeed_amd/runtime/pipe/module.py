"""Pipeline-parallel model description: layer specs, partitioning, tied layers.

Reference parity: runtime/pipe/module.py (``LayerSpec`` :30, ``TiedLayerSpec`` :68, ``PipelineModule``
:86-693: ``_partition_layers`` :393 with ``uniform``/``parameters``/``type:regex``, tied-module groups
:420-470, activation checkpoint interval, ``loss_fn``). Each rank builds ONLY its stage's layers; the
parameter counts used by the ``parameters`` partitioner come from building the specs on the meta device,
so partitioning a 70B model allocates nothing.
"""
import re
from functools import partial

import torch
import torch.nn as nn

from ... import comm as dist
from ...utils import groups
from ...utils.logging import log_dist


class PipelineError(Exception):
    pass


class LayerSpec:
    """Deferred layer construction: ``LayerSpec(nn.Linear, 4096, 4096)``."""

    def __init__(self, typename, *module_args, **module_kwargs):
        if not issubclass(typename, nn.Module):
            raise RuntimeError("LayerSpec only supports torch.nn.Module types.")
        self.typename = typename
        self.module_args = module_args
        self.module_kwargs = module_kwargs

    def __repr__(self):
        return f"LayerSpec({self.typename.__name__})"

    def build(self, log=False):
        if log:
            log_dist(f"building {self}", ranks=[0])
        return self.typename(*self.module_args, **self.module_kwargs)


class TiedLayerSpec(LayerSpec):
    """A layer whose ``tied_weight_attr`` parameter(s) are shared by every stage holding ``key``."""

    def __init__(self, key, typename, *module_args, forward_fn=None, tied_weight_attr=("weight", ),
                 **module_kwargs):
        super().__init__(typename, *module_args, **module_kwargs)
        self.key = key
        self.forward_fn = forward_fn
        self.tied_weight_attr = (tied_weight_attr, ) if isinstance(tied_weight_attr, str) else tuple(tied_weight_attr)


def _count_params(spec):
    if isinstance(spec, nn.Module):
        return sum(p.numel() for p in spec.parameters() if p.requires_grad)
    if isinstance(spec, LayerSpec):
        with torch.device("meta"):
            m = spec.build()
        return sum(p.numel() for p in m.parameters() if p.requires_grad)
    return 0


def partition_uniform(num_items, num_parts):
    parts = [0] * (num_parts + 1)
    chunk, extra = divmod(num_items, num_parts)
    for p in range(num_parts):
        parts[p + 1] = parts[p] + chunk + (1 if p < extra else 0)
    return parts


def partition_balanced(weights, num_parts):
    """Contiguous split minimising the heaviest part (binary search on the bottleneck)."""
    n = len(weights)
    prefix = [0]
    for w in weights:
        prefix.append(prefix[-1] + w)

    def parts_for(limit):
        bounds, start = [0], 0
        while start < n:
            end = start + 1
            while end < n and prefix[end + 1] - prefix[start] <= limit:
                end += 1
            bounds.append(end)
            start = end
        return bounds

    lo, hi = max(weights) if weights else 0, prefix[-1]
    while lo < hi:
        mid = (lo + hi) // 2
        if len(parts_for(mid)) - 1 <= num_parts:
            hi = mid
        else:
            lo = mid + 1
    bounds = parts_for(lo)
    while len(bounds) - 1 < num_parts:
        # fewer parts than stages: split the part with the most layers (keeps every stage non-empty)
        sizes = [(bounds[i + 1] - bounds[i], i) for i in range(len(bounds) - 1)]
        size, i = max(sizes)
        if size <= 1:
            bounds.append(n)  # more stages than layers: trailing empty stages
            continue
        bounds.insert(i + 1, bounds[i] + size // 2)
    return bounds


class PipelineModule(nn.Module):

    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seed_layers=False,
                 seed_fn=None, base_seed=1234, partition_method="parameters", activation_checkpoint_interval=0,
                 activation_checkpoint_func=None, checkpointable_layers=None, dynamic_shape=False):
        super().__init__()
        if num_stages is None and topology is None:
            raise RuntimeError("must provide num_stages or topology")
        if not dist.is_initialized():
            dist.init_distributed()
        if topology is not None:
            num_stages = topology.get_dim("pipe")
        self.num_stages = int(num_stages)
        if groups._State.topo is None or groups._State.topo.get_dim("pipe") != self.num_stages:
            tp = topology.get_dim("model") if topology is not None and "model" in topology.axes else 1
            groups.reset()
            groups.initialize(tp=tp, pp=self.num_stages)
        from .topology import PipelineParallelGrid
        self._grid = PipelineParallelGrid()
        self._topo = groups.get_topology()
        self.stage_id = self._grid.get_stage_id()
        self.global_rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        self.loss_fn = loss_fn
        self.seed_layers = seed_layers
        self.seed_fn = seed_fn
        self.base_seed = base_seed
        self.activation_checkpoint_interval = activation_checkpoint_interval
        self.activation_checkpoint_func = activation_checkpoint_func
        self.checkpointable_layers = checkpointable_layers
        self._layer_specs = list(layers)
        self._num_layers = len(self._layer_specs)
        self._partition_layers(partition_method)
        self.forward_funcs = []
        self.fwd_map = {}
        self.tied_modules = nn.ModuleDict()
        self.tied_weight_attrs = {}
        self._build()

    # ------------------------------------------------------------------------------------
    def _partition_layers(self, method):
        P = self.num_stages
        m = method.lower()
        if m == "uniform":
            self.parts = partition_uniform(self._num_layers, P)
        elif m == "parameters":
            self.parts = partition_balanced([_count_params(s) for s in self._layer_specs], P)
        elif m.startswith("type:"):
            pat = method.split(":", 1)[1]
            w = [1 if re.search(pat, (s.typename.__name__ if isinstance(s, LayerSpec) else type(s).__name__),
                                re.IGNORECASE) else 0 for s in self._layer_specs]
            self.parts = partition_balanced(w, P)
        elif m == "profile":
            raise NotImplementedError("partition_method 'profile' is not implemented")
        else:
            raise NotImplementedError(f"partition_method {method}")
        assert len(self.parts) == P + 1
        log_dist(f"pipeline partition ({method}): {self.parts}", ranks=[0])

    def _build(self):
        lo, hi = self.parts[self.stage_id], self.parts[self.stage_id + 1]
        self._local_start, self._local_stop = lo, hi
        for idx in range(lo, hi):
            spec = self._layer_specs[idx]
            if self.seed_layers:
                (self.seed_fn or torch.manual_seed)(self.base_seed + idx)
            if isinstance(spec, TiedLayerSpec):
                if spec.key not in self.tied_modules:
                    self.tied_modules[spec.key] = spec.build()
                    self.tied_weight_attrs[spec.key] = spec.tied_weight_attr
                mod = self.tied_modules[spec.key]
                fn = partial(spec.forward_fn, mod) if spec.forward_fn is not None else mod
                self.forward_funcs.append(fn)
                self.fwd_map[f"tied:{spec.key}"] = len(self.forward_funcs) - 1
            elif isinstance(spec, LayerSpec):
                mod = spec.build()
                name = str(idx)
                self.add_module(name, mod)
                self.forward_funcs.append(mod)
                self.fwd_map[name] = len(self.forward_funcs) - 1
            elif isinstance(spec, nn.Module):
                self.add_module(str(idx), spec)
                self.forward_funcs.append(spec)
            elif callable(spec):
                self.forward_funcs.append(spec)
            else:
                raise ValueError(f"layer {idx}: unsupported spec {type(spec)}")
        self._tied_groups = self._index_tied_modules()

    def _index_tied_modules(self):
        """{key: (process group, owner global ranks)} for keys present on more than one stage."""
        out = {}
        keys = sorted({s.key for s in self._layer_specs if isinstance(s, TiedLayerSpec)})
        me = self._topo.get_coord(self.global_rank)
        for key in keys:
            stages = sorted({self.stage_owner(i) for i, s in enumerate(self._layer_specs)
                             if isinstance(s, TiedLayerSpec) and s.key == key})
            # one group per (data, seq, model) coordinate; every rank creates every group (collective)
            for c, r in sorted(self._topo.mapping.items()):
                coord = dict(zip(self._topo.axes, c))
                if coord["pipe"] != 0:
                    continue
                ranks = [self._topo.get_rank(**dict(coord, pipe=s)) for s in stages]
                g = dist.new_group(ranks=ranks) if len(ranks) > 1 and self.world_size > 1 else None
                if all(coord[a] == me[a] for a in self._topo.axes if a != "pipe") and self.stage_id in stages:
                    out[key] = (g, ranks)
        return out

    def stage_owner(self, layer_idx):
        for s in range(self.num_stages):
            if self.parts[s] <= layer_idx < self.parts[s + 1]:
                return s
        raise RuntimeError(f"layer {layer_idx} not owned by any stage")

    def tied_parameters(self, key):
        mod = self.tied_modules[key]
        return [getattr(mod, a) for a in self.tied_weight_attrs[key]]

    def sync_tied_weights(self):
        """Broadcast tied weights from the lowest owning stage (reference module.py:420-440)."""
        for key, (g, ranks) in self._tied_groups.items():
            if g is None:
                continue
            for p in self.tied_parameters(key):
                dist.broadcast(p.data, ranks[0], group=g)

    def allreduce_tied_weight_gradients(self):
        """Sum tied-parameter gradients over the owning stages (reference module.py:454-460)."""
        for key, (g, _) in self._tied_groups.items():
            if g is None:
                continue
            for p in self.tied_parameters(key):
                if p.grad is not None:
                    dist.all_reduce(p.grad, group=g)

    # ------------------------------------------------------------------------------------
    def forward(self, forward_input):
        x = forward_input

        def run(start, end):

            def exec_range(*inputs):
                h = inputs[0] if len(inputs) == 1 else inputs
                for fn in self.forward_funcs[start:end]:
                    h = fn(h)
                return h

            return exec_range

        n = len(self.forward_funcs)
        interval = self.activation_checkpoint_interval
        if interval == 0 or not self.training:
            return run(0, n)(x)
        from ..activation_checkpointing.checkpointing import checkpoint
        ckpt = self.activation_checkpoint_func or checkpoint
        for start in range(0, n, interval):
            end = min(start + interval, n)
            args = x if isinstance(x, tuple) else (x, )
            if self._is_checkpointable(self.forward_funcs[start:end]):
                x = ckpt(run(start, end), *args)
            else:
                x = run(start, end)(*args)
        return x

    def _is_checkpointable(self, funcs):
        if self.checkpointable_layers is not None:
            return all(type(f).__name__ in self.checkpointable_layers for f in funcs)
        params = [f.parameters() for f in funcs if isinstance(f, nn.Module)]
        return any(len(list(p)) > 0 for p in params)

    def num_pipeline_stages(self):
        return self.num_stages

    def topology(self):
        return self._topo

    def mpu(self):
        return self._grid

    def _local_layers(self):
        """[(local index, module)] of this stage's parameterised layers (tied modules under their first index)."""
        out, seen = [], set()
        for idx in range(self._local_start, self._local_stop):
            spec = self._layer_specs[idx]
            mod = None
            if isinstance(spec, TiedLayerSpec):
                mod = self.tied_modules[spec.key] if spec.key not in seen else None
                seen.add(spec.key)
            elif str(idx) in self._modules:
                mod = self._modules[str(idx)]
            if mod is not None and any(True for _ in mod.parameters()):
                out.append((idx - self._local_start, mod))
        return out

    def save_state_dict(self, save_dir, checkpoint_engine=None, exclude_frozen_params=False):
        """One ``layer_XX[-model_YY]-model_states.pt`` per parameterised layer of this stage (the reference's
        layer-wise pipeline checkpoint, pipe/module.py save_state_dict): written by data-parallel rank 0 of each
        stage / model-parallel slice."""
        import os
        if self._grid.get_data_parallel_rank() != 0:
            return
        os.makedirs(save_dir, exist_ok=True)
        for li, mod in self._local_layers():
            sd = {k: v.detach().clone().cpu() for k, v in mod.state_dict().items()}
            if exclude_frozen_params:
                frozen = {n for n, p in mod.named_parameters() if not p.requires_grad}
                sd = {k: v for k, v in sd.items() if k not in frozen}
            path = self.ckpt_layer_path(save_dir, li)
            (checkpoint_engine.save(sd, path) if checkpoint_engine is not None else torch.save(sd, path))

    def load_state_dir(self, load_dir, checkpoint_engine=None, strict=True):
        """Load the layer files ``save_state_dict`` wrote into this stage's layers."""
        for li, mod in self._local_layers():
            path = self.ckpt_layer_path(load_dir, li)
            sd = (checkpoint_engine.load(path, map_location="cpu") if checkpoint_engine is not None else
                  torch.load(path, map_location="cpu", weights_only=True))
            mod.load_state_dict(sd, strict=strict)
        self.sync_tied_weights() if self.num_stages > 1 else None

    def ckpt_layer_path(self, ckpt_dir, local_layer_idx):
        import os
        idx = local_layer_idx + self._local_start
        rank_repr = f"-model_{groups.get_model_parallel_rank():02d}" if groups.get_model_parallel_world_size() > 1 \
            else ""
        return os.path.join(ckpt_dir, f"layer_{idx:02d}{rank_repr}-model_states.pt")
