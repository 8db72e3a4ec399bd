"""hcache_deepspeed_amd -- an MI355X-native training / serving framework with the capabilities of
zhangzuo21/Hcache_DeepSpeed (DeepSpeed 0.16.8 + the HCache host-side hidden-state cache).

Drop-in usage::

    import hcache_deepspeed_amd as deepspeed
    engine, optimizer, dataloader, lr_scheduler = deepspeed.initialize(model=model, config=ds_config)

Reference parity: deepspeed/__init__.py (``initialize`` :69-230, ``add_config_arguments`` :233-281,
``init_inference`` :284-366, ``tp_model_init`` :369-398).
"""
import argparse
import os

# Device->host copies (activation spills, HCache latents) run as the HIP runtime's blit kernel, which otherwise spreads
# one copy over as many workgroups as it has chunks and takes CUs from the kernels it overlaps: a 32k-token Llama-3-8B
# step spilling 25 GiB ran its forward 56 % longer. PCIe bounds the copy, so 16 workgroups still saturate it, and with
# this limit the measured cost of a spill is ~0.01 ms per GB (profiles/r4/copy_engine_ab_r4f.txt). It only takes
# effect when it is in the environment before torch loads the HIP runtime (set here after `import torch`, spills
# measured 2-6 ms/GB: profiles/r4/plan32k_pkg_import_default_r4h.txt), so bench.py and the launcher set it first;
# this import covers a script that imports the package before torch. An explicit value is kept.
import sys as _sys


def _hip_runtime_loaded():
    """Is the HIP runtime library already mapped into this process (torch loads it at import)?"""
    try:
        with open("/proc/self/maps") as f:
            return any("libamdhip64" in line for line in f)
    except OSError:
        return "torch" in _sys.modules


# the limit is in effect if the runtime is not loaded yet (set just below, read when it loads) or if the variable was
# already in the environment at this point -- set by the launcher, bench.py, or the user before importing torch
BLIT_LIMIT_EARLY = "DEBUG_CLR_LIMIT_BLIT_WG" in os.environ or not _hip_runtime_loaded()
os.environ.setdefault("DEBUG_CLR_LIMIT_BLIT_WG", "16")

from .version import __version__, __version_major__, __version_minor__, __version_patch__  # noqa: F401
from . import comm  # noqa: F401
from .comm import init_distributed  # noqa: F401
from .runtime import zero  # noqa: F401
from .runtime.config import DeepSpeedConfig  # noqa: F401
from .runtime.engine import DeepSpeedEngine  # noqa: F401
from .runtime.lr_schedules import VALID_LR_SCHEDULES  # noqa: F401
from .utils.logging import logger, log_dist  # noqa: F401
from .runtime.activation_checkpointing import checkpointing  # noqa: F401
from . import ops  # noqa: F401
from .accelerator import get_accelerator  # noqa: F401
from .runtime.config import ConfigError as DeepSpeedConfigError  # noqa: F401
from .runtime.lr_schedules import add_tuning_arguments  # noqa: F401
from .runtime.compiler import is_compile_supported  # noqa: F401
from .utils.init_on_device import OnDevice  # noqa: F401
from .pipe import PipelineModule  # noqa: F401
from .runtime.pipe.engine import PipelineEngine  # noqa: F401
from .runtime.hybrid_engine import DeepSpeedHybridEngine  # noqa: F401
from .inference.engine import InferenceEngine  # noqa: F401
from .inference.config import DeepSpeedInferenceConfig  # noqa: F401
from .ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer  # noqa: F401
from .module_inject import replace_transformer_layer, revert_transformer_layer, set_autotp_mode  # noqa: F401
from . import comm as dist  # noqa: F401  (reference: ``deepspeed.dist``)
from typing import Callable as _Callable, Dict as _Dict, Iterable as _Iterable, Union as _Union

import torch as _torch

TORCH_DISTRIBUTED_DEFAULT_PORT = 29500
ADAM_OPTIMIZER, LAMB_OPTIMIZER = "adam", "lamb"  # reference runtime/config.py optimizer-name constants
# reference __init__.py:30-31: what ``initialize(optimizer=..., lr_scheduler=...)`` accepts besides instances
DeepSpeedOptimizerCallable = _Callable[[_Union[_Iterable[_torch.nn.Parameter], _Dict[str, _Iterable]]],
                                       _torch.optim.Optimizer]
DeepSpeedSchedulerCallable = _Callable[[_torch.optim.Optimizer], _torch.optim.lr_scheduler.LRScheduler]


def _git_info():
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    try:
        h = subprocess.run(["git", "rev-parse", "--short", "HEAD"], cwd=root, capture_output=True, text=True,
                           timeout=5).stdout.strip()
        b = subprocess.run(["git", "rev-parse", "--abbrev-ref", "HEAD"], cwd=root, capture_output=True, text=True,
                           timeout=5).stdout.strip()
        return h or "unknown", b or "unknown"
    except Exception:  # noqa: BLE001 -- no git in the environment
        return "unknown", "unknown"


git_hash, git_branch = _git_info()
from .runtime import domino  # noqa: F401

version = __version__


def initialize(args=None, model=None, optimizer=None, model_parameters=None, training_data=None, lr_scheduler=None,
               distributed_port=29500, mpu=None, dist_init_required=None, collate_fn=None, config=None, mesh_param=None,
               config_params=None):
    """Returns ``(engine, engine.optimizer, engine.training_dataloader, engine.lr_scheduler)``."""
    assert model is not None, "deepspeed.initialize requires a model"
    if config is None:
        config = config_params
    if config is None and args is not None:
        config = getattr(args, "deepspeed_config", None)
    init_distributed(distributed_port=distributed_port, dist_init_required=dist_init_required)
    cfg = DeepSpeedConfig(config, mpu=mpu)
    if mesh_param is not None:
        # (data_parallel, sequence_parallel) device mesh (reference __init__.py:141-148): the SP extent becomes the
        # Ulysses group size; ZeRO then shards over the dp x sp sequence-data-parallel group
        dp, sp = (int(x) for x in mesh_param)
        if dp * sp != comm.get_world_size():
            raise ValueError(f"mesh_param {mesh_param} does not cover the world size {comm.get_world_size()}")
        cfg.sequence_parallel_size = sp
    from .runtime.pipe.module import PipelineModule
    if isinstance(model, PipelineModule):
        from .runtime.pipe.engine import PipelineEngine
        engine = PipelineEngine(args=args, model=model, optimizer=optimizer, model_parameters=model_parameters,
                                training_data=training_data, lr_scheduler=lr_scheduler, mpu=model.mpu(),
                                dist_init_required=dist_init_required, collate_fn=collate_fn, config=config,
                                config_class=cfg)
    elif (cfg.hybrid_engine or {}).get("enabled", False):
        from .runtime.hybrid_engine import DeepSpeedHybridEngine
        engine = DeepSpeedHybridEngine(args=args, model=model, optimizer=optimizer, model_parameters=model_parameters,
                                       training_data=training_data, lr_scheduler=lr_scheduler, mpu=mpu,
                                       dist_init_required=dist_init_required, collate_fn=collate_fn, config=config,
                                       config_class=cfg)
    else:
        engine = DeepSpeedEngine(args=args, model=model, optimizer=optimizer, model_parameters=model_parameters,
                                 training_data=training_data, lr_scheduler=lr_scheduler, mpu=mpu,
                                 dist_init_required=dist_init_required, collate_fn=collate_fn, config=config,
                                 config_class=cfg)
    return engine, engine.optimizer, engine.training_dataloader, engine.lr_scheduler


def _add_core_arguments(parser):
    group = parser.add_argument_group("DeepSpeed", "DeepSpeed configurations")
    group.add_argument("--deepspeed", default=False, action="store_true",
                       help="Enable DeepSpeed (helper flag for user code, no impact on DeepSpeed backend)")
    group.add_argument("--deepspeed_config", default=None, type=str, help="DeepSpeed json configuration file.")
    group.add_argument("--deepscale", default=False, action="store_true", help=argparse.SUPPRESS)
    group.add_argument("--deepscale_config", default=None, type=str, help=argparse.SUPPRESS)
    return parser


def add_config_arguments(parser):
    return _add_core_arguments(parser)


def default_inference_config():
    from .inference.config import DeepSpeedInferenceConfig
    return DeepSpeedInferenceConfig().to_dict()


def init_inference(model, config=None, **kwargs):
    """Inference engine (kernel injection / AutoTP analogue). kwargs override config keys."""
    from .inference.engine import InferenceEngine
    from .inference.config import DeepSpeedInferenceConfig
    cfg = dict(config or {})
    cfg.update(kwargs)
    import torch.nn as _nn
    if not isinstance(model, _nn.Module) and any(hasattr(model, a) for a in ("unet", "vae", "text_encoder")):
        # a diffusion pipeline (reference replace_module.generic_injection): UNet / VAE / CLIP text encoder are
        # wrapped in place with HIP-graph replay and the fused attention processor
        from .inference.diffusers import inject_pipeline
        inject_pipeline(model, enable_cuda_graph=bool(cfg.get("enable_cuda_graph", True)))
        return model
    return InferenceEngine(model, config=DeepSpeedInferenceConfig(**cfg))


def tp_model_init(model, tp_size, dtype, config=None, **kwargs):
    """AutoTP training entry: shard nn.Linear layers over a tensor-parallel group of ``tp_size``."""
    from .parallel.tp import TpTrainingManager
    return TpTrainingManager(model=model, tp_size=tp_size, dtype=dtype).module
