"""DeepCompile (reference deepspeed/compile/): profile-guided ZeRO schedule passes over the unit trace.
See backend.py for how a schedule is produced and passes.py for the passes."""
from .backend import DeepCompileBackend
from .passes import (CompiledSchedule, UnitGraph, compile_schedule, plan_param_offload, plan_state_offload,
                     plan_state_reload,
                     schedule_prefetch, selective_gather, zero3_compile)
from .profiler import CommPredictor, UnitProbe, profile_allgather
