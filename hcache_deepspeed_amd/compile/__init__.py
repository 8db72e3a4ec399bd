"""DeepCompile (reference deepspeed/compile/): profile-guided ZeRO schedule passes over the unit trace.
See backend.py for how a schedule is produced and passes.py for the passes."""
from .backend import DeepCompileBackend
from .passes import (CompiledSchedule, UnitGraph, compile_schedule, schedule_prefetch, selective_gather,
                     zero1_compile, zero3_compile)
from .profiler import CommPredictor, UnitProbe, profile_allgather
