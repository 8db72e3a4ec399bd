"""Test-only fault injection: fail rank ``k`` at global step ``n`` to exercise launcher failure propagation,
collective-timeout handling and checkpoint resume (SURVEY.md §5.3 — the reference has no fault injection; its
launcher kills the process tree on any child failure, launcher/launch.py:317-355).

Enable with the environment variable ``HDS_FAULT_INJECT="<rank>:<step>[:<mode>]"`` (several specs separated by
``,``) or the config section ``{"fault_injection": {"rank": k, "step": n, "mode": "raise"}}``. Modes:

* ``raise``  — raise :class:`InjectedFault` from ``engine.step()`` after the optimizer step of global step ``n``
  (the Python-level failure path: exception handlers, ``monitored_barrier`` diagnostics);
* ``exit``   — ``os._exit(17)`` without cleanup (a crashed worker: peers see their collectives fail);
* ``hang``   — sleep forever (a stuck worker: peers hit the collective timeout ``DEEPSPEED_TIMEOUT``).

Faults fire once per process. Nothing is injected unless configured.
"""
import os
import time

from ..utils.logging import logger


class InjectedFault(RuntimeError):
    pass


def _parse(spec):
    out = []
    for part in filter(None, (s.strip() for s in spec.split(","))):
        f = part.split(":")
        out.append((int(f[0]), int(f[1]), f[2] if len(f) > 2 else "raise"))
    return out


class FaultInjector:

    def __init__(self, config=None):
        specs = _parse(os.environ.get("HDS_FAULT_INJECT", ""))
        cfg = config or {}
        if cfg.get("rank") is not None and cfg.get("step") is not None:
            specs.append((int(cfg["rank"]), int(cfg["step"]), cfg.get("mode", "raise")))
        for _, _, mode in specs:
            if mode not in ("raise", "exit", "hang"):
                raise ValueError(f"unknown fault mode {mode!r}")
        self.specs = specs
        self.fired = False

    @property
    def enabled(self):
        return bool(self.specs) and not self.fired

    def maybe_fire(self, rank, step):
        if not self.enabled:
            return
        for r, s, mode in self.specs:
            if r == rank and s == step:
                self.fired = True
                logger.warning(f"[fault injection] rank {rank} step {step}: {mode}")
                if mode == "exit":
                    os._exit(17)
                if mode == "hang":
                    while True:
                        time.sleep(3600)
                raise InjectedFault(f"injected fault at rank {rank} step {step}")
