"""ZeRO-3 fetch / prefetch event profiler (reference runtime/zero/partitioned_param_profiler.py :10):
counts and times fetch, prefetch, wait and release events with their element counts."""
from ...utils.logging import log_dist


class PartitionedParameterProfiler:

    class EventCounter:

        def __init__(self, name):
            self.name = name
            self.reset()

        def reset(self):
            self.count = 0
            self.num_elem = 0

        def increment(self, numel):
            self.count += 1
            self.num_elem += numel

    def __init__(self, timers):
        self.timers = timers
        self.event_counters = {}

    def reset_events(self):
        for c in self.event_counters.values():
            c.reset()

    def start_event(self, name):
        if self.timers is None:
            return
        if name not in self.event_counters:
            self.event_counters[name] = PartitionedParameterProfiler.EventCounter(name)
        self.timers(name).start()

    def stop_event(self, name, num_elem):
        if self.timers is None:
            return
        assert name in self.event_counters, f"unknown event {name}"
        self.event_counters[name].increment(num_elem)
        self.timers(name).stop()

    def _log_timers(self):
        if self.timers is None:
            return
        self.timers.log(names=list(self.event_counters.keys()))

    def _log_event_counters(self):
        for c in self.event_counters.values():
            log_dist(f"{c.name}: count = {c.count}, numel = {c.num_elem}", ranks=[0])

    def log_events(self):
        self._log_event_counters()
        self._log_timers()
