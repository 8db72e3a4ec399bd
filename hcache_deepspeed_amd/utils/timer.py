"""Wall-clock timers (reference: utils/timer.py SynchronizedWallClockTimer :32-160, ThroughputTimer :199-313).

On GPU the timers use HIP events on the current stream, so a timed region does not force a device
synchronisation until it is read.
"""
import time

import torch

from .logging import log_dist


class _Timer:

    def __init__(self, name, use_events):
        self.name = name
        self.use_events = use_events
        self.elapsed_ = 0.0
        self.started = False
        self._events = []
        self._t0 = None

    def start(self):
        if self.started:
            return
        if self.use_events:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events.append([e, None])
        else:
            self._t0 = time.perf_counter()
        self.started = True

    def stop(self, reset=False, record=False):
        if not self.started:
            return
        if self.use_events:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events[-1][1] = e
        else:
            self.elapsed_ += time.perf_counter() - self._t0
        self.started = False

    def _flush(self):
        if self.use_events and self._events:
            done = [p for p in self._events if p[1] is not None]
            if done:
                done[-1][1].synchronize()
                for s, e in done:
                    self.elapsed_ += s.elapsed_time(e) / 1e3
                self._events = [p for p in self._events if p[1] is None]

    def reset(self):
        self.elapsed_ = 0.0
        self._events = []
        self.started = False

    def elapsed(self, reset=True):
        started = self.started
        if started:
            self.stop()
        self._flush()
        v = self.elapsed_
        if reset:
            self.reset()
        if started:
            self.start()
        return v

    def mean(self):
        return self.elapsed(reset=False)


class SynchronizedWallClockTimer:

    def __init__(self):
        self.timers = {}
        self.use_events = torch.cuda.is_available()

    def __call__(self, name):
        if name not in self.timers:
            self.timers[name] = _Timer(name, self.use_events)
        return self.timers[name]

    def get_timers(self):
        return self.timers

    def log(self, names, normalizer=1.0, reset=True, memory_breakdown=False, ranks=None):
        s = "time (ms)"
        for n in names:
            if n in self.timers:
                s += f" | {n}: {self.timers[n].elapsed(reset=reset) * 1000.0 / normalizer:.2f}"
        log_dist(s, ranks=ranks or [0])

    def get_mean(self, names, normalizer=1.0, reset=True):
        return {n: self.timers[n].elapsed(reset=reset) * 1000.0 / normalizer for n in names if n in self.timers}


class NoopTimer:

    class _T:

        def start(self):
            pass

        def stop(self, **kw):
            pass

        def reset(self):
            pass

        def elapsed(self, **kw):
            return 0.0

        def mean(self):
            return 0.0

    def __init__(self):
        self.t = self._T()

    def __call__(self, name):
        return self.t

    def get_timers(self):
        return {}

    def log(self, *a, **k):
        pass

    def get_mean(self, *a, **k):
        return {}


class ThroughputTimer:
    """samples/s (and tokens/s when ``tokens_per_sample`` given) with warm-up steps excluded."""

    def __init__(self, batch_size, start_step=2, steps_per_output=50, monitor_memory=False, logging_fn=None,
                 tokens_per_sample=None):
        self.batch_size = batch_size
        self.start_step = start_step
        self.steps_per_output = steps_per_output
        self.tokens_per_sample = tokens_per_sample
        self.global_step_count = 0
        self.micro_step_count = 0
        self.total_elapsed_time = 0.0
        self.step_elapsed_time = 0.0
        self._t0 = None
        self.started = False

    def start(self):
        self.started = True
        if self.global_step_count >= self.start_step:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self._t0 = time.perf_counter()

    def stop(self, global_step=False, report_speed=True):
        if not self.started:
            return
        self.started = False
        self.micro_step_count += 1
        if global_step:
            self.global_step_count += 1
        if self._t0 is not None:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            dt = time.perf_counter() - self._t0
            self.total_elapsed_time += dt
            self.step_elapsed_time += dt
            self._t0 = None

    def avg_samples_per_sec(self):
        steps = self.global_step_count - self.start_step
        if steps > 0 and self.total_elapsed_time > 0:
            return self.batch_size * steps / self.total_elapsed_time
        return float("-inf")
