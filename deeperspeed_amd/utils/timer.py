"""Timers (reference parity: deepspeed/utils/timer.py:19-182).

MI355X design: the reference synchronises the whole device at every start/stop
(`timer.py:29-41`).  Here GPU-side intervals are measured with HIP events recorded on
the current stream, resolved lazily when `elapsed()` is read, so timing never inserts a
host sync into the training loop.  On CPU (tests) wall clock is used.
"""

import time

import torch

from .logging import log_dist

try:
    import psutil
    PSUTILS_INSTALLED = True
except ImportError:  # pragma: no cover
    PSUTILS_INSTALLED = False


def _gpu():
    return torch.cuda.is_available()


class _Timer:
    def __init__(self, name):
        self.name_ = name
        self.elapsed_ = 0.0  # seconds, resolved
        self.started_ = False
        self.start_time = 0.0
        self._pending = []  # list of (start_event, end_event)
        self._start_ev = None
        self.use_events = _gpu()

    def start(self):
        assert not self.started_, f"timer {self.name_} has already been started"
        if self.use_events:
            self._start_ev = torch.cuda.Event(enable_timing=True)
            self._start_ev.record()
        self.start_time = time.time()
        self.started_ = True

    def stop(self, reset=False, record=False):
        assert self.started_, f"timer {self.name_} is not started"
        if self.use_events:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._pending.append((self._start_ev, ev))
            self._start_ev = None
        else:
            self.elapsed_ += time.time() - self.start_time
        self.started_ = False
        if reset:
            self.reset()

    def _resolve(self):
        if self._pending:
            for s, e in self._pending:
                e.synchronize()
                self.elapsed_ += s.elapsed_time(e) / 1000.0
            self._pending = []

    def reset(self):
        self.elapsed_ = 0.0
        self._pending = []
        self.started_ = False

    def elapsed(self, reset=True):
        started = self.started_
        if started:
            self.stop()
        self._resolve()
        e = self.elapsed_
        if reset:
            self.reset()
        if started:
            self.start()
        return e

    def mean(self):
        return self.elapsed(reset=False)


class SynchronizedWallClockTimer:
    """Group of named timers; same names/log format as the reference."""

    Timer = _Timer

    def __init__(self):
        self.timers = {}

    def __call__(self, name):
        if name not in self.timers:
            self.timers[name] = _Timer(name)
        return self.timers[name]

    @staticmethod
    def memory_usage():
        if not _gpu():
            return ""
        alloc = "mem_allocated: {:.4f} GB".format(torch.cuda.memory_allocated() / (1024 ** 3))
        max_alloc = "max_mem_allocated: {:.4f} GB".format(torch.cuda.max_memory_allocated() / (1024 ** 3))
        cache = "cache_allocated: {:.4f} GB".format(torch.cuda.memory_reserved() / (1024 ** 3))
        max_cache = "max_cache_allocated: {:.4f} GB".format(torch.cuda.max_memory_reserved() / (1024 ** 3))
        return " | {} | {} | {} | {}".format(alloc, max_alloc, cache, max_cache)

    def log(self, names, normalizer=1.0, reset=True, memory_breakdown=False, ranks=None):
        assert normalizer > 0.0
        string = "time (ms)"
        for name in names:
            if name in self.timers:
                elapsed_time = self.timers[name].elapsed(reset=reset) * 1000.0 / normalizer
                string += " | {}: {:.2f}".format(name, elapsed_time)
        if memory_breakdown:
            string += self.memory_usage()
        log_dist(string, ranks=ranks or [0])

    def get_timers_value(self, names, normalizer=1.0, reset=True):
        """DeeperSpeed addition (timer.py:84-102): return {name: ms} instead of logging."""
        out = {}
        for name in names:
            if name in self.timers:
                out[name] = self.timers[name].elapsed(reset=reset) * 1000.0 / normalizer
        return out


class ThroughputTimer:
    """Samples/sec over the steps after a warm-up (behaviour of reference timer.py:105-182).

    No host synchronisation on the hot path: each micro-step brackets itself with two HIP
    events on the current stream; the events are only resolved (one event wait) when a rate
    is reported or read, i.e. every `steps_per_output` steps.  On CPU wall clock is used.
    """

    def __init__(self, batch_size, num_workers=1, start_step=2, steps_per_output=50, monitor_memory=False,
                 logging_fn=None):
        self.batch_size = 1 if batch_size is None else batch_size
        self.num_workers = num_workers
        self.start_step = start_step
        self.steps_per_output = steps_per_output
        self.monitor_memory = monitor_memory
        self.logging = logging_fn or (lambda msg: log_dist(msg, ranks=[0]))
        self.epoch_count = 0
        self.local_step_count = 0
        self.total_step_count = 0
        self.total_elapsed_time = 0.0
        self.started = False
        self.initialized = False
        self._open = None  # start marker of the interval being measured
        self._closed = []  # finished (start, end) markers not yet folded into total_elapsed_time

    def update_epoch_count(self):
        self.epoch_count += 1
        self.local_step_count = 0

    @staticmethod
    def _mark():
        if _gpu():
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.time()

    def _fold(self, keep=0):
        """Fold finished intervals into the total; `keep` most recent ones stay pending (their
        end events may still be in flight, the older ones have long completed)."""
        done, self._closed = self._closed[:len(self._closed) - keep], self._closed[len(self._closed) - keep:]
        for a, b in done:
            if isinstance(a, float):
                self.total_elapsed_time += b - a
            else:
                b.synchronize()
                self.total_elapsed_time += a.elapsed_time(b) / 1000.0

    def start(self):
        self.initialized = True
        self.started = True
        self._open = self._mark() if self.total_step_count >= self.start_step else None

    def stop(self, report_speed=True):
        if not self.started:
            return
        self.started = False
        self.total_step_count += 1
        self.local_step_count += 1
        if self._open is not None and self.total_step_count > self.start_step:
            self._closed.append((self._open, self._mark()))
            if len(self._closed) > 64:  # bound the pending list on ranks that never report
                self._fold(keep=8)
        self._open = None
        if report_speed and self.local_step_count % self.steps_per_output == 0:
            self.logging(f"{self.epoch_count}/{self.local_step_count}, SamplesPerSec={self.avg_samples_per_sec()}")
            if self.monitor_memory and PSUTILS_INSTALLED:
                vm, sw = psutil.virtual_memory(), psutil.swap_memory()
                self.logging(f"{self.epoch_count}/{self.local_step_count}, vm percent: {vm.percent}, "
                             f"swap percent: {sw.percent}")

    def avg_samples_per_sec(self):
        self._fold()
        measured = self.total_step_count - self.start_step
        if measured <= 0 or self.total_elapsed_time <= 0:
            return float("-inf")
        return self.batch_size * self.num_workers * measured / self.total_elapsed_time
