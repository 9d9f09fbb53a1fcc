"""Pipeline schedules: pure-Python generators of per-step instruction lists.

Reference parity: deepspeed/runtime/pipe/schedule.py:1-482 (same instruction vocabulary and
the same interleaved 1F1B timeline, so a given (micro_batches, stages, stage_id) yields the
same command stream).  Timeline used here, for global step t on stage s of P stages:

    forward  micro-batch  t//2 - s//2                 when (t - s) is even
    backward micro-batch  (t+1)//2 - P + (s+1)//2     when (t - s) is odd

Even and odd stages are thus always in opposite phases, which is what lets every
send be matched by the neighbour's recv within the same step without deadlock.
"""

from __future__ import annotations

from abc import ABC, abstractmethod


def _is_even(x):
    return x % 2 == 0


def _is_odd(x):
    return x % 2 != 0


class PipeInstruction:
    """Base class of instructions; kwargs become attributes (namedtuple-like)."""

    def __init__(self, **kwargs):
        self.name = self.__class__.__name__
        self.kwargs = kwargs
        for k, v in kwargs.items():
            setattr(self, k, v)

    def __repr__(self):
        args = ", ".join(f"{k}={v}" for k, v in self.kwargs.items())
        return f"{self.name}({args})"

    def __eq__(self, other):
        return type(self) is type(other) and self.kwargs == other.kwargs

    def __hash__(self):
        return hash((self.name, tuple(sorted(self.kwargs.items()))))


class OptimizerStep(PipeInstruction):
    """Performs one step with the optimizer and zeros gradients."""


class ReduceGrads(PipeInstruction):
    """Reduce the computed gradients among data-parallel processes within the stage."""


class ReduceTiedGrads(PipeInstruction):
    """Reduce the gradients of tied modules within a pipeline-parallel group."""


class BufferOpInstruction(PipeInstruction):
    def __init__(self, buffer_id, **kwargs):
        super().__init__(buffer_id=buffer_id, **kwargs)


class LoadMicroBatch(BufferOpInstruction):
    """Load a micro-batch into a buffer (first and last stages)."""


class ForwardPass(BufferOpInstruction):
    """Compute a forward pass."""


class BackwardPass(BufferOpInstruction):
    """Compute a backward pass and accumulate gradients."""


class SendActivation(BufferOpInstruction):
    """Send activations to the next stage in the pipeline."""


class RecvActivation(BufferOpInstruction):
    """Receive activations from the previous stage in the pipeline."""


class SendGrad(BufferOpInstruction):
    """Send computed gradients to the previous pipeline stage."""


class RecvGrad(BufferOpInstruction):
    """Receive computed gradients the next pipeline stage."""


class PipeSchedule(ABC):
    def __init__(self, micro_batches, stages, stage_id):
        self.micro_batches = micro_batches
        self.stages = stages
        self.stage_id = stage_id
        self.prev_stage = stage_id - 1
        self.next_stage = stage_id + 1

    @abstractmethod
    def steps(self):
        """Yield a list of PipeInstructions for each step of the schedule."""

    def num_pipe_buffers(self):
        return self.micro_batches

    def _valid_micro_batch(self, micro_batch_id):
        return 0 <= micro_batch_id < self.micro_batches

    def _valid_stage(self, stage_id):
        return 0 <= stage_id < self.stages

    @property
    def stage(self):
        return self.stage_id

    @property
    def num_stages(self):
        return self.stages

    @property
    def num_micro_batches(self):
        return self.micro_batches

    @property
    def is_first_stage(self):
        return self.stage_id == 0

    @property
    def is_last_stage(self):
        return self.stage_id == self.stages - 1

    def _buffer_idx(self, micro_batch_id):
        assert self._valid_micro_batch(micro_batch_id)
        return micro_batch_id % self.num_pipe_buffers()

    def __iter__(self):
        self.it = None
        return self

    def __next__(self):
        if self.it is None:
            self.it = self.steps()
        return next(self.it)


class InferenceSchedule(PipeSchedule):
    """Forward-only pipeline: stage s handles micro-batch t - s at step t, two rotating
    buffers, even stages send-then-recv and odd stages recv-then-send."""

    def steps(self):
        for t in range(self.micro_batches + self.stages - 1):
            mb = t - self.stage_id
            even = _is_even(self.stage_id)
            recv_buf = t % 2 if even else (t + 1) % 2
            send_buf = (t + 1) % 2 if even else t % 2
            cmds = []
            if (self.is_first_stage or self.is_last_stage) and self._valid_micro_batch(mb):
                cmds.append(LoadMicroBatch(recv_buf))
            send = [SendActivation(send_buf)] if (self._valid_stage(self.next_stage) and
                                                  self._valid_micro_batch(mb - 1)) else []
            recv = [RecvActivation(recv_buf)] if (self._valid_stage(self.prev_stage) and
                                                  self._valid_micro_batch(mb)) else []
            cmds.extend(send + recv if even else recv + send)
            if self._valid_micro_batch(mb):
                cmds.append(ForwardPass(recv_buf))
            yield cmds

    def num_pipe_buffers(self):
        return 2


class TrainSchedule(PipeSchedule):
    """Interleaved 1F1B training schedule (gradient accumulation across micro-batches)."""

    def _step_to_micro_batch(self, step_id):
        s, P = self.stage_id, self.stages
        if _is_even(step_id - s):
            return step_id // 2 - s // 2, True
        return (step_id + 1) // 2 - P + (s + 1) // 2, False

    def steps(self):
        total = 2 * (self.micro_batches + self.stages - 1)
        prev_mb = -1
        for t in range(total):
            mb, is_fwd = self._step_to_micro_batch(t)
            cur_ok, prev_ok = self._valid_micro_batch(mb), self._valid_micro_batch(prev_mb)
            cur_buf = self._buffer_idx(mb) if cur_ok else None
            prev_buf = self._buffer_idx(prev_mb) if prev_ok else None
            cmds = []
            if is_fwd:
                if cur_ok and self._valid_stage(self.prev_stage):
                    cmds.append(RecvActivation(cur_buf))
                if prev_ok and self._valid_stage(self.prev_stage):
                    cmds.append(SendGrad(prev_buf))
            else:
                if prev_ok and self._valid_stage(self.next_stage):
                    cmds.append(SendActivation(prev_buf))
                if cur_ok and self._valid_stage(self.next_stage):
                    cmds.append(RecvGrad(cur_buf))
            if (self.is_first_stage or self.is_last_stage) and is_fwd and cur_ok:
                cmds.append(LoadMicroBatch(cur_buf))
            if cur_ok:
                cmds.append(ForwardPass(cur_buf) if is_fwd else BackwardPass(cur_buf))
            if t == total - 1:
                cmds.extend([ReduceTiedGrads(), ReduceGrads(), OptimizerStep()])
            prev_mb = mb
            yield cmds

    def num_pipe_buffers(self):
        """As many buffers as the distance from this stage to the last stage (>= 2)."""
        return max(2, min(self.stages - self.stage_id + 1, self.micro_batches))


class DataParallelSchedule(PipeSchedule):
    """Plain data parallelism with gradient accumulation (one buffer)."""

    def steps(self):
        for step_id in range(self.micro_batches):
            cmds = [LoadMicroBatch(buffer_id=0), ForwardPass(buffer_id=0), BackwardPass(buffer_id=0)]
            if step_id == self.micro_batches - 1:
                cmds.extend([ReduceGrads(), OptimizerStep()])
            yield cmds

    def num_pipe_buffers(self):
        return 1
