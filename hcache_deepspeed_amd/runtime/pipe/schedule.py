"""Pipeline schedules as instruction streams.

Reference parity: runtime/pipe/schedule.py (``PipeSchedule``, ``InferenceSchedule``, ``TrainSchedule``
:189-299, ``DataParallelSchedule``, the ``PipeInstruction`` family). The reference TrainSchedule walks
a 2*(M+S-1) step grid and lets even/odd stages order their sends/receives. Here the 1F1B order is
generated directly per stage (warm-up forwards, steady one-forward-one-backward, cool-down backwards)
and every group of *adjacent* communication instructions is issued by the engine as ONE batched
P2P call (``batch_isend_irecv`` -> one RCCL group over xGMI): a stage's "send my activation to
stage s+1" and "receive the gradient from stage s+1" travel in the same group on the two directions
of the same xGMI link, so a step never waits for a neighbour to finish an unrelated transfer.
"""


class PipeInstruction:

    def __init__(self, **kwargs):
        self.name = type(self).__name__
        self.kwargs = kwargs
        for k, v in kwargs.items():
            setattr(self, k, v)

    def __repr__(self):
        args = ", ".join(f"{k}={v}" for k, v in self.kwargs.items())
        return f"{self.name}({args})"

    def __eq__(self, other):
        return type(self) is type(other) and self.kwargs == other.kwargs


class OptimizerStep(PipeInstruction):
    pass


class ReduceGrads(PipeInstruction):
    pass


class ReduceTiedGrads(PipeInstruction):
    pass


class BufferOpInstruction(PipeInstruction):

    def __init__(self, buffer_id, **kwargs):
        super().__init__(buffer_id=buffer_id, **kwargs)


class LoadMicroBatch(BufferOpInstruction):
    pass


class ForwardPass(BufferOpInstruction):
    pass


class BackwardPass(BufferOpInstruction):
    pass


class SendActivation(BufferOpInstruction):
    pass


class RecvActivation(BufferOpInstruction):
    pass


class SendGrad(BufferOpInstruction):
    pass


class RecvGrad(BufferOpInstruction):
    pass


COMM_INSTRUCTIONS = (SendActivation, RecvActivation, SendGrad, RecvGrad)


class PipeSchedule:
    """Yields lists of instructions ("steps") for one stage of a ``stages``-deep pipeline."""

    def __init__(self, micro_batches, stages, stage_id):
        self.micro_batches = micro_batches
        self.stages = stages
        self.stage_id = stage_id
        self.prev_stage = stage_id - 1
        self.next_stage = stage_id + 1

    def steps(self):
        raise NotImplementedError

    def num_pipe_buffers(self):
        return self.micro_batches

    @property
    def is_first_stage(self):
        return self.stage_id == 0

    @property
    def is_last_stage(self):
        return self.stage_id == self.stages - 1

    def _valid_micro_batch(self, mb):
        return 0 <= mb < self.micro_batches

    def _valid_stage(self, s):
        return 0 <= s < self.stages

    def __iter__(self):
        return iter(self.steps())


class InferenceSchedule(PipeSchedule):
    """Forward-only fill/drain: every micro-batch flows through the stages in order."""

    def steps(self):
        for mb in range(self.micro_batches):
            cmds = []
            if self.is_first_stage or self.is_last_stage:
                cmds.append(LoadMicroBatch(mb))
            if not self.is_first_stage:
                cmds.append(RecvActivation(mb))
            cmds.append(ForwardPass(mb))
            if not self.is_last_stage:
                cmds.append(SendActivation(mb))
            yield cmds

    def num_pipe_buffers(self):
        return 2


class TrainSchedule(PipeSchedule):
    """1F1B: ``stages - stage_id - 1`` warm-up forwards, then alternate forward/backward, then drain.

    Peak in-flight activations per stage = warm-up + 1 (<= stages), independent of ``micro_batches``.
    """

    def num_pipe_buffers(self):
        return max(2, min(self.stages - self.stage_id, self.micro_batches))

    def _fwd(self, mb):
        cmds = []
        if self.is_first_stage or self.is_last_stage:
            cmds.append(LoadMicroBatch(mb))
        cmds.append(ForwardPass(mb))
        return cmds

    def steps(self):
        M = self.micro_batches
        first, last = self.is_first_stage, self.is_last_stage
        warmup = min(self.stages - self.stage_id - 1, M)
        steady = M - warmup
        f = b = 0
        for _ in range(warmup):
            cmds = [] if first else [RecvActivation(f)]
            cmds += self._fwd(f)
            if not last:
                cmds.append(SendActivation(f))
            f += 1
            yield cmds
        if steady > 0 and not first:
            yield [RecvActivation(f)]
        for i in range(steady):
            cmds = self._fwd(f)
            if not last:
                cmds += [SendActivation(f), RecvGrad(b)]
            cmds.append(BackwardPass(b))
            f += 1
            tail = []
            if not first:
                tail.append(SendGrad(b))
                if i < steady - 1:
                    tail.append(RecvActivation(f))
            b += 1
            yield cmds + tail
        for _ in range(warmup):
            cmds = [] if last else [RecvGrad(b)]
            cmds.append(BackwardPass(b))
            if not first:
                cmds.append(SendGrad(b))
            b += 1
            yield cmds
        yield [ReduceTiedGrads(), ReduceGrads(), OptimizerStep()]


class DataParallelSchedule(PipeSchedule):
    """Single-stage 'pipeline': plain gradient accumulation."""

    def steps(self):
        for mb in range(self.micro_batches):
            cmds = [LoadMicroBatch(mb), ForwardPass(mb), BackwardPass(mb)]
            if mb == self.micro_batches - 1:
                cmds += [ReduceGrads(), OptimizerStep()]
            yield cmds

    def num_pipe_buffers(self):
        return 1
