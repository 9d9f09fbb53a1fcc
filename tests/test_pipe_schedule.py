"""Pipeline schedules (reference analogue: tests/unit/test_pipe_schedule.py)."""

import pytest

import deeperspeed_amd.runtime.pipe.schedule as schedule


def _count_type(cmds, classtype):
    return len([c for c in cmds if type(c) == classtype])


def test_pipe_inference_schedule_singlestage():
    sched = schedule.InferenceSchedule(micro_batches=4, stages=1, stage_id=0)
    assert sched.num_micro_batches == 4
    full = list(iter(sched))
    for idx, cmds in enumerate(full):
        assert len(cmds) == 2
        assert type(cmds[0]) == schedule.LoadMicroBatch
        assert type(cmds[1]) == schedule.ForwardPass
        assert cmds[0].buffer_id == cmds[1].buffer_id
    assert len(full) == sched.num_micro_batches


def test_pipe_train_schedule_singlestage():
    sched = schedule.TrainSchedule(micro_batches=4, stages=1, stage_id=0)
    full = list(iter(sched))
    for idx, cmds in enumerate(full):
        if (idx % 2) != 0:
            assert (len(cmds) == 1) or (len(cmds) == 4)
            assert type(cmds[0]) == schedule.BackwardPass
        else:
            assert len(cmds) == 2
            assert type(cmds[0]) == schedule.LoadMicroBatch
            assert type(cmds[1]) == schedule.ForwardPass
            assert cmds[0].buffer_id == cmds[1].buffer_id
    assert len(full) == sched.num_micro_batches * 2


@pytest.mark.parametrize("micro_batches", [1, 3, 8, 10])
def test_pipe_inference_schedule_firststage(micro_batches, stages=3):
    sched = schedule.InferenceSchedule(micro_batches=micro_batches, stages=stages, stage_id=0)
    full = list(iter(sched))
    for idx, cmds in enumerate(full):
        if idx < micro_batches:
            assert _count_type(cmds, schedule.LoadMicroBatch) == 1
            assert _count_type(cmds, schedule.ForwardPass) == 1
        else:
            assert len(cmds) <= 1
        if 0 < idx <= micro_batches:
            assert _count_type(cmds, schedule.SendActivation) == 1
    assert len(full) == micro_batches + stages - 1


@pytest.mark.parametrize("micro_batches", [1, 3, 8, 10])
def test_pipe_inference_schedule_midstage(micro_batches, stages=3):
    sched = schedule.InferenceSchedule(micro_batches=micro_batches, stages=stages, stage_id=1)
    full = list(iter(sched))
    for idx, cmds in enumerate(full):
        if idx < sched.stage or idx > sched.stage + micro_batches:
            assert len(cmds) == 0
            continue
        assert _count_type(cmds, schedule.LoadMicroBatch) == 0
        if idx <= sched.stage + micro_batches - 1:
            assert _count_type(cmds, schedule.ForwardPass) == 1
            assert _count_type(cmds, schedule.RecvActivation) == 1
        if idx > sched.stage:
            assert _count_type(cmds, schedule.SendActivation) == 1
    assert len(full) == micro_batches + stages - 1


@pytest.mark.parametrize("micro_batches", [1, 3, 8, 10])
def test_pipe_inference_schedule_laststage(micro_batches, stages=3):
    sched = schedule.InferenceSchedule(micro_batches=micro_batches, stages=stages, stage_id=2)
    full = list(iter(sched))
    for idx, cmds in enumerate(full):
        if idx < sched.stage or idx > sched.stage + micro_batches:
            assert len(cmds) == 0
            continue
        assert _count_type(cmds, schedule.LoadMicroBatch) == 1
        assert _count_type(cmds, schedule.ForwardPass) == 1
        assert _count_type(cmds, schedule.RecvActivation) == 1
        assert _count_type(cmds, schedule.SendActivation) == 0
    assert len(full) == micro_batches + stages - 1


def _simulate(micro_batches, stages):
    """Every send must be matched by the neighbour's recv in the same step, forward
    activations of micro-batch m must be produced before they are consumed, and each
    stage must run exactly one forward and one backward per micro-batch."""
    scheds = [list(schedule.TrainSchedule(micro_batches, stages, s)) for s in range(stages)]
    total = 2 * (micro_batches + stages - 1)
    for s in range(stages):
        assert len(scheds[s]) == total
        fwd = sum(_count_type(c, schedule.ForwardPass) for c in scheds[s])
        bwd = sum(_count_type(c, schedule.BackwardPass) for c in scheds[s])
        assert fwd == micro_batches and bwd == micro_batches
        assert type(scheds[s][-1][-1]) == schedule.OptimizerStep
    for t in range(total):
        for s in range(stages - 1):
            a = scheds[s][t]
            b = scheds[s + 1][t]
            assert _count_type(a, schedule.SendActivation) == _count_type(b, schedule.RecvActivation), (t, s)
            assert _count_type(b, schedule.SendGrad) == _count_type(a, schedule.RecvGrad), (t, s)


@pytest.mark.parametrize("micro_batches,stages", [(1, 2), (4, 2), (8, 4), (3, 5), (16, 8)])
def test_train_schedule_matches_across_stages(micro_batches, stages):
    _simulate(micro_batches, stages)


def test_num_pipe_buffers():
    assert schedule.TrainSchedule(8, 4, 0).num_pipe_buffers() == 5
    assert schedule.TrainSchedule(8, 4, 3).num_pipe_buffers() == 2
    assert schedule.TrainSchedule(1, 4, 0).num_pipe_buffers() == 2
    assert schedule.InferenceSchedule(8, 4, 1).num_pipe_buffers() == 2
    assert schedule.DataParallelSchedule(4, 1, 0).num_pipe_buffers() == 1
