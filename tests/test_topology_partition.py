"""Topology rank math and layer partitioners (reference: test_topology.py, test_partition.py)."""

import pytest
import torch

from common import distributed_test
from deeperspeed_amd.parallel.topology import (PipeDataParallelTopology, PipeModelDataParallelTopology,
                                               PipelineParallelGrid, ProcessTopology, _prime_factors)
from deeperspeed_amd.runtime.utils import PartitionedTensor, partition_balanced, partition_uniform


def test_topology_2d():
    topo = ProcessTopology(axes=["row", "col"], dims=[2, 2])
    assert topo.world_size() == 4
    assert topo.get_rank(row=0, col=0) == 0
    assert topo.get_rank(row=0, col=1) == 1
    assert topo.get_rank(row=1, col=0) == 2
    assert topo.get_rank(row=1, col=1) == 3
    assert topo.get_axis_list(axis="row", idx=0) == [0, 1]
    assert topo.get_axis_list(axis="col", idx=0) == [0, 2]


def test_topology_dims():
    topo = ProcessTopology(axes=["a", "b", "c"], dims=[2, 3, 4])
    assert topo.world_size() == 24
    assert topo.get_dim("a") == 2 and topo.get_dim("b") == 3 and topo.get_dim("c") == 4
    assert topo.get_dim("missing") == 0


def test_topology_match():
    topo = ProcessTopology(axes=["pipe", "data", "model"], dims=[2, 2, 2])
    assert topo.filter_match(pipe=0, data=1) == [2, 3]
    assert topo.filter_match(pipe=1) == [4, 5, 6, 7]


def test_topology_rank_repr():
    topo = ProcessTopology(axes=["a", "b"], dims=[2, 2])
    assert topo.get_rank_repr(rank=0) == "a_00-b_00"
    assert topo.get_rank_repr(rank=3) == "a_01-b_01"
    assert topo.get_rank_repr(rank=3, omit_axes=["a"]) == "b_01"
    assert topo.get_rank_repr(rank=3, inner_sep="+", outer_sep="|") == "a+01|b+01"
    topo = PipeModelDataParallelTopology(num_pp=2, num_dp=2, num_mp=2)
    assert topo.get_rank_repr(rank=0) == "model_00"
    assert topo.get_rank_repr(rank=1) == "model_01"
    assert topo.get_rank_repr(rank=4, omit_axes=[]) == "pipe_01-data_00-model_00"


def test_topology_3d_comm_lists():
    topo = ProcessTopology(axes=["pipe", "data", "model"], dims=[2, 2, 2])
    assert topo.get_axis_comm_lists("pipe") == [[0, 4], [1, 5], [2, 6], [3, 7]]
    assert topo.get_axis_comm_lists("data") == [[0, 2], [1, 3], [4, 6], [5, 7]]
    assert topo.get_axis_comm_lists("model") == [[0, 1], [2, 3], [4, 5], [6, 7]]
    assert topo.get_axis_comm_lists("jeff") == []
    assert topo.get_coord(7) == topo.ProcessCoord(pipe=1, data=1, model=1)


def test_primes():
    assert _prime_factors(1) == []
    assert _prime_factors(12) == [2, 2, 3]
    assert _prime_factors(97) == [97]
    with pytest.raises(ValueError):
        _prime_factors(0)


def _grid_body():
    import torch.distributed as dist
    topo = PipeDataParallelTopology(num_pp=2, num_dp=2)
    grid = PipelineParallelGrid(topology=topo)
    rank = dist.get_rank()
    assert grid.get_stage_id() == rank // 2
    assert grid.get_data_parallel_id() == rank % 2
    assert grid.get_pipe_parallel_world_size() == 2
    assert grid.get_data_parallel_world_size() == 2
    assert grid.stage_to_global(stage_id=0) == rank % 2
    assert grid.stage_to_global(stage_id=1) == 2 + rank % 2
    t = torch.tensor([float(rank)])
    dist.all_reduce(t, group=grid.get_data_parallel_group())
    assert t.item() == (0 + 1 if rank < 2 else 2 + 3)
    t = torch.tensor([float(rank)])
    dist.all_reduce(t, group=grid.get_pipe_parallel_group())
    assert t.item() == (rank % 2) * 2 + 2
    # PartitionedTensor over the data group round-trips
    x = torch.arange(13, dtype=torch.float32) * (1 + rank % 2 * 0)
    part = PartitionedTensor(x, group=grid.get_data_parallel_group())
    full = part.full()
    assert torch.equal(full, x)
    meta = part.to_meta()
    again = PartitionedTensor.from_meta(meta, part.data(), group=grid.get_data_parallel_group(), device="cpu")
    assert torch.equal(again.full(), x)


def test_grid_4ranks():
    from common import run_distributed
    run_distributed(_grid_body, 4)


def test_partition_uniform():
    assert partition_uniform(num_items=7, num_parts=4) == [0, 1, 2, 3, 7]  # last part takes the remainder
    assert partition_uniform(num_items=4, num_parts=4) == [0, 1, 2, 3, 4]
    assert partition_uniform(num_items=2, num_parts=4) == [0, 1, 2, 2, 2]
    assert partition_uniform(num_items=8, num_parts=4) == [0, 2, 4, 6, 8]


def _part_weight(weights, parts):
    return [sum(weights[parts[i]:parts[i + 1]]) for i in range(len(parts) - 1)]


@pytest.mark.parametrize("weights,num_parts", [([1] * 8, 4), ([1, 2, 3, 4, 5, 6, 7, 8], 3), ([0, 1, 1, 1, 0], 2),
                                                ([10, 1, 1, 1, 1, 10], 3), ([1] * 50 + [5], 7)])
def test_partition_balanced_is_optimal(weights, num_parts):
    parts = partition_balanced(weights, num_parts)
    assert parts[0] == 0 and parts[-1] == len(weights) and len(parts) == num_parts + 1
    assert all(parts[i] <= parts[i + 1] for i in range(num_parts))
    best = max(_part_weight(weights, parts))
    # brute force for the optimal bottleneck on small inputs
    import itertools
    n = len(weights)
    if n <= 12:
        opt = min(max(_part_weight(weights, [0, *c, n])) for c in itertools.combinations_with_replacement(range(n + 1),
                                                                                                         num_parts - 1)
                  if list(c) == sorted(c))
        assert best == opt
    assert best <= sum(weights) / num_parts + max(weights)
