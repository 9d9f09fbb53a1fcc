"""Process topologies and the 3D parallel grid (pipe x data x model).

Reference parity: deepspeed/runtime/pipe/topology.py:13-467 -- `ProcessTopology` (row-major
rank <-> named-coordinate mapping, axis comm lists, filtering, rank repr for checkpoint
names), `PipeDataParallelTopology`, `PipeModelDataParallelTopology` (axes
['pipe','data','model'], data before model) and `PipelineParallelGrid`, the `mpu` object
consumed by the engine (model-parallel group = every rank sharing a data-parallel index,
i.e. pipe x tensor; slice group = tensor axis; p2p groups between adjacent stages).

MI355X note: with 8 GPUs on one xGMI mesh every placement is one hop, so the axis order is
chosen for determinism/compatibility, not for link locality.
"""

from __future__ import annotations

import itertools
from collections import namedtuple
from typing import Dict, List

import torch.distributed as dist


class ProcessTopology:
    def __init__(self, axes: List[str], dims: List[int]):
        self.axes = list(axes)
        self.dims = list(dims)
        self.ProcessCoord = namedtuple("ProcessCoord", self.axes)
        self.mapping: Dict = {}
        self._by_rank: Dict[int, tuple] = {}
        for rank, coord in enumerate(itertools.product(*[range(d) for d in self.dims])):
            key = self.ProcessCoord(*coord)
            self.mapping[key] = rank
            self._by_rank[rank] = key

    def get_rank(self, **coord_kwargs):
        if len(coord_kwargs) != len(self.axes):
            raise ValueError("get_rank() does not support slices. Use filter_match())")
        key = self.ProcessCoord(**coord_kwargs)
        assert key in self.mapping, f"key {coord_kwargs} invalid"
        return self.mapping[key]

    def get_axis_names(self):
        return self.axes

    def get_rank_repr(self, rank, omit_axes=("data", "pipe"), inner_sep="_", outer_sep="-"):
        omit = frozenset(omit_axes)
        coord = self.get_coord(rank)
        return outer_sep.join(f"{ax}{inner_sep}{getattr(coord, ax):02d}" for ax in self.axes if ax not in omit)

    def get_dim(self, axis):
        return self.dims[self.axes.index(axis)] if axis in self.axes else 0

    def get_coord(self, rank):
        if rank not in self._by_rank:
            raise ValueError(f"rank {rank} not found in topology.")
        return self._by_rank[rank]

    def get_axis_comm_lists(self, axis):
        """Lists of ranks that differ only along `axis` (one list per combination of the others)."""
        if axis not in self.axes:
            return []
        others = [a for a in self.axes if a != axis]
        out = []
        for combo in itertools.product(*[range(self.get_dim(a)) for a in others]):
            fixed = dict(zip(others, combo))
            out.append([self.mapping[self.ProcessCoord(**fixed, **{axis: i})] for i in range(self.get_dim(axis))])
        return out

    def filter_match(self, **filter_kwargs):
        return [r for key, r in self.mapping.items() if all(getattr(key, k) == v for k, v in filter_kwargs.items())]

    def get_axis_list(self, axis, idx):
        axis_num = self.axes.index(axis)
        return [self.mapping[k] for k in self.mapping.keys() if k[axis_num] == idx]

    def world_size(self):
        n = 1
        for d in self.dims:
            n *= d
        return n

    def __str__(self):
        return str(self.mapping)


def _prime_factors(n):
    if n <= 0:
        raise ValueError("Values must be strictly positive.")
    out, p = [], 2
    while n > 1:
        while n % p == 0:
            out.append(p)
            n //= p
        p += 1
    return out


class PipeDataParallelTopology(ProcessTopology):
    """pipe x data (data innermost so DP neighbours are adjacent ranks)."""

    def __init__(self, num_pp, num_dp):
        super().__init__(axes=["pipe", "data"], dims=[num_pp, num_dp])


class PipeModelDataParallelTopology(ProcessTopology):
    """pipe x data x model (tensor-parallel innermost)."""

    def __init__(self, num_pp, num_mp, num_dp):
        super().__init__(axes=["pipe", "data", "model"], dims=[num_pp, num_dp, num_mp])


class PipelineParallelGrid:
    """The mpu of pipeline/3D runs: process groups and rank queries per axis."""

    def __init__(self, topology=None, process_group=None):
        self.global_rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        if topology is not None:
            self._topo = topology
        else:
            num_pp = num_dp = 1
            for i, p in enumerate(_prime_factors(self.world_size)):
                if i % 2 == 0:
                    num_pp *= p
                else:
                    num_dp *= p
            self._topo = PipeDataParallelTopology(num_dp=num_dp, num_pp=num_pp)
        self.data_parallel_size = max(self._topo.get_dim("data"), 1)
        self.pipe_parallel_size = max(self._topo.get_dim("pipe"), 1)
        self.model_parallel_size = max(self._topo.get_dim("model"), 1)
        assert self._is_grid_valid(), "Invalid Grid"
        self.stage_id = self.get_stage_id()
        self.data_parallel_id = self.get_data_parallel_id()

        # "model parallel" group of the engine: all ranks with the same data index (pipe x model)
        self.ds_model_proc_group, self.ds_model_rank = None, -1
        for dp in range(self.data_parallel_size):
            ranks = sorted(self._topo.get_axis_list(axis="data", idx=dp))
            g = dist.new_group(ranks=ranks)
            if self.global_rank in ranks:
                self.ds_model_proc_group = g
                self.ds_model_world_size = len(ranks)
                self.ds_model_rank = ranks.index(self.global_rank)
        assert self.ds_model_rank > -1 and self.ds_model_proc_group is not None

        self.dp_group, self.dp_groups = [], self._topo.get_axis_comm_lists("data")
        for ranks in self.dp_groups:
            g = dist.new_group(ranks=ranks)
            if self.global_rank in ranks:
                self.dp_group, self.dp_proc_group = ranks, g

        self.is_first_stage = self.stage_id == 0
        self.is_last_stage = self.stage_id == self.pipe_parallel_size - 1
        self.p2p_groups = self._build_p2p_groups()

        self.pp_group, self.pp_proc_group = [], None
        self.pipe_groups = self._topo.get_axis_comm_lists("pipe")
        for ranks in self.pipe_groups:
            g = dist.new_group(ranks=ranks)
            if self.global_rank in ranks:
                self.pp_group, self.pp_proc_group = ranks, g
        assert self.pp_proc_group is not None

        if self.model_parallel_size == 1:
            for r in range(self.world_size):
                g = dist.new_group(ranks=[r])
                if r == self.global_rank:
                    self.slice_group, self.slice_proc_group = [r], g
        else:
            self.model_groups = self._topo.get_axis_comm_lists("model")
            for ranks in self.model_groups:
                g = dist.new_group(ranks=ranks)
                if self.global_rank in ranks:
                    self.slice_group, self.slice_proc_group = ranks, g

    def get_stage_id(self):
        return self._topo.get_coord(rank=self.global_rank).pipe

    def get_data_parallel_id(self):
        return self._topo.get_coord(rank=self.global_rank).data

    def _build_p2p_groups(self):
        """Per pipe comm list, the (stage i, stage i+1 mod P) rank pairs."""
        comm_lists = self._topo.get_axis_comm_lists("pipe")
        groups = []
        for rank in range(self.world_size):
            for lst in comm_lists:
                assert len(lst) == self.pipe_parallel_size
                if rank in lst:
                    idx = lst.index(rank)
                    groups.append([lst[idx], lst[(idx + 1) % self.pipe_parallel_size]])
        assert len(groups) == self.world_size
        return groups

    def _is_grid_valid(self):
        n = 1
        for ax in self._topo.get_axis_names():
            n *= self._topo.get_dim(ax)
        return n == dist.get_world_size()

    def stage_to_global(self, stage_id, **kwargs):
        me = self._topo.get_coord(self.global_rank)._asdict()
        me.update(pipe=stage_id, **kwargs)
        return self._topo.get_rank(**me)

    def topology(self):
        return self._topo

    def get_global_rank(self):
        return self.global_rank

    def get_pipe_parallel_rank(self):
        return self.get_stage_id()

    def get_pipe_parallel_world_size(self):
        return self.pipe_parallel_size

    def get_pipe_parallel_group(self):
        return self.pp_proc_group

    def get_data_parallel_rank(self):
        return self.data_parallel_id

    def get_data_parallel_world_size(self):
        return self.data_parallel_size

    def get_data_parallel_src_rank(self):
        return self.dp_group[0] if self.dp_group else 0

    def get_data_parallel_group(self):
        return self.dp_proc_group

    def get_model_parallel_rank(self):
        return self.ds_model_rank

    def get_model_parallel_world_size(self):
        return self.ds_model_world_size

    def get_model_parallel_group(self):
        return self.ds_model_proc_group

    def get_slice_parallel_rank(self):
        if "model" in self._topo.get_axis_names():
            return self._topo.get_coord(rank=self.global_rank).model
        return 0

    def get_slice_parallel_world_size(self):
        return self.model_parallel_size

    def get_slice_parallel_group(self):
        return self.slice_proc_group
