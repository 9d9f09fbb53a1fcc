"""PipelineModule: a model written as a list of layers, each pipeline stage owning a slice.

Behavioural parity with deepspeed/runtime/pipe/module.py:19-589:
* `LayerSpec(cls, *args, **kw)` defers construction so a stage builds only its own layers;
  `TiedLayerSpec(key, cls, ..., forward_fn, tied_weight_attr)` shares one module between
  the stages that use `key` (embedding / LM head): weights broadcast from the lowest stage
  at construction, gradients all-reduced over the stages by `allreduce_tied_weight_gradients`.
* partition methods `uniform`, `parameters` (balanced by trainable parameter count) and
  `type:<regex>` (balanced by the number of layers whose class name matches).
* `activation_checkpoint_interval` recomputes groups of that many consecutive layers; the
  DeeperSpeed `checkpointable_layers` list restricts which groups qualify.
* `seed_layers` seeds each layer's construction and each forward deterministically.
* checkpoints: one file per layer, `layer_XX[-<rank repr>]-model_states.pt`, written by
  data-parallel rank 0; `ckpt_prefix` for the stage's engine state.

Structure here: the stage plan (partition boundaries) is computed once by `_plan_stages`;
the local layers are `_Slot` records (callable + owning module or tie key); the forward is a
precomputed list of `_Segment`s (range + whether it is recomputed), run by one loop, so no
closures are rebuilt per micro-batch.
"""

from __future__ import annotations

import os
import re
from dataclasses import dataclass, field
from functools import partial
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ...parallel.topology import PipeDataParallelTopology, PipelineParallelGrid
from ...utils.logging import logger
from .. import utils as ds_utils
from ..activation_checkpointing import checkpointing


class PipelineError(Exception):
    """Errors related to the use of deepspeed.PipelineModule."""


class LayerSpec:
    """A layer to be built later: `LayerSpec(nn.Linear, 8, 4)` -> `nn.Linear(8, 4)` on the
    owning stage only."""

    def __init__(self, typename, *module_args, **module_kwargs):
        if not (isinstance(typename, type) and issubclass(typename, nn.Module)):
            raise RuntimeError("LayerSpec only supports torch.nn.Module types.")
        self.typename = typename
        self.module_args = module_args
        self.module_kwargs = module_kwargs
        self.global_rank = dist.get_rank() if dist.is_initialized() else -1

    def __repr__(self):
        return ds_utils.call_to_str(self.typename.__name__, *self.module_args, **self.module_kwargs)

    def build(self, log=False):
        if log:
            logger.info(f"RANK={self.global_rank} building {self!r}")
        return self.typename(*self.module_args, **self.module_kwargs)


class TiedLayerSpec(LayerSpec):
    """A layer whose module (and `tied_weight_attr` parameter) is shared by every position
    using the same `key`; `forward_fn(module, x)` lets a position use it differently (e.g.
    the LM head reading the embedding matrix)."""

    def __init__(self, key, typename, *module_args, forward_fn=None, tied_weight_attr="weight", **module_kwargs):
        super().__init__(typename, *module_args, **module_kwargs)
        self.key = key
        self.forward_fn = forward_fn
        self.tied_weight_attr = tied_weight_attr


@dataclass
class _Slot:
    index: int                      # global layer index
    fn: Callable                    # what forward calls
    module: Optional[nn.Module]     # registered submodule (None for tied layers / plain callables)
    tie_key: Optional[str] = None


@dataclass
class _Segment:
    start: int
    stop: int
    recompute: bool


@dataclass
class _TieGroup:
    ranks: List[int]
    group: object
    weight_attr: str
    module: nn.Module = field(repr=False)

    def __getitem__(self, k):  # dict-style access kept for callers written against the reference
        return {"ranks": self.ranks, "group": self.group, "weight_attr": self.weight_attr, "module": self.module}[k]


def _layer_name(layer) -> Optional[str]:
    if isinstance(layer, LayerSpec):
        return layer.typename.__name__
    if isinstance(layer, nn.Module):
        return type(layer).__name__
    return getattr(layer, "__name__", None)


def _trainable_numel(layer) -> int:
    if isinstance(layer, LayerSpec):
        mod = layer.build()
        n = sum(p.numel() for p in mod.parameters() if p.requires_grad)
        del mod
        return n
    if isinstance(layer, nn.Module):
        return sum(p.numel() for p in layer.parameters() if p.requires_grad)
    return 0


def _plan_stages(specs, num_stages: int, method: str) -> List[int]:
    """Stage boundaries (len num_stages + 1) for the layer list under a partition method."""
    method = method.lower()
    n = len(specs)
    if method == "uniform":
        return ds_utils.partition_uniform(num_items=n, num_parts=num_stages)
    if method == "parameters":
        return ds_utils.partition_balanced(weights=[_trainable_numel(s) for s in specs], num_parts=num_stages)
    if method.startswith("type:"):
        rx = re.compile(method.split(":", 1)[1], re.IGNORECASE)
        hits = [1 if (_layer_name(s) is not None and rx.search(_layer_name(s))) else 0 for s in specs]
        if not any(hits):
            raise RuntimeError(f"Partitioning '{method[5:]}' found no valid layers to partition.")
        return ds_utils.partition_balanced(weights=hits, num_parts=num_stages)
    raise NotImplementedError(f"Partitioning method {method} not implemented.")


class PipelineModule(nn.Module):
    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seed_layers=False, seed_fn=None,
                 base_seed=1234, partition_method="parameters", activation_checkpoint_interval=0,
                 activation_checkpoint_func=checkpointing.checkpoint, checkpointable_layers=None):
        super().__init__()
        if num_stages is None and topology is None:
            raise RuntimeError("must provide num_stages or topology")
        if checkpointable_layers is not None and not isinstance(checkpointable_layers, list):
            raise TypeError("checkpointable_layers must be a list of class names")
        if not dist.is_initialized():
            from ...utils.distributed import init_distributed
            init_distributed()
        self.loss_fn = loss_fn
        self.seed_layers = seed_layers
        self.seed_fn = seed_fn
        self.base_seed = base_seed
        self.micro_offset = 0
        self.curr_layer = -1
        self.activation_checkpoint_func = activation_checkpoint_func
        self.checkpointable_layers = checkpointable_layers

        self.world_group = dist.new_group(ranks=range(dist.get_world_size()))
        self.global_rank = dist.get_rank(group=self.world_group)
        self.world_size = dist.get_world_size(group=self.world_group)
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if topology is None:
            if self.world_size % num_stages:
                raise RuntimeError(f"num_stages ({num_stages}) must divide distributed world size ({self.world_size})")
            topology = PipeDataParallelTopology(num_pp=num_stages, num_dp=self.world_size // num_stages)
        self._topo = topology
        self.num_stages = topology.get_dim("pipe")
        self._grid = PipelineParallelGrid(process_group=self.world_group, topology=topology)
        self.stage_id = topology.get_coord(self.global_rank).pipe

        self._layer_specs = list(layers)
        self._num_layers = len(self._layer_specs)
        self.parts = _plan_stages(self._layer_specs, self.num_stages, partition_method)
        self._local_start, self._local_stop = self.parts[self.stage_id], self.parts[self.stage_id + 1]
        if self.global_rank == 0:
            for s in range(self.num_stages):
                logger.info(f"stage={s} layers={self.parts[s + 1] - self.parts[s]}")

        self.tied_modules = nn.ModuleDict()
        self.tied_weight_attrs: Dict[str, str] = {}
        self._slots: List[_Slot] = [self._materialize(i) for i in range(self._local_start, self._local_stop)]
        # a stage's parameters are its own: norms / overflow checks reduce over the pipe group
        for p in self.parameters():
            p.model_parallel = True
        if torch.cuda.is_available():
            self.to(f"cuda:{self.local_rank % max(1, torch.cuda.device_count())}")
        self.tied_comms = self._make_tie_groups()
        self._synchronize_tied_weights()
        self.activation_checkpoint_interval = activation_checkpoint_interval

    # ------------------------------------------------------------------ construction
    def _seed(self, value):
        (self.seed_fn or ds_utils.set_random_seed)(value)

    def _materialize(self, idx) -> _Slot:
        spec = self._layer_specs[idx]
        if self.seed_layers:
            self._seed(self.base_seed + idx)
        if isinstance(spec, PipelineModule):
            raise NotImplementedError("nested PipelineModule layers are not supported")
        if isinstance(spec, TiedLayerSpec):
            if spec.key not in self.tied_modules:
                self.tied_modules[spec.key] = spec.build()
                self.tied_weight_attrs[spec.key] = spec.tied_weight_attr
            mod = self.tied_modules[spec.key]
            fn = mod if spec.forward_fn is None else partial(spec.forward_fn, mod)
            return _Slot(idx, fn, None, spec.key)
        if isinstance(spec, LayerSpec):
            spec = spec.build()
        if isinstance(spec, nn.Module):
            self.add_module(str(idx), spec)
            return _Slot(idx, spec, spec)
        return _Slot(idx, spec, None)  # plain callable (e.g. a lambda reshaping the activations)

    @property
    def forward_funcs(self) -> List[Callable]:
        return [s.fn for s in self._slots]

    def _make_tie_groups(self) -> Dict[str, _TieGroup]:
        """One process group per (tie key, data-parallel / model-parallel coordinate) spanning
        the stages that hold the key; every rank creates every group (collective)."""
        out: Dict[str, _TieGroup] = {}
        if self.num_stages == 1:
            return out
        keys = sorted({s.key for s in self._layer_specs if isinstance(s, TiedLayerSpec)})
        g = self._grid
        for key in keys:
            stages = sorted({self.stage_owner(i) for i, s in enumerate(self._layer_specs)
                             if isinstance(s, TiedLayerSpec) and s.key == key})
            for dp in range(g.data_parallel_size):
                for mp in range(g.model_parallel_size):
                    coord = {"data": dp, "model": mp} if g.model_parallel_size > 1 else {"data": dp}
                    ranks = [g.stage_to_global(stage_id=s, **coord) for s in stages]
                    pg = dist.new_group(ranks=ranks)
                    if self.global_rank not in ranks:
                        continue
                    out[key] = _TieGroup(ranks, pg, self.tied_weight_attrs[key], self.tied_modules[key])
                    if self.global_rank != ranks[0]:
                        # replicated copy: counted once (on the first stage) in grad norms
                        for p in self.tied_modules[key].parameters():
                            p.model_parallel = False
        return out

    def _synchronize_tied_weights(self):
        for t in self.tied_comms.values():
            dist.broadcast(getattr(t.module, t.weight_attr).data, src=min(t.ranks), group=t.group)

    def allreduce_tied_weight_gradients(self):
        for t in self.tied_comms.values():
            w = getattr(t.module, t.weight_attr)
            if w.grad is not None:
                dist.all_reduce(w.grad, group=t.group)

    # ------------------------------------------------------------------ forward
    @property
    def activation_checkpoint_interval(self):
        return self._ckpt_interval

    @activation_checkpoint_interval.setter
    def activation_checkpoint_interval(self, interval):
        if interval < 0:
            raise ValueError("activation_checkpoint_interval must be >= 0")
        self._ckpt_interval = int(interval)
        self._segments = self._make_segments()

    def set_checkpoint_interval(self, interval):
        self.checkpoint_interval = interval
        self.activation_checkpoint_interval = interval

    def _make_segments(self) -> List[_Segment]:
        n = len(self._slots)
        k = self._ckpt_interval
        if k == 0:
            return [_Segment(0, n, False)] if n else []
        return [_Segment(s, min(s + k, n), self._is_checkpointable(self.forward_funcs[s:min(s + k, n)]))
                for s in range(0, n, k)]

    def _is_checkpointable(self, funcs):
        if self.checkpointable_layers is not None:
            return all(type(f).__name__ in self.checkpointable_layers for f in funcs)
        if type(self).__name__ == "GPT2ModelPipe":  # DeeperSpeed special case for GPT-NeoX
            return all("ParallelTransformerLayerPipe" in type(f).__name__ for f in funcs)
        return any(any(True for _ in f.parameters()) for f in funcs if isinstance(f, nn.Module))

    def _run_range(self, seg: _Segment, micro: int, *inputs):
        x = inputs[0] if len(inputs) == 1 else inputs
        for slot in self._slots[seg.start:seg.stop]:
            self.curr_layer = slot.index
            if self.seed_layers:
                self._seed(self.base_seed * micro + slot.index)
            x = slot.fn(x)
        return x

    def forward(self, forward_input):
        self.micro_offset += 1
        micro = self.micro_offset + 1
        x = forward_input
        for seg in self._segments:
            args = x if isinstance(x, tuple) else (x,)
            if seg.recompute:
                x = self.activation_checkpoint_func(partial(self._run_range, seg, micro), *args)
            else:
                x = self._run_range(seg, micro, *args)
        return x

    # ------------------------------------------------------------------ topology queries
    def partitions(self):
        return self.parts

    def stage_owner(self, layer_idx):
        if not 0 <= layer_idx < self._num_layers:
            raise IndexError(f"layer {layer_idx} out of range [0, {self._num_layers})")
        for s in range(self.num_stages):
            if self.parts[s] <= layer_idx < self.parts[s + 1]:
                return s
        raise RuntimeError(f"Layer {layer_idx} not owned? parts={self.parts}")

    def topology(self):
        return self._topo

    def mpu(self):
        return self._grid

    def num_pipeline_stages(self):
        return self.num_stages

    # ------------------------------------------------------------------ checkpoints
    def ckpt_prefix(self, checkpoints_path, tag):
        coord = self._topo.get_coord(rank=self.global_rank)
        parts = [f"{a}_{getattr(coord, a):02d}" for a in self._topo.get_axis_names() if a != "data"]
        return os.path.join(checkpoints_path, str(tag), "-".join(["module"] + parts))

    def ckpt_layer_path(self, ckpt_dir, local_layer_idx):
        rank_repr = self._topo.get_rank_repr(rank=self.global_rank)
        name = f"layer_{local_layer_idx + self._local_start:02d}" + (f"-{rank_repr}" if rank_repr else "")
        return os.path.join(ckpt_dir, name + "-model_states.pt")

    def _stateful(self):
        """Positions that own a layer file: whatever forward calls, when it has a state dict
        (reference pipe/module.py:546-567 walks forward_funcs the same way).  A TiedLayerSpec
        position with a forward_fn calls a partial, so it writes no file: the tied module is
        saved (and restored, then broadcast to its tie group) by the position that calls it
        directly -- GPT-NeoX's tied embedding / LM head."""
        for local, slot in enumerate(self._slots):
            obj = slot.fn
            if hasattr(obj, "state_dict") and hasattr(obj, "load_state_dict"):
                yield local, obj

    def save_state_dict(self, save_dir):
        if self._grid.data_parallel_id != 0:
            return
        os.makedirs(save_dir, exist_ok=True)
        for local, obj in self._stateful():
            host = {k: v.detach().cpu().clone() if torch.is_tensor(v) else v for k, v in obj.state_dict().items()}
            torch.save(host, self.ckpt_layer_path(save_dir, local))

    def load_state_dir(self, load_dir, strict=True):
        for local, obj in self._stateful():
            path = self.ckpt_layer_path(load_dir, local)
            obj.load_state_dict(torch.load(path, map_location="cpu", weights_only=True), strict=strict)
            if self._grid.data_parallel_id == 0:
                logger.info(f"RANK={self.global_rank} Loaded layer={local + self._local_start} file={path}")
        self._synchronize_tied_weights()
