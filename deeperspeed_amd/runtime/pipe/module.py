"""PipelineModule: a model expressed as a sequence of layers partitioned over pipeline stages.

Reference parity: deepspeed/runtime/pipe/module.py:19-589 -- `LayerSpec` (lazy construction so
each stage only builds its own layers), `TiedLayerSpec` (weights shared across stages, e.g.
embedding / LM head, with gradient all-reduce and initial broadcast), partition methods
`uniform`, `parameters`, `type:<regex>`, per-stage activation checkpointing at
`activation_checkpoint_interval` layers (DeeperSpeed `checkpointable_layers`), per-layer
checkpoint files `layer_XX[-model_YY]-model_states.pt` written by data-parallel rank 0,
and `seed_layers` deterministic per-layer seeding.
"""

from __future__ import annotations

import os
import re
from functools import partial

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
    """Deferred construction of a layer: `LayerSpec(nn.Linear, 8, 4)` builds `nn.Linear(8, 4)`
    only on the stage that owns it."""

    def __init__(self, typename, *module_args, **module_kwargs):
        self.typename = typename
        self.module_args = module_args
        self.module_kwargs = module_kwargs
        if not issubclass(typename, nn.Module):
            raise RuntimeError("LayerSpec only supports torch.nn.Module types.")
        self.global_rank = dist.get_rank() if dist.is_initialized() else -1

    def __repr__(self):
        return ds_utils.call_to_str(self.typename.__name__, *self.module_args, **self.module_kwargs)

    def build(self, log=False):
        if log:
            logger.info(f"RANK={self.global_rank} building {repr(self)}")
        return self.typename(*self.module_args, **self.module_kwargs)


class TiedLayerSpec(LayerSpec):
    def __init__(self, key, typename, *module_args, forward_fn=None, tied_weight_attr="weight", **module_kwargs):
        super().__init__(typename, *module_args, **module_kwargs)
        self.key = key
        self.forward_fn = forward_fn
        self.tied_weight_attr = tied_weight_attr


class PipelineModule(nn.Module):
    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seed_layers=False, seed_fn=None,
                 base_seed=1234, partition_method="parameters", activation_checkpoint_interval=0,
                 activation_checkpoint_func=checkpointing.checkpoint, checkpointable_layers=None):
        super().__init__()
        if num_stages is None and topology is None:
            raise RuntimeError("must provide num_stages or topology")
        self.micro_offset = 0
        self.loss_fn = loss_fn
        self.seed_layers = seed_layers
        self.seed_fn = seed_fn
        self.base_seed = base_seed
        if not dist.is_initialized():
            from ...utils.distributed import init_distributed
            init_distributed()
        self.world_group = dist.new_group(ranks=range(dist.get_world_size()))
        self.global_rank = dist.get_rank(group=self.world_group)
        self.world_size = dist.get_world_size(group=self.world_group)
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if topology:
            self._topo = topology
            self.num_stages = self._topo.get_dim("pipe")
        else:
            self.num_stages = num_stages
            if self.world_size % self.num_stages != 0:
                raise RuntimeError(f"num_stages ({self.num_stages}) must divide distributed world size "
                                   f"({self.world_size})")
            self._topo = PipeDataParallelTopology(num_pp=num_stages, num_dp=self.world_size // num_stages)
        self._grid = PipelineParallelGrid(process_group=self.world_group, topology=self._topo)
        self.stage_id = self._topo.get_coord(self.global_rank).pipe
        self._layer_specs = list(layers)
        self._num_layers = len(self._layer_specs)
        self._local_start = 0
        self._local_stop = None
        self._partition_layers(method=partition_method)
        self.forward_funcs = []
        self.tied_modules = nn.ModuleDict()
        self.tied_weight_attrs = {}
        self._build()
        if torch.cuda.is_available():
            self.to(f"cuda:{self.local_rank % max(1, torch.cuda.device_count())}")
        self.tied_comms = self._index_tied_modules()
        self._synchronize_tied_weights()
        self.activation_checkpoint_interval = activation_checkpoint_interval
        self.activation_checkpoint_func = activation_checkpoint_func
        if checkpointable_layers is not None:
            assert isinstance(checkpointable_layers, list)
        self.checkpointable_layers = checkpointable_layers

    def _build(self):
        for local_idx, layer in enumerate(self._layer_specs[self._local_start:self._local_stop]):
            layer_idx = local_idx + self._local_start
            if self.seed_layers:
                (self.seed_fn or ds_utils.set_random_seed)(self.base_seed + layer_idx)
            if isinstance(layer, PipelineModule):
                raise NotImplementedError("RECURSIVE BUILD NOT YET IMPLEMENTED")
            elif isinstance(layer, nn.Module):
                self.forward_funcs.append(layer)
                self.add_module(str(layer_idx), layer)
            elif isinstance(layer, TiedLayerSpec):
                if layer.key not in self.tied_modules:
                    self.tied_modules[layer.key] = layer.build()
                    self.tied_weight_attrs[layer.key] = layer.tied_weight_attr
                mod = self.tied_modules[layer.key]
                self.forward_funcs.append(mod if layer.forward_fn is None else partial(layer.forward_fn, mod))
            elif isinstance(layer, LayerSpec):
                module = layer.build()
                self.forward_funcs.append(module)
                self.add_module(str(layer_idx), module)
            else:
                self.forward_funcs.append(layer)
        # pipeline params are distinct per stage: "model parallel" for the norm reductions
        for p in self.parameters():
            p.model_parallel = True

    def _count_layer_params(self):
        counts = [0] * len(self._layer_specs)
        for idx, layer in enumerate(self._layer_specs):
            if isinstance(layer, LayerSpec):
                mod = layer.build()
                counts[idx] = sum(p.numel() for p in mod.parameters() if p.requires_grad)
                del mod
            elif isinstance(layer, nn.Module):
                counts[idx] = sum(p.numel() for p in layer.parameters() if p.requires_grad)
        return counts

    def _find_layer_type(self, layername):
        rx = re.compile(layername, re.IGNORECASE)
        idxs = []
        for idx, layer in enumerate(self._layer_specs):
            if isinstance(layer, LayerSpec):
                name = layer.typename.__name__
            elif isinstance(layer, nn.Module):
                name = layer.__class__.__name__
            else:
                name = getattr(layer, "__name__", None)
                if name is None:
                    continue
            if rx.search(name):
                idxs.append(idx)
        if not idxs:
            raise RuntimeError(f"Partitioning '{layername}' found no valid layers to partition.")
        return idxs

    def forward(self, forward_input):
        self.micro_offset += 1

        def exec_range_func(start, end):
            local_micro_offset = self.micro_offset + 1

            def exec_func(*inputs):
                if len(inputs) == 1:
                    inputs = inputs[0]
                for idx, layer in enumerate(self.forward_funcs[start:end]):
                    self.curr_layer = idx + self._local_start
                    if self.seed_layers:
                        (self.seed_fn or ds_utils.set_random_seed)(self.base_seed * local_micro_offset +
                                                                    self.curr_layer)
                    inputs = layer(inputs)
                return inputs

            return exec_func

        if self.activation_checkpoint_interval == 0:
            return exec_range_func(0, len(self.forward_funcs))(forward_input)
        x = forward_input
        n = len(self.forward_funcs)
        for s in range(0, n, self.activation_checkpoint_interval):
            e = min(s + self.activation_checkpoint_interval, n)
            if not isinstance(x, tuple):
                x = (x,)
            if self._is_checkpointable(self.forward_funcs[s:e]):
                x = self.activation_checkpoint_func(exec_range_func(s, e), *x)
            else:
                x = exec_range_func(s, e)(*x)
        return x

    def _partition_layers(self, method="uniform"):
        num_stages = self._topo.get_dim("pipe")
        stage_id = self._topo.get_coord(self.global_rank).pipe
        method = method.lower()
        if method == "uniform":
            self.parts = ds_utils.partition_uniform(num_items=len(self._layer_specs), num_parts=num_stages)
        elif method == "parameters":
            self.parts = ds_utils.partition_balanced(weights=self._count_layer_params(), num_parts=num_stages)
        elif method.startswith("type:"):
            weights = [0] * len(self._layer_specs)
            for idx in self._find_layer_type(method.split(":", 1)[1]):
                weights[idx] = 1
            self.parts = ds_utils.partition_balanced(weights=weights, num_parts=num_stages)
        else:
            raise NotImplementedError(f"Partitioning method {method} not implemented.")
        if self.global_rank == 0:
            for stage in range(num_stages):
                start, stop = self.parts[stage], self.parts[stage + 1]
                logger.info(f"stage={stage} layers={stop - start}")
        self._set_bounds(start=self.parts[stage_id], stop=self.parts[stage_id + 1])

    def allreduce_tied_weight_gradients(self):
        for key, comm in self.tied_comms.items():
            weight = getattr(self.tied_modules[key], comm["weight_attr"])
            if weight.grad is not None:
                dist.all_reduce(weight.grad, group=comm["group"])

    def _synchronize_tied_weights(self):
        for key, comm in self.tied_comms.items():
            dist.broadcast(getattr(comm["module"], comm["weight_attr"]).data, src=min(comm["ranks"]),
                           group=comm["group"])

    def _index_tied_modules(self):
        tied_comms = {}
        if self._topo.get_dim("pipe") == 1:
            return tied_comms
        specs = self._layer_specs
        for key in sorted(set(s.key for s in specs if isinstance(s, TiedLayerSpec))):
            tied_layers = [i for i, s in enumerate(specs) if isinstance(s, TiedLayerSpec) and s.key == key]
            tied_stages = sorted(set(self.stage_owner(i) for i in tied_layers))
            for dp in range(self._grid.data_parallel_size):
                for mp in range(self._grid.model_parallel_size):
                    kw = dict(data=dp, model=mp) if self._grid.model_parallel_size > 1 else dict(data=dp)
                    ranks = [self._grid.stage_to_global(stage_id=s, **kw) for s in tied_stages]
                    group = dist.new_group(ranks=ranks)
                    if self.global_rank in ranks:
                        assert key in self.tied_modules
                        tied_comms[key] = {"ranks": ranks, "group": group,
                                           "weight_attr": self.tied_weight_attrs[key],
                                           "module": self.tied_modules[key]}
                        if self.global_rank != ranks[0]:
                            for p in self.tied_modules[key].parameters():
                                p.model_parallel = False
        return tied_comms

    def partitions(self):
        return self.parts

    def stage_owner(self, layer_idx):
        assert 0 <= layer_idx < self._num_layers
        for stage in range(self._topo.get_dim("pipe")):
            if self.parts[stage] <= layer_idx < self.parts[stage + 1]:
                return stage
        raise RuntimeError(f"Layer {layer_idx} not owned? parts={self.parts}")

    def _set_bounds(self, start=None, stop=None):
        self._local_start = start
        self._local_stop = stop

    def set_checkpoint_interval(self, interval):
        assert interval >= 0
        self.checkpoint_interval = interval
        self.activation_checkpoint_interval = interval

    def topology(self):
        return self._topo

    def mpu(self):
        return self._grid

    def num_pipeline_stages(self):
        return self._topo.get_dim("pipe")

    def ckpt_prefix(self, checkpoints_path, tag):
        rank_name = "module"
        coord = self._grid._topo.get_coord(rank=self.global_rank)
        for dim in [a for a in self._grid._topo.get_axis_names() if a != "data"]:
            rank_name += f"-{dim}_{getattr(coord, dim):02d}"
        return os.path.join(checkpoints_path, str(tag), rank_name)

    def ckpt_layer_path(self, ckpt_dir, local_layer_idx):
        idx = local_layer_idx + self._local_start
        path = os.path.join(ckpt_dir, f"layer_{idx:02d}")
        rank_repr = self._grid._topo.get_rank_repr(rank=self.global_rank)
        if rank_repr != "":
            path += f"-{rank_repr}"
        return path + "-model_states.pt"

    def save_state_dict(self, save_dir):
        if self._grid.data_parallel_id != 0:
            return
        os.makedirs(save_dir, exist_ok=True)
        for idx, layer in enumerate(self.forward_funcs):
            if not hasattr(layer, "state_dict"):
                continue
            torch.save({k: (v.detach().cpu().clone() if torch.is_tensor(v) else v)
                        for k, v in layer.state_dict().items()}, self.ckpt_layer_path(save_dir, idx))

    def load_state_dir(self, load_dir, strict=True):
        for idx, layer in enumerate(self.forward_funcs):
            if not hasattr(layer, "load_state_dict"):
                continue
            path = self.ckpt_layer_path(load_dir, idx)
            layer.load_state_dict(torch.load(path, map_location="cpu", weights_only=True), strict=strict)
            if self._grid.data_parallel_id == 0:
                logger.info(f"RANK={self.global_rank} Loaded layer={idx + self._local_start} file={path}")
        self._synchronize_tied_weights()

    def _is_checkpointable(self, funcs):
        if self.checkpointable_layers is not None:
            return all(f.__class__.__name__ in self.checkpointable_layers for f in funcs)
        if self.__class__.__name__ == "GPT2ModelPipe":
            return all("ParallelTransformerLayerPipe" in f.__class__.__name__ for f in funcs)
        return any(len(list(f.parameters())) > 0 for f in funcs if isinstance(f, nn.Module))
