"""PipelineEngine: executes Train/Inference schedules for a PipelineModule.

Reference parity: deepspeed/runtime/pipe/engine.py:52-1316 -- `train_batch(data_iter,
layers_to_hook)`, `eval_batch(data_iter, return_logits, layers_to_hook)` and DeeperSpeed's
`inference_batch` returning (logits, presents) broadcast over the pipe group, loss
aggregation over the data-parallel group + broadcast along the pipe, tied-weight gradient
reduction, first-send tensor metadata handshake, fp32 activation/gradient transfer for bf16
(`fp32_allreduce`), the GPT-NeoX bool attention-mask transport hack, timer-value return,
per-layer checkpoint files.  ZeRO stages >= 2 are rejected like the reference.

MI355X design: stage transfers are RCCL send/recv pairs (`batch_isend_irecv`) over the
direct xGMI link between the two stage GPUs; data-parallel gradient reduction is done by
the flat-arena optimizer with reductions launched during the *last* micro-batch's
backward (overlapped), not by a separate pass after the schedule.
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ...ops import linear as _linear_ops
from ...utils.logging import logger, log_dist
from ...utils.timer import ThroughputTimer
from ..engine import DeepSpeedEngine
from ..utils import PartitionedTensor
from . import p2p, schedule
from .module import PipelineModule

_DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32, torch.bool,
           torch.uint8, torch.int16, torch.int8]
_META_SLOTS = 16
_META_DIMS = 8


def is_even(number):
    return number % 2 == 0


class PipelineEngine(DeepSpeedEngine):
    def __init__(self, *super_args, **super_kwargs):
        super().__init__(*super_args, **super_kwargs)
        assert isinstance(self.module, PipelineModule), "model must base PipelineModule"
        assert self.zero_optimization_stage() < 2, "ZeRO-2 and ZeRO-3 are incompatible with pipeline parallelism"
        self.enable_backward_allreduce = False
        self.eval_return_logits = False
        self.outputs = None
        assert not self.elasticity_enabled(), "Elasticity is not currently supported with pipeline parallelism."
        self.micro_batch_size = self.train_micro_batch_size_per_gpu()
        self.micro_batches = self.gradient_accumulation_steps()
        self.grid = self.module._grid
        self.global_rank = self.grid.get_global_rank()
        assert self.dp_world_size == self.grid.data_parallel_size
        assert self.train_batch_size() == self.micro_batch_size * self.micro_batches * self.grid.data_parallel_size
        self.num_stages = self.grid.pipe_parallel_size
        self.stage_id = self.grid.get_stage_id()
        self.prev_stage = self.stage_id - 1
        self.next_stage = self.stage_id + 1
        self.data_iterator = None
        self.batch_fn = None
        self._force_grad_boundary = False
        self.batch_timer = ThroughputTimer(batch_size=self.micro_batch_size * self.micro_batches,
                                           num_workers=self.dp_world_size, logging_fn=self.tput_log,
                                           monitor_memory=False, steps_per_output=self.steps_per_print())
        if self.training_data:
            self._build_data_iter(self.training_data)
        self.is_pipe_parallel = self.grid.pipe_parallel_size > 1
        self.is_data_parallel = self.grid.data_parallel_size > 1
        self.is_model_parallel = self.grid.model_parallel_size > 1
        self.is_pipe_partitioned = self.is_model_parallel
        self.is_grad_partitioned = False

        num_params = sum(p.numel() for p in self.module.parameters() if p.requires_grad)
        unique = num_params
        for tie in self.module.tied_comms.values():
            if self.global_rank != min(tie.ranks):
                unique -= sum(p.numel() for p in tie.module.parameters())
        t = torch.LongTensor([num_params, unique]).to(self.device)
        dist.all_reduce(t, group=self.grid.get_model_parallel_group())
        total, uniq = t.tolist()
        if self.grid.data_parallel_id == 0:
            logger.info(f"RANK={self.global_rank} STAGE={self.stage_id} "
                        f"LAYERS={self.module._local_stop - self.module._local_start} "
                        f"[{self.module._local_start}, {self.module._local_stop}) STAGE_PARAMS={num_params} "
                        f"({num_params / 1e6:0.3f}M) TOTAL_PARAMS={total} ({total / 1e6:0.3f}M) "
                        f"UNIQUE_PARAMS={uniq} ({uniq / 1e6:0.3f}M)")
        if self.is_pipe_parallel:
            p2p.init_process_groups(self.grid)
        self.num_pipe_buffers = 0
        self.pipe_buffers = {"inputs": [], "labels": [], "outputs": [], "output_tensors": []}
        self.pipe_recv_buf = None
        self.grad_layer = None
        self.meta_buffer = None
        self.first_output_send = True
        self.first_gradient_send = True
        self.timer_values = None
        self.loss = torch.tensor(0.0).to(self.device)
        self.total_loss = None
        self.agg_loss = torch.tensor(0.0, requires_grad=False).to(self.device)
        self.dp_group_loss = torch.tensor(0.0, requires_grad=False).to(self.device)
        if self._config.pipeline["activation_checkpoint_interval"] > 0:
            self.module.activation_checkpoint_interval = self._config.pipeline["activation_checkpoint_interval"]
        if self.is_last_stage():
            self.loss_model = self.module.loss_fn
        self.has_attention_mask = self.module.__class__.__name__ == "GPT2ModelPipe"
        self._recv_meta = None
        self._bw_count = 0
        # asynchronous p2p (DSA_PIPE_ASYNC_P2P=0 restores blocking transfers): sends are left in
        # flight across the following compute, receives are waited by their consumer, and a
        # receive is posted ahead of the compute instruction before it when no other p2p op
        # lies in between (the per-pair order both ranks issue stays identical: no deadlock)
        self._async_p2p = os.environ.get("DSA_PIPE_ASYNC_P2P", "1") != "0"
        self._pending_sends = []
        self._recv_handles = {}
        self._prefetched = {}
        self.p2p_trace = None  # set to a list to record (instruction, sends in flight, receives in flight)
        # warm-up handshake between neighbours (establishes the RCCL p2p channels)
        if self.is_pipe_parallel:
            if is_even(self.stage_id):
                if not self.is_last_stage():
                    p2p.send(self.loss, self.next_stage)
                if not self.is_first_stage():
                    p2p.recv(self.loss, self.prev_stage)
            else:
                if not self.is_first_stage():
                    p2p.recv(self.loss, self.prev_stage)
                if not self.is_last_stage():
                    p2p.send(self.loss, self.next_stage)

    # ------------------------------------------------------------------ config helpers
    def _fp32_comm(self):
        return self.precision() == torch.bfloat16 and self.allreduce_always_fp32()

    def set_has_attention_mask(self, value):
        assert isinstance(value, bool)
        self.has_attention_mask = value

    def _build_data_iter(self, dataset):
        sampler = torch.utils.data.distributed.DistributedSampler(dataset, num_replicas=self.dp_world_size,
                                                                  rank=self.mpu.get_data_parallel_rank(),
                                                                  shuffle=False)
        loader = self.deepspeed_io(dataset, data_sampler=sampler)
        from ..dataloader import RepeatingLoader
        self.set_dataloader(RepeatingLoader(loader))

    # ------------------------------------------------------------------ reductions
    def _exec_reduce_tied_grads(self):
        self.module.allreduce_tied_weight_gradients()

    def _exec_reduce_grads(self):
        self._force_grad_boundary = True
        if hasattr(self.optimizer, "reduce_epilogue"):
            self.optimizer.reduce_epilogue()
        elif self.is_data_parallel:
            self.buffered_allreduce_fallback(elements_per_buffer=500000000)
        self._force_grad_boundary = False

    def _reserve_pipe_buffers(self, num_buffers):
        if self.num_pipe_buffers >= num_buffers:
            return
        for key in self.pipe_buffers:
            self.pipe_buffers[key].extend([None] * (num_buffers - self.num_pipe_buffers))
        self.num_pipe_buffers = num_buffers

    # ------------------------------------------------------------------ batch APIs
    def train_batch(self, data_iter=None, layers_to_hook=None):
        if not torch._C.is_grad_enabled():
            raise RuntimeError("train_batch() requires gradients enabled. Use eval_batch() instead.")
        if layers_to_hook is not None:
            self.register_forward_hook(layers_to_hook)
        if data_iter:
            self.set_dataiterator(data_iter)
        self.module.train()
        self.total_loss = None
        self._bw_count = 0
        self.timers("train_batch").start()
        sched = schedule.TrainSchedule(micro_batches=self.micro_batches, stages=self.num_stages,
                                       stage_id=self.stage_id)
        self._exec_schedule(sched)
        self.agg_train_loss = self._aggregate_total_loss()
        self.timers("train_batch").stop()
        if self.global_steps % self.steps_per_print() == 0:
            elapsed = self.timers("train_batch").elapsed(reset=True)
            if self.global_rank == 0:
                iter_time = elapsed / self.steps_per_print()
                tput = self.train_batch_size() / iter_time
                print(f"steps: {self.global_steps} loss: {self.agg_train_loss:0.4f} iter time (s): {iter_time:0.3f} "
                      f"samples/sec: {tput:0.3f}")
            if self.wall_clock_breakdown():
                vals = {}
                for k in ("comms", "step", "forward", "backward"):
                    if k in self.timers.timers:
                        vals["pct_" + {"step": "optimizer_step", "forward": "fwd"}.get(k, k)] = \
                            self.timers(k).elapsed(reset=False) / max(elapsed, 1e-9) * 100
                vals.update(self.timers.get_timers_value(list(self.timers.timers.keys())))
                self.timer_values = vals
        if self.tensorboard_enabled() and self.global_rank == 0:
            self.summary_writer.add_scalar("Train/Samples/train_loss", self.agg_train_loss.mean().item(),
                                           self.global_samples)
            if self.global_steps % self.steps_per_print() == 0:
                self.summary_writer.flush()
        if layers_to_hook is not None:
            self.register_forward_hook([])
        return self.agg_train_loss

    def eval_batch(self, data_iter, return_logits=False, layers_to_hook=None):
        self.eval_return_logits = return_logits
        self.module.eval()
        self.total_loss = None
        if layers_to_hook is not None:
            self.register_forward_hook(layers_to_hook)
        train_iterator = self.data_iterator
        self.set_dataiterator(data_iter)
        sched = schedule.InferenceSchedule(micro_batches=self.micro_batches, stages=self.num_stages,
                                           stage_id=self.stage_id)
        with torch.no_grad():
            self._exec_schedule(sched)
        self.agg_eval_loss = self._aggregate_total_loss()
        if self.tensorboard_enabled() and self.global_rank == 0:
            self.summary_writer.add_scalar("Train/Samples/eval_loss", self.agg_eval_loss.mean().item(),
                                           self.global_samples)
            self.summary_writer.flush()
        self.set_dataiterator(train_iterator)
        if layers_to_hook is not None:
            self.register_forward_hook([])
        self.eval_return_logits = False
        if return_logits:
            outputs, self.outputs = self.outputs, None
            return self.agg_eval_loss, outputs
        return self.agg_eval_loss

    def inference_batch(self, data_iter, layers_to_hook=None):
        """GPT-NeoX inference: returns (logits, presents) on every stage of the pipe group."""
        self.module.eval()
        self.total_loss = None
        if self.micro_batches > 1:
            log_dist("WARNING: setting g.a.s to 1 in inference", ranks=[0])
            self.micro_batches = 1
        train_batch_fn = self.batch_fn
        self.set_batch_fn(lambda x: x)
        self.first_output_send = True
        self.pipe_recv_buf = None
        self._recv_meta = None
        if self.is_data_parallel:
            raise NotImplementedError("Inference not yet implemented for pipeline + data parallel")
        train_iterator = self.data_iterator
        self.set_dataiterator(data_iter)
        if layers_to_hook is not None:
            self.register_forward_hook(layers_to_hook)
        sched = schedule.InferenceSchedule(micro_batches=self.micro_batches, stages=self.num_stages,
                                           stage_id=self.stage_id)
        with torch.no_grad():
            self._exec_schedule(sched)
        comm_dtype = torch.float32 if self.precision() == torch.bfloat16 else self.precision()
        src_rank = self.grid.stage_to_global(self.num_stages - 1)
        if self.is_last_stage():
            logits, presents = self.total_loss
            shapes = torch.LongTensor([logits.dim()] + list(logits.shape) + [0] * (8 - logits.dim()) +
                                      [presents.dim()] + list(presents.shape) + [0] * (8 - presents.dim()))
            shapes = shapes.to(self.device)
        else:
            shapes = torch.zeros(18, dtype=torch.long, device=self.device)
        dist.broadcast(shapes, src=src_rank)
        s = shapes.tolist()
        lshape, pshape = s[1:1 + s[0]], s[10:10 + s[9]]
        if self.is_last_stage():
            logits = logits.detach().to(comm_dtype).contiguous()
            presents = presents.detach().to(comm_dtype).contiguous()
        else:
            logits = torch.zeros(lshape, dtype=comm_dtype, device=self.device)
            presents = torch.zeros(pshape, dtype=comm_dtype, device=self.device)
        if self.is_pipe_parallel:
            dist.broadcast(logits, src=src_rank, group=self.grid.get_pipe_parallel_group())
            dist.broadcast(presents, src=src_rank, group=self.grid.get_pipe_parallel_group())
        logits, presents = logits.to(self.precision()), presents.to(self.precision())
        self.set_dataiterator(train_iterator)
        self.set_batch_fn(train_batch_fn)
        if layers_to_hook is not None:
            self.register_forward_hook([])
        return logits, presents

    def is_first_stage(self):
        return self.stage_id == 0

    def is_last_stage(self):
        return self.stage_id == self.num_stages - 1

    def _aggregate_total_loss(self):
        if self.is_last_stage():
            loss = self._scale_loss_by_gas(self.total_loss)
            self.dp_group_loss = loss.clone().detach()
            agg = self.dp_group_loss.clone().detach()
            if self.is_data_parallel:
                dist.all_reduce(agg, group=self.mpu.get_data_parallel_group())
                agg /= self.dp_world_size
            assert self.global_rank in self.grid.pp_group
            losses = torch.stack([self.dp_group_loss, agg]).float()
            if self.is_pipe_parallel:
                dist.broadcast(losses, src=self.global_rank, group=self.mpu.get_pipe_parallel_group())
        else:
            src_rank = self.grid.stage_to_global(self.num_stages - 1)
            assert src_rank in self.grid.pp_group
            losses = torch.empty(2, dtype=torch.float32, device=self.device)
            dist.broadcast(losses, src=src_rank, group=self.grid.get_pipe_parallel_group())
            self.dp_group_loss = losses[0].clone().detach()
            agg = losses[1].clone().detach()
        return agg

    def _scale_loss_by_gas(self, prescaled_loss):
        if isinstance(prescaled_loss, torch.Tensor):
            return prescaled_loss / self.gradient_accumulation_steps()
        if isinstance(prescaled_loss, (tuple, list)):
            return type(prescaled_loss)(l / self.gradient_accumulation_steps() for l in prescaled_loss)
        return prescaled_loss

    def set_dataloader(self, loader):
        if self.is_first_stage() or self.is_last_stage():
            self.training_dataloader = loader
            self.data_iterator = iter(self.training_dataloader)

    def set_dataiterator(self, iterator):
        if self.is_first_stage() or self.is_last_stage():
            self.training_dataloader = None
            self.data_iterator = iterator

    def set_batch_fn(self, fn):
        self.batch_fn = fn

    def is_gradient_accumulation_boundary(self):
        return self._force_grad_boundary

    def log_for_device(self, *msg):
        logger.info(f"RANK={dist.get_rank()} STAGE={self.stage_id} DATA={self.grid.data_parallel_id} " +
                    " ".join(str(m) for m in msg))

    def tput_log(self, *msg):
        if self.global_rank == 0 and self.global_steps % self.steps_per_print() == 0:
            print(*msg)

    def _next_batch(self):
        batch = next(self.data_iterator) if self.data_iterator is not None else None
        if self.batch_fn:
            batch = self.batch_fn(batch)
        return batch

    # ------------------------------------------------------------------ instructions
    def _exec_forward_pass(self, buffer_id):
        self.tput_timer.start()
        self.mem_status("BEFORE FWD", reset_max=True)
        self._wait_recv(("act", buffer_id))
        inputs = self.pipe_buffers["inputs"][buffer_id]
        if isinstance(inputs, tuple):
            inputs = tuple(t.clone() if torch.is_tensor(t) else t for t in inputs)
        elif torch.is_tensor(inputs):
            inputs = inputs.clone()
        if self.is_pipe_partitioned and not self.is_first_stage() and isinstance(inputs, tuple) and \
                len(inputs) >= 2 and torch.is_tensor(inputs[0]) and inputs[0].dtype == torch.long:
            part = PartitionedTensor.from_meta(meta=inputs[0], local_part=inputs[1],
                                               group=self.grid.get_slice_parallel_group())
            inputs = (part.full(),) + tuple(inputs[2:])
            inputs[0].requires_grad = True
            self.pipe_buffers["inputs"][buffer_id] = inputs
        self._zero_grads(inputs)
        if self.wall_clock_breakdown():
            self.timers("forward").start()
        outputs = super().forward(inputs)
        if self.wall_clock_breakdown():
            self.timers("forward").stop()
        if self.is_pipe_partitioned and not self.is_last_stage():
            if isinstance(outputs, tuple):
                first = outputs[0]
            else:
                first = outputs
            part = PartitionedTensor(tensor=first, group=self.grid.get_slice_parallel_group())
            first.data = torch.zeros(1, device=first.device)
            self.pipe_buffers["output_tensors"][buffer_id] = first
            rest = outputs[1:] if isinstance(outputs, tuple) else ()
            outputs = (part.to_meta(), part.data(), *rest)
        self.pipe_buffers["outputs"][buffer_id] = outputs
        if self.is_last_stage():
            if self._compute_loss and self.loss_model is not None:
                labels = self.pipe_buffers["labels"][buffer_id]
                self.loss = self.loss_model(outputs, labels)
            else:
                self.loss = outputs
            if self.eval_return_logits:
                self.outputs = outputs
            if isinstance(self.loss, torch.Tensor):
                if self.total_loss is None:
                    self.total_loss = torch.zeros_like(self.loss)
                self.total_loss += self.loss.detach()
            else:
                if self.total_loss is None:
                    self.total_loss = [torch.zeros_like(l) for l in self.loss]
                for i, l in enumerate(self.loss):
                    self.total_loss[i] += l.detach()

    def _exec_backward_pass(self, buffer_id):
        assert self.optimizer is not None, "must provide optimizer during init in order to use backward"
        self._bw_count += 1
        boundary = self._bw_count == self.micro_batches
        if hasattr(self.optimizer, "is_gradient_accumulation_boundary"):
            self.optimizer.is_gradient_accumulation_boundary = boundary
        if self.wall_clock_breakdown():
            self.timers("backward_microstep").start()
            self.timers("backward").start()
        if self.is_last_stage():
            loss = self.loss / self.gradient_accumulation_steps()
            if hasattr(self.optimizer, "backward") and (self.zero_optimization() or self.fp16_enabled()):
                self.optimizer.backward(loss)
            else:
                loss.backward()
        else:
            outputs = self.pipe_buffers["outputs"][buffer_id]
            if self.is_pipe_partitioned:
                outputs = (self.pipe_buffers["output_tensors"][buffer_id],) + tuple(
                    outputs[2:] if isinstance(outputs, tuple) else ())
            self._wait_recv(("grad", buffer_id))
            grads = self.grad_layer
            if isinstance(outputs, tuple):
                out_t = [t for t in outputs if torch.is_tensor(t) and t.is_floating_point() and t.requires_grad]
                assert len(out_t) == len(grads)
                torch.autograd.backward(tensors=out_t, grad_tensors=grads)
            else:
                torch.autograd.backward(tensors=(outputs,), grad_tensors=(grads[0],))
            if hasattr(self.optimizer, "mark_new_gradients"):
                self.optimizer.mark_new_gradients()  # persistent buffers hold fresh gradients again
        _linear_ops.end_backward_pass()  # pre-transposed operands never outlive their backward
        self.pipe_buffers["output_tensors"][buffer_id] = None
        self.pipe_buffers["outputs"][buffer_id] = None
        if self.wall_clock_breakdown():
            self.timers("backward").stop()
            self.timers("backward_microstep").stop()

    def _exec_load_micro_batch(self, buffer_id):
        if self.wall_clock_breakdown():
            self.timers("batch_input").start()
        batch = self._next_batch()
        if self.is_first_stage():
            data = batch[0]
            if torch.is_tensor(data):
                loaded = data.clone().detach().to(self.device)
                loaded.requires_grad = loaded.is_floating_point()
            else:
                loaded = []
                for x in data:
                    if torch.is_tensor(x):
                        x = x.clone().detach().to(self.device)
                        x.requires_grad = x.is_floating_point()
                    loaded.append(x)
                loaded = tuple(loaded)
                if self.has_attention_mask:
                    loaded = loaded[:-1] + (loaded[-1].bool(),)
            self.pipe_buffers["inputs"][buffer_id] = loaded
        if self.is_last_stage():
            lab = batch[1]
            if torch.is_tensor(lab):
                lab = lab.to(self.device)
            elif isinstance(lab, (list, tuple)):
                lab = tuple(x.to(self.device) if torch.is_tensor(x) else x for x in lab)
            self.pipe_buffers["labels"][buffer_id] = lab
        if self.wall_clock_breakdown():
            self.timers("batch_input").stop()

    # ------------------------------------------------------------------ p2p with metadata
    def _as_list(self, x):
        return list(x) if isinstance(x, tuple) else [x]

    def _send_tensor_meta(self, buffer, recv_stage):
        items = self._as_list(buffer)
        assert len(items) <= _META_SLOTS
        meta = torch.zeros(2 + _META_SLOTS * (2 + _META_DIMS), dtype=torch.long)
        meta[0] = 1 if isinstance(buffer, tuple) else 0
        meta[1] = len(items)
        for i, t in enumerate(items):
            base = 2 + i * (2 + _META_DIMS)
            dt = t.dtype
            if self._fp32_comm() and dt == torch.bfloat16:
                dt = torch.float32
            meta[base] = _DTYPES.index(dt)
            meta[base + 1] = t.dim()
            meta[base + 2: base + 2 + t.dim()] = torch.tensor(list(t.shape), dtype=torch.long)
        p2p.send(meta.to(self.device), recv_stage)

    def _recv_tensor_meta(self, send_stage):
        meta = torch.zeros(2 + _META_SLOTS * (2 + _META_DIMS), dtype=torch.long, device=self.device)
        p2p.recv(meta, send_stage)
        m = meta.tolist()
        is_tuple, n = m[0], m[1]
        specs = []
        for i in range(n):
            base = 2 + i * (2 + _META_DIMS)
            dt = _DTYPES[m[base]]
            nd = m[base + 1]
            specs.append((dt, tuple(m[base + 2: base + 2 + nd])))
        return bool(is_tuple), specs

    def _exec_send_activations(self, buffer_id):
        if self.wall_clock_breakdown():
            self.timers("pipe_send_output").start()
        outputs = self.pipe_buffers["outputs"][buffer_id]
        if self.has_attention_mask and isinstance(outputs, tuple):
            outputs = outputs[:-1] + (outputs[-1].half() if outputs[-1].dtype == torch.bool else outputs[-1],)
        if self.first_output_send:
            self.first_output_send = False
            self._send_tensor_meta(outputs, self.next_stage)
        items = [t.detach() for t in self._as_list(outputs)]
        self._track_send(p2p.send_many(items, self.next_stage, fp32_comm=self._fp32_comm(),
                                       async_op=self._async_p2p))
        if self.wall_clock_breakdown():
            self.timers("pipe_send_output").stop()

    def _exec_send_grads(self, buffer_id):
        if self.wall_clock_breakdown():
            self.timers("pipe_send_grad").start()
        inputs = self.pipe_buffers["inputs"][buffer_id]
        if self.is_grad_partitioned:
            raise NotImplementedError
        grads = []
        for t in self._as_list(inputs):
            if torch.is_tensor(t) and t.is_floating_point() and t.requires_grad:
                grads.append(t.grad if t.grad is not None else torch.zeros_like(t))
        self._track_send(p2p.send_many(grads, self.prev_stage, fp32_comm=self._fp32_comm(),
                                       async_op=self._async_p2p))
        self.pipe_buffers["inputs"][buffer_id] = None
        if self.wall_clock_breakdown():
            self.timers("pipe_send_grad").stop()

    def _exec_recv_activations(self, buffer_id):
        if self.wall_clock_breakdown():
            self.timers("pipe_recv_input").start()
        if self._recv_meta is None:
            self._recv_meta = self._recv_tensor_meta(self.prev_stage)
        is_tuple, _ = self._recv_meta
        pre = self._prefetched.pop(("act", buffer_id), None)
        handle, bufs = pre if pre is not None else self._post_recv_activations()
        if handle is not None:
            self._recv_handles[("act", buffer_id)] = handle
        for b in bufs:
            if b.is_floating_point():
                b.requires_grad_(True)
        if self.has_attention_mask and is_tuple:
            # the bool mask travels as a half tensor: converted once it has arrived
            self._wait_recv(("act", buffer_id))
            bufs[-1] = bufs[-1].detach().bool()
        self.pipe_buffers["inputs"][buffer_id] = tuple(bufs) if is_tuple else bufs[0]
        if self.wall_clock_breakdown():
            self.timers("pipe_recv_input").stop()

    def _exec_recv_grads(self, buffer_id):
        if self.wall_clock_breakdown():
            self.timers("pipe_recv_grad").start()
        outputs = self.pipe_buffers["outputs"][buffer_id]
        if self.is_pipe_partitioned:
            outputs = (self.pipe_buffers["output_tensors"][buffer_id],) + tuple(
                outputs[2:] if isinstance(outputs, tuple) else ())
        targets = [t for t in self._as_list(outputs) if torch.is_tensor(t) and t.is_floating_point() and
                   t.requires_grad]
        pre = self._prefetched.pop(("grad", buffer_id), None)
        if pre is not None:
            handle, self.grad_layer = pre
        else:
            self.grad_layer = [torch.empty_like(t) for t in targets]
            handle = p2p.recv_many(self.grad_layer, self.next_stage, fp32_comm=self._fp32_comm(),
                                   async_op=self._async_p2p)
        if handle is not None:
            self._recv_handles[("grad", buffer_id)] = handle
        if self.wall_clock_breakdown():
            self.timers("pipe_recv_grad").stop()

    # ------------------------------------------------------------------ asynchronous p2p
    def _post_recv_activations(self):
        _, specs = self._recv_meta
        bufs = []
        for dt, shape in specs:
            tgt = self.precision() if (dt == torch.float32 and self._fp32_comm()) else dt
            bufs.append(torch.empty(shape, dtype=tgt, device=self.device))
        handle = p2p.recv_many(bufs, self.prev_stage, fp32_comm=self._fp32_comm(), async_op=self._async_p2p)
        return handle, bufs

    def _post_recv_grads(self, buffer_id):
        outputs = self.pipe_buffers["outputs"][buffer_id]
        if outputs is None:
            return None
        if self.is_pipe_partitioned:
            outputs = (self.pipe_buffers["output_tensors"][buffer_id],) + tuple(
                outputs[2:] if isinstance(outputs, tuple) else ())
        targets = [t for t in self._as_list(outputs) if torch.is_tensor(t) and t.is_floating_point() and
                   t.requires_grad]
        bufs = [torch.empty_like(t) for t in targets]
        return p2p.recv_many(bufs, self.next_stage, fp32_comm=self._fp32_comm(), async_op=True), bufs

    def _prefetch(self, cmd):
        """Post a later receive now (its buffers are installed by the instruction itself)."""
        bid = cmd.kwargs["buffer_id"]
        if isinstance(cmd, schedule.RecvActivation):
            if self._recv_meta is not None and ("act", bid) not in self._prefetched:
                self._prefetched[("act", bid)] = self._post_recv_activations()
        elif isinstance(cmd, schedule.RecvGrad) and ("grad", bid) not in self._prefetched:
            pre = self._post_recv_grads(bid)
            if pre is not None:
                self._prefetched[("grad", bid)] = pre

    def _wait_recv(self, key):
        h = self._recv_handles.pop(key, None)
        if h is not None:
            h.wait()

    def _track_send(self, handle):
        if handle is None or handle.done:
            return
        self._pending_sends.append(handle)
        while len(self._pending_sends) > 4:  # bound the activations kept alive by transfers
            self._pending_sends.pop(0).wait()

    def _drain_p2p(self):
        for h in self._pending_sends:
            h.wait()
        self._pending_sends = []
        for h in self._recv_handles.values():
            h.wait()
        self._recv_handles = {}

    @staticmethod
    def _plan_prefetch(flat):
        """{i: [j, ...]}: receive instruction j is posted just before compute instruction i.
        A receive moves up over compute / data-loading instructions only, never over another
        p2p op or a collective, so both ranks of every pair keep issuing their transfers in the
        schedule's order."""
        compute = (schedule.ForwardPass, schedule.BackwardPass)
        movable = compute + (schedule.LoadMicroBatch,)
        plan = {}
        for j, cmd in enumerate(flat):
            if not isinstance(cmd, (schedule.RecvActivation, schedule.RecvGrad)):
                continue
            k, target = j - 1, None
            while k >= 0 and isinstance(flat[k], movable):
                if isinstance(flat[k], compute):
                    target = k
                    break
                k -= 1
            if target is not None:
                # a gradient receive needs its forward's outputs: never above that forward
                if isinstance(cmd, schedule.RecvGrad) and isinstance(flat[target], schedule.ForwardPass) and \
                        flat[target].kwargs["buffer_id"] == cmd.kwargs["buffer_id"]:
                    continue
                plan.setdefault(target, []).append(j)
        return plan

    def _exec_optimizer_step(self, lr_kwargs=None):
        if self.wall_clock_breakdown():
            self.timers("step_microstep").start()
            self.timers("step").start()
        self._force_grad_boundary = True
        self._take_model_step(lr_kwargs)
        self._force_grad_boundary = False
        if self.wall_clock_breakdown():
            self.timers("step").stop()
            self.timers("step_microstep").stop()

    def _zero_grads(self, inputs):
        for t in self._as_list(inputs):
            if torch.is_tensor(t) and t.is_leaf and t.grad is not None:
                t.grad.data.zero_()

    # ------------------------------------------------------------------ disabled DeepSpeedEngine APIs
    _curr_ckpt_path = None
    _loads_module_from_dir = True

    def forward(self, *args, **kwargs):
        raise PipelineError("Only train_batch() is accessible in pipeline mode.")

    def backward(self, *args, **kwargs):
        raise PipelineError("Only train_batch() is accessible in pipeline mode.")

    def step(self, *args, **kwargs):
        raise PipelineError("Only train_batch() is accessible in pipeline mode.")

    def mem_status(self, msg, print_rank=-1, reset_max=False):
        return

    # ------------------------------------------------------------------ checkpoints (per-layer files)
    def module_state_dict(self):
        assert isinstance(self.module, PipelineModule)
        assert self._curr_ckpt_path is not None, "PipelineEngine expects module_state_dict() to be called from " \
                                                 "save_checkpoint()"
        self.module.save_state_dict(self._curr_ckpt_path)
        return None

    def load_module_state_dict(self, state_dict, strict=True):
        if state_dict is not None and not isinstance(state_dict, str):
            super().load_module_state_dict(state_dict, strict)
            return
        self.module.load_state_dir(load_dir=self._curr_ckpt_path, strict=strict)
        if hasattr(self.optimizer, "refresh_from_params"):
            self.optimizer.refresh_from_params()

    def save_checkpoint(self, save_dir, tag=None, client_state=None, save_latest=True):
        tag = f"global_step{self.global_steps}" if tag is None else str(tag)
        import os
        self._curr_ckpt_path = os.path.join(save_dir, tag)
        try:
            return super().save_checkpoint(save_dir, tag, client_state, save_latest)
        finally:
            self._curr_ckpt_path = None

    def load_checkpoint(self, load_dir, tag=None, load_module_strict=True, load_optimizer_states=True,
                        load_lr_scheduler_states=True):
        import os
        if tag is None:
            latest = os.path.join(load_dir, "latest")
            if os.path.isfile(latest):
                tag = open(latest).read().strip()
        self._curr_ckpt_path = os.path.join(load_dir, str(tag))
        try:
            return super().load_checkpoint(load_dir, tag, load_module_strict, load_optimizer_states,
                                           load_lr_scheduler_states)
        finally:
            self._curr_ckpt_path = None

    _INSTRUCTION_MAP = {
        schedule.OptimizerStep: _exec_optimizer_step,
        schedule.ReduceGrads: _exec_reduce_grads,
        schedule.ReduceTiedGrads: _exec_reduce_tied_grads,
        schedule.LoadMicroBatch: _exec_load_micro_batch,
        schedule.ForwardPass: _exec_forward_pass,
        schedule.BackwardPass: _exec_backward_pass,
        schedule.SendActivation: _exec_send_activations,
        schedule.RecvActivation: _exec_recv_activations,
        schedule.SendGrad: _exec_send_grads,
        schedule.RecvGrad: _exec_recv_grads,
    }

    def _exec_schedule(self, pipe_schedule):
        self._reserve_pipe_buffers(pipe_schedule.num_pipe_buffers())
        self._compute_loss = True
        flat = [cmd for step_cmds in pipe_schedule for cmd in step_cmds]
        plan = self._plan_prefetch(flat) if (self._async_p2p and self.is_pipe_parallel) else {}
        try:
            for i, cmd in enumerate(flat):
                if type(cmd) not in self._INSTRUCTION_MAP:
                    raise RuntimeError(f"{self.__class__.__name__} does not understand instruction {repr(cmd)}")
                if isinstance(cmd, schedule.OptimizerStep):
                    self._drain_p2p()
                for j in plan.get(i, ()):
                    self._prefetch(flat[j])
                if self.p2p_trace is not None and isinstance(cmd, (schedule.ForwardPass, schedule.BackwardPass)):
                    self.p2p_trace.append((type(cmd).__name__, cmd.kwargs["buffer_id"], len(self._pending_sends),
                                           len(self._prefetched) + len(self._recv_handles)))
                self._exec_instr = self._INSTRUCTION_MAP[type(cmd)].__get__(self, PipelineEngine)
                self._exec_instr(**cmd.kwargs)
        finally:
            self._drain_p2p()
            self._prefetched = {}


class PipelineError(Exception):
    """Errors related to the use of deepspeed.PipelineEngine."""
