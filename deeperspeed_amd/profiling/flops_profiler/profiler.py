"""Per-module FLOPs / MACs / latency / parameter profiler.

Reference parity: deepspeed/profiling/flops_profiler/profiler.py:1-868 (`FlopsProfiler`,
`get_model_profile`, `print_model_profile`, `print_model_aggregated_profile`, the *_to_string
helpers).  Like the reference, `get_total_flops()` counts multiply-accumulates (MACs) and the
printed FLOPs are 2 * MACs.

Design (no monkey-patching of torch.nn.functional): a `TorchDispatchMode` sees every aten op
issued while profiling and prices it from a formula table (mm/addmm/bmm/baddbmm/conv/sdpa +
elementwise / normalisation / softmax ops), and the framework's own HIP kernels (flash
attention, fused LayerNorm, bias-GeLU, cross-entropy, rotary) report their cost through
`record_native_macs` because they are invisible to the aten dispatcher.  Module forward
pre/post hooks snapshot a global counter, so a module's count includes its children;
latencies are measured between device-synchronised hooks.
"""

from __future__ import annotations

import time
from functools import reduce
from typing import Dict, Optional

import torch
import torch.nn as nn
from torch.utils._python_dispatch import TorchDispatchMode

_ACTIVE: Optional["_Counter"] = None


def _prod(xs):
    return reduce(lambda a, b: a * b, xs, 1)


def record_native_macs(macs: float):
    """Called by deeperspeed_amd.ops.native for HIP kernels (no-op unless profiling)."""
    if _ACTIVE is not None:
        _ACTIVE.macs += macs


class _Counter(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.macs = 0.0

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        try:
            self.macs += _aten_macs(func, args, kwargs, out)
        except Exception:  # pragma: no cover - never break the model for a statistic
            pass
        return out


_ELEMENTWISE_1 = {"relu", "gelu", "silu", "sigmoid", "tanh", "add", "sub", "mul", "div", "neg", "exp", "log",
                  "dropout", "native_dropout", "hardtanh", "leaky_relu", "elu", "pow", "sqrt", "rsqrt", "clamp"}


def _aten_macs(func, args, kwargs, out) -> float:
    name = func.__name__.split(".")[0] if hasattr(func, "__name__") else str(func)
    name = name.rstrip("_")
    if name == "mm":
        a, b = args[0], args[1]
        return a.shape[0] * a.shape[1] * b.shape[1]
    if name == "addmm":
        a, b = args[1], args[2]
        return a.shape[0] * a.shape[1] * b.shape[1]  # bias add is not a MAC (reference linear formula)
    if name in ("bmm", "baddbmm"):
        a, b = (args[0], args[1]) if name == "bmm" else (args[1], args[2])
        return a.shape[0] * a.shape[1] * a.shape[2] * b.shape[2]
    if name in ("convolution", "_convolution", "cudnn_convolution", "miopen_convolution"):
        x, w = args[0], args[1]
        transposed = bool(args[6]) if len(args) > 6 else False
        if transposed:
            return x.numel() * _prod(w.shape[1:])
        return out.numel() * _prod(w.shape[1:])
    if name in ("_scaled_dot_product_flash_attention", "_scaled_dot_product_efficient_attention",
                "scaled_dot_product_attention", "_scaled_dot_product_flash_attention_for_cpu"):
        q, k = args[0], args[1]
        return 2 * _prod(q.shape[:-1]) * k.shape[-2] * q.shape[-1]
    if name in ("_softmax", "softmax", "_log_softmax", "log_softmax"):
        return out.numel()
    if name in ("native_layer_norm", "native_batch_norm", "_native_batch_norm_legit", "native_group_norm"):
        return 5 * args[0].numel()  # reference counts 5 ops per element for norms
    if name in _ELEMENTWISE_1:
        return out.numel() if torch.is_tensor(out) else 0
    return 0


class FlopsProfiler:
    """Measure the model's forward pass: MACs, latency and parameter count per module."""

    def __init__(self, model: nn.Module):
        self.model = model
        self._handles = []
        self._counter = None
        self.started = False
        self.flops = 0
        self.params = 0

    # ------------------------------------------------------------------ lifecycle
    def start_profile(self, ignore_list=None):
        global _ACTIVE
        self.reset_profile()
        ignore = tuple(ignore_list or ())
        sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)

        def pre(module, inp):
            if ignore and isinstance(module, ignore):
                return
            sync()
            module.__start_macs__ = self._counter.macs
            module.__start_time__ = time.time()

        def post(module, inp, out):
            if ignore and isinstance(module, ignore):
                return
            sync()
            module.__flops__ += self._counter.macs - module.__start_macs__
            module.__duration__ += time.time() - module.__start_time__

        for m in self.model.modules():
            self._handles.append(m.register_forward_pre_hook(pre))
            self._handles.append(m.register_forward_hook(post))
        self._counter = _Counter()
        self._counter.__enter__()
        _ACTIVE = self._counter
        from ...ops import native
        native._flop_sink = record_native_macs
        self.started = True

    def stop_profile(self):
        global _ACTIVE
        if self._counter is not None:
            self._counter.__exit__(None, None, None)
            self._counter_macs = self._counter.macs
        _ACTIVE = None
        from ...ops import native
        native._flop_sink = None
        for h in self._handles:
            h.remove()
        self._handles = []

    def end_profile(self):
        self.stop_profile()
        for m in self.model.modules():
            for a in ("__flops__", "__params__", "__duration__", "__start_macs__", "__start_time__"):
                if hasattr(m, a):
                    delattr(m, a)
        self.started = False

    def reset_profile(self):
        for m in self.model.modules():
            m.__flops__ = 0
            m.__duration__ = 0.0
            m.__params__ = sum(_pnumel(p) for p in m.parameters() if p.requires_grad)

    # ------------------------------------------------------------------ totals
    def get_total_flops(self, as_string=False):
        """Total MACs of the profiled forward passes (reference naming)."""
        v = getattr(self.model, "__flops__", 0)
        return macs_to_string(v) if as_string else v

    def get_total_macs(self, as_string=False):
        return self.get_total_flops(as_string)

    def get_total_duration(self, as_string=False):
        v = getattr(self.model, "__duration__", 0.0)
        return duration_to_string(v) if as_string else v

    def get_total_params(self, as_string=False):
        v = getattr(self.model, "__params__", 0)
        return params_to_string(v) if as_string else v

    # ------------------------------------------------------------------ reports
    def print_model_profile(self, profile_step=1, module_depth=-1, top_modules=3, detailed=True, output_file=None):
        macs, dur, params = self.get_total_flops(), self.get_total_duration(), self.get_total_params()
        self.flops, self.params = macs, params
        lines = ["", "-------------------------- DeepSpeed Flops Profiler --------------------------",
                 "Summary of forward pass:",
                 "{:<60}  {:<8}".format("Profile step: ", profile_step),
                 "{:<60}  {:<8}".format("Number of parameters: ", params_to_string(params)),
                 "{:<60}  {:<8}".format("Number of multiply-accumulate operations (MACs): ", num_to_string(macs)),
                 "{:<60}  {:<8}".format("Number of floating point operations ( = 2 * MACs): ", num_to_string(2 * macs)),
                 "{:<60}  {:<8}".format("Latency: ", duration_to_string(dur)),
                 "{:<60}  {:<8}".format("Floating point operations per second(FLOPS): ",
                                        flops_to_string(2 * macs / dur if dur > 0 else 0))]
        lines += self._aggregated_lines(module_depth, top_modules)
        if detailed:
            lines += ["", "------------------------------ Detailed Profile ------------------------------",
                      "Each module profile is listed after its name in the following order:",
                      "number of parameters, percentage of total parameters, number of multiply-accumulate "
                      "operations (MACs), percentage of total MACs, latency, percentage of total latency, "
                      "number of floating point operations per second (FLOPS, computed as 2 * MACs / latency).", ""]
            lines += self._tree_lines(self.model, "", macs, dur, params)
        lines.append("------------------------------------------------------------------------------")
        text = "\n".join(lines)
        if output_file:
            with open(output_file, "w") as f:
                f.write(text + "\n")
        else:
            print(text)
        return text

    def print_model_aggregated_profile(self, module_depth=-1, top_modules=3):
        text = "\n".join(self._aggregated_lines(module_depth, top_modules))
        print(text)
        return text

    def _tree_lines(self, module, indent, tot_macs, tot_dur, tot_params, name="model"):
        f = getattr(module, "__flops__", 0)
        d = getattr(module, "__duration__", 0.0)
        p = getattr(module, "__params__", 0)
        stats = ", ".join([params_to_string(p), f"{100 * p / max(tot_params, 1):.2f}% Params",
                           macs_to_string(f), f"{100 * f / max(tot_macs, 1):.2f}% MACs", duration_to_string(d),
                           f"{100 * d / tot_dur if tot_dur else 0:.2f}% latency",
                           flops_to_string(2 * f / d if d else 0)])
        out = [f"{indent}({name}): {type(module).__name__}({stats})"]
        for cname, child in module.named_children():
            out += self._tree_lines(child, indent + "  ", tot_macs, tot_dur, tot_params, cname)
        return out

    def _aggregated_lines(self, module_depth, top_modules):
        info: Dict[int, Dict[str, list]] = {}

        def walk(m, depth):
            info.setdefault(depth, {})
            e = info[depth].setdefault(type(m).__name__, [0, 0, 0.0])
            e[0] += getattr(m, "__params__", 0)
            e[1] += getattr(m, "__flops__", 0)
            e[2] += getattr(m, "__duration__", 0.0)
            for c in m.children():
                walk(c, depth + 1)

        walk(self.model, 0)
        if not info:
            return []
        depth = max(info) if module_depth == -1 else min(module_depth, max(info))
        d = info[depth]
        top = lambda i: sorted(d.items(), key=lambda kv: kv[1][i], reverse=True)[:top_modules]  # noqa: E731
        return ["", "----------------------------- Aggregated Profile -----------------------------",
                f"Top {top_modules} modules in terms of params, MACs or latency at different model depths:",
                f"depth {depth}:",
                "    params      - " + str({k: params_to_string(v[0]) for k, v in top(0)}),
                "    MACs        - " + str({k: macs_to_string(v[1]) for k, v in top(1)}),
                "    fwd latency - " + str({k: duration_to_string(v[2]) for k, v in top(2)})]


def _pnumel(p):
    return p.ds_numel if hasattr(p, "ds_numel") else p.numel()


# ---------------------------------------------------------------------- string helpers
def num_to_string(num, precision=2):
    for div, unit in ((1e9, " G"), (1e6, " M"), (1e3, " K")):
        if num // div > 0:
            return str(round(num / div, precision)) + unit
    return str(num)


def _units(value, units, precision, table, suffix):
    if units is None:
        for div, u in table:
            if value // div > 0:
                return str(round(value / div, precision)) + " " + u + suffix
        return str(value) + " " + suffix
    div = dict((u, d) for d, u in table).get(units, 1)
    return str(round(value / div, precision)) + " " + units + suffix


_SI = ((1e12, "T"), (1e9, "G"), (1e6, "M"), (1e3, "K"))


def macs_to_string(macs, units=None, precision=2):
    return _units(macs, units, precision, _SI, "MACs")


def flops_to_string(flops, units=None, precision=2):
    return _units(flops, units, precision, _SI, "FLOPS")


def params_to_string(params_num, units=None, precision=2):
    return _units(params_num, units, precision, ((1e9, "G"), (1e6, "M"), (1e3, "k")), "").strip()


def duration_to_string(duration, units=None, precision=2):
    if units is None:
        if duration > 1:
            return str(round(duration, precision)) + " s"
        if duration * 1e3 > 1:
            return str(round(duration * 1e3, precision)) + " ms"
        if duration * 1e6 > 1:
            return str(round(duration * 1e6, precision)) + " us"
        return str(duration)
    return str(round(duration * {"us": 1e6, "ms": 1e3}.get(units, 1), precision)) + " " + units


def get_module_flops(module):
    return getattr(module, "__flops__", 0)


def get_model_profile(model, input_res=None, input_constructor=None, print_profile=True, detailed=True,
                      module_depth=-1, top_modules=3, warm_up=1, as_string=True, output_file=None,
                      ignore_modules=None, args=None, kwargs=None):
    """Profile one forward pass; returns (macs, params) like the reference (strings when
    `as_string`)."""
    assert isinstance(model, nn.Module)
    dev = next(model.parameters()).device

    def make_inputs():
        if input_constructor is not None:
            r = input_constructor(input_res)
            return ((), r) if isinstance(r, dict) else ((r,) if torch.is_tensor(r) else tuple(r), {})
        if args is not None or kwargs is not None:
            return tuple(args or ()), dict(kwargs or {})
        return (torch.ones(()).new_empty((1, *input_res), device=dev),), {}

    model.eval()
    with torch.no_grad():
        for _ in range(warm_up):
            a, k = make_inputs()
            model(*a, **k)
        prof = FlopsProfiler(model)
        prof.start_profile(ignore_list=ignore_modules)
        a, k = make_inputs()
        model(*a, **k)
        macs, params = prof.get_total_flops(), prof.get_total_params()
        if print_profile:
            prof.print_model_profile(profile_step=warm_up, module_depth=module_depth, top_modules=top_modules,
                                     detailed=detailed, output_file=output_file)
        prof.end_profile()
    if as_string:
        return macs_to_string(macs), params_to_string(params)
    return macs, params
