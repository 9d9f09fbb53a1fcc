"""Host-side time (median of the last 20 calls) per training-step phase of the BERT bench (no device syncs inside the step):
which Python paths keep the GPU waiting.  Wraps the engine's forward / backward / step and the
optimizer pieces with perf_counter and prints mean milliseconds per call as one JSON line."""
import json
import os
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

acc = defaultdict(list)


def wrap(obj, name, tag):
    fn = getattr(obj, name)

    def w(*a, **k):
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[tag].append(time.perf_counter() - t)
    setattr(obj, name, w)


def main():
    from deeperspeed_amd.runtime.fp16 import unfused_optimizer as uo
    from deeperspeed_amd.ops.lamb import fused_lamb as fl
    from deeperspeed_amd.runtime import engine as eng
    from deeperspeed_amd.runtime import utils as ru
    wrap(uo.FP16_UnfusedOptimizer, "step", "opt.step")
    wrap(uo.FP16_UnfusedOptimizer, "zero_grad", "opt.zero_grad")
    wrap(uo.FP16_UnfusedOptimizer, "_device_coef", "opt._device_coef")
    wrap(fl.FusedLamb, "step", "lamb.step")
    wrap(fl.FusedLamb, "_multi_step", "lamb._multi_step")
    wrap(eng.DeepSpeedEngine, "forward", "engine.forward")
    wrap(eng.DeepSpeedEngine, "backward", "engine.backward")
    wrap(eng.DeepSpeedEngine, "step", "engine.step")
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    import runpy
    runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench_bert.py"), run_name="__main__")
    # steady state: median over the last 20 calls of each (after the warmup steps)
    import statistics
    print(json.dumps({k: round(1e3 * statistics.median(v[-20:]), 3) for k, v in acc.items()}), flush=True)


if __name__ == "__main__":
    main()
