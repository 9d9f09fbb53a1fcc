"""Which HIP streams share a hardware queue with the compute stream?

HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware queues; streams on one queue execute in
submission order, so a side stream's cross-stream wait (a barrier packet) stalls every stream on
its queue.  Test per candidate: a bounded spin kernel on the compute stream, then a tiny kernel
on the candidate.  On a separate queue the tiny kernel finishes while the spin still runs; on a
shared queue it finishes after it.

    python scripts/probe_hw_queues.py   -> one JSON line per candidate stream
"""

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deeperspeed_amd.ops import native  # noqa: E402


def spin_cycles_for(ms):
    torch.cuda.synchronize()
    t = time.time()
    torch.cuda._sleep(1_000_000)
    torch.cuda.synchronize()
    per = (time.time() - t) / 1_000_000
    return int(ms / 1000.0 / max(per, 1e-12))


def shares_queue(a, b, cycles):
    torch.cuda.synchronize()
    ea, eb = torch.cuda.Event(), torch.cuda.Event()
    with torch.cuda.stream(a):
        torch.cuda._sleep(cycles)
        ea.record(a)
    with torch.cuda.stream(b):
        torch.cuda._sleep(100)
        eb.record(b)
    eb.synchronize()
    a_done = ea.query()
    torch.cuda.synchronize()
    return bool(a_done)


def main():
    hip = native.hip_ops()
    least, greatest = hip.stream_priority_range()
    print(json.dumps({"priority_range": {"least": least, "greatest": greatest},
                      "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)
    cycles = spin_cycles_for(30.0)
    comp = torch.cuda.current_stream()
    cands = []
    for i in range(6):
        cands.append((f"torch_default_{i}", torch.cuda.Stream()))
    for i in range(2):
        cands.append((f"torch_prio_high_{i}", torch.cuda.Stream(priority=-1)))
    for prio in sorted({least, 0, greatest}):
        for i in range(4):
            cands.append((f"hip_prio{prio}_{i}", torch.cuda.ExternalStream(hip.priority_stream(prio))))
    for name, s in cands:
        r = {"stream": name, "shares_compute_queue": shares_queue(comp, s, cycles)}
        print(json.dumps(r), flush=True)
    # low-priority streams among themselves
    lows = [s for n, s in cands if n.startswith(f"hip_prio{least}_")]
    for i in range(1, len(lows)):
        print(json.dumps({"pair": f"low0-low{i}", "shared": shares_queue(lows[0], lows[i], cycles)}), flush=True)


if __name__ == "__main__":
    main()
