#!/usr/bin/env python
"""Headline benchmark: GPT-NeoX-20B, ZeRO-3, bf16, synthetic data, random-init weights.

Metric (BASELINE.json): tokens/sec for the whole node at N = 1/2/4/8 MI355X (weak scaling:
the per-GPU micro-batch and gradient-accumulation are fixed as N grows).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Each step is a full training step through the framework: forward + backward of every
micro-batch, ZeRO-3 all-gathers / reduce-scatters over RCCL, global-norm clipping, fused Adam
on the fp32 master, bf16 parameter refresh.  A memory planner picks the layout per N: on one
GPU the 20B model's states only fit as 14 B/param (compact fp32 master = bf16 weight + int16
residual) with activation recompute; with N >= 2 the shards shrink, recompute turns off and
the spare HBM keeps gathered parameters resident across micro-batches
(stage3_max_live_parameters).

`--pipe P` switches to BASELINE config 4 (PipelineModule PP=P x DP=N/P, ZeRO-1 or 1-bit
Adam via `--optimizer onebitadam`).

Rank 0 prints ONE JSON line.  `vs_baseline` divides by the only DeeperSpeed-derived
number BASELINE.md gives for this model/metric (410 tokens/s per GPU: the reference's best
published ZeRO-3 efficiency of 49 TFLOPS/GPU applied to 20B at 6N FLOPs/token), times N.
"""

import argparse
import json
import os
import sys
import time

# stdout carries exactly one line, the result JSON: everything else printed to fd 1 (framework
# logs, the RCCL banner written by the C library) goes to stderr; emit_result() writes to the
# original stdout
_RESULT_FD = os.dup(1)
sys.stdout.flush()
os.dup2(2, 1)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def emit_result(out):
    os.write(_RESULT_FD, (json.dumps(out) + "\n").encode())

REF_TOKENS_PER_GPU = 410.0  # BASELINE.md "North-star planning targets (derived)"
# 1-bit Adam / LAMB (BASELINE config 4).  Their update has no bias correction (reference
# deepspeed/runtime/fp16/onebit/adam.py:197-265, mirrored in runtime/fp16/onebit/adam.py), so the
# variance frozen at freeze_step is (1 - beta2^k) E[g^2]: after the old 2 warm-up steps at
# beta2 = 0.999 that is 2e-3 E[g^2], and the compressed momentum then moves every element by
# ~20x lr per step -- the PP rehearsals ended at loss 115-1,548 from 11.6.  The reference advises
# freeze_step 400-23,000 at beta2 0.999 (docs/_tutorials/onebit-adam.md:87,187); a benchmark
# cannot afford that many untimed steps, so it runs GPT-NeoX's beta2 = 0.95 (its 20B config) and
# freezes after 16 steps, when the variance estimate holds 1 - 0.95^16 = 56 % of E[g^2].
ONEBIT_FREEZE = 16
ONEBIT_BETAS = [0.9, 0.95]
# a run whose final loss is non-finite or above this multiple of its first warmup loss is marked
# "diverged": true in the result line
DIVERGED_RATIO = 1.2
# memory margins (GiB): below the device for the measured fit / stash (allocator variance on another
# box), on each moment tier, and the headroom the first fit grant keeps back
MEM_FLOOR_GIB = 3.0
STASH_MARGIN_GIB = 2.0
STASH_FLOOR_GIB = 1.5
TIER_MARGIN_GIB = 6.0
FIT_MARGIN_GIB = 1.0
HOST_MOMENTS_GIB = [0.0]  # set from --host-moments-gib


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--model", type=str, default="gpt-neox-20b")
    p.add_argument("--micro-batch", type=int, default=None)
    p.add_argument("--grad-accum", type=int, default=None)
    p.add_argument("--seq", type=int, default=2048)
    p.add_argument("--zero", type=int, default=3)
    p.add_argument("--offload", type=str, default="auto", choices=["auto", "none", "compact", "master", "all", "nvme", "moments"],
                   help="moments: Adam moments in pinned host memory, compact master + grads in HBM (6 B/param)")
    p.add_argument("--ckpt", type=str, default="auto", choices=["auto", "on", "off"],
                   help="activation checkpointing; auto = off when activations fit in HBM next to the shards")
    p.add_argument("--layers", type=int, default=None, help="override depth (memory experiments only)")
    p.add_argument("--hidden", type=int, default=None, help="override width (peak-params runs; heads = hidden/128)")
    p.add_argument("--sparse", type=str, default=None,
                   help="block-sparse attention mode (bigbird|fixed|bslongformer|variable|local) - BASELINE config 5")
    p.add_argument("--block", type=int, default=64, help="sparse attention block size")
    p.add_argument("--nvme-path", type=str, default="/tmp/dsa_nvme", help="ZeRO-Infinity swap folder (--offload nvme)")
    p.add_argument("--profile-steps", type=int, default=0, help="extra steps under torch.profiler (0 = off)")
    p.add_argument("--local_rank", type=int, default=None)
    p.add_argument("--max-live", type=float, default=None,
                   help="override stage3_max_live_parameters (default: planned from spare HBM)")
    p.add_argument("--pipe", type=int, default=1,
                   help="pipeline stages (BASELINE config 4: --model gpt3-6.7b --pipe 4 on 8 GPUs = PP4 x DP2)")
    p.add_argument("--optimizer", type=str, default="adam", choices=["adam", "onebitadam", "onebitlamb", "lamb"],
                   help="1-bit optimizers run without ZeRO (reference restriction)")
    p.add_argument("--freeze-step", type=int, default=None,
                   help="1-bit optimizers: full-precision warm-up steps before compression (default "
                        f"{ONEBIT_FREEZE}; the untimed warmup is extended past it so every timed step is a "
                        "compressed one)")
    p.add_argument("--force-sharded", action="store_true",
                   help="ZeRO-3 on one GPU: run the gather / reduce-scatter unit path over a world-1 RCCL "
                        "communicator instead of binding parameters to their shards")
    p.add_argument("--resident-grads", type=str, default="auto", choices=["auto", "on", "off"],
                   help="keep gradients resident across micro-batches, one reduce-scatter per step "
                        "(auto: when the spare HBM holds a bf16 copy of the gradients)")
    p.add_argument("--dist-backend", type=str, default="nccl",
                   help="nccl (= RCCL); gloo only to rehearse N ranks sharing one GPU (forced on CPU)")
    p.add_argument("--host-moments-layers", type=str, default="auto",
                   help="Adam moments of the LM head and the last K transformer layers in pinned host memory, "
                        "streamed through HBM during the step (frees 8 B/param of HBM for the activation stash); "
                        "head: the LM head only; auto: 1 for the 20B single-GPU bound ZeRO-3 run (1 / 2 / 3 measured "
                        "8,936 / 8,895 / 8,647 "
                        "tok/s, profiles/r4w_notes.md), else 0")
    p.add_argument("--moments-tiers", type=str, default="auto",
                   help="--offload moments: where the Adam moments live, per layer, in the order HBM -> pinned host "
                        "-> NVMe file (--nvme-path).  auto: HBM headroom, then the host budget "
                        "(--host-moments-gib, default min(available - 24 GiB, 215 GiB)), then the free disk; "
                        "host: everything in pinned host memory")
    p.add_argument("--stash", type=str, default="auto", choices=["auto", "attn", "off"],
                   help="selective recompute from measured headroom (one-GPU recompute runs): auto = attention "
                        "outputs, then fc1 outputs with what is left; attn = attention only; off = full recompute")
    p.add_argument("--stash-offload", action="store_true",
                   help="park the attention stash of the layers HBM cannot hold in pinned host memory "
                        "(measured slower on MI355X: profiles/aux/host_stash_ab.log)")
    p.add_argument("--mlp-host-layers", type=int, default=0,
                   help="one-GPU recompute runs: the first K layers without an HBM fc1 stash park their fc1 "
                        "output in pinned host memory (copy engines) instead of recomputing the fc1 GEMM")
    p.add_argument("--park-backlog", type=int, default=6,
                   help="host-parked stashes whose device->host copy may be outstanding before the compute "
                        "stream waits (bounds the HBM they pin)")
    p.add_argument("--host-moments-gib", type=float, default=0.0,
                   help="--offload moments: pinned-host budget of the moment tiers (0: min(available - 24, 215) GiB)")
    p.add_argument("--overlap-step", type=str, default="on", choices=["on", "off"],
                   help="bound single-rank ZeRO-3: the fused Adam step overlaps the next forward (side stream)")
    p.add_argument("--memtrace", action="store_true", help="log HBM after every warmup phase and per layer")
    p.add_argument("--emulate-world", type=int, default=0,
                   help="one process runs rank 0 of an N-rank ZeRO job at full depth: shards, buckets, "
                        "micro-batch, recompute and memory fit planned for N ranks, collectives replaced by "
                        "local stand-ins that write the same bytes (utils/comm.py).  Reports EMULATED per-rank "
                        "tokens/s, the collective bytes per step and the xGMI rate full overlap needs")
    p.add_argument("--fp32-reduce", type=str, default="auto", choices=["auto", "on", "off"],
                   help="reduce bf16 gradients in fp32 (DeeperSpeed's bf16 default fp32_allreduce; "
                        "tests/test_zero_reduce_precision.py measures what bf16 reduction costs).  auto: on "
                        "for N >= 2 -- the emulated N = 2 / 4 / 8 ranks measured -2.3 / -2.1 / +0.1 %% per-rank "
                        "throughput and 33.5 vs 22.3 GB/s of xGMI at N = 8 (profiles/r6a_emulated_world_notes.md); "
                        "one rank reduces nothing")
    return p.parse_args()


def plan_memory(cfg, mb, seq, world, offload, ckpt, ga=1):
    """Bytes of HBM one rank needs: ZeRO-3 model states + activations + transient buffers.

    States per parameter: bf16 weight shard 2 B + gradient shard + fp32 moments 8 B + fp32
    master 4 B (2 B int16 residual with compact_master, 0 B when offloaded).  The gradient
    shard is bf16 (2 B) on one rank (gradients accumulate in place into the bound shard) and
    fp32 (4 B) for N >= 2 with gradient accumulation (reduce-scattered micro-batch gradients
    are summed in fp32).  Measured on MI355X (--memtrace, profiles/aux/memtrace_*.log):
    20B, N=1, compact, recompute on -> planned 279 GiB, peak 274.7 GiB; activations of one
    GPT-NeoX layer without recompute = 32.0 * s * b * h bytes (budgeted as 34), one s*b*h
    layer input with it.  Transients: two gathered ZeRO-3 units, the logits (bf16 + grad,
    fused HIP cross-entropy) and allocator slack."""
    p = cfg.num_params()
    grad = 4 if (world > 1 and ga > 1) else 2
    per_param = {"none": 14, "compact": 12, "master": 10, "all": 2, "nvme": 2, "moments": 4}[offload] + grad
    states = p * per_param / world
    sbh = seq * mb * cfg.hidden_size
    act_layer = 2 * sbh if ckpt else 34 * sbh
    acts = cfg.num_layers * act_layer + (34 * sbh if ckpt else 0)
    logits = seq * mb * cfg.vocab_size * 4  # bf16 logits + bf16 grad (fused HIP cross-entropy)
    transient = 2 * 2 * 2e8 * 2 + logits + 2 * 2**30
    return states + acts + transient


def plan_moment_tiers(model, P, hbm_free, nvme_path):
    """Peak-parameter layout (--offload moments): budgets of the three moment tiers from what this
    box measures (HBM headroom under the plan, host memory, free disk at --nvme-path), then
    runtime/memory_fit.split_moment_tiers assigns the model's blocks to them in order."""
    import shutil
    from deeperspeed_amd.runtime import memory_fit
    margin = TIER_MARGIN_GIB * 2**30
    hbm = max(0.0, hbm_free - margin)
    try:
        import psutil
        avail = psutil.virtual_memory().available
    except Exception:  # noqa: BLE001
        avail = 1 << 50
    host = HOST_MOMENTS_GIB[0] * 2**30 or min(avail - 24 * 2**30, 215 * 2**30)
    os.makedirs(nvme_path, exist_ok=True)
    disk = max(0.0, shutil.disk_usage(nvme_path).free - TIER_MARGIN_GIB * 2**30)
    blocks = [[model.embed_in]] + [[l] for l in model.layers] + [[model.final_layer_norm, model.embed_out]]
    blocks = [[p for m in mods for p in m.parameters()] for mods in blocks]
    try:
        groups, rec = memory_fit.split_moment_tiers(blocks, {"gpu": hbm, "cpu": host, "nvme": disk})
    except memory_fit.TierShortfall as e:
        raise SystemExit(f"[bench] {e}")
    log(f"moment tiers: HBM {rec['gpu']['gib']} GiB, pinned host {rec['cpu']['gib']} GiB, NVMe "
        f"{rec['nvme']['gib']} GiB ({nvme_path}); budgets {rec['budget_gib']}")
    return groups, rec


def log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


# A rank that hangs (an RCCL collective that never completes, a stuck kernel) must not burn a
# multi-GPU slot for the process-group timeout: every rank beats a heartbeat per phase / warmup /
# timed step (one stderr line + a file the spawning parent watches) and a watchdog thread ends
# the rank -- after printing its last heartbeat and every thread's Python stack -- when no beat
# came for DSA_BENCH_WATCHDOG_S seconds.  Its non-zero exit makes torchrun, or spawn_ranks
# below, stop the whole job.  Warmup steps beat once per micro-batch phase (forward / backward /
# step), so the default limit stays below a 180 s silence guard of the job's supervisor and a
# stall leaves every rank's stacks behind, not a killed job without evidence.
WATCHDOG_S = float(os.environ.get("DSA_BENCH_WATCHDOG_S", "150"))
PG_TIMEOUT_S = float(os.environ.get("DSA_BENCH_PG_TIMEOUT_S", "600"))


class Heartbeat:
    def __init__(self, rank, limit_s=WATCHDOG_S):
        import threading
        self.rank = rank
        self.limit = limit_s
        self.last = "start"
        self.t = time.time()
        self.path = None
        d = os.environ.get("DSA_BENCH_HB_DIR")
        if d:
            self.path = os.path.join(d, f"rank{rank}")
        self._write()
        if limit_s > 0:
            threading.Thread(target=self._watch, name="bench-watchdog", daemon=True).start()

    def _write(self):
        if self.path:
            tmp = self.path + ".tmp"
            with open(tmp, "w") as f:
                f.write(f"{self.t:.3f} {self.last}\n")
            os.replace(tmp, self.path)

    def beat(self, what, quiet=False, **info):
        self.last = what + "".join(f" {k}={v}" for k, v in info.items())
        self.t = time.time()
        if not quiet:
            print(f"[hb] rank={self.rank} {self.last}", file=sys.stderr, flush=True)
        self._write()

    def _watch(self):
        import faulthandler
        while True:
            time.sleep(min(5.0, self.limit / 4))
            idle = time.time() - self.t
            if idle > self.limit:
                print(f"[bench] WATCHDOG rank {self.rank}: no progress for {idle:.0f}s "
                      f"(limit {self.limit:.0f}s, DSA_BENCH_WATCHDOG_S); last heartbeat: {self.last}; "
                      f"Python stacks follow", file=sys.stderr, flush=True)
                try:
                    from deeperspeed_amd.utils import comm
                    print(f"[bench] WATCHDOG rank {self.rank}: {comm.progress()}", file=sys.stderr, flush=True)
                except Exception:  # noqa: BLE001 - diagnostics only
                    pass
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                os._exit(124)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`bench.py --gpus N` without an external launcher: start N rank processes of this script,
    one per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment), relay rank 0's
    result line, and stop every rank as soon as one fails (the contract of the framework's own
    launcher, launcher/launch.py; reference deepspeed/launcher/launch.py:121-175).  The parent
    never initialises HIP: only the rank processes touch the GPU."""
    import signal
    import subprocess
    import threading
    import tempfile
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
    hb_dir = tempfile.mkdtemp(prefix="dsa_bench_hb_")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR=addr, MASTER_PORT=port, DSA_BENCH_HB_DIR=hb_dir)
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else 2,
                                      start_new_session=True))
    lines = []
    reader = threading.Thread(target=lambda: lines.extend(procs[0].stdout.readlines()), daemon=True)
    reader.start()

    def signal_all(sig):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except (ProcessLookupError, PermissionError):
                    pass

    def stop_all(grace=30.0):
        signal_all(signal.SIGTERM)
        signal_all(signal.SIGCONT)  # a stopped rank handles its SIGTERM only once resumed
        deadline = time.time() + grace
        while any(p.poll() is None for p in procs) and time.time() < deadline:
            time.sleep(0.2)
        signal_all(signal.SIGKILL)

    def on_signal(signum, frame):
        stop_all(10.0)
        sys.exit(128 + signum)

    def heartbeats():
        out = {}
        for r in range(n):
            try:
                with open(os.path.join(hb_dir, f"rank{r}")) as f:
                    t, _, what = f.read().strip().partition(" ")
                out[r] = (float(t), what)
            except (OSError, ValueError):
                out[r] = (None, "no heartbeat yet")
        return out

    signal.signal(signal.SIGINT, on_signal)
    signal.signal(signal.SIGTERM, on_signal)
    rc = 0
    # parent-side watchdog: covers a rank that cannot run its own (stopped, wedged in a driver
    # call holding the GIL); a little longer than the ranks' own limit so theirs fires first
    limit = WATCHDOG_S + 60.0 if WATCHDOG_S > 0 else 0.0
    started = time.time()
    while True:
        codes = [p.poll() for p in procs]
        bad = next(((r, c) for r, c in enumerate(codes) if c not in (None, 0)), None)
        if bad is not None:
            r, c = bad
            rc = c if c > 0 else 128 - c
            print(f"[bench] rank {r} exited with status {c}; stopping the other ranks", file=sys.stderr, flush=True)
            for rr, (t, what) in heartbeats().items():
                print(f"[bench]   rank {rr} last heartbeat: {what}", file=sys.stderr, flush=True)
            stop_all()
            break
        if all(c == 0 for c in codes):
            break
        if limit > 0:
            now = time.time()
            hb = heartbeats()
            stale = [r for r, (t, _) in hb.items() if codes[r] is None and now - (t or started) > limit]
            if stale:
                print(f"[bench] WATCHDOG: rank(s) {stale} made no progress for {limit:.0f}s; stopping all ranks",
                      file=sys.stderr, flush=True)
                for rr, (t, what) in hb.items():
                    age = f"{now - t:.0f}s ago" if t else "never"
                    print(f"[bench]   rank {rr} last heartbeat ({age}): {what}", file=sys.stderr, flush=True)
                stop_all(10.0)
                rc = 124
                break
        time.sleep(0.2)
    for p in procs:
        p.wait()
    reader.join(timeout=10)
    import shutil
    shutil.rmtree(hb_dir, ignore_errors=True)
    if rc == 0:
        for ln in lines:
            os.write(_RESULT_FD, ln)
    return rc


def main():
    args = parse()
    HOST_MOMENTS_GIB[0] = args.host_moments_gib
    if args.fp32_reduce == "auto":
        n_ranks = args.emulate_world or int(os.environ.get("WORLD_SIZE", "0") or 0) or args.gpus
        args.fp32_reduce = "on" if n_ranks > 1 else "off"
    launched = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if launched == 0 and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = launched or 1
    emulated = args.emulate_world if args.emulate_world > 1 else 0
    if emulated:
        if world != 1:
            raise SystemExit("[bench] --emulate-world runs as ONE process (no launcher, --gpus 1)")
        if args.pipe != 1 or args.zero != 3:
            raise SystemExit("[bench] --emulate-world emulates the ZeRO-3 data-parallel bench only")
        world = emulated  # every plan below is the N-rank job's; the process group stays world 1
    elif world != args.gpus:
        log(f"--gpus {args.gpus} differs from the launcher's WORLD_SIZE={world}; using {world}")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("DSA_SKIP_MODEL_BROADCAST", "1")  # identical seeded init on every rank

    import deeperspeed_amd as ds
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    from deeperspeed_amd.ops import native
    from deeperspeed_amd.runtime import memory_fit

    on_gpu = torch.cuda.is_available()
    hb = Heartbeat(int(os.environ["RANK"]))
    if world > 1 and not emulated and int(os.environ["RANK"]) == 0 and on_gpu:
        # rank 0 logs RCCL's version, topology, channel and ring setup once (stdout of the C
        # library is redirected to stderr above), so a multi-GPU record shows how it was wired
        os.environ.setdefault("NCCL_DEBUG", "INFO")
        os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,GRAPH,ENV")
    from datetime import timedelta
    ds.init_distributed(dist_backend=args.dist_backend if on_gpu else "gloo", timeout=timedelta(seconds=PG_TIMEOUT_S))
    rank = dist.get_rank()
    hb.beat("process group up", backend=dist.get_backend(), world=world)
    if emulated:
        from deeperspeed_amd.utils import comm as _comm
        _comm.set_emulated_world(emulated)
        log(f"EMULATED world {emulated}: this process is rank 0 of a {emulated}-rank job; collectives are "
            f"local stand-ins (values meaningless, memory / kernels / collective sequence are the rank's)")
    if rank == 0 and world > 1 and not emulated:
        try:
            rccl = ".".join(map(str, torch.cuda.nccl.version())) if on_gpu else None
        except Exception:  # noqa: BLE001 - informational only
            rccl = "unknown"
        log(f"world={world} backend={dist.get_backend()} rccl={rccl} pg_timeout={PG_TIMEOUT_S:.0f}s "
            f"watchdog={WATCHDOG_S:.0f}s HSA_ENABLE_IPC_MODE_LEGACY={os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY')} "
            + " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith(("NCCL_", "RCCL_"))))
    if os.environ.get("DSA_BENCH_FAIL_RANK") == str(rank):  # teardown test hook (tests/test_bench_contract.py)
        raise SystemExit(7)
    if on_gpu:
        # one rank per GPU; more ranks than GPUs (a rehearsal of the N-GPU path on one card)
        # share the device and split its memory budget
        ndev = torch.cuda.device_count()
        local = int(os.environ["LOCAL_RANK"]) % ndev
        share = -(-int(os.environ.get("LOCAL_WORLD_SIZE", "1")) // ndev)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        native.hip_ops()  # fail loudly if the HIP extension is missing
        hbm = torch.cuda.get_device_properties(local).total_memory
    else:  # CPU / gloo: the plumbing of the contract (tests), no memory planning
        local, share, dev, hbm = 0, 1, torch.device("cpu"), float(1 << 60)

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    def reserved_peak():
        return torch.cuda.max_memory_reserved(local) if on_gpu else 0

    def device_peak():
        """Peak HBM of this rank: the allocator's reserved peak plus what lives outside it
        (RCCL buffers, runtime); the outside part is only attributable with one rank per GPU."""
        if not on_gpu:
            return 0
        outside = 0
        if share == 1:
            free, total = torch.cuda.mem_get_info(local)
            outside = max(0, (total - free) - torch.cuda.memory_reserved(local))
        return reserved_peak() + outside

    over = {"num_layers": args.layers} if args.layers else {}
    if args.hidden:
        over.update(hidden_size=args.hidden, num_heads=args.hidden // 128)
    if args.sparse:
        over["sparse_attention"] = {"mode": args.sparse, "block": args.block}
    cfg = get_config(args.model, max_seq_len=args.seq, checkpoint_activations=True, **over)
    big = get_config(args.model).num_params() > 5e9  # batch shape of the full model, also under --layers
    budget = 0.97 * hbm / share
    reserve = 0.03 * hbm / share  # allocator fragmentation, RCCL / runtime buffers
    P = cfg.num_params()

    def layout(mb, ga):
        """Model-state layout for one (micro-batch, grad-accum): compact fp32 master (bf16
        weight + int16 residual: exact, same Adam bytes as a separate fp32 master, 2 B/param
        less) > everything in HBM > fp32 master on the host; then recompute only if needed."""
        offload = args.offload
        if offload == "auto":
            offload = "none" if not on_gpu else next(
                (o for o in ("compact", "none", "master")
                 if plan_memory(cfg, mb, args.seq, world, o, True, ga) < budget), "master")
        ckpt = args.ckpt
        if ckpt == "auto":
            ckpt = "off" if plan_memory(cfg, mb, args.seq, world, offload, False, ga) < budget else "on"
        return offload, ckpt, plan_memory(cfg, mb, args.seq, world, offload, ckpt == "on", ga)

    # Per-GPU work is fixed at 16 sequences per optimizer step for the big models (weak
    # scaling).  When the shards are small enough (N >= 4 for 20B), micro-batch 8 x 2 runs
    # without recompute and leaves room to keep every gathered unit resident: hipBLASLt is ~4 %
    # faster at M = 16384 tokens than at 8192 (profiles/aux/gemm_m16k.log) and the
    # per-micro-batch ZeRO-3 gradient reduce-scatters halve.  Otherwise micro-batch 4 x 4.
    # Smaller models (GPT-NeoX 1.3B, BASELINE config 2) run the 16 sequences as one micro-batch:
    # 16 x 1 measured 109.7k vs 104.6k tok/s for 8 x 2 on one MI355X (profiles/r4b_*), larger GEMMs
    # and no accumulation pass
    if args.micro_batch or args.grad_accum or not big:
        mb = args.micro_batch or (4 if big else 16 // (args.grad_accum or 1))
        ga = args.grad_accum or (4 if big else max(1, 16 // mb))
        offload, ckpt, planned = layout(mb, ga)
    else:
        for mb, ga in ((8, 2), (4, 4)):
            offload, ckpt, planned = layout(mb, ga)
            if ckpt == "off" and planned + 2 * P + reserve < budget:
                break
    cfg.checkpoint_activations = ckpt == "on"
    # ZeRO-3 retention (stage3_max_live_parameters) and resident gradients only buy speed.
    # They are sized from MEASUREMENT (runtime/memory_fit.py): the first warmup step runs lean
    # (none of either), its measured peak decides what the rest of HBM is granted to, and every
    # later warmup step gives back retention, then resident gradients, then halves the
    # micro-batch if the peak comes within MEM_FLOOR_GIB of the device.
    sharded = world > 1 or args.force_sharded
    fit = None
    if args.zero == 3 and sharded and ckpt == "off" and on_gpu and args.pipe == 1:
        fit = memory_fit.FitState(params=P, world=world, micro_batch=mb, grad_accum=ga,
                                  auto_live=args.max_live is None, auto_resident=args.resident_grads == "auto")
    live = int(args.max_live) if args.max_live is not None else (0 if fit else int(min(P, 1e9)))
    resident = args.resident_grads == "on"
    if fit is not None:
        fit.live, fit.resident = live, resident
    floor = MEM_FLOOR_GIB * 2**30
    limit = hbm / share - floor
    # gloo rehearsal of an N-GPU job on one GPU: gloo's asynchronous collectives on device tensors
    # stalled for ~50 s when several ZeRO reductions were in flight (profiles/r5a_notes.md), so the
    # rehearsal waits for each collective as it is issued (RCCL runs keep the overlap)
    gloo_gpu = on_gpu and args.dist_backend == "gloo" and not emulated
    zcfg = {"stage": args.zero, "overlap_comm": not gloo_gpu, "reduce_scatter": True, "reduce_bucket_size": int(2e8),
            "stage3_prefetch_bucket_size": int(5e8), "stage3_param_persistence_threshold": int(1e6),
            "stage3_unit_max_numel": int(2e8), "stage3_max_live_parameters": live,
            "stage3_max_reuse_distance": int(2 * P)}
    if args.force_sharded:
        # the bypass accumulates micro-batch gradients in bf16 in the bound shard; the forced
        # sharded path does the same (an fp32 shard would not fit next to 20B's states)
        zcfg.update(stage3_force_sharded=True, grad_accum_dtype="param")
    if resident:
        zcfg["resident_grads"] = True
    # bound single-rank ZeRO-3: the fused Adam step overlaps the next forward (side stream,
    # per-bucket events); --overlap-step off keeps the serial step
    if (world == 1 and not args.force_sharded and offload in ("compact", "none") and on_gpu
            and args.overlap_step == "on"):
        zcfg["overlap_step"] = True
    if offload == "compact":
        zcfg["compact_master"] = True
    elif offload == "moments":
        zcfg["compact_master"] = True
        zcfg["offload_optimizer"] = {"device": "cpu", "pin_memory": True, "states": "moments",
                                     "nvme_path": args.nvme_path}
    elif offload == "nvme":
        zcfg["offload_optimizer"] = {"device": "nvme", "nvme_path": args.nvme_path, "pin_memory": True,
                                     "states": "all"}
    elif offload != "none":
        zcfg["offload_optimizer"] = {"device": "cpu", "pin_memory": True, "states": offload}
    conf = {
        "train_micro_batch_size_per_gpu": mb,
        "gradient_accumulation_steps": ga,
        "optimizer": {"type": "Adam", "params": {"lr": 1e-4, "betas": [0.9, 0.95], "eps": 1e-8,
                                                  "weight_decay": 0.01}},
        "fp16": {"enabled": True, "type": "bfloat16"},
        "fp32_allreduce": args.fp32_reduce == "on",
        "gradient_clipping": 1.0,
        "zero_optimization": zcfg,
        "steps_per_print": 1000000,
        "wall_clock_breakdown": False,
    }
    log(f"model={args.model} params={P / 1e9:.2f}B world={world} mb={mb} ga={ga} seq={args.seq} "
        f"zero={args.zero} offload={offload} ckpt={ckpt} live={live / 1e9:.1f}B resident_grads={resident} "
        f"measured_fit={fit is not None} force_sharded={args.force_sharded} hbm={hbm / 2**30:.0f} GiB "
        f"planned={planned / 2**30:.0f} GiB")
    if args.pipe > 1:
        return run_pipeline(args, cfg, mb, ga, world, rank, dev, hb)
    t0 = time.time()
    torch.manual_seed(1234)
    model = GPTNeoX(cfg, device=dev, dtype=torch.bfloat16)
    log(f"model built in {time.time() - t0:.1f}s")
    hb.beat("model built")
    # Host moments (MI355X extension, runtime/zero/sharded_base.py _host_moments_step): on one GPU
    # the 20B states leave ~16 GiB for activations, so 18 of 44 layers recompute their attention.
    # The LM head and the last K layers are the parameters with the most slack between their final
    # gradient (early in the last micro-batch's backward) and their next read (late in the next
    # forward): their Adam moments live in pinned host memory and stream through HBM on the copy
    # engines during the overlapped step, and the 8 B/param freed goes to the attention stash.
    hm = args.host_moments_layers
    # (only where the freed HBM buys attention stash: with --stash off host moments only add the PCIe
    # phase to the step)
    k_host = (1 if (world == 1 and args.zero == 3 and offload == "compact" and ckpt == "on" and big and on_gpu
                    and not args.force_sharded and args.pipe == 1
                    and args.stash != "off") else 0) if hm == "auto" else \
        (0.5 if hm == "head" else int(hm))  # "head": the LM head only
    params = model.parameters()
    host_numel = 0
    tiers = None
    if offload == "moments" and on_gpu and args.moments_tiers != "host":
        params, tiers = plan_moment_tiers(model, P, budget - planned, args.nvme_path)
    if k_host > 0:
        host_mods = [model.embed_out] + (list(model.layers[-int(k_host):]) if k_host >= 1 else [])
        tail = {id(p) for m in host_mods for p in m.parameters()}
        host_numel = sum(p.numel() for p in model.parameters() if id(p) in tail)
        params = [{"params": [p for p in model.parameters() if id(p) not in tail]},
                  {"params": [p for p in model.parameters() if id(p) in tail], "host_moments": True}]
        log(f"host moments: LM head + last {int(k_host)} layers = {host_numel / 1e9:.2f}B params "
            f"({8 * host_numel / 2**30:.1f} GiB of Adam moments in pinned host memory)")
    engine, _, _, _ = ds.initialize(model=model, model_parameters=params, config_params=conf)
    del model
    log(f"engine ready in {time.time() - t0:.1f}s" +
        (f", mem={torch.cuda.memory_allocated() / 2**30:.1f} GiB" if on_gpu else ""))
    hb.beat("engine ready")

    def peak_gib():
        return round(torch.cuda.max_memory_allocated() / 2**30, 1) if on_gpu else 0.0

    g = torch.Generator(device=dev)
    g.manual_seed(4321 + rank)
    batches = []

    def make_batches():
        batches[:] = [torch.randint(0, cfg.vocab_size, (mb, args.seq), device=dev, generator=g) for _ in range(ga)]

    make_batches()

    def train_step():
        loss = None
        for i in range(ga):
            loss = engine(batches[i], labels=batches[i])
            engine.backward(loss)
            engine.step()
            if gloo_gpu:
                sync()  # gloo rehearsal: bounded work in flight per rank (see zcfg above)
        return loss

    def timed_step():
        """Warmup step with synchronised per-phase timing (outside the timed region)."""
        ph = {"fwd": 0.0, "bwd": 0.0, "step": 0.0}
        loss = None
        for i in range(ga):
            for name, fn in (("fwd", lambda: engine(batches[i], labels=batches[i])),
                             ("bwd", lambda: engine.backward(loss)), ("step", engine.step)):
                sync()
                t = time.time()
                r = fn()
                sync()
                ph[name] += time.time() - t
                hb.beat(f"warmup micro {i} {name} done", s=round(time.time() - t, 2), quiet=not verbose_hb)
                if name == "fwd":
                    loss = r
                if memtrace:
                    log(f"mem after micro {i} {name}: {torch.cuda.memory_allocated() / 2**30:.2f} GiB "
                        f"(peak {torch.cuda.max_memory_allocated() / 2**30:.2f})")
        return loss, ph

    memtrace = args.memtrace and on_gpu
    verbose_hb = world > 1
    if memtrace:  # per-layer activation footprint of the first forward (planner calibration)
        layers = [m for m in engine.module.modules() if type(m).__name__ == "NeoXTransformerLayer"]
        marks = []

        def _mark(m, inp, out, idx=[0]):
            if len(marks) < len(layers):
                marks.append(torch.cuda.memory_allocated())
                if len(marks) in (1, 2, len(layers)):
                    log(f"mem after layer {len(marks) - 1} fwd: {marks[-1] / 2**30:.2f} GiB")
                if len(marks) == len(layers) and len(marks) > 2:
                    log(f"activation bytes/layer = {(marks[-1] - marks[1]) / (len(marks) - 2) / 2**20:.1f} MiB "
                        f"= {(marks[-1] - marks[1]) / (len(marks) - 2) / (args.seq * mb * cfg.hidden_size):.2f} sbh")
        for m in layers:
            m.register_forward_hook(_mark)

    stashed = 0
    stashed_mlp = 0
    parked_mlp = 0

    def plan_stash():
        """Selective recompute from MEASURED headroom: after a warmup step with full recompute,
        HBM left above the allocator's reserved peak (minus a margin) keeps the attention
        q, k, v, output and LSE of as many layers as fit (NeoXAttention.stash_outputs), so their
        recompute skips the QKV GEMM, rotary split and flash forward."""
        if not cfg.checkpoint_activations or not on_gpu or args.stash == "off":
            return 0
        layers = [m for m in engine.module.modules() if type(m).__name__ == "NeoXTransformerLayer"]
        per_layer = 4 * mb * args.seq * cfg.hidden_size * 2 + mb * cfg.num_heads * args.seq * 4
        margin = STASH_MARGIN_GIB * 2**30
        free = hbm / share - reserved_peak() - margin
        per_mlp = mb * args.seq * cfg.intermediate_size * 2
        k_park = max(0, min(len(layers), args.mlp_host_layers))
        if k_park:
            # HBM the parked fc1 outputs pin: the device->host backlog and the backward's prefetch
            from deeperspeed_amd.models.gpt_neox import STASH_PREFETCH_DEPTH
            free -= (args.park_backlog + STASH_PREFETCH_DEPTH + 1) * per_mlp
        n = int(max(0, min(len(layers), free // per_layer)))
        for m in layers[-n:] if n else []:
            m.attention.stash_outputs = True
        # then the MLP: the fc1 output u [tokens, 4h] of as many layers as still fit (saves the fc1
        # GEMM of their recompute; about the same GEMM time per GiB as the attention stash)
        n_mlp = 0
        if n == len(layers) and args.stash == "auto":
            n_mlp = int(max(0, min(len(layers), (free - n * per_layer) // per_mlp)))
            for m in layers[-n_mlp:] if n_mlp else []:
                m.mlp.stash_outputs = True
        nonlocal stashed_mlp, parked_mlp
        stashed_mlp = n_mlp
        log(f"selective recompute: {n}/{len(layers)} layers keep attention outputs, {n_mlp} keep the fc1 output "
            f"({(n * per_layer + n_mlp * per_mlp) / 2**30:.1f} GiB; reserved peak {reserved_peak() / 2**30:.1f} GiB)")
        if k_park:
            from deeperspeed_amd.runtime.activation_checkpointing import host_stash as hs
            hs.host_stash().max_backlog = args.park_backlog
            park = [m for m in layers[:k_park] if not m.mlp.stash_outputs]
            for m in park:
                m.mlp.stash_outputs = True
                m.mlp.stash_offload = True
            parked_mlp = len(park)
            log(f"selective recompute: the first {len(park)} layers park their fc1 output in pinned host memory "
                f"({len(park) * per_mlp / 2**30:.1f} GiB per micro-batch each way over PCIe, backlog "
                f"{args.park_backlog})")
        # the remaining layers park their stash in pinned host memory (copy engines over PCIe,
        # prefetched back by the recompute of the layers above): opt-in, --stash-offload -- on the
        # measured box the PCIe copies throttled the forward (profiles/aux/host_stash_ab.log)
        if args.stash_offload and n < len(layers):
            from deeperspeed_amd.runtime.activation_checkpointing import host_stash as hs
            hs.host_stash().max_backlog = 6
            for m in layers[: len(layers) - n]:
                m.attention.stash_outputs = True
                m.attention.stash_offload = True
            log(f"selective recompute: {len(layers) - n} more layers park theirs in pinned host memory "
                f"({(len(layers) - n) * per_layer / 2**30:.1f} GiB)")
        torch.cuda.reset_peak_memory_stats()
        return n

    def check_stash(n):
        """Safety check after the first step WITH the stash: if the allocator's reserved peak
        came within STASH_FLOOR_GIB of the HBM budget, give stashed layers
        back (first-stashed first) until the measured overshoot is covered, so allocator
        variance on another box cannot push a timed step into an out-of-memory error."""
        if n <= 0:
            return n
        nonlocal stashed_mlp
        layers = [m for m in engine.module.modules() if type(m).__name__ == "NeoXTransformerLayer"]
        per_layer = 4 * mb * args.seq * cfg.hidden_size * 2 + mb * cfg.num_heads * args.seq * 4
        sfloor = STASH_FLOOR_GIB * 2**30
        over = reserved_peak() - (hbm / share - sfloor)
        if over <= 0:
            return n
        if stashed_mlp:  # the MLP stashes go back first
            per_mlp = mb * args.seq * cfg.intermediate_size * 2
            drop = min(stashed_mlp, int(-(-over // per_mlp)))
            for m in layers[len(layers) - stashed_mlp: len(layers) - stashed_mlp + drop]:
                m.mlp._stash.clear()
                m.mlp.stash_outputs = False
            stashed_mlp -= drop
            over -= drop * per_mlp
            torch.cuda.empty_cache()
            log(f"stash safety: {drop} MLP stash(es) given back ({stashed_mlp} kept)")
            if over <= 0:
                return n
        drop = min(n, int(-(-over // per_layer)))
        offload = any(l.attention.stash_offload for l in layers)
        for m in layers[len(layers) - n: len(layers) - n + drop]:
            m.attention._stash.clear()
            if offload:
                m.attention.stash_offload = True  # parked in host memory instead of HBM
            else:
                m.attention.stash_outputs = False
        torch.cuda.empty_cache()
        log(f"stash safety: reserved peak {reserved_peak() / 2**30:.1f} GiB is within "
            f"{sfloor / 2**30:.1f} GiB of the budget; {drop} layer(s) back to full recompute ({n - drop} stashed)")
        return n - drop

    def refit(i):
        """Measured memory fit after warmup step i (see `fit` above).  Returns True when the
        configuration changed (one more untimed step must run with it before timing)."""
        nonlocal mb, ga
        # every rank must take the same decision (collective order): act on the most
        # constrained rank's measurement
        h = torch.tensor([limit - device_peak()], device=dev, dtype=torch.float64)
        dist.all_reduce(h, op=dist.ReduceOp.MIN)
        head = float(h.item())
        if i == 0:
            grow_margin = FIT_MARGIN_GIB * 2**30
            acts = memory_fit.grow(fit, head - grow_margin)
        else:
            acts = memory_fit.shrink(fit, -head) if head < 0 else []
        if not acts:
            return False
        measured = device_peak()
        if memory_fit.apply(engine, acts):
            mb, ga = fit.micro_batch, fit.grad_accum
            make_batches()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
        log(f"memory fit after warmup {i}: peak {measured / 2**30:.1f} GiB measured, headroom "
            f"{head / 2**30:.1f} GiB -> {acts} (live={fit.live / 1e9:.2f}B resident={fit.resident} mb={mb} ga={ga})")
        return True

    i, extra = 0, 0
    first_loss = None
    while i < args.warmup + extra:
        if os.environ.get("DSA_BENCH_STOP_RANK") == str(rank) and i == 1:
            # watchdog test hook (tests/test_bench_contract.py): this rank freezes mid-run
            import signal
            os.kill(os.getpid(), signal.SIGSTOP)
        ts = time.time()
        loss, ph = timed_step()
        if i == 0:
            first_loss = float(loss.detach())
        log(f"warmup {i} loss={float(loss.detach()):.4f} {time.time() - ts:.2f}s "
            + " ".join(f"{k}={v:.2f}s" for k, v in ph.items())
            + (f" peak={torch.cuda.max_memory_allocated() / 2**30:.1f} GiB"
               f" reserved={reserved_peak() / 2**30:.1f} GiB device={device_peak() / 2**30:.1f} GiB" if on_gpu else "")
            + (f" zero3_pool={engine.optimizer._pool.held * 2 / 2**30:.1f} GiB"
               if hasattr(engine.optimizer, "_pool") else ""))
        hb.beat(f"warmup {i} done", peak_gib=peak_gib(),
                fit=[list(x) for x in fit.actions] if fit is not None else None)
        changed = False
        if fit is not None:
            changed = refit(i)
        elif i == 0 and args.warmup >= 2:
            stashed = plan_stash()
        elif i == 1 and stashed:
            stashed = check_stash(stashed)
        if changed and i == args.warmup + extra - 1 and extra < 3:
            extra += 1  # the timed steps never run a configuration no warmup step has run
        i += 1

    dist.barrier()
    sync()
    if on_gpu:  # trace markers around the timed steps (scripts/prof_summary.py --timed)
        native.hip_ops().profile_marker(1)
    from deeperspeed_amd.utils import comm as _comm
    _comm.reset_bytes()
    t_start = time.time()
    for i in range(args.steps):
        loss = train_step()
        hb.beat(f"timed step {i} queued", peak_gib=peak_gib())  # host-side only: no sync in the loop
    sync()
    dist.barrier()
    elapsed = time.time() - t_start
    hb.beat("timed steps done", seconds=round(elapsed, 2))
    if on_gpu:
        native.hip_ops().profile_marker(2)
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    if args.profile_steps > 0:
        from torch.profiler import ProfilerActivity, profile
        stacks = True
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                     with_stack=stacks) as prof:
            for _ in range(args.profile_steps):
                train_step()
            sync()
        if rank == 0:
            os.makedirs("gpurun_out", exist_ok=True)
            with open("gpurun_out/torch_profile.txt", "w") as f:
                f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
                f.write("\n\nby input shape\n")
                f.write(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=120,
                                                                           max_name_column_width=60,
                                                                           max_shapes_column_width=120))
                if stacks:  # where the fills / copies come from (python call sites)
                    f.write("\n\nfill / zero / copy call sites\n")
                    for e in prof.key_averages(group_by_stack_n=6):
                        if any(k in e.key for k in ("fill_", "zero_", "copy_", "aten::zeros", "aten::cat", "aten::add",
                                                    "aten::add_")):
                            f.write(f"{e.key} count={e.count} device_us={e.device_time_total:.0f}\n")
                            for fr in e.stack:
                                f.write(f"    {fr}\n")

    global_batch = mb * ga * world
    tokens = global_batch * args.seq * args.steps
    tps = tokens / elapsed
    flops_tok = cfg.flops_per_token(args.seq, recompute=False)
    ms_step = elapsed / args.steps * 1000.0
    opt = engine.optimizer
    full_model = args.model == "gpt-neox-20b" and not (args.hidden or args.layers)
    zpath = None
    if args.zero == 3:
        zpath = "sharded" if (world > 1 or args.force_sharded) else "bound-single-rank"
    out = {
        "metric": ("tokens/sec (node) GPT-NeoX-20B ZeRO-3" if full_model and args.zero == 3
                   else f"tokens/sec {args.model} ZeRO-{args.zero}" + (
                       f" reshaped to {P / 1e9:.1f}B (hidden {cfg.hidden_size}, {cfg.num_layers} layers)"
                       if (args.hidden or args.layers) else ""))
                  + (f" block-sparse {args.sparse} seq{args.seq}" if args.sparse else ""),
        "value": round(tps, 2),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(tps / (REF_TOKENS_PER_GPU * world), 3) if full_model and args.zero == 3 else None,
        "dtype": "bf16",
        "data": "synthetic random tokens, random-init weights",
        "diverged": None if emulated else diverged(first_loss, float(loss.detach())),
        "config": {"model": args.model, "global_batch": global_batch, "seq_len": args.seq,
                   "parallelism": f"zero{args.zero}-dp{world}", "micro_batch": mb, "grad_accum": ga,
                   "offload": offload, "activation_checkpointing": ckpt == "on", "sparse_attention": args.sparse,
                   "attention_density": round(cfg.attention_density(args.seq), 4),
                   "params_per_gpu": round(P / world / 1e9, 3),
                   "model_tflops_per_gpu": round(tps * flops_tok / world / 1e12, 1),
                   "final_loss": round(float(loss.detach()), 4),
                   "first_warmup_loss": round(first_loss, 4) if first_loss is not None else None,
                   "peak_hbm_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1) if on_gpu else None,
                   "planned_hbm_gib": round(planned / 2**30, 1),
                   "stashed_attention_layers": stashed,
                   "stashed_mlp_layers": stashed_mlp,
                   "host_parked_mlp_layers": parked_mlp,
                   "host_stashed_attention_layers": sum(1 for m in engine.module.modules()
                                                        if getattr(m, "stash_offload", False)),
                   "zero3_path": zpath,
                   "max_live_parameters": getattr(opt, "max_live_parameters", None) if args.zero == 3 else None,
                   "resident_grads": bool(getattr(opt, "resident_grads", False)) if args.zero == 3 else None,
                   "memory_fit_actions": [list(a) for a in fit.actions] if fit is not None else None,
                   "fp32_reduce": args.fp32_reduce == "on",
                   "dist_backend": dist.get_backend(),
                   "overlap_step": bool(zcfg.get("overlap_step", False)),
                   "host_moments_params": host_numel,
                   "moment_tiers": tiers,
                   "peak_host_rss_gib": round(_peak_rss() / 2**30, 1),
                   "lt_gemm": _lt_summary() if on_gpu else None,
                   "baseline_note": "vs_baseline = value / (410 tok/s/GPU * N): BASELINE.md's derived target "
                                    "(reference's best published ZeRO-3 49 TFLOPS/GPU on V100 at 6N FLOPs/token); "
                                    "BASELINE.json publishes no number for this metric"},
    }
    if emulated:
        out = emulated_record(out, args, emulated, mb, ga, ms_step, _comm.bytes_by_kind(), flops_tok)
    if rank == 0:
        emit_result(out)
    dist.barrier()
    dist.destroy_process_group()


def emulated_record(out, args, n, mb, ga, ms_step, nbytes, flops_tok):
    """Result of --emulate-world N: the measured step of ONE rank of the N-rank job (collectives
    replaced by local stand-ins), the collective bytes that rank moves per step, and the xGMI
    rate those bytes need to hide under the step.  Ring model (runtime/comm/bucket_sizing.py): a
    ring all-gather / reduce-scatter of B bytes sends (N-1)/N * B per rank; RCCL over the 7 xGMI
    links of an MI355X is ASSUMED to sustain 300 GB/s per rank (bucket_sizing.DEFAULT_BETA_BPS,
    not measured here: one GPU cannot run a multi-rank RCCL job).  The projection is labelled as
    such: per-rank step time if the collectives overlap fully, else the modelled comm time."""
    from deeperspeed_amd.runtime.comm import bucket_sizing
    steps = max(1, args.steps)
    per = {k: v / steps for k, v in nbytes.items()}
    ag, rs = per.get("all_gather", 0.0), per.get("reduce_scatter", 0.0)
    t_step = ms_step / 1000.0
    beta = bucket_sizing.DEFAULT_BETA_BPS
    sent = (n - 1) / n * (ag + rs)
    # the reduce-scatter input doubles with --fp32-reduce on (fp32 staging of bf16 gradients)
    rs_fp32 = rs if args.fp32_reduce == "on" else 2 * rs
    sent_fp32 = (n - 1) / n * (ag + rs_fp32)
    tokens_rank = mb * ga * args.seq
    proj_step = max(t_step, sent / beta)
    proj_step_fp32 = max(t_step, sent_fp32 / beta)
    out = dict(out)
    out["metric"] = (f"EMULATED per-rank tokens/sec: rank 0 of an N={n} GPT-NeoX-20B ZeRO-3 job on one GPU "
                     f"(collectives replaced by local stand-ins; not a node measurement)")
    out["value"] = round(tokens_rank / t_step, 2)
    out["n_gpus"] = 1
    out["vs_baseline"] = None
    out["emulated_world"] = n
    cfg = dict(out["config"])
    cfg["parallelism"] = f"zero3-dp{n} (emulated rank 0)"
    cfg["model_tflops_per_gpu"] = round(tokens_rank / t_step * flops_tok / 1e12, 1)
    cfg["final_loss_note"] = "stand-in collectives: the loss is not meaningful"
    out["config"] = cfg
    gib = 2**30
    out["comm_per_rank_per_step"] = {
        "all_gather_gib": round(ag / gib, 2), "reduce_scatter_gib": round(rs / gib, 2),
        "all_reduce_mib": round(per.get("all_reduce", 0.0) / 2**20, 3),
        "ring_bytes_sent_gib": round(sent / gib, 2),
        "xgmi_gbps_needed_for_full_overlap": round(sent / t_step / 1e9, 1),
        "ring_bytes_sent_gib_fp32_reduce": round(sent_fp32 / gib, 2),
        "xgmi_gbps_needed_fp32_reduce": round(sent_fp32 / t_step / 1e9, 1),
        "assumed_xgmi_gbps_per_rank": beta / 1e9,
        "modelled_comm_s": round(sent / beta, 3), "modelled_comm_s_fp32_reduce": round(sent_fp32 / beta, 3),
    }
    out["projection"] = {
        "label": "PROJECTION, not a measurement: node tok/s = N x per-rank tokens / max(measured step, "
                 "modelled ring time at the assumed xGMI rate)",
        "node_tokens_per_s": round(n * tokens_rank / proj_step, 1),
        "node_tokens_per_s_fp32_reduce": round(n * tokens_rank / proj_step_fp32, 1),
    }
    return out


def _peak_rss():
    """Peak resident host memory of this process (bytes): pinned moments, staging, the runtime."""
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024


def _lt_summary():
    """How many GEMM problems the hipBLASLt wrapper tuned, and how many picked a solution from the
    measured table (ops/lt_tune.py) over the heuristic's candidates."""
    try:
        from deeperspeed_amd.ops import lt_tune, native
        if not lt_tune.ENABLED:
            return {"enabled": False}
        ch = native.hip_ops().lt_choices()
    except Exception as e:  # diagnostics only
        return {"error": repr(e)}
    return {"enabled": True, "problems": len(ch), "table_wins": sum(1 for c in ch if c[10]),
            "routes": {"fwd": lt_tune.FWD}}


def _optimizer_block(args):
    if args.optimizer == "adam":
        return {"type": "Adam", "params": {"lr": 1e-4, "betas": [0.9, 0.95], "eps": 1e-8, "weight_decay": 0.01}}
    if args.optimizer == "lamb":
        return {"type": "Lamb", "params": {"lr": 1e-3, "weight_decay": 0.01}}
    name = {"onebitadam": "OneBitAdam", "onebitlamb": "OneBitLamb"}[args.optimizer]
    freeze = ONEBIT_FREEZE if args.freeze_step is None else args.freeze_step
    return {"type": name, "params": {"lr": 1e-4, "betas": list(ONEBIT_BETAS), "freeze_step": freeze,
                                     "comm_backend_name": "nccl"}}


def diverged(first, last):
    import math
    return not math.isfinite(last) or (first is not None and math.isfinite(first) and last > DIVERGED_RATIO * first)


def run_pipeline(args, cfg, mb, ga, world, rank, dev, hb):
    """BASELINE config 4: GPT-NeoX/GPT-3 as a PipelineModule, PP=args.pipe x DP=world/pipe,
    1F1B schedule with `ga` micro-batches per step, p2p activations over RCCL, ZeRO-1 (Adam)
    or 1-bit Adam/LAMB on the data-parallel group."""
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.gpt_neox import to_pipeline
    from deeperspeed_amd.runtime.pipe.topology import PipeDataParallelTopology
    assert world % args.pipe == 0, f"world {world} not divisible by --pipe {args.pipe}"
    dp = world // args.pipe
    onebit = args.optimizer.startswith("onebit")
    cfg.checkpoint_activations = False  # the pipeline module checkpoints per layer itself
    torch.manual_seed(1234)
    topo = PipeDataParallelTopology(num_pp=args.pipe, num_dp=dp)
    model = to_pipeline(cfg, num_stages=None, topology=topo, activation_checkpoint_interval=1 if args.ckpt != "off" else 0)
    conf = {"train_micro_batch_size_per_gpu": mb, "gradient_accumulation_steps": ga,
            "optimizer": _optimizer_block(args), "fp16": {"enabled": True, "type": "bfloat16"},
            "fp32_allreduce": False, "gradient_clipping": 0.0 if onebit else 1.0, "steps_per_print": 1000000}
    if not onebit:
        conf["zero_optimization"] = {"stage": 1, "reduce_bucket_size": int(2e8)}
    t0 = time.time()
    engine, _, _, _ = ds.initialize(model=model, model_parameters=[p for p in model.parameters()],
                                    config_params=conf)
    log(f"pipeline PP={args.pipe} DP={dp} stage={engine.stage_id} params/stage="
        f"{sum(p.numel() for p in engine.module.parameters()) / 1e9:.2f}B optimizer={args.optimizer} "
        f"ready in {time.time() - t0:.1f}s")
    g = torch.Generator(device=dev)
    g.manual_seed(4321 + engine.grid.get_data_parallel_id())
    batches = [torch.randint(0, cfg.vocab_size, (mb, args.seq), device=dev, generator=g) for _ in range(ga)]

    def train_step():
        return engine.train_batch(iter([(b, b) for b in batches]))

    on_gpu = dev.type == "cuda"

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    hb.beat("pipeline engine ready")
    # a 1-bit run times compressed steps only: the untimed warmup runs past the freeze step
    freeze = _optimizer_block(args)["params"]["freeze_step"] if onebit else 0
    warmup = max(args.warmup, freeze + 1) if onebit else args.warmup
    if warmup != args.warmup:
        log(f"1-bit: {warmup} untimed warmup steps (freeze_step {freeze}), so the timed steps are compressed")
    first = None
    for i in range(warmup):
        ts = time.time()
        loss = train_step()
        sync()
        if first is None:
            first = float(loss)
        log(f"warmup {i} loss={float(loss):.4f} {time.time() - ts:.2f}s"
            + (f" peak={torch.cuda.max_memory_allocated() / 2**30:.1f} GiB" if on_gpu else ""))
        hb.beat(f"warmup {i} done", peak_gib=round(torch.cuda.max_memory_allocated() / 2**30, 1) if on_gpu else 0.0)
    dist.barrier()
    sync()
    timed_losses = []
    t_start = time.time()
    for i in range(args.steps):
        loss = train_step()
        timed_losses.append(loss.detach() if isinstance(loss, torch.Tensor) else loss)
        hb.beat(f"timed step {i} done")
    sync()
    dist.barrier()
    t = torch.tensor([time.time() - t_start], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    timed_losses = [round(float(l), 4) for l in timed_losses]
    global_batch = mb * ga * dp
    tps = global_batch * args.seq * args.steps / elapsed
    out = {
        "metric": f"tokens/sec {args.model} PipelineModule PP{args.pipe}xDP{dp} {args.optimizer}",
        "value": round(tps, 2), "unit": "tokens/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1000.0, 2), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic random tokens, random-init weights",
        "diverged": diverged(first, timed_losses[-1]),
        "config": {"model": args.model, "global_batch": global_batch, "seq_len": args.seq,
                   "parallelism": f"pp{args.pipe}-dp{dp}" + ("" if onebit else "-zero1"), "micro_batch": mb,
                   "grad_accum": ga, "optimizer": args.optimizer,
                   "optimizer_params": _optimizer_block(args)["params"], "warmup_steps_run": warmup,
                   "first_warmup_loss": round(first, 4) if first is not None else None,
                   "timed_losses": timed_losses,
                   "model_tflops_per_gpu": round(tps * cfg.flops_per_token(args.seq) / world / 1e12, 1),
                   "final_loss": round(float(loss.detach()), 4),
                   "dist_backend": dist.get_backend(),
                   "peak_hbm_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1) if on_gpu else None},
    }
    if rank == 0:
        emit_result(out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
