"""`ds_report`: environment + native-op compatibility report (reference parity:
deepspeed/env_report.py:1-109), for the ROCm / MI355X stack."""

import os
import shutil
import subprocess

GREEN, RED, YELLOW, END = "\033[92m", "\033[91m", "\033[93m", "\033[0m"
OKAY, WARNING, FAIL = f"{GREEN}[OKAY]{END}", f"{YELLOW}[WARNING]{END}", f"{RED}[FAIL]{END}"
INFO = "[INFO]"


def _cmd(args):
    try:
        return subprocess.check_output(args, stderr=subprocess.DEVNULL, timeout=20).decode().strip()
    except Exception:
        return None


def op_report():
    from .ops import builder
    rows = [("op name", "built", "compatible")]
    for name, spec in builder._ext_specs().items():
        built = builder.is_built(name)
        tool = "hipcc" if spec["kind"] == "hip" else "g++"
        compatible = shutil.which(os.path.join(builder.ROCM, "bin", "hipcc")) is not None if tool == "hipcc" \
            else shutil.which("g++") is not None
        rows.append((name, OKAY if built else f"{YELLOW}[NO]{END}", OKAY if compatible else FAIL))
    print("-" * 50)
    print("deeperspeed_amd native op report (in-tree, gfx950)")
    print("-" * 50)
    for r in rows:
        print(f"{r[0]:<20} {r[1]:<22} {r[2]}")
    print("-" * 50)
    from .ops.builder import ALL_OPS
    print("op builders: " + ", ".join(sorted(ALL_OPS)))


def debug_report():
    import torch
    from .version import __version__
    hip = getattr(torch.version, "hip", None)
    rows = [("torch install path", os.path.dirname(torch.__file__)), ("torch version", torch.__version__),
            ("torch hip version", hip), ("rocm path", os.environ.get("ROCM_PATH", "/opt/rocm")),
            ("hipcc version", (_cmd(["/opt/rocm/bin/hipcc", "--version"]) or "n/a").splitlines()[-1]),
            ("deeperspeed_amd install path", os.path.dirname(os.path.abspath(__file__))),
            ("deeperspeed_amd version", __version__),
            ("visible GPUs (device_count)", torch.cuda.device_count()),
            ("rccl (nccl backend) available", torch.distributed.is_nccl_available())]
    print("DeepSpeed general environment info:")
    for k, v in rows:
        print(f"{k + ' ':.<40} {v}")


def main():
    op_report()
    debug_report()


if __name__ == "__main__":
    main()
