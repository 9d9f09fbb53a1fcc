"""Which hipBLASLt epilogues have algorithms on this build (bf16 TN GEMM at the NeoX-20B MLP shape)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deeperspeed_amd.ops import native
ops = native.hip_ops()
torch.cuda.init()
for name, code, aux in (("DEFAULT", 1, False), ("BIAS", 4, False), ("GELU", 32, False), ("GELU_BIAS", 36, False),
                        ("GELU_AUX", 160, True), ("GELU_AUX_BIAS", 164, True), ("DGELU", 192, True),
                        ("DGELU_BGRAD", 208, True), ("BGRADA", 256, False), ("BGRADB", 512, False)):
    print(name, ops.lt_algo_count(24576, 8192, 6144, code, aux), flush=True)
