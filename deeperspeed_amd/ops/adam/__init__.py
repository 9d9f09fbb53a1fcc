from .cpu_adam import DeepSpeedCPUAdam
from .fused_adam import FusedAdam
