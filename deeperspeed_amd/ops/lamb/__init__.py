from .fused_lamb import FusedLamb
