"""ZeRO-Infinity NVMe swapping (reference: deepspeed/runtime/swap_tensor/*)."""
