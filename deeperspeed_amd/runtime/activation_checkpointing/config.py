"""`activation_checkpointing` config section (reference: activation_checkpointing/config.py:27-103)."""

from ..config_utils import DeepSpeedConfigObject

ACT_CHKPT = "activation_checkpointing"
ACT_CHKPT_DEFAULT = {
    "partition_activations": False,
    "number_checkpoints": None,
    "contiguous_memory_optimization": False,
    "synchronize_checkpoint_boundary": False,
    "profile": False,
    "cpu_checkpointing": False,
}


class DeepSpeedActivationCheckpointingConfig(DeepSpeedConfigObject):
    def __init__(self, param_dict):
        d = dict(ACT_CHKPT_DEFAULT)
        d.update(param_dict.get(ACT_CHKPT, {}) or {})
        self.partition_activations = d["partition_activations"]
        self.contiguous_memory_optimization = d["contiguous_memory_optimization"]
        self.cpu_checkpointing = d["cpu_checkpointing"]
        self.number_checkpoints = d["number_checkpoints"]
        self.profile = d["profile"]
        self.synchronize_checkpoint_boundary = d["synchronize_checkpoint_boundary"]
