"""`deeperspeed_amd.pipe` (reference: deepspeed/pipe/__init__.py)."""

from ..parallel.topology import ProcessTopology
from ..runtime.pipe.module import LayerSpec, PipelineModule, TiedLayerSpec
