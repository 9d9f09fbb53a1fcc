"""Import path of the reference (deepspeed/runtime/pipe/topology.py); the implementation
lives in deeperspeed_amd/parallel/topology.py."""

from ...parallel.topology import *  # noqa: F401,F403
from ...parallel.topology import (PipeDataParallelTopology, PipelineParallelGrid, PipeModelDataParallelTopology,
                                  ProcessTopology)
