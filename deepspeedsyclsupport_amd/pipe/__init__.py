"""`deepspeed.pipe` import path parity."""
from ..runtime.pipe import LayerSpec, PipelineModule, TiedLayerSpec  # noqa: F401
from ..runtime.pipe.topology import ProcessTopology  # noqa: F401
