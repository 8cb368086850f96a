from .module import PipelineModule, LayerSpec, TiedLayerSpec  # noqa: F401
from .topology import ProcessTopology, PipeDataParallelTopology, PipeModelDataParallelTopology  # noqa: F401
