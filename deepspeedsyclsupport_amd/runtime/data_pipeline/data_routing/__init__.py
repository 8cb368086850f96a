from .basic_layer import RandomLayerTokenDrop
from .scheduler import RandomLTDScheduler
