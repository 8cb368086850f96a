from .autotuner import Autotuner, ResourceManager
