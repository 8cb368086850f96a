from .base_tuner import BaseTuner  # noqa: F401
from .index_based_tuner import GridSearchTuner, RandomTuner  # noqa: F401
from .model_based_tuner import ModelBasedTuner  # noqa: F401
