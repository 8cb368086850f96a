"""Data efficiency: curriculum learning, curriculum data sampling, random layerwise token dropping."""
from .curriculum_scheduler import CurriculumScheduler
