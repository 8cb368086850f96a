"""Scheduling verdicts for the ragged engine (reference `inference/v2/scheduling_utils.py`)."""
from enum import Enum


class SchedulingResult(Enum):
    Success = 0
    EngineSequenceLimitExceeded = 1
    BatchSequenceLimitExceeded = 2
    BatchTokenLimitExceeded = 3
    KVCacheLimitExceeded = 4
    SequenceTokenLimitExceeded = 5


class SchedulingError(RuntimeError):

    def __init__(self, result: SchedulingResult) -> None:
        self.result = result
        super().__init__(f"Batch scheduling failed with result {result}")
