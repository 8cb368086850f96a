"""Logger of the ragged inference engine (reference `inference/v2/logging.py`)."""
import logging

from ...utils.logging import LoggerFactory

inf_logger = None


def inference_logger(level: int = logging.INFO) -> logging.Logger:
    global inf_logger
    if inf_logger is None:
        inf_logger = LoggerFactory.create_logger(name="DS-Inference", level=level)
        inf_logger.debug("Inference logger created.")
    return inf_logger
