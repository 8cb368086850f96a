from .constants import *  # noqa: F401,F403
