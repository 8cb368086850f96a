"""Exception types of the reference's `utils/exceptions.py`."""


class DeprecatedException(Exception):
    pass
