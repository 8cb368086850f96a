from .cpu_adagrad import DeepSpeedCPUAdagrad  # noqa: F401
