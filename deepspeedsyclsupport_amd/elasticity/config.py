"""Elasticity config section (reference `elasticity/config.py`, `constants.py`: same keys and defaults)."""
ELASTICITY = "elasticity"
LATEST_ELASTICITY_VERSION = 0.2
MINIMUM_DEEPSPEED_VERSION = "0.3.8"
DEEPSPEED_ELASTICITY_CONFIG = "DEEPSPEED_ELASTICITY_CONFIG"


class ElasticityError(Exception):
    pass


class ElasticityConfigError(ElasticityError):
    pass


class ElasticityIncompatibleWorldSize(ElasticityError):
    pass


class ElasticityConfig:
    """{"enabled", "max_train_batch_size", "micro_batch_sizes", "min_gpus", "max_gpus", "min_time", "version",
    "prefer_larger_batch", "ignore_non_elastic_batch_info", "num_gpus_per_node", "model_parallel_size"}"""

    def __init__(self, d):
        self.enabled = d.get("enabled", False)
        if self.enabled:
            if "max_train_batch_size" not in d:
                raise ElasticityConfigError("Elasticity config missing max_train_batch_size")
            if "micro_batch_sizes" not in d:
                raise ElasticityConfigError("Elasticity config missing micro_batch_sizes")
        self.max_acceptable_batch_size = d.get("max_train_batch_size", 2000)
        self.micro_batches = d.get("micro_batch_sizes", [2, 4, 6])
        if not isinstance(self.micro_batches, list) or not all(isinstance(m, int) and m > 0
                                                               for m in self.micro_batches):
            raise ElasticityConfigError(f"micro_batch_sizes must be a list of positive ints, got {self.micro_batches}")
        self.min_gpus = d.get("min_gpus", 1)
        self.max_gpus = d.get("max_gpus", 10000)
        if self.min_gpus < 1 or self.max_gpus < 1:
            raise ElasticityConfigError("min_gpus / max_gpus must be >= 1")
        if self.max_gpus < self.min_gpus:
            raise ElasticityConfigError("max_gpus must be >= min_gpus")
        self.model_parallel_size = d.get("model_parallel_size", 1)
        self.num_gpus_per_node = d.get("num_gpus_per_node", 1)
        self.min_time = d.get("min_time", 0)
        if self.min_time < 0:
            raise ElasticityConfigError("min_time must be >= 0")
        self.version = d.get("version", LATEST_ELASTICITY_VERSION)
        self.prefer_larger_batch_size = d.get("prefer_larger_batch", True)
        self.ignore_non_elastic_batch_info = d.get("ignore_non_elastic_batch_info", False)

    def repr(self):
        return self.__dict__

    def __repr__(self):
        return str(self.__dict__)
