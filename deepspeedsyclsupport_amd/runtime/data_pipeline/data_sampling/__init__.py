from .data_sampler import DeepSpeedDataSampler
