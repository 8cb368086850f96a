"""Reference `elasticity/utils.py`."""


def is_torch_elastic_compatible():
    """torch.distributed.elastic (the agent `DSElasticAgent` builds on) needs torch >= 1.11."""
    import torch
    major, minor = (int(x) for x in torch.__version__.split(".")[:2])
    return (major, minor) >= (1, 11)
