"""`ds_elastic`: print the elastic batch / GPU-count plan of a config (reference `bin/ds_elastic`)."""
import argparse
import json

from .elasticity import compute_elastic_config


def main(argv=None):
    p = argparse.ArgumentParser(prog="ds_elastic")
    p.add_argument("-c", "--config", required=True, help="DeepSpeed config json")
    p.add_argument("-w", "--world-size", type=int, default=0, help="intended / current world size")
    args = p.parse_args(argv)
    with open(args.config) as f:
        ds_config = json.load(f)
    from .. import __version__
    bar = "-" * 42
    print(f"{bar}\nElasticity config:\n{bar}")
    print(json.dumps(ds_config.get("elasticity", {}), indent=4, sort_keys=True))
    if args.world_size > 0:
        bs, gpus, mb = compute_elastic_config(ds_config, __version__, world_size=args.world_size,
                                              return_microbatch=True)
        print(f"{bar}\nCalculated results for world size {args.world_size}:\n{bar}")
        print(f"final_batch_size .... {bs}\nvalid_gpus .......... {gpus}\nmicro_batch_size .... {mb}")
    else:
        bs, gpus = compute_elastic_config(ds_config, __version__)
        print(f"{bar}\nCalculated results:\n{bar}")
        print(f"final_batch_size .... {bs}\nvalid_gpus .......... {gpus}")
    return 0
