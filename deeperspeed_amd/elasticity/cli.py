"""`ds_elastic` entry point (reference bin/ds_elastic): print the elastic batch configuration
of a DeepSpeed JSON config, optionally for one world size."""

import argparse
import json

from ..version import __version__
from .elasticity import compute_elastic_config


def main(argv=None):
    p = argparse.ArgumentParser(prog="ds_elastic")
    p.add_argument("-c", "--config", type=str, required=True, help="DeepSpeed config json")
    p.add_argument("-w", "--world-size", type=int, default=0, help="Intended/current world size")
    a = p.parse_args(argv)
    with open(a.config) as f:
        cfg = json.load(f)
    print("-" * 50)
    print("Elastic config:", json.dumps(cfg.get("elasticity", {}), indent=2))
    if a.world_size > 0:
        bs, gpus, mbs = compute_elastic_config(cfg, __version__, world_size=a.world_size)
        print(f"final_batch_size .... {bs}\nvalid_gpus .......... {gpus}\nmicro_batch_size .... {mbs}")
    else:
        bs, gpus = compute_elastic_config(cfg, __version__)
        print(f"final_batch_size .... {bs}\nvalid_gpus .......... {gpus}")


if __name__ == "__main__":
    main()
