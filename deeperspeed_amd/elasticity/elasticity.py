"""Elastic batch-size planning (reference parity: deepspeed/elasticity/elasticity.py:19-334).

Given a set of acceptable micro-batch sizes and a maximum global batch, choose the global
batch that is divisible by the largest number of GPU counts in [min_gpus, max_gpus], so a
job can be rescheduled on any of those counts without changing convergence (only the
gradient-accumulation factor changes).
"""

import json
import math
import os
import re
from functools import reduce

from ..utils.logging import logger
from ..version import __version__
from .config import (ElasticityConfig, ElasticityConfigError, ElasticityError, ElasticityIncompatibleWorldSize)
from .constants import (DEEPSPEED_ELASTICITY_CONFIG, ELASTICITY, ENABLED, ENABLED_DEFAULT, LATEST_ELASTICITY_VERSION,
                        MINIMUM_DEEPSPEED_VERSION)


# Thirty-eight smallest highly composite numbers (supports batch sizes up to ~720K).
HCN_LIST = [1, 2, 4, 6, 12, 24, 36, 48, 60, 120, 180, 240, 360, 720, 840, 1260, 1680, 2520, 5040, 7560, 10080,
            15120, 20160, 25200, 27720, 45360, 50400, 55440, 83160, 110880, 166320, 221760, 277200, 332640,
            498960, 554400, 665280, 720720]


def get_candidate_batch_sizes(base_list, max_acceptable_batch_size):
    """For each base, the largest base*HCN not exceeding the cap (deduplicated)."""
    cands = set()
    for base in base_list:
        best = base
        for h in HCN_LIST:
            if base * h > max_acceptable_batch_size:
                break
            best = base * h
        cands.add(best)
    return list(cands)


def get_valid_gpus(batch_size, micro_batches, min_valid_gpus, max_valid_gpus):
    """GPU counts g in range such that batch_size = mb * gas * g for some listed mb."""
    valid = set()
    for mb in micro_batches:
        if batch_size % mb:
            continue
        max_g = batch_size // mb
        for g in [max_g] + [i for i in range(1, max_g // 2 + 1) if max_g % i == 0]:
            if min_valid_gpus <= g <= max_valid_gpus:
                valid.add(g)
    return sorted(valid)


def get_best_candidates(candidate_batch_sizes, micro_batches, min_gpus, max_gpus, prefer_larger):
    best_count, best_gpus = 0, None
    best_bs = int(min(micro_batches))
    for bs in candidate_batch_sizes:
        gpus = get_valid_gpus(bs, micro_batches, min_gpus, max_gpus)
        better_tie = (prefer_larger and bs > best_bs) or (not prefer_larger and bs < best_bs)
        if len(gpus) > best_count or (len(gpus) == best_count and better_tie):
            best_count, best_gpus, best_bs = len(gpus), gpus, bs
    return best_bs, best_gpus


def _get_compatible_gpus_v01(micro_batches, max_acceptable_batch_size, min_gpus=None, max_gpus=None,
                             prefer_larger=True):
    min_gpus = 1 if min_gpus is None else min_gpus
    if max_gpus is None:
        max_gpus = int(max_acceptable_batch_size / min(micro_batches))
    assert all(mb <= max_acceptable_batch_size for mb in micro_batches), \
        f"All micro batches must be <= max_acceptable_batch_size: {max_acceptable_batch_size}"
    lcm = reduce(lambda a, b: a * b // math.gcd(a, b), micro_batches)
    bases = list(micro_batches) + [lcm]
    cands = get_candidate_batch_sizes(bases, max_acceptable_batch_size)
    return get_best_candidates(cands, micro_batches, min_gpus, max_gpus, prefer_larger)


def _parse_version(version_str):
    m = re.search(r"^(\d+)\.(\d+)(?:\.(\d+))?", version_str)
    assert m is not None, f"expected major.minor[.patch] version, got {version_str}"
    return int(m.group(1)), int(m.group(2)), int(m.group(3) or 0)


def _compatible_ds_version_check(target_deepspeed_version: str):
    if _parse_version(target_deepspeed_version) < _parse_version(MINIMUM_DEEPSPEED_VERSION):
        raise ElasticityError(f"Target deepspeed version of {target_deepspeed_version} is not compatible with "
                              f"minimum version {MINIMUM_DEEPSPEED_VERSION} supporting elasticity.")
    return True


def elasticity_enabled(ds_config: dict):
    return bool(ds_config.get(ELASTICITY, {}).get(ENABLED, ENABLED_DEFAULT)) if ELASTICITY in ds_config else False


def ensure_immutable_elastic_config(runtime_elastic_config_dict: dict):
    """The scheduler-seen config (env DEEPSPEED_ELASTICITY_CONFIG) must match the runtime one."""
    if DEEPSPEED_ELASTICITY_CONFIG not in os.environ:
        logger.warning("Unable to find DEEPSPEED_ELASTICITY_CONFIG environment variable, cannot guarantee "
                       "resource scheduler will scale this job using compatible GPU counts.")
        return
    sched = ElasticityConfig(json.loads(os.environ[DEEPSPEED_ELASTICITY_CONFIG]))
    run = ElasticityConfig(runtime_elastic_config_dict)
    for attr in ("max_acceptable_batch_size", "micro_batches", "version"):
        if getattr(run, attr) != getattr(sched, attr):
            raise ElasticityConfigError(f"Elastic config '{attr}={getattr(sched, attr)}' seen by resource scheduler "
                                        f"does not match config passed to runtime {attr}={getattr(run, attr)}")


def compute_elastic_config(ds_config: dict, target_deepspeed_version: str, world_size=0):
    """Return (final_batch_size, valid_gpus[, micro_batch_size if world_size > 0])."""
    if not isinstance(ds_config, dict):
        raise ValueError(f"Expected ds_config to be a dictionary but received a {type(ds_config)}")
    if ELASTICITY not in ds_config:
        raise ElasticityConfigError(f"'{ELASTICITY}' is missing from config json, please add it if running an "
                                    "elastic training job.")
    ecd = ds_config[ELASTICITY]
    if not ecd.get(ENABLED, ENABLED_DEFAULT):
        raise ElasticityConfigError("Elasticity is disabled, please enable it ('enabled':true) if running an "
                                    "elastic training job.")
    ec = ElasticityConfig(ecd)
    if float(ec.version) > LATEST_ELASTICITY_VERSION:
        raise ElasticityConfigError(f"Attempting to run elasticity version {ec.version} but runtime only supports "
                                    f"up to {LATEST_ELASTICITY_VERSION}")
    if not _compatible_ds_version_check(target_deepspeed_version):
        raise ElasticityError(f"Unable to run elasticity on target deepspeed version of {target_deepspeed_version}")
    if float(ec.version) != 0.1:
        raise NotImplementedError(f"Unable to find elastic logic for version: {ec.version}")
    final_bs, valid_gpus = _get_compatible_gpus_v01(ec.micro_batches, ec.max_acceptable_batch_size, ec.min_gpus,
                                                    ec.max_gpus, ec.prefer_larger_batch_size)
    final_bs = int(final_bs)
    if world_size > 0:
        if world_size not in valid_gpus:
            raise ElasticityIncompatibleWorldSize(f"World size ({world_size}) is not valid with the current list of "
                                                  f"valid GPU counts: {valid_gpus}")
        mbs = None
        for mb in sorted(set(ec.micro_batches), reverse=True):
            if (final_bs // world_size) % mb == 0:
                mbs = mb
                break
        assert mbs is not None, (f"Unable to find divisible micro batch size world_size={world_size}, "
                                 f"final_batch_size={final_bs}, micro_batches={ec.micro_batches}.")
        return final_bs, valid_gpus, mbs
    return final_bs, valid_gpus
