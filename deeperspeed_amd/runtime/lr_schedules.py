"""Learning-rate schedules selectable by name in the config.

Reference parity: deepspeed/runtime/lr_schedules.py (LRRangeTest :301, OneCycle :408,
WarmupLR :677 with logarithmic warm-up, WarmupDecayLR :761, CLI tuning arguments and
`get_config_from_args`).  All schedules share one small base class here; each only
defines its per-iteration learning-rate (and momentum) curve.
"""

import argparse
import math

from torch.optim import Optimizer

from ..utils.logging import logger

LR_SCHEDULE = "lr_schedule"
LR_RANGE_TEST = "LRRangeTest"
ONE_CYCLE = "OneCycle"
WARMUP_LR = "WarmupLR"
WARMUP_DECAY_LR = "WarmupDecayLR"
VALID_LR_SCHEDULES = [LR_RANGE_TEST, ONE_CYCLE, WARMUP_LR, WARMUP_DECAY_LR]

LR_RANGE_TEST_MIN_LR = "lr_range_test_min_lr"
LR_RANGE_TEST_STEP_RATE = "lr_range_test_step_rate"
LR_RANGE_TEST_STEP_SIZE = "lr_range_test_step_size"
LR_RANGE_TEST_STAIRCASE = "lr_range_test_staircase"
EDGE_VALUE = "edge_value"
MID_VALUE = "mid_value"
CYCLE_FIRST_STEP_SIZE = "cycle_first_step_size"
CYCLE_FIRST_STAIR_COUNT = "cycle_first_stair_count"
CYCLE_SECOND_STEP_SIZE = "cycle_second_step_size"
CYCLE_SECOND_STAIR_COUNT = "cycle_second_stair_count"
DECAY_STEP_SIZE = "decay_step_size"
CYCLE_MIN_LR = "cycle_min_lr"
CYCLE_MAX_LR = "cycle_max_lr"
DECAY_LR_RATE = "decay_lr_rate"
CYCLE_MIN_MOM = "cycle_min_mom"
CYCLE_MAX_MOM = "cycle_max_mom"
DECAY_MOM_RATE = "decay_mom_rate"
WARMUP_MIN_LR = "warmup_min_lr"
WARMUP_MAX_LR = "warmup_max_lr"
WARMUP_NUM_STEPS = "warmup_num_steps"
TOTAL_NUM_STEPS = "total_num_steps"


def add_tuning_arguments(parser):
    g = parser.add_argument_group("Convergence Tuning", "Convergence tuning configurations")
    g.add_argument("--lr_schedule", type=str, default=None, help="LR schedule for training.")
    g.add_argument("--lr_range_test_min_lr", type=float, default=0.001, help="Starting lr value.")
    g.add_argument("--lr_range_test_step_rate", type=float, default=1.0, help="scaling rate for LR range test.")
    g.add_argument("--lr_range_test_step_size", type=int, default=1000, help="training steps per LR change.")
    g.add_argument("--lr_range_test_staircase", type=bool, default=False, help="use staircase scaling for LR range test.")
    g.add_argument("--cycle_first_step_size", type=int, default=1000, help="size of first step of 1Cycle schedule.")
    g.add_argument("--cycle_first_stair_count", type=int, default=-1, help="first stair count for 1Cycle schedule.")
    g.add_argument("--cycle_second_step_size", type=int, default=-1, help="size of second step of 1Cycle schedule.")
    g.add_argument("--cycle_second_stair_count", type=int, default=-1, help="second stair count for 1Cycle schedule.")
    g.add_argument("--decay_step_size", type=int, default=1000, help="size of intervals for applying post cycle decay.")
    g.add_argument("--cycle_min_lr", type=float, default=0.01, help="1Cycle LR lower bound.")
    g.add_argument("--cycle_max_lr", type=float, default=0.1, help="1Cycle LR upper bound.")
    g.add_argument("--decay_lr_rate", type=float, default=0.0, help="post cycle LR decay rate.")
    g.add_argument("--cycle_momentum", default=False, action="store_true", help="Enable 1Cycle momentum schedule.")
    g.add_argument("--cycle_min_mom", type=float, default=0.8, help="1Cycle momentum lower bound.")
    g.add_argument("--cycle_max_mom", type=float, default=0.9, help="1Cycle momentum upper bound.")
    g.add_argument("--decay_mom_rate", type=float, default=0.0, help="post cycle momentum decay rate.")
    g.add_argument("--warmup_min_lr", type=float, default=0, help="WarmupLR minimum/initial LR value")
    g.add_argument("--warmup_max_lr", type=float, default=0.001, help="WarmupLR maximum LR value.")
    g.add_argument("--warmup_num_steps", type=int, default=1000, help="WarmupLR step count for LR warmup.")
    return parser


def parse_arguments():
    parser = argparse.ArgumentParser()
    parser = add_tuning_arguments(parser)
    lr_sched_args, unknown_args = parser.parse_known_args()
    return lr_sched_args, unknown_args


_ARG_GROUPS = {
    LR_RANGE_TEST: [LR_RANGE_TEST_MIN_LR, LR_RANGE_TEST_STEP_RATE, LR_RANGE_TEST_STEP_SIZE, LR_RANGE_TEST_STAIRCASE],
    ONE_CYCLE: [CYCLE_FIRST_STEP_SIZE, CYCLE_FIRST_STAIR_COUNT, CYCLE_SECOND_STEP_SIZE, CYCLE_SECOND_STAIR_COUNT,
                DECAY_STEP_SIZE, CYCLE_MIN_LR, CYCLE_MAX_LR, DECAY_LR_RATE, CYCLE_MIN_MOM, CYCLE_MAX_MOM,
                DECAY_MOM_RATE],
    WARMUP_LR: [WARMUP_MIN_LR, WARMUP_MAX_LR, WARMUP_NUM_STEPS],
}


def override_params(args, params):
    for keys in _ARG_GROUPS.values():
        for k in keys:
            if hasattr(args, k) and getattr(args, k) is not None:
                params[k] = getattr(args, k)


def get_config_from_args(args):
    if not hasattr(args, LR_SCHEDULE) or args.lr_schedule is None:
        return None, "--{} not specified on command line".format(LR_SCHEDULE)
    if args.lr_schedule not in VALID_LR_SCHEDULES:
        return None, "{} is not supported LR schedule".format(args.lr_schedule)
    config = {"type": args.lr_schedule, "params": {}}
    keys = _ARG_GROUPS.get(args.lr_schedule, _ARG_GROUPS[WARMUP_LR])
    for k in keys:
        if hasattr(args, k) and getattr(args, k) is not None:
            config["params"][k] = getattr(args, k)
    return config, None


def get_lr_from_config(config):
    if "type" not in config:
        return None, "LR schedule type not defined in config"
    if "params" not in config:
        return None, "LR schedule params not defined in config"
    lr_schedule, lr_params = config["type"], config["params"]
    if lr_schedule not in VALID_LR_SCHEDULES:
        return None, "{} is not a valid LR schedule".format(lr_schedule)
    if lr_schedule == LR_RANGE_TEST:
        return lr_params[LR_RANGE_TEST_MIN_LR], ""
    if lr_schedule == ONE_CYCLE:
        return lr_params[CYCLE_MAX_LR], ""
    return lr_params[WARMUP_MAX_LR], ""


def get_torch_optimizer(optimizer):
    """Unwrap DeepSpeed optimizer wrappers to the torch.optim.Optimizer holding param_groups."""
    if isinstance(optimizer, Optimizer):
        return optimizer
    if hasattr(optimizer, "optimizer") and isinstance(optimizer.optimizer, Optimizer):
        return optimizer.optimizer
    if hasattr(optimizer, "param_groups"):
        return optimizer
    raise TypeError("{} is not a subclass of torch.optim.Optimizer".format(type(optimizer).__name__))


def _per_group(optimizer, value, name):
    n = len(optimizer.param_groups)
    if isinstance(value, (list, tuple)):
        if len(value) != n:
            raise ValueError(f"expected {n} value for {name}, got {value}")
        return list(value)
    return [value] * n


class _IterSchedule:
    """Base: per-batch schedule driven by `last_batch_iteration`."""

    def __init__(self, optimizer, last_batch_iteration=-1):
        self.optimizer = get_torch_optimizer(optimizer)
        self.last_batch_iteration = last_batch_iteration

    def get_lr(self):
        raise NotImplementedError

    def get_mom(self):
        return None

    def get_last_lr(self):
        assert getattr(self, "_last_lr", None) is not None, "need to call step() first"
        return self._last_lr

    def _apply(self, lrs, moms=None):
        for g, lr in zip(self.optimizer.param_groups, lrs):
            g["lr"] = lr
        if moms is not None:
            for g, m in zip(self.optimizer.param_groups, moms):
                g["betas"] = m
        self._last_lr = [g["lr"] for g in self.optimizer.param_groups]

    def step(self, batch_iteration=None):
        self.last_batch_iteration = self.last_batch_iteration + 1 if batch_iteration is None else batch_iteration
        self._apply(self.get_lr(), self.get_mom())

    def state_dict(self):
        return {"last_batch_iteration": self.last_batch_iteration}

    def load_state_dict(self, sd):
        self.last_batch_iteration = sd["last_batch_iteration"]


class LRRangeTest(_IterSchedule):
    """lr = min_lr * (1 + step_rate * interval), interval = (it+1)/step_size (floored if staircase)."""

    def __init__(self, optimizer, lr_range_test_min_lr=1e-3, lr_range_test_step_size=2000,
                 lr_range_test_step_rate=1.0, lr_range_test_staircase=False, last_batch_iteration=-1):
        super().__init__(optimizer, last_batch_iteration)
        self.min_lr = _per_group(self.optimizer, lr_range_test_min_lr, "lr_range_test_min_lr")
        self.step_size = lr_range_test_step_size
        self.step_rate = lr_range_test_step_rate
        self.staircase = lr_range_test_staircase
        if last_batch_iteration == -1:
            self._apply(self.min_lr)

    def _interval(self):
        x = float(self.last_batch_iteration + 1) / self.step_size
        return math.floor(x) if self.staircase else x

    def get_lr(self):
        inc = 1 + self.step_rate * self._interval()
        return [m * inc for m in self.min_lr]


class OneCycle(_IterSchedule):
    """Triangular cycle min->max->min over (first + second) steps, then decay."""

    def __init__(self, optimizer, cycle_min_lr, cycle_max_lr, decay_lr_rate=0.0, cycle_first_step_size=2000,
                 cycle_second_step_size=None, cycle_first_stair_count=0, cycle_second_stair_count=None,
                 decay_step_size=0, cycle_momentum=True, cycle_min_mom=0.8, cycle_max_mom=0.9, decay_mom_rate=0.0,
                 last_batch_iteration=-1):
        super().__init__(optimizer, last_batch_iteration)
        first = float(cycle_first_step_size)
        second = float(cycle_second_step_size) if cycle_second_step_size is not None else first
        self.total_size = first + second
        self.step_ratio = first / self.total_size
        self.first_stair_count = cycle_first_stair_count
        self.second_stair_count = cycle_first_stair_count if cycle_second_stair_count is None \
            else cycle_second_stair_count
        self.decay_step_size = decay_step_size
        n = len(self.optimizer.param_groups)
        self.min_lrs = [cycle_min_lr] * n
        self.max_lrs = [cycle_max_lr] * n
        self.decay_lr_rate = decay_lr_rate
        if last_batch_iteration == -1:
            for lr, g in zip(self.min_lrs, self.optimizer.param_groups):
                g["lr"] = lr
        self.cycle_momentum = cycle_momentum
        if cycle_momentum:
            if "betas" not in self.optimizer.defaults:
                logger.warning(f"cycle_momentum is disabled because optimizer {type(self.optimizer).__name__} "
                               "does not support momentum, no betas attribute in defaults")
                self.cycle_momentum = False
            else:
                self.decay_mom_rate = decay_mom_rate
                self.min_moms = [(cycle_min_mom, 0.99)] * n
                self.max_moms = [(cycle_max_mom, 0.99)] * n
                if last_batch_iteration == -1:
                    for m, g in zip(self.min_moms, self.optimizer.param_groups):
                        g["betas"] = m

    def _scale(self):
        it = self.last_batch_iteration + 1
        cycle = math.floor(1 + it / self.total_size)
        x = 1.0 + it / self.total_size - cycle
        return x / self.step_ratio if x <= self.step_ratio else (x - 1) / (self.step_ratio - 1)

    def get_lr(self):
        if self.last_batch_iteration < self.total_size:
            s = self._scale()
            return [lo + (hi - lo) * s for lo, hi in zip(self.min_lrs, self.max_lrs)]
        it = self.last_batch_iteration - self.total_size + 1
        factor = 1 + self.decay_lr_rate * (it / self.decay_step_size)
        return [lo / factor for lo in self.min_lrs]

    def get_mom(self):
        if not self.cycle_momentum:
            return None
        if self.last_batch_iteration < self.total_size:
            s = self._scale()
            return [(hi[0] - (hi[0] - lo[0]) * s, lo[1]) for lo, hi in zip(self.min_moms, self.max_moms)]
        it = self.last_batch_iteration - self.total_size + 1
        factor = 1 + self.decay_mom_rate * (it / self.decay_step_size)
        return [(b0 * factor, b1) for b0, b1 in self.max_moms]


class WarmupLR(_IterSchedule):
    """Logarithmic warm-up from min_lr to max_lr over warmup_num_steps, then constant."""

    def __init__(self, optimizer, warmup_min_lr=0.0, warmup_max_lr=0.001, warmup_num_steps=1000,
                 last_batch_iteration=-1):
        super().__init__(optimizer, last_batch_iteration)
        self.min_lrs = _per_group(self.optimizer, warmup_min_lr, "min_lr")
        self.max_lrs = _per_group(self.optimizer, warmup_max_lr, "max_lr")
        self.delta_lrs = [hi - lo for hi, lo in zip(self.max_lrs, self.min_lrs)]
        self.warmup_num_steps = max(2, warmup_num_steps)
        self.inverse_log_warm_up = 1.0 / math.log(self.warmup_num_steps)

    def _get_gamma(self):
        if self.last_batch_iteration < self.warmup_num_steps:
            return self.inverse_log_warm_up * math.log(self.last_batch_iteration + 1)
        return 1.0

    def get_lr(self):
        if self.last_batch_iteration < 0:
            logger.warning("Attempting to get learning rate from scheduler before it has started")
            return [0.0]
        gamma = self._get_gamma()
        return [lo + d * gamma for lo, d in zip(self.min_lrs, self.delta_lrs)]


class WarmupDecayLR(WarmupLR):
    """WarmupLR followed by linear decay to 0 at total_num_steps."""

    def __init__(self, optimizer, total_num_steps, warmup_min_lr=0.0, warmup_max_lr=0.001, warmup_num_steps=1000,
                 last_batch_iteration=-1):
        self.total_num_steps = total_num_steps
        super().__init__(optimizer, warmup_min_lr, warmup_max_lr, warmup_num_steps, last_batch_iteration)
        if self.total_num_steps < self.warmup_num_steps:
            logger.warning(f"total_num_steps {total_num_steps} is less than warmup_num_steps {warmup_num_steps}")

    def _get_gamma(self):
        if self.last_batch_iteration < self.warmup_num_steps:
            return self.inverse_log_warm_up * math.log(self.last_batch_iteration + 1)
        return max(0.0, float(self.total_num_steps - self.last_batch_iteration) /
                   float(max(1.0, self.total_num_steps - self.warmup_num_steps)))
