"""Tiny models and data helpers for engine tests (reference: tests/unit/simple_model.py)."""

import json
import os

import torch
import torch.nn as nn


class SimpleModel(nn.Module):
    def __init__(self, hidden_dim, empty_grad=False):
        super().__init__()
        self.linear = nn.Linear(hidden_dim, hidden_dim)
        self.linear2 = nn.Linear(hidden_dim, hidden_dim)
        if empty_grad:
            self.linear_unused = nn.Linear(hidden_dim, hidden_dim)
        self.cross_entropy_loss = nn.CrossEntropyLoss()

    def forward(self, x, y):
        h = self.linear2(torch.relu(self.linear(x)))
        return self.cross_entropy_loss(h.float(), y)


class LinearStack(nn.Module):
    def __init__(self, input_dim=32, hidden_dim=64, output_dim=16, num_layers=4):
        super().__init__()
        self.input_layer = nn.Linear(input_dim, hidden_dim)
        self.layers = nn.ModuleList([nn.Linear(hidden_dim, hidden_dim, bias=False) for _ in range(num_layers)])
        self.output_layer = nn.Linear(hidden_dim, output_dim)
        self.loss_fn = nn.CrossEntropyLoss()

    def forward(self, x, y):
        x = self.input_layer(x)
        for layer in self.layers:
            x = torch.relu(layer(x))
        return self.loss_fn(self.output_layer(x).float(), y)


def random_batches(n, batch, hidden_dim, seed=0, dtype=torch.float32, classes=None):
    g = torch.Generator()
    g.manual_seed(seed)
    classes = classes or hidden_dim
    return [(torch.randn(batch, hidden_dim, generator=g).to(dtype), torch.randint(0, classes, (batch,), generator=g))
            for _ in range(n)]


def base_config(stage=0, dtype="bfloat16", mb=2, ga=1, opt="Adam", lr=1e-2, **zero):
    cfg = {"train_micro_batch_size_per_gpu": mb, "gradient_accumulation_steps": ga,
           "optimizer": {"type": opt, "params": {"lr": lr}}, "steps_per_print": 1000}
    if dtype is not None:
        cfg["fp16"] = {"enabled": True, "type": dtype}
        if dtype == "bfloat16":
            cfg["fp32_allreduce"] = False
    if stage:
        z = {"stage": stage}
        z.update(zero)
        cfg["zero_optimization"] = z
    return cfg


def args_from_dict(tmpdir, config_dict):
    path = os.path.join(str(tmpdir), "ds_config.json")
    with open(path, "w") as f:
        json.dump(config_dict, f)

    class Args:
        pass

    a = Args()
    a.deepspeed = True
    a.deepspeed_config = path
    a.local_rank = 0
    return a
