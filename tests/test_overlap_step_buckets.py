"""runtime/overlap_step.py forward_order_buckets: parameters grouped in module-registration
(forward) order into buckets of at least `bucket_numel` elements, each parameter exactly once
(tied weights counted at their first owner), orphans last."""

import torch

from deeperspeed_amd.runtime.overlap_step import forward_order_buckets


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = torch.nn.Embedding(10, 8)           # 80
        self.l1 = torch.nn.Linear(8, 8)                # 64 + 8
        self.l2 = torch.nn.Linear(8, 8)                # 64 + 8
        self.head = torch.nn.Linear(8, 10, bias=False)
        self.head.weight = self.emb.weight            # tied (registered again under head)


def test_forward_order_buckets_cover_each_parameter_once():
    net = _Net()
    orphan = torch.nn.Parameter(torch.zeros(3))
    params = list(net.parameters()) + [orphan]
    buckets = forward_order_buckets(net, params, bucket_numel=70)

    def idx(t):
        return next(i for i, p in enumerate(params) if p is t)

    flat = [i for b in buckets for i in b]
    assert sorted(flat) == list(range(len(params)))  # every parameter once
    assert flat[0] == idx(net.emb.weight)    # forward order: the embedding first
    assert buckets[-1] == [idx(orphan)]      # not owned by the module tree: last bucket
    for b in buckets[:-2]:                            # all but the trailing ones reach the size
        assert sum(params[i].numel() for i in b) >= 70
