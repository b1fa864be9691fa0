"""The reference's own CPU compute path, for the timed CPU baseline -- TEST/BENCH
INFRASTRUCTURE ONLY.

Only tests/ and bench.py's cpu_baseline leg may import this module. The product path
(two_towers_amd/) never calls it.

oracle/cpu_ref.py restates the reference arithmetic with explicit GRU cells (a parity
checker, slow by design: a Python loop per time step). What the reference actually runs
on a CPU is PyTorch's ATen modules: nn.GRU (enhanced_two_tower.py:17-33, called :51,
:57), nn.Linear / nn.LayerNorm / nn.ReLU (:36-48), F.normalize + matmul + cross_entropy
(:72-82), F.cosine_similarity + topk (:102-133), torch.optim.Adam (train_enhanced.py:43,
:63). This module assembles exactly those third-party modules with the reference's
parameter layout (the same 44 state_dict keys), so `bench.py` can time the reference's
CPU step rather than the checker's. It is pinned to the golden vectors of the reference
run in tests/test_oracle_golden.py.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class AtenTwoTower(nn.Module):
    """EnhancedTwoTowerModel's modules and forward (enhanced_two_tower.py:13-65)."""

    def __init__(self, embedding_dim: int, hidden_dim: int):
        super().__init__()

        def gru():
            return nn.GRU(embedding_dim, 2 * hidden_dim, num_layers=2, batch_first=True, bidirectional=True,
                          dropout=0.1)

        def head():
            return nn.Sequential(nn.Linear(4 * hidden_dim, 2 * hidden_dim), nn.LayerNorm(2 * hidden_dim), nn.ReLU(),
                                 nn.Linear(2 * hidden_dim, hidden_dim))

        self.query_encoder, self.doc_encoder = gru(), gru()
        self.query_proj, self.doc_proj = head(), head()

    @staticmethod
    def _encode(enc, proj, x):
        _, hn = enc(x)
        return proj(torch.cat((hn[-2], hn[-1]), 1))

    def forward(self, q, d):
        return self._encode(self.query_encoder, self.query_proj, q), self._encode(self.doc_encoder, self.doc_proj, d)


def infonce(q, d, temperature=0.07):
    """InfoNCELoss (enhanced_two_tower.py:72-82)."""
    s = F.normalize(q, p=2, dim=1) @ F.normalize(d, p=2, dim=1).t() / temperature
    return F.cross_entropy(s, torch.arange(q.shape[0]))


def hardneg_margin(q, d, k=5, margin=0.2):
    """The config-3 composition as the reference spells it: get_hard_negatives per query
    (cosine_similarity, positive set to -1, topk; enhanced_two_tower.py:123-133), then
    MarginRankingLoss with those negatives (:102-121)."""
    with torch.no_grad():
        idx = []
        for i in range(q.shape[0]):
            sims = F.cosine_similarity(q[i].unsqueeze(0), d)
            sims[i] = -1
            idx.append(sims.topk(k).indices)
        idx = torch.stack(idx)
    neg = d[idx.reshape(-1)]
    pos = F.cosine_similarity(q, d)
    negs = F.cosine_similarity(q.unsqueeze(1).expand(-1, k, -1), neg.view(q.shape[0], k, -1), dim=2).mean(1)
    return torch.clamp(margin - pos + negs, min=0).mean()
