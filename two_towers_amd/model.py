"""EnhancedTwoTowerModel on the MI355X HIP path.

Mirrors enhanced_two_tower.py:13-65: same constructor, same submodule names
(query_encoder / doc_encoder are nn.GRU parameter holders, query_proj / doc_proj are
the nn.Sequential heads), hence the same 44 state_dict keys and the same default
initialisation for a given torch seed. forward / encode_* run the fused tower kernels
(two_towers_amd/towers.py) instead of nn.GRU / nn.Linear.

Extensions over the reference surface (all opt-in):
  - inputs may be [B, T] int token ids when an embedding table is attached
    (set_embedding_table): the Word2Vec gather then runs on the GPU;
  - set_compute_dtype(torch.bfloat16) selects bf16 storage with fp32 accumulation.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import dist, ops
from .towers import TowerCfg, run_towers


class EnhancedTwoTowerModel(nn.Module):
    def __init__(self, embedding_dim: int, hidden_dim: int):
        super().__init__()
        self.query_encoder = nn.GRU(input_size=embedding_dim, hidden_size=hidden_dim * 2, num_layers=2,
                                    batch_first=True, bidirectional=True, dropout=0.1)
        self.doc_encoder = nn.GRU(input_size=embedding_dim, hidden_size=hidden_dim * 2, num_layers=2,
                                  batch_first=True, bidirectional=True, dropout=0.1)
        self.query_proj = nn.Sequential(nn.Linear(hidden_dim * 4, hidden_dim * 2), nn.LayerNorm(hidden_dim * 2),
                                        nn.ReLU(), nn.Linear(hidden_dim * 2, hidden_dim))
        self.doc_proj = nn.Sequential(nn.Linear(hidden_dim * 4, hidden_dim * 2), nn.LayerNorm(hidden_dim * 2),
                                      nn.ReLU(), nn.Linear(hidden_dim * 2, hidden_dim))
        self.embedding_dim = embedding_dim
        self.hidden_dim = hidden_dim
        self.compute_dtype = torch.float32
        self.process_group = None  # data-parallel group (None: the default group when initialised)
        self.overlap_grad_allreduce = False  # DP: sum gradients inside the backward (opt-in)
        self._table = None  # not a parameter/buffer: keeps state_dict identical to the reference

    # ---------------------------------------------------------------- options
    def set_compute_dtype(self, dtype: torch.dtype):
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("compute dtype must be torch.float32 or torch.bfloat16")
        self.compute_dtype = dtype
        return self

    def set_process_group(self, group, overlap_grad_allreduce: bool = False):
        """Data-parallel group the batch is split over. The dropout masks depend on it:
        rank r's rows draw the masks of global rows r*B .. r*B+B-1, as one process running
        the whole global batch would (so the ranks never repeat each other's masks).

        overlap_grad_allreduce (opt-in): the backward sums the gradients across the group
        itself, the head + layer-1 bucket overlapping the layer-0 BPTT
        (dist.OverlapReducer), and dist.allreduce_grads then skips them. The backward then
        contains collectives, so every rank must run it, and no other reducer (DDP, a
        manual all_reduce) may sum the same gradients again. Off, the gradients stay
        per-rank and dist.allreduce_grads (or DDP) sums them after the backward."""
        self.process_group = group
        self.overlap_grad_allreduce = overlap_grad_allreduce
        return self

    def set_embedding_table(self, table: torch.Tensor | None):
        """Attach a device Word2Vec table [V, E] (any float dtype); token-id inputs then
        gather rows on the GPU. Stored padded in the compute dtype (built on first use;
        the source tensor may be dropped after that)."""
        if table is None:
            self._table = None
            self._table_src = None
            return self
        if table.dim() != 2 or table.shape[1] != self.embedding_dim:
            raise ValueError(f"table must be [V, {self.embedding_dim}]")
        self._table_src = table
        self._table = None
        return self

    def _device_table(self, device):
        src = getattr(self, "_table_src", None)
        if src is None:
            return None
        dt = self.compute_dtype
        ep = ops.pad_cols(self.embedding_dim, dt)
        t = self._table
        if t is None or t.dtype != dt or t.device != device or t.shape[1] != ep:
            t = torch.zeros(src.shape[0], ep, dtype=dt, device=device)
            t[:, : self.embedding_dim] = src.to(device=device, dtype=dt)
            t.real_cols = self.embedding_dim  # for algorithmic-byte accounting (timing.py)
            self._table = t
        return t

    # ------------------------------------------------------------------ compute
    def _tower_params(self, which: str):
        enc = self.query_encoder if which == "query" else self.doc_encoder
        proj = self.query_proj if which == "query" else self.doc_proj
        g = [getattr(enc, n) for n in _GRU_ORDER]
        hd = [proj[0].weight, proj[0].bias, proj[1].weight, proj[1].bias, proj[3].weight, proj[3].bias]
        return g + hd

    def _cfg(self, ntowers, encs):
        drops = {float(e.dropout) if self.training else 0.0 for e in encs}
        if len(drops) != 1:
            return None
        return TowerCfg(ntowers, self.embedding_dim, 2 * self.hidden_dim, self.hidden_dim, self.compute_dtype,
                        drops.pop(), rank=dist.rank_world(self.process_group)[0])

    def _run(self, which, xs):
        encs = [self.query_encoder if w == "query" else self.doc_encoder for w in which]
        cfg = self._cfg(len(which), encs)
        if cfg is None:  # different dropout per tower: run them one at a time
            return tuple(self._run([w], [x])[0] for w, x in zip(which, xs))
        params = []
        for w in which:
            params.extend(self._tower_params(w))
        table = self._device_table(xs[0].device) if xs[0].dtype in (torch.int32, torch.int64) else None
        return run_towers(cfg, table, xs, params, self.process_group,
                          self.overlap_grad_allreduce and torch.is_grad_enabled())

    def encode_query(self, query_emb):
        return self._run(["query"], [query_emb])[0]

    def encode_doc(self, doc_emb):
        return self._run(["doc"], [doc_emb])[0]

    def forward(self, query_emb, doc_emb):
        if query_emb.shape[:2] == doc_emb.shape[:2] and query_emb.dtype == doc_emb.dtype:
            q, d = self._run(["query", "doc"], [query_emb, doc_emb])
            return q, d
        return self.encode_query(query_emb), self.encode_doc(doc_emb)


_GRU_ORDER = [f"{w}_l{layer}{sfx}" for layer in (0, 1) for sfx in ("", "_reverse")
              for w in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]

# Name used by validate_enhanced.py:7 and compare_models.py:7.
EnhancedTwoTower = EnhancedTwoTowerModel
