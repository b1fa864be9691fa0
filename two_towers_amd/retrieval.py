"""Batched retrieval and MRR@k (the metric of validate_enhanced.py:19-126).

The reference encodes every document in its own forward pass (validate_enhanced.py:
61-71, one EnhancedDataset per text, max_length 30), scores one query at a time with
F.cosine_similarity and takes torch.topk(10) (:73-80), then averages 1/rank of the
first relevant document (:104-110). Here documents and queries are encoded in large
batches through the fused towers, and scoring + top-k is the fused tt_hardneg_topk
kernel (cosine GEMM + per-row top-k) with a stated tie-break: equal scores rank the
lower document index first.
"""
from __future__ import annotations

from typing import Sequence

import torch

from .data import encode_batch
from .losses import mine_hard_negatives


@torch.no_grad()
def encode_texts(model, texts: Sequence[str], vocab, kind: str, max_length: int = 30, batch: int = 4096,
                 device="cuda") -> torch.Tensor:
    """[len(texts), h] fp32 tower outputs; kind is 'query' or 'doc'."""
    was = model.training
    model.eval()
    outs = []
    enc = model.encode_query if kind == "query" else model.encode_doc
    for i in range(0, len(texts), batch):
        ids = encode_batch(texts[i:i + batch], vocab, max_length).to(device)
        outs.append(enc(ids))
    model.train(was)
    return torch.cat(outs, 0)


@torch.no_grad()
def topk_cosine(query_vecs: torch.Tensor, doc_vecs: torch.Tensor, k: int = 10, compute_dtype=torch.float32):
    """Top-k documents per query by cosine similarity: (indices int64 [Q,k], scores [Q,k])."""
    idx, val = mine_hard_negatives(query_vecs, doc_vecs, label_offset=-1, k=k, compute_dtype=compute_dtype,
                                   return_values=True)
    return idx.long(), val


def mrr_at_k(top_idx: torch.Tensor, relevant: Sequence[set]) -> float:
    """Mean over queries of 1/rank of the first relevant document in top_idx (0 if none)."""
    total = 0.0
    rows = top_idx.cpu().tolist()
    for row, rel in zip(rows, relevant):
        for rank, j in enumerate(row, 1):
            if j in rel:
                total += 1.0 / rank
                break
    return total / max(len(rows), 1)
