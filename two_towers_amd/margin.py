"""The margin model family (margin_two_tower.py / train_margin.py) on the HIP path.

  TwoTowerModel(embedding_dim, hidden_dim)   margin_two_tower.py:9-68
        two nn.GRU(E, hidden_dim, 2 layers, bidirectional, dropout 0.1) encoders and ONE
        projection Sequential(Linear(2H,H), LayerNorm(H), ReLU, Dropout(0.1)) shared by
        both towers; same submodule names, hence the same state_dict keys and the same
        default initialisation for a given torch seed. forward returns the normalised
        (q, d) pair in training mode and the cosine matrix q·dᵀ in eval mode
        (compute_similarity, :37-48); encode_query / encode_doc return the raw
        projection output (:50-62).
  InfoNCELoss(temperature=0.07)              margin_two_tower.py:70-85 (the same
        computation as the enhanced InfoNCE: losses.InfoNCELoss).
  SimpleDataset(queries, docs, word2vec)     margin_two_tower.py:87-161, including the
        structural-marker rewriting of text_to_embedding; margin_ids / MarginIdDataset
        are its int32 row-id form for the GPU gather.

GPU layout: the GRU towers are the fused TowersFn with cfg.head "none" (they return
cat(h_fwd_final, h_rev_final) = cat(hidden[-2], hidden[-1]), :59-61); query and doc rows
are then stacked into one [2B, 2H] batch for tt_proj_head1_fwd/bwd, so the shared head
runs as one GEMM + one fused LayerNorm/ReLU/Dropout pass and its weight gradients are
the two towers' sum by construction. Normalisation is tt_l2norm; the eval-mode
similarity matrix is a tt_gemm.
"""
from __future__ import annotations

import re
from typing import List

import numpy as np
import torch
import torch.nn as nn
from torch.utils.data import Dataset

from . import _lib, dist, ops, timing
from ._lib import Head1BwdIO, Head1FwdIO, call, dtype_code, stream_ptr
from .losses import InfoNCELoss
from .model import _GRU_ORDER
from .towers import HEAD_DT, LN_EPS, TowerCfg, run_towers

NORM_EPS = 1e-12  # F.normalize default


class _SharedHeadFn(torch.autograd.Function):
    """(x [rows, 2H] fp32, w1, b1, ln_g, ln_b) -> relu(LN(x w1^T + b1)) * dropout, [rows, H]."""

    @staticmethod
    def forward(ctx, x, w1, b1, ln_g, ln_b, drop_p):
        _lib.require_gpu(x, w1, b1, ln_g, ln_b)
        dev = x.device
        rows, C = x.shape[0], w1.shape[0]
        if x.shape[1] != 2 * C or tuple(w1.shape) != (C, 2 * C):
            raise ValueError(f"projection expects x [rows, {2 * C}] and weight [{C}, {2 * C}]")
        x = x.to(HEAD_DT).contiguous()
        w = w1.detach().to(HEAD_DT).contiguous()
        b = b1.detach().float().contiguous()
        g = ln_g.detach().float().contiguous()
        be = ln_b.detach().float().contiguous()
        p1 = torch.empty(rows, C, dtype=HEAD_DT, device=dev)
        mean = torch.empty(rows, dtype=torch.float32, device=dev)
        rstd = torch.empty(rows, dtype=torch.float32, device=dev)
        out = torch.empty(rows, C, dtype=torch.float32, device=dev)
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if drop_p > 0 else 0
        # rows are [queries; docs] stacked locally, so no single row offset maps them onto
        # the global batch: data-parallel ranks draw from rank-distinct seeds instead
        rank = dist.rank_world(None)[0]
        if rank:
            seed = (seed ^ (0x9E3779B9 * rank)) & 0x7FFFFFFF
        io = Head1FwdIO()
        io.x, io.w1, io.b1, io.ln_g, io.ln_b = x.data_ptr(), w.data_ptr(), b.data_ptr(), g.data_ptr(), be.data_ptr()
        io.p1, io.mean, io.rstd, io.out = p1.data_ptr(), mean.data_ptr(), rstd.data_ptr(), out.data_ptr()
        with timing.region("margin_head_fwd", 2, 2.0 * rows * C * 2 * C, 4.0 * rows * (2 * C + 3 * C)):
            call("tt_proj_head1_fwd", dtype_code(HEAD_DT), io, rows, C, LN_EPS, float(drop_p), seed, stream_ptr(dev))
        ctx.save = (x, w, g, be, p1, mean, rstd)
        ctx.cfg = (float(drop_p), seed)
        return out

    @staticmethod
    def backward(ctx, gout):
        x, w, g, be, p1, mean, rstd = ctx.save
        drop_p, seed = ctx.cfg
        dev = x.device
        rows, C = p1.shape
        gout = gout.float().contiguous()
        dx = torch.empty(rows, 2 * C, dtype=torch.float32, device=dev)
        dw1 = torch.empty(C, 2 * C, dtype=torch.float32, device=dev)
        db1 = torch.empty(C, dtype=torch.float32, device=dev)
        dg = torch.empty(C, dtype=torch.float32, device=dev)
        dbeta = torch.empty(C, dtype=torch.float32, device=dev)
        lib = _lib.load()
        ws = torch.empty(lib.tt_proj_head1_bwd_ws_size(dtype_code(HEAD_DT), rows, C), dtype=torch.uint8, device=dev)
        io = Head1BwdIO()
        io.x, io.w1, io.ln_g, io.ln_b = x.data_ptr(), w.data_ptr(), g.data_ptr(), be.data_ptr()
        io.p1, io.mean, io.rstd, io.dout, io.dx = (p1.data_ptr(), mean.data_ptr(), rstd.data_ptr(), gout.data_ptr(),
                                                   dx.data_ptr())
        io.dw1, io.db1, io.dg, io.dbeta, io.ws = (dw1.data_ptr(), db1.data_ptr(), dg.data_ptr(), dbeta.data_ptr(),
                                                  ws.data_ptr())
        call("tt_proj_head1_bwd", dtype_code(HEAD_DT), io, rows, C, drop_p, seed, stream_ptr(dev))
        ctx.save = None
        return dx, dw1, db1, dg, dbeta, None


class _NormalizeFn(torch.autograd.Function):
    """F.normalize(x, p=2, dim=1) (margin_two_tower.py:39-40) on tt_l2norm."""

    @staticmethod
    def forward(ctx, x):
        _lib.require_gpu(x)
        x = x.float().contiguous()
        y, y32, norm = ops.l2norm_fwd(x, NORM_EPS, torch.float32)
        ctx.save = (y32, norm)
        return y32

    @staticmethod
    def backward(ctx, gy):
        y32, norm = ctx.save
        return ops.l2norm_bwd(gy.float().contiguous(), y32, norm, NORM_EPS)


def normalize(x: torch.Tensor) -> torch.Tensor:
    return _NormalizeFn.apply(x)


def similarity_matrix(qn: torch.Tensor, dn: torch.Tensor) -> torch.Tensor:
    """qn dnᵀ [Q, D] fp32 (margin_two_tower.py:47) on tt_gemm."""
    _lib.require_gpu(qn, dn)
    qn = qn.float().contiguous()
    dn = dn.float().contiguous()
    Q, h = qn.shape
    D = dn.shape[0]
    out = torch.empty(Q, D, dtype=torch.float32, device=qn.device)
    ops.gemm([qn], [dn], [out], m=Q, n=D, k=h, lda=h, ldb=h, ldc=D, a_kouter=False, b_kouter=False,
             dtype=torch.float32, out_dtype=torch.float32)
    return out


class TwoTowerModel(nn.Module):
    def __init__(self, embedding_dim: int, hidden_dim: int):
        super().__init__()
        self.query_encoder = nn.GRU(input_size=embedding_dim, hidden_size=hidden_dim, num_layers=2,
                                    batch_first=True, bidirectional=True, dropout=0.1)
        self.doc_encoder = nn.GRU(input_size=embedding_dim, hidden_size=hidden_dim, num_layers=2,
                                  batch_first=True, bidirectional=True, dropout=0.1)
        self.projection = nn.Sequential(nn.Linear(hidden_dim * 2, hidden_dim), nn.LayerNorm(hidden_dim), nn.ReLU(),
                                        nn.Dropout(0.1))
        self.embedding_dim = embedding_dim
        self.hidden_dim = hidden_dim
        self.compute_dtype = torch.float32
        self._table = None
        self._table_src = None
        self.process_group = None
        self.overlap_grad_allreduce = False

    # ---------------------------------------------------------------- options
    def set_process_group(self, group, overlap_grad_allreduce: bool = False):
        """Data-parallel group; as EnhancedTwoTowerModel.set_process_group (the opt-in
        overlap sums the GRU gradients inside the backward; the shared projection's are
        left to dist.allreduce_grads)."""
        self.process_group = group
        self.overlap_grad_allreduce = overlap_grad_allreduce
        return self

    def set_compute_dtype(self, dtype: torch.dtype):
        """dtype of the GRU towers (fp32 or bf16 storage, fp32 accumulation); the shared
        projection head always runs in fp32."""
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("compute dtype must be torch.float32 or torch.bfloat16")
        self.compute_dtype = dtype
        return self

    def set_embedding_table(self, table: torch.Tensor | None):
        """Attach a device Word2Vec table [V, E]; [B, T] int token-id inputs (margin_ids)
        then gather rows on the GPU."""
        if table is not None and (table.dim() != 2 or table.shape[1] != self.embedding_dim):
            raise ValueError(f"table must be [V, {self.embedding_dim}]")
        self._table_src = table
        self._table = None
        return self

    def _device_table(self, device):
        if self._table_src is None:
            return None
        dt = self.compute_dtype
        ep = ops.pad_cols(self.embedding_dim, dt)
        t = self._table
        if t is None or t.dtype != dt or t.device != device or t.shape[1] != ep:
            t = torch.zeros(self._table_src.shape[0], ep, dtype=dt, device=device)
            t[:, : self.embedding_dim] = self._table_src.to(device=device, dtype=dt)
            t.real_cols = self.embedding_dim
            self._table = t
        return t

    # ------------------------------------------------------------------ compute
    def _towers(self, which, xs):
        """cat(hidden[-2], hidden[-1]) [B, 2H] fp32 per requested tower."""
        encs = [self.query_encoder if w == "query" else self.doc_encoder for w in which]
        drops = {float(e.dropout) if self.training else 0.0 for e in encs}
        if len(drops) != 1 or xs[0].shape[:2] != xs[-1].shape[:2] or xs[0].dtype != xs[-1].dtype:
            return tuple(self._towers([w], [x])[0] for w, x in zip(which, xs))
        cfg = TowerCfg(len(which), self.embedding_dim, self.hidden_dim, self.hidden_dim, self.compute_dtype,
                       drops.pop(), head="none", rank=dist.rank_world(getattr(self, "process_group", None))[0])
        params = []
        for e in encs:
            params.extend(getattr(e, n) for n in _GRU_ORDER)
        table = self._device_table(xs[0].device) if xs[0].dtype in (torch.int32, torch.int64) else None
        return run_towers(cfg, table, xs, params, getattr(self, "process_group", None),
                          getattr(self, "overlap_grad_allreduce", False) and torch.is_grad_enabled())

    def _project(self, vecs):
        """The shared projection over the row-stacked towers; returns one [B_i, H] per tower."""
        p = self.projection
        drop_p = float(p[3].p) if self.training else 0.0
        x = vecs[0] if len(vecs) == 1 else torch.cat(vecs, 0)
        out = _SharedHeadFn.apply(x, p[0].weight, p[0].bias, p[1].weight, p[1].bias, drop_p)
        return out.split([v.shape[0] for v in vecs], 0)

    def encode(self, emb, encoder):
        which = "query" if encoder is self.query_encoder else "doc"
        return self._project(self._towers([which], [emb]))[0]

    def encode_query(self, query_emb):
        return self.encode(query_emb, self.query_encoder)

    def encode_doc(self, doc_emb):
        return self.encode(doc_emb, self.doc_encoder)

    def compute_similarity(self, query_vec, doc_vec):
        query_vec = normalize(query_vec)
        doc_vec = normalize(doc_vec)
        if self.training:
            return query_vec, doc_vec
        return similarity_matrix(query_vec, doc_vec)

    def forward(self, query_emb, doc_emb):
        q, d = self._project(self._towers(["query", "doc"], [query_emb, doc_emb]))
        return self.compute_similarity(q, d)


# ------------------------------------------------------------------------- data
_MARKERS = [
    (re.compile(r"\b(is|are|refers?\s+to)\s+(?:a|an|the)\b"), "IS"),
    (re.compile(r"\b(contains?|has|have|includes?)\b"), "HAS"),
    (re.compile(r"\b(part|component|element)\s+of\b"), "PART_OF"),
    (re.compile(r"\b(controls?|regulates?|manages?)\b"), "CONTROLS"),
    (re.compile(r"\b(functions?|works?|operates?)\b"), "FUNCTIONS"),
    (re.compile(r"(\d+(?:\.\d+)?)\s*([a-zA-Z]+)"), r"\1_\2"),
]


def margin_tokens(text: str) -> List[str]:
    """The lookup sequence of SimpleDataset.text_to_embedding (margin_two_tower.py:97-139):
    the text is lower-cased before every rewrite (so the markers end up lower-case), and
    processed word i is tried after ORIGINAL word i (positional, even when a rewrite has
    merged words), the processed one only when it differs."""
    original = text.lower().split()
    t = text
    for pat, rep in _MARKERS:
        t = pat.sub(rep, t.lower())
    out = []
    for i, word in enumerate(t.split()):
        if i < len(original):
            out.append(original[i])
        if word != original[i]:
            out.append(word)
    return out


def margin_ids(text: str, vocab, max_length: int = 30) -> List[int]:
    """text_to_embedding as row ids: in-vocabulary lookups in order, a single zero row
    (-1) if none, then pad with -1 / truncate to max_length."""
    index = vocab.index if hasattr(vocab, "index") and isinstance(vocab.index, dict) else vocab
    ids = [index[w] for w in margin_tokens(text) if w in index]
    if not ids:
        ids = [-1]
    return ids[:max_length] + [-1] * (max_length - len(ids[:max_length]))


class SimpleDataset(Dataset):
    def __init__(self, queries: List[str], docs: List[str], word2vec, max_length: int = 30):
        super().__init__()
        self.queries = queries
        self.docs = docs
        self.word2vec = word2vec
        self.max_length = max_length
        self.embedding_dim = word2vec.vector_size

    @staticmethod
    def text_to_embedding(text: str, word2vec, max_length: int = 30) -> torch.Tensor:
        rows = []
        for w in margin_tokens(text):
            try:
                rows.append(np.asarray(word2vec[w], dtype=np.float32))
            except KeyError:
                continue
        out = np.zeros((max_length, word2vec.vector_size), dtype=np.float32)
        for i, r in enumerate(rows[:max_length]):
            out[i] = r
        return torch.from_numpy(out)

    def __len__(self):
        return len(self.queries)

    def __getitem__(self, idx):
        return (self.text_to_embedding(self.queries[idx], self.word2vec, self.max_length),
                self.text_to_embedding(self.docs[idx], self.word2vec, self.max_length))


class MarginIdDataset(Dataset):
    """SimpleDataset returning int32 id rows (margin_ids) for the GPU gather."""

    def __init__(self, queries: List[str], docs: List[str], vocab, max_length: int = 30):
        self.queries, self.docs, self.vocab, self.max_length = queries, docs, vocab, max_length

    def __len__(self):
        return len(self.queries)

    def __getitem__(self, idx):
        return (torch.tensor(margin_ids(self.queries[idx], self.vocab, self.max_length), dtype=torch.int32),
                torch.tensor(margin_ids(self.docs[idx], self.vocab, self.max_length), dtype=torch.int32))


__all__ = ["TwoTowerModel", "InfoNCELoss", "SimpleDataset", "MarginIdDataset", "margin_tokens", "margin_ids",
           "normalize", "similarity_matrix"]
