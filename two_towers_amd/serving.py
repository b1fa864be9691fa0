"""Serving search over cached document embeddings (server/python-api/app.py).

The reference service (app.py:41-70) encodes every validation document once, one
document per forward pass, caches the [N, H] matrix, and per request (app.py:85-123)
encodes the query, takes F.cosine_similarity against all cached rows and torch.topk(3),
returning text (first 200 characters + "..." when longer), score, is_ground_truth (the
document text is among the query's paired documents) and rank.

SearchIndex does the same on the HIP path, laid out for serving:
  - documents are encoded in large batches through the fused towers (GPU gather of
    margin_ids rows, one launch sequence per batch of up to 4096 documents);
  - the cached matrix is stored already L2-normalised (eps 1e-8, F.cosine_similarity's)
    in the scoring dtype and stays resident in HBM, so a request is one query encode,
    one fused pass over the resident matrix (tt_search_topk: per-lane scores and top-k,
    no score matrix, for up to 64 queries at once; a GEMM + column-split top-k beyond);
  - ties rank the lower document index first (torch.topk leaves them unspecified).

make_app(index) builds the FastAPI app with the reference's request/response models
(QueryRequest, SearchResult, SearchResponse) and POST /search.
"""

from typing import Dict, List, Optional, Sequence

import torch

from . import _lib, ops, timing
from ._lib import call, dtype_code, stream_ptr

COS_EPS = 1e-8  # F.cosine_similarity default
TOP_K = 3  # app.py:100


def snippet(text: str) -> str:
    """app.py:109: first 200 characters + '...' when the document is longer."""
    return text[:200] + "..." if len(text) > 200 else text


def format_results(docs: Sequence[str], ground_truth: Sequence[str], idx: Sequence[int], scores: Sequence[float]):
    """app.py:104-115 for one query: list of {text, score, is_ground_truth, rank}."""
    gt = set(ground_truth)
    return [{"text": snippet(docs[j]), "score": float(s), "is_ground_truth": docs[j] in gt, "rank": r + 1}
            for r, (j, s) in enumerate(zip(idx, scores))]


def query_to_docs_map(queries: Sequence[str], docs: Sequence[str]) -> Dict[str, List[str]]:
    """app.py:30-36: every paired document of a query text."""
    m: Dict[str, List[str]] = {}
    for q, d in zip(queries, docs):
        m.setdefault(q, []).append(d)
    return m


class SearchIndex:
    """Resident, normalised document embeddings of a margin TwoTowerModel (or any model
    with encode_query / encode_doc taking [B, T] token ids)."""

    def __init__(self, model, vocab, docs: Sequence[str], *, queries: Optional[Sequence[str]] = None,
                 paired_docs: Optional[Sequence[str]] = None, max_length: int = 30, batch: int = 4096,
                 score_dtype=torch.float32, device="cuda", doc_vectors: Optional[torch.Tensor] = None,
                 tokenize=None):
        from .margin import margin_ids
        self.model = model
        self.vocab = vocab
        self.docs = list(docs)
        self.max_length = max_length
        self.batch = batch
        self.score_dtype = score_dtype
        self.device = torch.device(device)
        self.tokenize = tokenize or margin_ids
        self.query_to_docs = query_to_docs_map(queries or [], paired_docs or [])
        if hasattr(model, "set_embedding_table") and getattr(model, "_table_src", None) is None:
            model.set_embedding_table(torch.from_numpy(vocab.vectors).to(self.device))
        raw = doc_vectors.to(self.device).float() if doc_vectors is not None else self.encode_docs(self.docs)
        if raw.shape[0] != len(self.docs):
            raise ValueError(f"{raw.shape[0]} cached vectors for {len(self.docs)} documents")
        self.doc_vectors = raw  # [N, H] fp32, the reference's cached doc_embeddings
        self.doc_normed, _, _ = ops.l2norm_fwd(raw.contiguous(), COS_EPS, score_dtype, want_f32=False)

    def _ids(self, texts: Sequence[str]) -> torch.Tensor:
        return torch.tensor([self.tokenize(t, self.vocab, self.max_length) for t in texts], dtype=torch.int32)

    @torch.no_grad()
    def _encode(self, texts: Sequence[str], kind: str) -> torch.Tensor:
        was = self.model.training
        self.model.eval()
        enc = self.model.encode_query if kind == "query" else self.model.encode_doc
        outs = [enc(self._ids(texts[i:i + self.batch]).to(self.device)) for i in range(0, len(texts), self.batch)]
        self.model.train(was)
        if not outs:
            return torch.empty(0, self.model.hidden_dim, device=self.device)
        return torch.cat(outs, 0).float()

    def encode_docs(self, texts: Sequence[str]) -> torch.Tensor:
        return self._encode(texts, "doc")

    def encode_queries(self, texts: Sequence[str]) -> torch.Tensor:
        return self._encode(texts, "query")

    @torch.no_grad()
    def topk(self, query_vecs: torch.Tensor, k: int = TOP_K):
        """Cosine top-k of each query row against the resident documents:
        (indices int64 [Q, k], scores fp32 [Q, k])."""
        _lib.require_gpu(query_vecs)
        nd = self.doc_normed.shape[0]
        if not 1 <= k <= min(16, nd):
            raise ValueError(f"top_k={k} needs 1 <= k <= min(16, {nd})")
        qn, _, _ = ops.l2norm_fwd(query_vecs.float().contiguous(), COS_EPS, torch.float32)
        Q, h = qn.shape
        idx = torch.empty(Q, k, dtype=torch.int32, device=qn.device)
        val = torch.empty(Q, k, dtype=torch.float32, device=qn.device)
        lib = _lib.load()
        dc = dtype_code(self.score_dtype)
        # large query batches go through a score block of at most 4 GiB per chunk
        step = Q if Q <= 64 else max(65, min(Q, (1 << 30) // max(nd, 1)))
        esz = 2 if self.score_dtype == torch.bfloat16 else 4
        for r0 in range(0, Q, step):
            r1 = min(Q, r0 + step)
            ws = torch.empty(max(lib.tt_search_ws_size(dc, r1 - r0, nd, h, k), 1), dtype=torch.uint8,
                             device=qn.device)
            with timing.region("search_topk", 1, 2.0 * (r1 - r0) * nd * h, float(esz * nd * h + 4 * (r1 - r0) * h)):
                call("tt_search_topk", dc, qn[r0:r1].data_ptr(), r1 - r0, self.doc_normed.data_ptr(), nd, h, k,
                     idx[r0:r1].data_ptr(), val[r0:r1].data_ptr(), ws.data_ptr(), stream_ptr(qn.device))
        return idx.long(), val

    def search_batch(self, queries: Sequence[str], top_k: int = TOP_K):
        idx, val = self.topk(self.encode_queries(queries), top_k)
        idx, val = idx.cpu().tolist(), val.cpu().tolist()
        return [{"query": q, "results": format_results(self.docs, self.query_to_docs.get(q, []), i, v)}
                for q, i, v in zip(queries, idx, val)]

    def search(self, query: str, top_k: int = TOP_K):
        """One /search request (app.py:86-120): {query, results}."""
        return self.search_batch([query], top_k)[0]

    # ---------------------------------------------------- doc-embedding cache
    def save(self, path: str):
        """The cached embeddings (app.py:64-65 DOC_EMBEDDINGS_CACHE) as a plain tensor file."""
        torch.save(self.doc_vectors.cpu(), path)

    @staticmethod
    def load_vectors(path: str) -> torch.Tensor:
        return torch.load(path, map_location="cpu", weights_only=True)


def make_app(index: SearchIndex):
    """FastAPI app with the reference's POST /search contract (app.py:72-123)."""
    from typing import List as _List

    from fastapi import FastAPI, HTTPException
    from pydantic import BaseModel

    class QueryRequest(BaseModel):
        query: str

    class SearchResult(BaseModel):
        text: str
        score: float
        is_ground_truth: bool
        rank: int

    class SearchResponse(BaseModel):
        query: str
        results: _List[SearchResult]

    app = FastAPI()

    @app.post("/search", response_model=SearchResponse)
    def search(request: QueryRequest):
        try:
            return index.search(request.query)
        except Exception as e:  # app.py:122-123
            raise HTTPException(status_code=500, detail=str(e))

    return app


__all__ = ["SearchIndex", "make_app", "format_results", "snippet", "query_to_docs_map"]
