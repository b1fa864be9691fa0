"""Serving /search (server/python-api/app.py:41-123) on the HIP path vs the oracle, which
encodes every document one at a time as the reference service does.

Tolerances: scores within 1e-4 absolute (fp32); rankings exact wherever the oracle's
top-(k+1) scores are separated by more than 1e-4 (closer gaps are reported as ties and
only their score is checked).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import cpu_ref  # noqa: E402
from two_towers_amd.data import Vocab  # noqa: E402
from two_towers_amd.margin import TwoTowerModel  # noqa: E402
from two_towers_amd.serving import SearchIndex  # noqa: E402

DEV = "cuda"


def corpus(seed, V=300, n_docs=400, n_q=24):
    rng = np.random.default_rng(seed)
    words = [f"t{i}" for i in range(V)] + ["is", "has", "controls", "part_of", "5_kg"]
    docs = []
    for i in range(n_docs):
        body = [words[j] for j in rng.integers(0, len(words), int(rng.integers(3, 40)))]
        docs.append(" ".join([f"t{i % V}", "is", "a"] + body + (["5 kg", "part of"] if i % 7 == 0 else [])))
    docs[3] = docs[3] + " " + "long " * 60  # > 200 characters
    qsel = rng.integers(0, n_docs, n_q)
    queries = [" ".join(docs[j].split()[:4]) for j in qsel]
    paired = [docs[j] for j in qsel]
    return words, docs, queries, paired


def oracle_encode(text, p, vocab_idx, table, kind, T):
    ids = cpu_ref.margin_text_to_ids(text, vocab_idx, T)
    emb = torch.from_numpy(cpu_ref.ids_to_embedding(ids, table)).unsqueeze(0)
    return cpu_ref.margin_encode(emb, p, kind)[0]


@pytest.mark.parametrize("H", [16, 64])
def test_search_matches_reference_service(H):
    E, T = 24, 30
    words, docs, queries, paired = corpus(30 + H)
    rng = np.random.default_rng(H)
    vecs = rng.standard_normal((len(words), E)).astype(np.float32)
    vocab = Vocab(words, vecs)
    torch.manual_seed(H)
    m = TwoTowerModel(E, H)
    p = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV).eval()
    index = SearchIndex(m, vocab, docs, queries=queries, paired_docs=paired, max_length=T, batch=128)
    vidx = vocab.index
    with torch.no_grad():
        doc_mat = torch.stack([oracle_encode(d, p, vidx, vecs, "doc", T) for d in docs])
    assert float((index.doc_vectors.cpu() - doc_mat).abs().max()) < 1e-4
    gt = {}
    for q, d in zip(queries, paired):
        gt.setdefault(q, []).append(d)
    got = index.search_batch(queries)
    assert got[0] == index.search(queries[0])
    checked = 0
    for q, res in zip(queries, got):
        with torch.no_grad():
            qv = oracle_encode(q, p, vidx, vecs, "query", T)
            ref = cpu_ref.search_results(qv, doc_mat, docs, gt.get(q, []), 4)
        assert res["query"] == q and len(res["results"]) == 3
        for a, b in zip(res["results"], ref):
            assert abs(a["score"] - b["score"]) < 1e-4
        gaps = np.diff([r["score"] for r in ref])
        if np.all(np.abs(gaps) > 1e-4):
            assert res["results"] == [dict(r, score=a["score"]) for r, a in zip(ref[:3], res["results"])]
            checked += 1
    assert checked >= len(queries) // 2


def test_search_bf16_scores_and_cache_roundtrip(tmp_path):
    E, H, T = 24, 32, 30
    words, docs, queries, paired = corpus(7)
    vecs = np.random.default_rng(8).standard_normal((len(words), E)).astype(np.float32)
    vocab = Vocab(words, vecs)
    torch.manual_seed(9)
    m = TwoTowerModel(E, H).to(DEV).eval()
    f32 = SearchIndex(m, vocab, docs, max_length=T)
    path = str(tmp_path / "doc_embeddings.pt")
    f32.save(path)
    bf = SearchIndex(m, vocab, docs, max_length=T, score_dtype=torch.bfloat16,
                     doc_vectors=SearchIndex.load_vectors(path))
    assert torch.equal(bf.doc_vectors, f32.doc_vectors)
    a = f32.search_batch(queries, top_k=5)
    b = bf.search_batch(queries, top_k=5)
    for x, y in zip(a, b):
        for rx, ry in zip(x["results"], y["results"]):
            assert abs(rx["score"] - ry["score"]) < 2e-2
        assert x["results"][0]["score"] == pytest.approx(y["results"][0]["score"], abs=2e-2)


def test_search_rejects_bad_k():
    words, docs, _, _ = corpus(1, n_docs=5)
    vocab = Vocab(words, np.ones((len(words), 8), np.float32))
    m = TwoTowerModel(8, 8).to(DEV).eval()
    index = SearchIndex(m, vocab, docs)
    with pytest.raises(ValueError):
        index.search("t1", top_k=6)
    assert len(index.search("t1", top_k=5)["results"]) == 5
