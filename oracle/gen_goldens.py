"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

TEST INFRASTRUCTURE ONLY. Run in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_goldens.py
The reference's enhanced_two_tower.py imports gensim.downloader at module level but only
dereferences it inside network loaders we never call, so a stub module satisfies the
import. The fixtures are data (inputs + expected outputs); no reference
source is copied. Weights are either small reference state_dicts (tiny models) or
regenerated procedurally on both sides (oracle.cpu_ref.counter_params).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("TT_REFERENCE", "/root/reference")
OUT = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)

from oracle import cpu_ref  # noqa: E402


def import_reference():
    g = types.ModuleType("gensim")
    gd = types.ModuleType("gensim.downloader")
    g.downloader = gd
    sys.modules.setdefault("gensim", g)
    sys.modules.setdefault("gensim.downloader", gd)
    sys.path.insert(0, REF)
    import enhanced_two_tower as et  # noqa: E402
    return et


def sd_arrays(prefix, sd):
    return {f"{prefix}{k}": v.detach().cpu().numpy().copy() for k, v in sd.items()}  # copy: .numpy() aliases


class FakeW2V(dict):
    """dict-backed Word2Vec: __getitem__ raises KeyError for OOV, has vector_size."""

    def __init__(self, words, vecs):
        super().__init__(zip(words, vecs))
        self.vector_size = vecs.shape[1]


def gen_tiny_model(et):
    torch.manual_seed(0)
    model = et.EnhancedTwoTowerModel(16, 8).eval()
    g = torch.Generator().manual_seed(11)
    q = torch.randn(16, 8, 16, generator=g)
    d = torch.randn(16, 8, 16, generator=g)
    qv, dv = model(q, d)
    loss = et.InfoNCELoss()(qv, dv)
    loss.backward()
    out = {"q": q.numpy(), "d": d.numpy(), "q_vec": qv.detach().numpy(), "d_vec": dv.detach().numpy(),
           "loss": np.float32(loss.item())}
    out.update(sd_arrays("w.", model.state_dict()))
    out.update({f"g.{k}": p.grad.numpy() for k, p in model.named_parameters()})
    np.savez_compressed(os.path.join(OUT, "tiny_model.npz"), **out)


def gen_tiny_train(et):
    torch.manual_seed(1)
    model = et.EnhancedTwoTowerModel(16, 8)  # train mode, as train_enhanced.py leaves it
    model.query_encoder.dropout = 0.0  # nn.GRU reads the attribute at call time
    model.doc_encoder.dropout = 0.0
    init = sd_arrays("w0.", model.state_dict())
    g = torch.Generator().manual_seed(12)
    batches = [(torch.randn(32, 10, 16, generator=g), torch.randn(32, 10, 16, generator=g)) for _ in range(4)]
    crit = et.InfoNCELoss()
    opt = torch.optim.Adam(model.parameters())
    losses = []
    for s in range(20):  # train_enhanced.py:54-69
        q, d = batches[s % 4]
        opt.zero_grad()
        qv, dv = model(q, d)
        loss = crit(qv, dv)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    out = dict(init)
    out.update(sd_arrays("w20.", model.state_dict()))
    out["losses"] = np.array(losses, dtype=np.float32)
    out["bq"] = np.stack([b[0].numpy() for b in batches])
    out["bd"] = np.stack([b[1].numpy() for b in batches])
    np.savez_compressed(os.path.join(OUT, "tiny_train.npz"), **out)


def gen_featurize(et):
    rng = np.random.default_rng(13)
    words = [f"w{i}" for i in range(50)] + ["hello", "world", "the"]
    vecs = rng.standard_normal((len(words), 8)).astype(np.float32)
    w2v = FakeW2V(words, vecs)
    texts = [
        "Hello World the w1 w2",            # case folding
        "hello OOVWORD world",              # OOV skipped, not zero-filled
        " ".join(f"w{i}" for i in range(12)),  # longer than max_length: truncated BEFORE OOV drop
        "zzz yyy xxx",                      # all OOV -> one zero row
        "",                                 # empty -> one zero row
        "oov1 oov2 oov3 oov4 oov5 oov6 w7",  # in-vocab word beyond max_length after OOVs -> dropped
        "w3\tw4\nw5  w6",                   # any whitespace splits
    ]
    ds = et.EnhancedDataset(texts, texts, w2v, max_length=6)
    embs = np.stack([ds.text_to_embedding(t).numpy() for t in texts])
    np.savez_compressed(os.path.join(OUT, "featurize.npz"), words=np.array(words), vecs=vecs,
                        texts=np.array(texts), max_length=np.int32(6), emb=embs)


def gen_full(et, E, h, T, B, name, seed):
    """Reference-size model with counter-hash weights (regenerated on both sides). The
    inputs are stored fp16-rounded and the reference ran on exactly those values."""
    p = cpu_ref.counter_params(E, h, seed)
    model = et.EnhancedTwoTowerModel(E, h).eval()
    model.load_state_dict(p)
    g = torch.Generator().manual_seed(seed + 100)
    q = (torch.randn(B, T, E, generator=g) * 0.5).half().float()
    d = (torch.randn(B, T, E, generator=g) * 0.5).half().float()
    qv, dv = model(q, d)
    loss = et.InfoNCELoss()(qv, dv)
    loss.backward()
    out = {"E": np.int32(E), "h": np.int32(h), "T": np.int32(T), "B": np.int32(B), "seed": np.int32(seed),
           "q": q.numpy().astype(np.float16), "d": d.numpy().astype(np.float16),
           "q_vec": qv.detach().numpy(), "d_vec": dv.detach().numpy(), "loss": np.float32(loss.item())}
    for k, prm in model.named_parameters():
        out[f"gnorm.{k}"] = np.float32(prm.grad.norm().item())
        out[f"gslice.{k}"] = prm.grad.reshape(-1)[:64].numpy()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)


def gen_losses(et):
    g = torch.Generator().manual_seed(14)
    out = {}
    for B in (8, 64, 256):
        h = 32
        q = torch.randn(B, h, generator=g)
        d = torch.randn(B, h, generator=g)
        k = 5 if B > 8 else 3
        n = torch.randn(B * k, h, generator=g)
        out[f"q{B}"], out[f"d{B}"], out[f"n{B}"] = q.numpy(), d.numpy(), n.numpy()
        for name, fn, args in (("infonce", et.InfoNCELoss(), (q, d)),
                               ("margin_inbatch", et.MarginRankingLoss(), (q, d)),
                               ("margin_explicit", et.MarginRankingLoss(), (q, d, n))):
            ts = [a.clone().requires_grad_(True) for a in args]
            loss = fn(*ts)
            loss.backward()
            out[f"{name}{B}.loss"] = np.float32(loss.item())
            for i, t in enumerate(ts):
                out[f"{name}{B}.grad{i}"] = t.grad.numpy()
        # the config-3 composition: looped get_hard_negatives over the in-batch docs
        qs, ds = q.clone().requires_grad_(True), d.clone().requires_grad_(True)
        idx = torch.stack([et.get_hard_negatives(qs[i].detach(), ds.detach(), i, k) for i in range(B)])
        loss = et.MarginRankingLoss()(qs, ds, ds[idx.reshape(-1)])
        loss.backward()
        out[f"hardneg{B}.idx"] = idx.numpy()
        out[f"hardneg{B}.loss"] = np.float32(loss.item())
        out[f"hardneg{B}.grad0"] = qs.grad.numpy()
        out[f"hardneg{B}.grad1"] = ds.grad.numpy()
    np.savez_compressed(os.path.join(OUT, "losses.npz"), k8=np.int32(3), **out)


def synth_corpus(rng, n_docs, n_queries, vocab_size, doc_len, q_len):
    """Docs with distinct leading tokens (no two docs share their first tokens, so
    their embeddings never tie); each query = a few words of its relevant doc + noise."""
    docs, queries, rel = [], [], []
    for i in range(n_docs):
        lead = [f"t{(i * 7919 + j * 104729) % vocab_size}" for j in range(2)]
        body = [f"t{x}" for x in rng.integers(0, vocab_size, doc_len - 2)]
        docs.append(" ".join(lead + body))
    for i in range(n_queries):
        j = int(rng.integers(0, n_docs))
        words = docs[j].split()
        pick = list(rng.choice(words, size=q_len - 1, replace=False)) + [f"t{int(rng.integers(0, vocab_size))}"]
        queries.append(" ".join(pick))
        rel.append(j)
    return docs, queries, rel


def gen_mrr(et):
    """Train a tiny reference model on a synthetic corpus, then score MRR@10 exactly as
    validate_enhanced.py:61-80,104-110 does (one doc per forward, cosine, top-10)."""
    rng = np.random.default_rng(15)
    V, E = 400, 16
    words = [f"t{i}" for i in range(V)]
    vecs = rng.standard_normal((V, E)).astype(np.float32)
    w2v = FakeW2V(words, vecs)
    docs, queries, rel = synth_corpus(rng, 1500, 150, V, 12, 4)
    torch.manual_seed(2)
    model = et.EnhancedTwoTowerModel(E, 8)
    model.query_encoder.dropout = 0.0
    model.doc_encoder.dropout = 0.0
    opt = torch.optim.Adam(model.parameters(), lr=3e-3)
    crit = et.InfoNCELoss()
    train_ds = et.EnhancedDataset(queries, [docs[j] for j in rel], w2v, max_length=12)
    for step in range(60):
        sel = rng.integers(0, len(queries), 64)
        q = torch.stack([train_ds[int(i)][0] for i in sel])
        d = torch.stack([train_ds[int(i)][1] for i in sel])
        opt.zero_grad()
        loss = crit(*model(q, d))
        loss.backward()
        opt.step()
    model.eval()

    def encode_text(text, kind):  # validate_enhanced.py:9-17 (max_length default 30)
        ds = et.EnhancedDataset([text], [text], w2v)
        emb = ds[0][0].unsqueeze(0)
        with torch.no_grad():
            return model.encode_query(emb) if kind == "query" else model.encode_doc(emb)

    doc_enc = torch.cat([encode_text(t, "doc") for t in docs], 0)
    mrr_sum = 0.0
    ranks = []
    for qi, qt in enumerate(queries):
        qv = encode_text(qt, "query")
        sims = torch.nn.functional.cosine_similarity(qv, doc_enc)
        top = torch.topk(sims, k=10)
        top_sorted = sorted(zip(top.values.tolist(), top.indices.tolist()), key=lambda x: (-x[0], x[1]))
        gaps = np.diff(sorted(sims.tolist(), reverse=True)[:11])
        assert np.all(np.abs(gaps) > 0), "score tie in the top-11: regenerate the corpus"
        mrr = 0.0
        for rank, (_, j) in enumerate(top_sorted, 1):
            if j == rel[qi]:
                mrr = 1.0 / rank
                break
        ranks.append(mrr)
        mrr_sum += mrr
    out = {"words": np.array(words), "vecs": vecs, "docs": np.array(docs), "queries": np.array(queries),
           "rel": np.array(rel, dtype=np.int32), "mrr": np.float64(mrr_sum / len(queries)),
           "rr": np.array(ranks), "doc_enc": doc_enc.numpy()}
    out.update(sd_arrays("w.", model.state_dict()))
    np.savez_compressed(os.path.join(OUT, "mrr_synth.npz"), **out)


def gen_dp(et):
    """Loss/grads of one global batch of 256, single process: the DP runs must match."""
    torch.manual_seed(3)
    model = et.EnhancedTwoTowerModel(16, 8).eval()
    g = torch.Generator().manual_seed(16)
    q = torch.randn(256, 6, 16, generator=g)
    d = torch.randn(256, 6, 16, generator=g)
    loss = et.InfoNCELoss()(*model(q, d))
    loss.backward()
    out = {"q": q.numpy(), "d": d.numpy(), "loss": np.float32(loss.item())}
    out.update(sd_arrays("w.", model.state_dict()))
    out.update({f"g.{k}": p.grad.numpy() for k, p in model.named_parameters()})
    np.savez_compressed(os.path.join(OUT, "dp_equiv.npz"), **out)


def gen_dp_step(et):
    """One full train_enhanced.py step (train_enhanced.py:58-63) on a global batch of 256,
    single process, for both losses the bench runs: InfoNCE, and the config-3
    composition (looped get_hard_negatives over the whole batch + MarginRankingLoss with
    those negatives). Loss, every parameter gradient and the weights after one
    Adam(lr=1e-3) step: an N-rank data-parallel step over the same 256 rows must
    reproduce them. Eval mode: the reference's dropout RNG is
    not reproducible by another backend."""
    g = torch.Generator().manual_seed(18)
    q = torch.randn(256, 6, 16, generator=g)
    d = torch.randn(256, 6, 16, generator=g)
    out = {"q": q.numpy(), "d": d.numpy()}
    for name in ("infonce", "hardneg"):
        torch.manual_seed(5)
        model = et.EnhancedTwoTowerModel(16, 8).eval()
        if name == "infonce":
            out.update(sd_arrays("w.", model.state_dict()))
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        opt.zero_grad()
        qv, dv = model(q, d)
        if name == "infonce":
            loss = et.InfoNCELoss()(qv, dv)
        else:
            idx = torch.stack([et.get_hard_negatives(qv[i].detach(), dv.detach(), i, 5) for i in range(256)])
            loss = et.MarginRankingLoss()(qv, dv, dv[idx.reshape(-1)])
            out["hardneg.idx"] = idx.numpy()
        loss.backward()
        out[f"{name}.loss"] = np.float32(loss.item())
        out.update({f"{name}.g.{k}": p.grad.numpy().copy() for k, p in model.named_parameters()})
        opt.step()
        out.update(sd_arrays(f"{name}.w1.", model.state_dict()))
    np.savez_compressed(os.path.join(OUT, "dp_step.npz"), **out)


def import_margin_reference():
    sys.path.insert(0, REF)
    import margin_two_tower as mt  # noqa: E402  (torch / numpy / re only)
    return mt


def gen_margin(mt):
    """margin_two_tower.TwoTowerModel: eval similarity matrix + encode_* outputs, and one
    train-mode InfoNCE(0.1) backward (train_margin.py) with every dropout set to 0."""
    torch.manual_seed(4)
    model = mt.TwoTowerModel(16, 8).eval()
    g = torch.Generator().manual_seed(17)
    q = torch.randn(12, 7, 16, generator=g)
    d = torch.randn(12, 7, 16, generator=g)
    with torch.no_grad():
        sim = model(q, d)
        eq = model.encode_query(q)
        ed = model.encode_doc(d)
    out = {"q": q.numpy(), "d": d.numpy(), "sim": sim.numpy(), "enc_q": eq.numpy(), "enc_d": ed.numpy()}
    out.update(sd_arrays("w.", model.state_dict()))
    model.train()
    model.query_encoder.dropout = 0.0
    model.doc_encoder.dropout = 0.0
    model.projection[3].p = 0.0
    qn, dn = model(q, d)
    loss = mt.InfoNCELoss(temperature=0.1)(qn, dn)
    loss.backward()
    out["qn"] = qn.detach().numpy()
    out["dn"] = dn.detach().numpy()
    out["loss"] = np.float32(loss.item())
    out.update({f"g.{k}": p.grad.numpy() for k, p in model.named_parameters()})
    np.savez_compressed(os.path.join(OUT, "margin_tiny.npz"), **out)

    # SimpleDataset.text_to_embedding: the marker rewrites and the original/processed
    # lookup order, with a vocabulary holding both original and rewritten tokens
    rng = np.random.default_rng(18)
    words = ["the", "heart", "is", "a", "muscle", "has", "contains", "4_chambers", "4", "chambers", "5_kg",
             "part_of", "brain", "controls", "functions", "cell", "an", "organ", "works", "3.5_mg", "dose",
             "refers", "to", "component", "of", "body", "are", "have", "includes", "element", "system"]
    vecs = rng.standard_normal((len(words), 6)).astype(np.float32)
    w2v = FakeW2V(words, vecs)
    texts = [
        "The heart is a muscle that contains 4 chambers",
        "the brain controls the body and works as an organ",
        "Dose: 3.5 mg or 5kg; 4chambers",
        "a cell is part of the body and refers to an element of a system",
        "Functions FUNCTION works worked operates",
        "heart\tmuscle\nbrain",
        "zzz qqq",
        "",
        "the " * 40,
    ]
    embs = np.stack([mt.SimpleDataset.text_to_embedding(t, w2v, 10).numpy() for t in texts])
    np.savez_compressed(os.path.join(OUT, "margin_featurize.npz"), words=np.array(words), vecs=vecs,
                        texts=np.array(texts), max_length=np.int32(10), emb=embs)


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(8)
    only = set(sys.argv[1:])
    if only:  # e.g. `gen_goldens.py margin` regenerates just those fixtures
        if "margin" in only:
            gen_margin(import_margin_reference())
        if "dp_step" in only:
            gen_dp_step(import_reference())
        return
    et = import_reference()
    gen_margin(import_margin_reference())
    gen_tiny_model(et)
    gen_tiny_train(et)
    gen_featurize(et)
    gen_losses(et)
    gen_dp(et)
    gen_dp_step(et)
    gen_mrr(et)
    gen_full(et, 300, 256, 64, 32, "full_h256_t64", 21)
    gen_full(et, 300, 512, 128, 8, "full_h512_t128", 22)
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
