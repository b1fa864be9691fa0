"""CPU ORACLE for the two-tower training step — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the timed CPU baseline. The product path
(two_towers_amd/) never calls it and has no CPU fallback.

A from-scratch restatement, in plain PyTorch-CPU with explicit GRU cell arithmetic
(no nn.GRU), of the reference algorithm in mateomarin/two_towers:
  - EnhancedTwoTowerModel            enhanced_two_tower.py:13-65
  - InfoNCELoss                      enhanced_two_tower.py:67-82
  - MarginRankingLoss                enhanced_two_tower.py:84-121
  - get_hard_negatives               enhanced_two_tower.py:123-133
  - EnhancedDataset.text_to_embedding enhanced_two_tower.py:144-166
  - the train_enhanced.py inner loop  train_enhanced.py:54-69 (Adam defaults)
  - margin TwoTowerModel              margin_two_tower.py:9-68 (shared projection head,
                                      compute_similarity), its InfoNCE :70-85 and
                                      SimpleDataset.text_to_embedding :96-153
  - MRR@10 of validate_enhanced.py    validate_enhanced.py:73-80,104-110
Pinned against golden vectors produced by running the reference itself
(oracle/gen_goldens.py -> tests/golden/*.npz; checked by tests/test_oracle_golden.py).

Dropout: the reference draws torch's RNG, which no other backend can reproduce. The
HIP path uses a counter-based mask keep(seed,row,col); `dropout_mask` restates it so
that dropout-on runs are checkable exactly. With p = 0 (or eval) both coincide with
the reference.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

# ---------------------------------------------------------------- dropout mask

def _u32(x):
    return np.asarray(x, dtype=np.uint64) & np.uint64(0xFFFFFFFF)


def tt_hash3(seed: int, row: np.ndarray, col: np.ndarray) -> np.ndarray:
    """Restates tt_hash3 in two_towers_amd/csrc/tt_common.h (uint32 wrap-around)."""
    m = np.uint64(0xFFFFFFFF)
    s = _u32(seed)
    r = _u32(row)
    c = _u32(col)
    h = ((s * np.uint64(0x9E3779B1)) & m) ^ ((r * np.uint64(0x85EBCA77)) & m) ^ \
        ((c * np.uint64(0xC2B2AE3D) + np.uint64(0x27D4EB2F)) & m)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x7FEB352D)) & m
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(0x846CA68B)) & m
    h ^= h >> np.uint64(16)
    return h


def dropout_mask(seed: int, rows: int, cols: int, p: float, row0: int = 0) -> np.ndarray:
    """Multiplier (0 or 1/(1-p)) for element (row, col); row = row0 + b*T + t, col in
    [0, 2H). row0 = rank * B * T on a data-parallel rank (tt_gru_fwd_rec.drop_row0)."""
    if p <= 0.0:
        return np.ones((rows, cols), dtype=np.float32)
    thresh = np.uint64(int(p * 16777216.0 + 0.5))
    r = np.arange(row0, row0 + rows, dtype=np.uint64)[:, None]
    c = np.arange(cols, dtype=np.uint64)[None, :]
    keep = (tt_hash3(seed, r, c) >> np.uint64(8)) >= thresh
    return np.where(keep, np.float32(1.0 / (1.0 - p)), np.float32(0.0)).astype(np.float32)

# ------------------------------------------------------------------- GRU math

def gru_direction(x: torch.Tensor, w_ih, w_hh, b_ih, b_hh, reverse: bool):
    """One direction of one nn.GRU layer (torch semantics, h0 = 0, no packing/masking).
    x [B, T, In] -> out [B, T, H]."""
    B, T, _ = x.shape
    H = w_hh.shape[1]
    gx = x @ w_ih.t() + b_ih  # [B, T, 3H]
    h = x.new_zeros(B, H)
    outs = [None] * T
    order = range(T - 1, -1, -1) if reverse else range(T)
    for t in order:
        gh = h @ w_hh.t() + b_hh
        xr, xz, xn = gx[:, t].split(H, dim=1)
        hr, hz, hn = gh.split(H, dim=1)
        r = torch.sigmoid(xr + hr)
        z = torch.sigmoid(xz + hz)
        n = torch.tanh(xn + r * hn)
        h = (1 - z) * n + z * h
        outs[t] = h
    return torch.stack(outs, 1)


def gru_encoder(x: torch.Tensor, p: dict, prefix: str, drop_p: float = 0.0, seed: int = 0):
    """2-layer bidirectional GRU (enhanced_two_tower.py:17-33). Returns h_n [4, B, H]
    in torch order (l0 fwd, l0 rev, l1 fwd, l1 rev) and the layer outputs."""
    B, T, _ = x.shape
    finals = []
    inp = x
    outs = []
    for layer in range(2):
        o = []
        for sfx, rev in (("", False), ("_reverse", True)):
            g = lambda n: p[f"{prefix}.{n}_l{layer}{sfx}"]
            od = gru_direction(inp, g("weight_ih"), g("weight_hh"), g("bias_ih"), g("bias_hh"), rev)
            o.append(od)
            finals.append(od[:, 0] if rev else od[:, T - 1])
        out = torch.cat(o, 2)
        outs.append(out)
        if layer == 0 and drop_p > 0.0:
            H2 = out.shape[2]
            m = torch.from_numpy(dropout_mask(seed, B * T, H2, drop_p)).to(out.dtype).view(B, T, H2)
            inp = out * m
        else:
            inp = out
    return torch.stack(finals, 0), outs


def proj_head(v: torch.Tensor, p: dict, prefix: str):
    """Linear(4h,2h) -> LayerNorm(2h) -> ReLU -> Linear(2h,h) (enhanced_two_tower.py:36-48)."""
    a = v @ p[f"{prefix}.0.weight"].t() + p[f"{prefix}.0.bias"]
    a = F.layer_norm(a, (a.shape[1],), p[f"{prefix}.1.weight"], p[f"{prefix}.1.bias"], 1e-5)
    a = torch.relu(a)
    return a @ p[f"{prefix}.3.weight"].t() + p[f"{prefix}.3.bias"]


def encode(x: torch.Tensor, p: dict, tower: str, drop_p: float = 0.0, seed: int = 0):
    """encode_query / encode_doc (enhanced_two_tower.py:50-60)."""
    enc = "query_encoder" if tower == "query" else "doc_encoder"
    proj = "query_proj" if tower == "query" else "doc_proj"
    hn, _ = gru_encoder(x, p, enc, drop_p, seed)
    v = torch.cat([hn[-2], hn[-1]], 1)
    return proj_head(v, p, proj)


def forward(q: torch.Tensor, d: torch.Tensor, p: dict, drop_p: float = 0.0, seeds=(0, 0)):
    """EnhancedTwoTowerModel.forward (enhanced_two_tower.py:62-65)."""
    return encode(q, p, "query", drop_p, seeds[0]), encode(d, p, "doc", drop_p, seeds[1])

# ------------------------------------------------------------- margin family

def margin_head(v: torch.Tensor, p: dict, drop_p: float = 0.0, seed: int = 0, row0: int = 0):
    """projection = Linear(2H,H) -> LayerNorm(H) -> ReLU -> Dropout (margin_two_tower.py:
    30-35), one set of weights for both towers. Dropout rows are counted from row0 in the
    query-then-doc stacking the HIP path uses."""
    a = v @ p["projection.0.weight"].t() + p["projection.0.bias"]
    a = F.layer_norm(a, (a.shape[1],), p["projection.1.weight"], p["projection.1.bias"], 1e-5)
    a = torch.relu(a)
    if drop_p > 0.0:
        m = dropout_mask(seed, row0 + a.shape[0], a.shape[1], drop_p)[row0:]
        a = a * torch.from_numpy(m).to(a.dtype)
    return a


def margin_encode(x: torch.Tensor, p: dict, tower: str, drop_p: float = 0.0, seed: int = 0):
    """TwoTowerModel.encode (margin_two_tower.py:58-62): cat(hidden[-2], hidden[-1])."""
    enc = "query_encoder" if tower == "query" else "doc_encoder"
    hn, _ = gru_encoder(x, p, enc, drop_p, seed)
    return margin_head(torch.cat([hn[-2], hn[-1]], 1), p)


def margin_forward(q: torch.Tensor, d: torch.Tensor, p: dict, training: bool):
    """TwoTowerModel.forward + compute_similarity (margin_two_tower.py:37-48, 64-68),
    dropout off: (normalize(q), normalize(d)) in training, qn dnᵀ in eval."""
    qn = normalize(margin_encode(q, p, "query"))
    dn = normalize(margin_encode(d, p, "doc"))
    return (qn, dn) if training else qn @ dn.t()


def margin_param_shapes(E: int, H: int):
    """state_dict layout of margin TwoTowerModel(E, H) (margin_two_tower.py:10-35)."""
    shapes = {}
    for enc in ("query_encoder", "doc_encoder"):
        for layer in range(2):
            inp = E if layer == 0 else 2 * H
            for sfx in ("", "_reverse"):
                shapes[f"{enc}.weight_ih_l{layer}{sfx}"] = (3 * H, inp)
                shapes[f"{enc}.weight_hh_l{layer}{sfx}"] = (3 * H, H)
                shapes[f"{enc}.bias_ih_l{layer}{sfx}"] = (3 * H,)
                shapes[f"{enc}.bias_hh_l{layer}{sfx}"] = (3 * H,)
    shapes["projection.0.weight"] = (H, 2 * H)
    shapes["projection.0.bias"] = (H,)
    shapes["projection.1.weight"] = (H,)
    shapes["projection.1.bias"] = (H,)
    return shapes


_MARGIN_RULES = (
    (r"\b(is|are|refers?\s+to)\s+(?:a|an|the)\b", "IS"),
    (r"\b(contains?|has|have|includes?)\b", "HAS"),
    (r"\b(part|component|element)\s+of\b", "PART_OF"),
    (r"\b(controls?|regulates?|manages?)\b", "CONTROLS"),
    (r"\b(functions?|works?|operates?)\b", "FUNCTIONS"),
    (r"(\d+(?:\.\d+)?)\s*([a-zA-Z]+)", r"\1_\2"),
)


def margin_text_to_ids(text: str, vocab: dict, max_length: int = 30):
    """SimpleDataset.text_to_embedding (margin_two_tower.py:96-153) as row ids: each rule
    is applied to the lower-cased result of the previous one; for processed word i the
    lookups are original word i, then processed word i when it differs; OOV lookups are
    skipped; one zero row if nothing was found; pad/truncate to max_length."""
    import re
    orig = text.lower().split()
    t = text
    for pat, rep in _MARGIN_RULES:
        t = re.sub(pat, rep, t.lower())
    ids = []
    for i, w in enumerate(t.split()):
        cands = ([orig[i]] if i < len(orig) else []) + ([w] if w != orig[i] else [])
        ids.extend(vocab[c] for c in cands if c in vocab)
    if not ids:
        ids = [-1]
    ids = ids[:max_length]
    return ids + [-1] * (max_length - len(ids))

def search_results(query_vec, doc_mat, docs, ground_truth, top_k=3):
    """The /search response body (server/python-api/app.py:94-115) for one encoded query:
    F.cosine_similarity against every cached row, top_k (ties: lower index first),
    text = first 200 chars + '...' when longer, is_ground_truth by text equality."""
    sims = F.cosine_similarity(query_vec.reshape(1, 1, -1), doc_mat.unsqueeze(0), dim=-1).reshape(-1)
    order = sorted(range(sims.shape[0]), key=lambda j: (-float(sims[j]), j))[:top_k]
    out = []
    for r, j in enumerate(order):
        text = docs[j][:200] + "..." if len(docs[j]) > 200 else docs[j]
        out.append({"text": text, "score": float(sims[j]), "is_ground_truth": docs[j] in ground_truth,
                    "rank": r + 1})
    return out

# ---------------------------------------------------------------------- losses

def normalize(x, eps=1e-12):
    """F.normalize(p=2) over the last dim: x / max(||x||, eps)."""
    return x / x.norm(dim=-1, keepdim=True).clamp_min(eps)


def infonce(q, d, temperature=0.07):
    """enhanced_two_tower.py:72-82."""
    qn, dn = normalize(q), normalize(d)
    s = qn @ dn.t() / temperature
    return F.cross_entropy(s, torch.arange(q.shape[0]))


def cosine(a, b, eps=1e-8):
    """F.cosine_similarity along the last dim."""
    return (normalize(a, eps) * normalize(b, eps)).sum(-1)


def margin_loss(q, pos, neg=None, margin=0.2, temperature=0.1):
    """MarginRankingLoss.forward (enhanced_two_tower.py:90-121)."""
    if neg is None:
        s = q @ pos.t() / temperature
        eye = torch.eye(q.shape[0], dtype=q.dtype)
        s = s - margin * (1 - eye)
        return F.cross_entropy(s, torch.arange(q.shape[0]))
    B = q.shape[0]
    k = neg.shape[0] // B
    pos_sim = cosine(q, pos)
    neg_sim = cosine(q.unsqueeze(1).expand(-1, k, -1), neg.view(B, k, -1)).mean(1)
    return torch.clamp(margin - pos_sim + neg_sim, min=0).mean()


def hard_negatives(qv, docs, positive_idx, k=5):
    """get_hard_negatives (enhanced_two_tower.py:123-133), ties -> lower index first."""
    with torch.no_grad():
        sims = cosine(qv.unsqueeze(0), docs)
        sims[positive_idx] = -1
        order = sorted(range(sims.shape[0]), key=lambda j: (-float(sims[j]), j))
        return torch.tensor(order[:k], dtype=torch.int64)


def hardneg_margin(q, d, k=5, margin=0.2):
    """The config-3 composition: per-row mining over the in-batch docs, then the
    explicit-negative MarginRankingLoss on the gathered rows."""
    idx = torch.stack([hard_negatives(q[i], d, i, k) for i in range(q.shape[0])])
    neg = d[idx.reshape(-1)]
    return margin_loss(q, d, neg, margin), idx

# ----------------------------------------------------------------- featurize

def text_to_ids(text: str, vocab: dict, max_length: int = 30):
    """EnhancedDataset.text_to_embedding (enhanced_two_tower.py:144-166) as row ids:
    truncate to max_length words BEFORE dropping OOV words, one zero row if none
    remain, pad with zero rows (-1) at the end."""
    words = text.lower().split()[:max_length]
    ids = [vocab[w] for w in words if w in vocab]
    if not ids:
        ids = [-1]
    ids = ids[:max_length]
    return ids + [-1] * (max_length - len(ids))


def ids_to_embedding(ids, table: np.ndarray) -> np.ndarray:
    out = np.zeros((len(ids), table.shape[1]), dtype=np.float32)
    for i, j in enumerate(ids):
        if j >= 0:
            out[i] = table[j]
    return out

# ------------------------------------------------------------------- training

def adam_steps(p: dict, batches, loss_fn, steps: int, lr=1e-3):
    """train_enhanced.py:58-63 with torch.optim.Adam defaults. Returns per-step losses."""
    params = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    opt = torch.optim.Adam(list(params.values()), lr=lr)
    losses = []
    for s in range(steps):
        q, d = batches[s % len(batches)]
        opt.zero_grad()
        loss = loss_fn(params, q, d)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    return losses, {k: v.detach() for k, v in params.items()}

# ------------------------------------------------------------------------ MRR

def mrr_at_10(query_vecs, doc_vecs, relevant):
    """validate_enhanced.py:73-80,104-110: cosine top-10, 1/rank of the first relevant."""
    sims = normalize(query_vecs, 1e-8) @ normalize(doc_vecs, 1e-8).t()
    total = 0.0
    for i in range(sims.shape[0]):
        order = sorted(range(sims.shape[1]), key=lambda j: (-float(sims[i, j]), j))[:10]
        rr = 0.0
        for rank, j in enumerate(order, 1):
            if j in relevant[i]:
                rr = 1.0 / rank
                break
        total += rr
    return total / sims.shape[0]

# ------------------------------------------------------- deterministic weights

def splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15))
    z = x
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def counter_uniform(seed: int, name: str, shape, bound: float) -> np.ndarray:
    """U(-bound, bound) from splitmix64(seed, crc(name), flat index): weights that both
    sides regenerate instead of shipping them."""
    import zlib
    n = int(np.prod(shape))
    with np.errstate(over="ignore"):
        key = np.uint64((seed * 1000003 + zlib.crc32(name.encode())) & 0xFFFFFFFFFFFFFFFF)
        x = splitmix64(np.arange(n, dtype=np.uint64) ^ splitmix64(np.array([key], dtype=np.uint64)))
    u = (x >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    return ((2.0 * u - 1.0) * bound).astype(np.float32).reshape(shape)


def reference_param_shapes(E: int, h: int):
    """state_dict layout of EnhancedTwoTowerModel(E, h) (enhanced_two_tower.py:13-48)."""
    H = 2 * h
    shapes = {}
    for enc in ("query_encoder", "doc_encoder"):
        for layer in range(2):
            inp = E if layer == 0 else 2 * H
            for sfx in ("", "_reverse"):
                shapes[f"{enc}.weight_ih_l{layer}{sfx}"] = (3 * H, inp)
                shapes[f"{enc}.weight_hh_l{layer}{sfx}"] = (3 * H, H)
                shapes[f"{enc}.bias_ih_l{layer}{sfx}"] = (3 * H,)
                shapes[f"{enc}.bias_hh_l{layer}{sfx}"] = (3 * H,)
    for proj in ("query_proj", "doc_proj"):
        shapes[f"{proj}.0.weight"] = (2 * h, 4 * h)
        shapes[f"{proj}.0.bias"] = (2 * h,)
        shapes[f"{proj}.1.weight"] = (2 * h,)
        shapes[f"{proj}.1.bias"] = (2 * h,)
        shapes[f"{proj}.3.weight"] = (h, 2 * h)
        shapes[f"{proj}.3.bias"] = (h,)
    return shapes


def counter_params(E: int, h: int, seed: int = 0) -> dict:
    """Procedural weights with PyTorch-default bounds (1/sqrt(fan)); LayerNorm affine
    around (1, 0) so that the norm path is exercised non-trivially."""
    out = {}
    H = 2 * h
    for name, shape in reference_param_shapes(E, h).items():
        if "encoder" in name:
            bound = 1.0 / math.sqrt(H)
            out[name] = torch.from_numpy(counter_uniform(seed, name, shape, bound))
        elif name.endswith(".1.weight"):
            out[name] = torch.from_numpy(1.0 + counter_uniform(seed, name, shape, 0.1))
        elif name.endswith(".1.bias"):
            out[name] = torch.from_numpy(counter_uniform(seed, name, shape, 0.1))
        else:
            fan = shape[1] if len(shape) == 2 else reference_param_shapes(E, h)[name.replace("bias", "weight")][1]
            out[name] = torch.from_numpy(counter_uniform(seed, name, shape, 1.0 / math.sqrt(fan)))
    return out
