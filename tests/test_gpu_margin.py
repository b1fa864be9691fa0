"""Margin model family (margin_two_tower.py) on the HIP path, against the golden vectors
made by running the reference (tests/golden/margin_tiny.npz) and against the oracle.

Tolerances: fp32 outputs 1e-4 relative (max-abs over max), gradients 2e-3 relative
(MFMA vs CPU accumulation order); bf16 towers: loss 2e-3 relative, gradient cosine
>= 0.998.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import two_towers_amd as tta  # noqa: E402
from oracle import cpu_ref  # noqa: E402
from two_towers_amd.margin import TwoTowerModel  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def golden_model():
    z = np.load(os.path.join(GOLD, "margin_tiny.npz"), allow_pickle=False)
    m = TwoTowerModel(16, 8)
    m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w.")})
    return z, m.to(DEV)


def test_margin_eval_similarity_and_encoders():
    z, m = golden_model()
    m.eval()
    q, d = torch.from_numpy(z["q"]).to(DEV), torch.from_numpy(z["d"]).to(DEV)
    with torch.no_grad():
        sim = m(q, d)
        eq = m.encode_query(q)
        ed = m.encode_doc(d)
    assert sim.shape == (12, 12)
    assert rel(sim, z["sim"]) < 1e-4
    assert rel(eq, z["enc_q"]) < 1e-4 and rel(ed, z["enc_d"]) < 1e-4


def test_margin_train_step_grads():
    """train_margin.py's step: InfoNCELoss(temperature=0.1) on the normalised pair, every
    dropout off (as the golden run)."""
    z, m = golden_model()
    m.train()
    m.query_encoder.dropout = 0.0
    m.doc_encoder.dropout = 0.0
    m.projection[3].p = 0.0
    qn, dn = m(torch.from_numpy(z["q"]).to(DEV), torch.from_numpy(z["d"]).to(DEV))
    loss = tta.InfoNCELoss(temperature=0.1)(qn, dn)
    loss.backward()
    assert rel(qn, z["qn"]) < 1e-4 and rel(dn, z["dn"]) < 1e-4
    assert abs(float(loss) - float(z["loss"])) < 1e-5 * max(1.0, abs(float(z["loss"])))
    for k, p in m.named_parameters():
        assert rel(p.grad, z[f"g.{k}"]) < 2e-3, k


@pytest.mark.parametrize("B,T,E,H", [(40, 6, 24, 16), (130, 9, 40, 64)])
def test_margin_dropout_matches_counter_masks(B, T, E, H):
    """GRU inter-layer dropout and the shared head's Dropout(0.1) both on: the oracle
    replays the counter masks from the seeds the model drew (2 tower seeds, then the
    head seed, from torch's CPU generator)."""
    torch.manual_seed(3)
    m = TwoTowerModel(E, H)
    p = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    m = m.to(DEV).train()
    g = torch.Generator().manual_seed(19)
    q = torch.randn(B, T, E, generator=g)
    d = torch.randn(B, T, E, generator=g)
    torch.manual_seed(123)
    qn, dn = m(q.to(DEV), d.to(DEV))
    loss = tta.InfoNCELoss(temperature=0.1)(qn, dn)
    loss.backward()
    torch.manual_seed(123)
    s = [int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) for _ in range(3)]
    hq, _ = cpu_ref.gru_encoder(q, p, "query_encoder", 0.1, s[0])
    hd, _ = cpu_ref.gru_encoder(d, p, "doc_encoder", 0.1, s[1])
    v = torch.cat([torch.cat([hq[-2], hq[-1]], 1), torch.cat([hd[-2], hd[-1]], 1)], 0)
    out = cpu_ref.margin_head(v, p, 0.1, s[2])
    rq, rd = cpu_ref.normalize(out[:B]), cpu_ref.normalize(out[B:])
    rl = cpu_ref.infonce(rq, rd, temperature=0.1)
    rl.backward()
    assert rel(qn, rq) < 1e-4 and rel(dn, rd) < 1e-4
    assert abs(float(loss) - float(rl)) < 1e-4 * max(1.0, abs(float(rl)))
    named = dict(m.named_parameters())
    worst = {k: rel(named[k].grad, p[k].grad) for k in p}
    assert max(worst.values()) < 2e-3, worst


def test_margin_bf16_towers_and_token_ids():
    """bf16 GRU towers fed by the GPU gather of margin_ids rows vs the fp32 oracle on
    the same bf16-rounded weights and table."""
    V, E, H, B, T = 300, 32, 64, 48, 10
    torch.manual_seed(5)
    m = TwoTowerModel(E, H)
    with torch.no_grad():
        for prm in m.parameters():
            prm.copy_(prm.to(torch.bfloat16).float())
    p = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(20)
    table = torch.randn(V, E, generator=g).to(torch.bfloat16).float()
    ids = torch.randint(-1, V, (2, B, T), generator=g, dtype=torch.int32)
    m = m.to(DEV).eval().set_compute_dtype(torch.bfloat16).set_embedding_table(table.to(DEV))
    m.train()
    m.query_encoder.dropout = 0.0
    m.doc_encoder.dropout = 0.0
    m.projection[3].p = 0.0
    qn, dn = m(ids[0].to(DEV), ids[1].to(DEV))
    loss = tta.InfoNCELoss(temperature=0.1)(qn, dn)
    loss.backward()

    def emb(x):
        e = table[x.clamp_min(0).long()]
        return e * (x >= 0).unsqueeze(-1).float()

    rq, rd = cpu_ref.margin_forward(emb(ids[0]), emb(ids[1]), p, training=True)
    rl = cpu_ref.infonce(rq, rd, temperature=0.1)
    rl.backward()
    assert abs(float(loss) - float(rl)) < 2e-3 * abs(float(rl))
    named = dict(m.named_parameters())
    for k in p:
        a, b = named[k].grad.double().cpu(), p[k].grad.double()
        cos = float((a * b).sum() / (a.norm() * b.norm() + 1e-30))
        assert cos >= 0.998, (k, cos)


def test_gru_width_must_be_multiple_of_8():
    m = TwoTowerModel(16, 12).to(DEV)
    with pytest.raises(ValueError, match="multiple of 8"):
        m.encode_query(torch.randn(2, 3, 16, device=DEV))


def test_margin_adam_steps_match_oracle():
    """train_margin.py:21-45 inner loop (Adam lr 1e-3, InfoNCE 0.1), 5 steps, dropout off."""
    torch.manual_seed(6)
    m = TwoTowerModel(16, 16)
    p0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV).train()
    m.query_encoder.dropout = 0.0
    m.doc_encoder.dropout = 0.0
    m.projection[3].p = 0.0
    g = torch.Generator().manual_seed(21)
    batches = [(torch.randn(24, 7, 16, generator=g), torch.randn(24, 7, 16, generator=g)) for _ in range(2)]
    opt = tta.Adam(m.parameters(), lr=1e-3)
    crit = tta.InfoNCELoss(temperature=0.1)
    losses = []
    for s in range(5):
        q, d = batches[s % 2]
        opt.zero_grad()
        loss = crit(*m(q.to(DEV), d.to(DEV)))
        loss.backward()
        opt.step()
        losses.append(float(loss))
    ref_losses, final = cpu_ref.adam_steps(
        p0, batches, lambda prm, q, d: cpu_ref.infonce(*cpu_ref.margin_forward(q, d, prm, True), temperature=0.1), 5)
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-4)
    sd = m.state_dict()
    for k, v in final.items():
        assert rel(sd[k], v) < 1e-3, k
