"""Pins the CPU oracle (oracle/cpu_ref.py) against golden vectors produced by running
the reference itself (oracle/gen_goldens.py). CPU only."""
import os

import numpy as np
import pytest
import torch

from oracle import cpu_ref

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)


def params(z, prefix):
    return {k[len(prefix):]: torch.from_numpy(z[k]).clone() for k in z.files if k.startswith(prefix)}


def close(a, b, rtol=1e-5, atol=1e-6):
    np.testing.assert_allclose(np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64), rtol=rtol, atol=atol)


def test_tiny_model():
    z = load("tiny_model")
    p = {k: v.requires_grad_(True) for k, v in params(z, "w.").items()}
    qv, dv = cpu_ref.forward(torch.from_numpy(z["q"]), torch.from_numpy(z["d"]), p)
    loss = cpu_ref.infonce(qv, dv)
    loss.backward()
    close(qv.detach(), z["q_vec"])
    close(dv.detach(), z["d_vec"])
    close(float(loss), z["loss"])
    for k, t in p.items():
        close(t.grad, z[f"g.{k}"], rtol=1e-4, atol=1e-6)


def test_tiny_train_adam():
    z = load("tiny_train")
    p = params(z, "w0.")
    batches = [(torch.from_numpy(z["bq"][i]), torch.from_numpy(z["bd"][i])) for i in range(4)]
    losses, final = cpu_ref.adam_steps(p, batches, lambda prm, q, d: cpu_ref.infonce(*cpu_ref.forward(q, d, prm)), 20)
    close(losses, z["losses"], rtol=1e-4)
    for k, v in final.items():
        close(v, z[f"w20.{k}"], rtol=1e-3, atol=1e-6)


def test_featurize():
    z = load("featurize")
    vocab = {str(w): i for i, w in enumerate(z["words"])}
    T = int(z["max_length"])
    for text, emb in zip(z["texts"], z["emb"]):
        ids = cpu_ref.text_to_ids(str(text), vocab, T)
        np.testing.assert_array_equal(cpu_ref.ids_to_embedding(ids, z["vecs"]), emb)


@pytest.mark.parametrize("B", [8, 64, 256])
def test_losses(B):
    z = load("losses")
    q, d, n = (torch.from_numpy(z[f"{c}{B}"]) for c in "qdn")
    for name, fn, args in (("infonce", cpu_ref.infonce, (q, d)), ("margin_inbatch", cpu_ref.margin_loss, (q, d)),
                           ("margin_explicit", cpu_ref.margin_loss, (q, d, n))):
        ts = [a.clone().requires_grad_(True) for a in args]
        loss = fn(*ts)
        loss.backward()
        close(float(loss), z[f"{name}{B}.loss"], rtol=1e-5)
        for i, t in enumerate(ts):
            close(t.grad, z[f"{name}{B}.grad{i}"], rtol=1e-4, atol=1e-7)
    k = 5 if B > 8 else 3
    qs, ds = q.clone().requires_grad_(True), d.clone().requires_grad_(True)
    loss, idx = cpu_ref.hardneg_margin(qs, ds, k)
    loss.backward()
    np.testing.assert_array_equal(idx.numpy(), z[f"hardneg{B}.idx"])
    close(float(loss), z[f"hardneg{B}.loss"])
    close(qs.grad, z[f"hardneg{B}.grad0"], atol=1e-7)
    close(ds.grad, z[f"hardneg{B}.grad1"], atol=1e-7)


def test_dp_equiv_batch():
    z = load("dp_equiv")
    p = {k: v.requires_grad_(True) for k, v in params(z, "w.").items()}
    loss = cpu_ref.infonce(*cpu_ref.forward(torch.from_numpy(z["q"]), torch.from_numpy(z["d"]), p))
    loss.backward()
    close(float(loss), z["loss"])
    for k, t in p.items():
        close(t.grad, z[f"g.{k}"], rtol=1e-4, atol=1e-6)


def test_reference_size_h256():
    z = load("full_h256_t64")
    E, h, seed = int(z["E"]), int(z["h"]), int(z["seed"])
    p = {k: v.requires_grad_(True) for k, v in cpu_ref.counter_params(E, h, seed).items()}
    q = torch.from_numpy(z["q"].astype(np.float32))
    d = torch.from_numpy(z["d"].astype(np.float32))
    qv, dv = cpu_ref.forward(q, d, p)
    loss = cpu_ref.infonce(qv, dv)
    loss.backward()
    close(qv.detach(), z["q_vec"], rtol=1e-4, atol=1e-5)
    close(float(loss), z["loss"], rtol=1e-5)
    for k, t in p.items():
        close(float(t.grad.norm()), z[f"gnorm.{k}"], rtol=1e-4)


def test_mrr_synth():
    z = load("mrr_synth")
    p = params(z, "w.")
    vocab = {str(w): i for i, w in enumerate(z["words"])}
    enc = lambda texts, kind: cpu_ref.encode(
        torch.from_numpy(np.stack([cpu_ref.ids_to_embedding(cpu_ref.text_to_ids(str(t), vocab, 30), z["vecs"])
                                   for t in texts])), p, kind)
    with torch.no_grad():
        dv = enc(z["docs"], "doc")
        qv = enc(z["queries"], "query")
    close(dv, z["doc_enc"], rtol=1e-4, atol=1e-5)
    mrr = cpu_ref.mrr_at_10(qv, dv, [{int(r)} for r in z["rel"]])
    assert abs(mrr - float(z["mrr"])) <= 0.002, (mrr, float(z["mrr"]))


def test_dropout_mask_statistics_and_determinism():
    m1 = cpu_ref.dropout_mask(7, 512, 64, 0.1)
    m2 = cpu_ref.dropout_mask(7, 512, 64, 0.1)
    m3 = cpu_ref.dropout_mask(8, 512, 64, 0.1)
    np.testing.assert_array_equal(m1, m2)
    assert (m1 != m3).any()
    frac = float((m1 == 0).mean())
    assert 0.09 < frac < 0.11
    assert set(np.unique(m1)) == {0.0, np.float32(1 / 0.9)}


def test_margin_model():
    """oracle.margin_* vs margin_two_tower.TwoTowerModel(16, 8) run by gen_goldens.py."""
    z = load("margin_tiny")
    p = {k: v.requires_grad_(True) for k, v in params(z, "w.").items()}
    assert set(p) == set(cpu_ref.margin_param_shapes(16, 8))
    q, d = torch.from_numpy(z["q"]), torch.from_numpy(z["d"])
    with torch.no_grad():
        close(cpu_ref.margin_forward(q, d, p, training=False), z["sim"])
        close(cpu_ref.margin_encode(q, p, "query"), z["enc_q"])
        close(cpu_ref.margin_encode(d, p, "doc"), z["enc_d"])
    qn, dn = cpu_ref.margin_forward(q, d, p, training=True)
    loss = cpu_ref.infonce(qn, dn, temperature=0.1)
    loss.backward()
    close(qn.detach(), z["qn"])
    close(dn.detach(), z["dn"])
    close(float(loss), z["loss"])
    for k, t in p.items():
        close(t.grad, z[f"g.{k}"], rtol=1e-4, atol=1e-6)


def test_margin_featurize():
    z = load("margin_featurize")
    vocab = {str(w): i for i, w in enumerate(z["words"])}
    T = int(z["max_length"])
    for text, emb in zip(z["texts"], z["emb"]):
        ids = cpu_ref.margin_text_to_ids(str(text), vocab, T)
        np.testing.assert_array_equal(cpu_ref.ids_to_embedding(ids, z["vecs"]), emb)


@pytest.mark.parametrize("loss", ["infonce", "hardneg"])
def test_dp_step(loss):
    """One full step (loss, 44 gradients, Adam update) of the global batch the DP test
    splits over ranks: the oracle reproduces the reference run (dp_step.npz)."""
    z = load("dp_step")
    p = {k: v.requires_grad_(True) for k, v in params(z, "w.").items()}
    qv, dv = cpu_ref.forward(torch.from_numpy(z["q"]), torch.from_numpy(z["d"]), p)
    if loss == "infonce":
        lv = cpu_ref.infonce(qv, dv)
    else:
        lv, idx = cpu_ref.hardneg_margin(qv, dv, 5, 0.2)
        np.testing.assert_array_equal(idx.numpy(), z["hardneg.idx"])
    close(float(lv), z[f"{loss}.loss"], rtol=1e-5)
    opt = torch.optim.Adam(list(p.values()), lr=1e-3)
    lv.backward()
    for k, t in p.items():  # max-abs error relative to the largest entry
        ref = z[f"{loss}.g.{k}"]
        assert float((t.grad - torch.from_numpy(ref)).abs().max()) <= 1e-4 * float(np.abs(ref).max()) + 1e-9, k
    opt.step()
    # Adam's first step is ~lr * sign(g): where |g| is near eps the update is sensitive
    # to the gradient's last bits, so the weights are compared to 1 % of lr
    for k, t in p.items():
        close(t.detach(), z[f"{loss}.w1.{k}"], rtol=0, atol=1e-5)


def test_aten_reference_path_matches_goldens():
    """oracle/aten_ref.py (the reference's ATen modules: nn.GRU, nn.Linear, nn.LayerNorm,
    the loss compositions) reproduces the reference run: it is the timed CPU baseline."""
    from oracle import aten_ref
    z = load("tiny_model")
    m = aten_ref.AtenTwoTower(16, 8).eval()
    m.load_state_dict({k: v for k, v in params(z, "w.").items()})
    qv, dv = m(torch.from_numpy(z["q"]), torch.from_numpy(z["d"]))
    loss = aten_ref.infonce(qv, dv)
    loss.backward()
    close(qv.detach(), z["q_vec"])
    close(float(loss), z["loss"])
    for k, p in m.named_parameters():
        close(p.grad, z[f"g.{k}"], rtol=1e-4, atol=1e-6)
    z = load("dp_step")
    m = aten_ref.AtenTwoTower(16, 8).eval()
    m.load_state_dict({k: v for k, v in params(z, "w.").items()})
    loss = aten_ref.hardneg_margin(*m(torch.from_numpy(z["q"]), torch.from_numpy(z["d"])))
    close(float(loss), z["hardneg.loss"], rtol=1e-5)


def test_dropout_mask_row_offset_is_a_slice_of_the_global_mask():
    """A data-parallel rank's mask rows (row0 = rank * B * T) are its slice of the
    single-process mask of the global batch, and different ranks get different masks."""
    full = cpu_ref.dropout_mask(1234, 4 * 60, 32, 0.1)
    for r in range(4):
        np.testing.assert_array_equal(cpu_ref.dropout_mask(1234, 60, 32, 0.1, row0=r * 60), full[r * 60:(r + 1) * 60])
    assert not np.array_equal(full[:60], full[60:120])
