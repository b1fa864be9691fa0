"""End-to-end data path on the GPU: word2vec .bin -> flat store -> pre-tokenized pair ids
-> train driver (both model families) -> checkpoint -> /search index."""
import struct

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from two_towers_amd import pretok, train, w2v  # noqa: E402
from two_towers_amd.margin import TwoTowerModel  # noqa: E402
from two_towers_amd.model import EnhancedTwoTowerModel  # noqa: E402
from two_towers_amd.serving import SearchIndex  # noqa: E402


def make_inputs(tmp_path, E=16, V=120, n=96):
    rng = np.random.default_rng(0)
    words = [f"t{i}" for i in range(V)]
    with open(tmp_path / "w2v.bin", "wb") as f:
        f.write(f"{V} {E}\n".encode())
        for w in words:
            f.write(w.encode() + b" " + struct.pack(f"<{E}f", *rng.standard_normal(E)) + b"\n")
    vocab = w2v.read_word2vec_format(str(tmp_path / "w2v.bin"))
    w2v.save_store(vocab, str(tmp_path / "store"))
    docs = [" ".join(f"t{x}" for x in rng.integers(0, V, 12)) for _ in range(n)]
    queries = [" ".join(d.split()[:3]) for d in docs]
    with open(tmp_path / "pairs.tsv", "w") as f:
        for q, d in zip(queries, docs):
            f.write(f"{q}\t{d}\n")
    return vocab, queries, docs


@pytest.mark.parametrize("family", ["enhanced", "margin"])
def test_pretokenized_training_and_search(tmp_path, family):
    vocab, queries, docs = make_inputs(tmp_path)
    tok = "margin" if family == "margin" else "enhanced"
    pretok.main(["--vocab", str(tmp_path / "store"), "--pairs", str(tmp_path / "pairs.tsv"), "--out",
                 str(tmp_path / "ids"), "--max-length", "12", "--tokenizer", tok, "--workers", "2"])
    out = train.main(["--model", family, "--ids", str(tmp_path / "ids"), "--vocab", str(tmp_path / "store"),
                      "--output_dir", str(tmp_path / "out"), "--num_epochs", "3", "--batch_size", "32",
                      "--hidden_dim", "16", "--log_every", "1"])
    ck = torch.load(f"{out}/best_model.pt", map_location="cpu", weights_only=True)
    if family == "margin":
        assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "loss"}
        m = TwoTowerModel(16, 16)
        m.load_state_dict(ck["model_state_dict"])
    else:
        m = EnhancedTwoTowerModel(16, 16)
        m.load_state_dict(ck)
    log = open(f"{out}/training.log").read()
    losses = [float(x.split("Average Loss: ")[1].split()[0]) for x in log.splitlines() if "Average Loss" in x]
    assert len(losses) == 3 and all(np.isfinite(losses))
    m = m.cuda().eval()
    index = SearchIndex(m, vocab, docs, queries=queries, paired_docs=docs, max_length=12,
                        tokenize=pretok._tokenizer(tok))
    res = index.search(queries[0])
    assert [r["rank"] for r in res["results"]] == [1, 2, 3]
    scores = [r["score"] for r in res["results"]]
    assert scores == sorted(scores, reverse=True) and -1.0001 <= scores[-1] <= scores[0] <= 1.0001


def test_bin_store_ids_and_device_gather_match_reference_featurization(tmp_path):
    """The whole data path pinned to the reference's own featurisation (featurize.npz,
    EnhancedDataset.text_to_embedding run by oracle/gen_goldens.py, and margin_featurize.npz,
    SimpleDataset): the fixture's word vectors written as word2vec.c binary bytes (header
    "V E\\n", then "word " + E little-endian float32 + "\\n" per row), read back, saved as the
    flat store, the texts pre-tokenized into id files, and the ids gathered on the GPU by
    tt_embed_gather through the model's table: every [T, E] row equals the reference's,
    bit for bit (fp32)."""
    import os

    from two_towers_amd import ops
    gold = os.path.join(os.path.dirname(__file__), "golden")
    for fixture, tok in (("featurize", "enhanced"), ("margin_featurize", "margin")):
        z = np.load(os.path.join(gold, fixture + ".npz"), allow_pickle=False)
        words, vecs = [str(w) for w in z["words"]], z["vecs"].astype(np.float32)
        V, E = vecs.shape
        path = tmp_path / f"{tok}.bin"
        with open(path, "wb") as f:
            f.write(f"{V} {E}\n".encode())
            for w, v in zip(words, vecs):
                f.write(w.encode("utf-8") + b" " + struct.pack(f"<{E}f", *v) + b"\n")
        vocab = w2v.read_word2vec_format(str(path))
        assert [w for w, _ in sorted(vocab.index.items(), key=lambda kv: kv[1])] == words
        assert np.array_equal(vocab.vectors, vecs)
        w2v.save_store(vocab, str(tmp_path / f"store_{tok}"))
        store = w2v.load_store(str(tmp_path / f"store_{tok}"))
        texts = [str(t) for t in z["texts"]]
        T = int(z["max_length"])
        pretok.pretokenize(texts, texts, store, str(tmp_path / f"ids_{tok}"), T, tok, workers=1)
        ds = pretok.PairIds(str(tmp_path / f"ids_{tok}"), store)
        ids = torch.stack([ds[i][0] for i in range(len(ds))]).cuda()
        m = EnhancedTwoTowerModel(E, 4).cuda()
        m.set_embedding_table(torch.from_numpy(np.array(store.vectors)).cuda())
        tab = m._device_table(ids.device)
        out = torch.empty(ids.numel(), tab.shape[1], device="cuda")
        ops.embed_gather(tab, ids.reshape(-1).to(torch.int32).contiguous(), out)
        got = out[:, :E].reshape(len(texts), T, E).cpu().numpy()
        np.testing.assert_array_equal(got, z["emb"])
