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
