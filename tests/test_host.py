"""Host-side logic on CPU: module surface, featurisation, data formats, C-ABI exports,
and that the product path refuses to run without the GPU."""
import os
import re

import numpy as np
import pytest
import torch

import two_towers_amd as tta
from oracle import cpu_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def test_state_dict_matches_reference_layout():
    m = tta.EnhancedTwoTowerModel(300, 256)
    ref = cpu_ref.reference_param_shapes(300, 256)
    sd = m.state_dict()
    assert sorted(sd) == sorted(ref) and len(sd) == 44
    for k, shp in ref.items():
        assert tuple(sd[k].shape) == shp, k
    assert sum(v.numel() for v in sd.values()) == 15_764_992
    assert tta.EnhancedTwoTower is tta.EnhancedTwoTowerModel


def test_same_init_as_reference_for_same_seed():
    # tiny_model.npz holds the reference's weights for torch.manual_seed(0), (16, 8)
    z = np.load(os.path.join(GOLD, "tiny_model.npz"))
    torch.manual_seed(0)
    m = tta.EnhancedTwoTowerModel(16, 8)
    for k, v in m.state_dict().items():
        np.testing.assert_array_equal(v.numpy(), z[f"w.{k}"], err_msg=k)


def test_enhanced_dataset_and_ids_match_reference():
    z = np.load(os.path.join(GOLD, "featurize.npz"))
    words = [str(w) for w in z["words"]]
    w2v = {w: z["vecs"][i] for i, w in enumerate(words)}

    class KV(dict):
        vector_size = z["vecs"].shape[1]

    T = int(z["max_length"])
    texts = [str(t) for t in z["texts"]]
    ds = tta.EnhancedDataset(texts, texts, KV(w2v), max_length=T)
    vocab = tta.Vocab(words, z["vecs"])
    for i, t in enumerate(texts):
        np.testing.assert_array_equal(ds[i][0].numpy(), z["emb"][i])
        ids = tta.encode_ids(t, vocab, T)
        assert len(ids) == T
        np.testing.assert_array_equal(cpu_ref.ids_to_embedding(ids, z["vecs"]), z["emb"][i])


def test_vocab_roundtrip(tmp_path):
    v = tta.Vocab(["a", "b", "c"], np.arange(6, dtype=np.float32).reshape(3, 2))
    path = str(tmp_path / "w2v.npz")
    v.save(path)
    w = tta.Vocab.load(path)
    assert w.index == v.index
    np.testing.assert_array_equal(w.vectors, v.vectors)
    assert tta.encode_ids("B zzz a", w, 4) == [1, 0, -1, -1]
    assert tta.encode_ids("zzz", w, 3) == [-1, -1, -1]


def test_msmarco_pairing_rule():
    samples = [
        {"query": "q1", "passages": {"passage_text": ["p1", "p2", "p3"], "is_selected": [0, 1, 1]}},
        {"query": "", "passages": {"passage_text": ["x"], "is_selected": [1]}},
        {"query": "q3"},
        {"query": "q4", "passages": {"passage_text": ["p4"], "is_selected": [0]}},
    ]
    assert tta.pairs_from_msmarco(samples) == (["q1", "q1"], ["p2", "p3"])


def header_functions():
    text = open(os.path.join(ROOT, "include", "tt_hip.h")).read()
    return sorted(set(re.findall(r"^(?:int|long|const char\*)\s+(tt_\w+)\(", text, re.M)))


def test_library_exports_every_header_symbol():
    from two_towers_amd import _lib
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(_lib.EXPORTED), set(names) ^ set(_lib.EXPORTED)
    assert lib.tt_version().decode().startswith("tt_hip")


def test_variant_switch_defaults_and_roundtrip():
    """The kernel-variant switches (tt_set_option / tt_get_option, host-only) default to the
    measured-fastest forms the bench and DESIGN.md quote, set and read back, and an unknown
    name is an error, not a silent no-op."""
    from two_towers_amd import _lib
    expect = {"gru_fwd_xc": 1, "gru_fwd_xs": 1, "gru_xc_coop": 0, "gemm_persist": 1, "gemm_bres": 1,
              "gemm_iepi": 1, "bres_rows": 32, "hn_scan_v": 5, "hn_map": 2, "hn_scan_gemm": 0, "hn_gemm": 0,
              "gemm_stream_out": 1, "gru_bwd_persist": 1}
    got = {k: _lib.get_option(k) for k in expect}
    assert got == expect, got
    old = _lib.set_option("hn_scan_v", 0)
    try:
        assert old == 5 and _lib.get_option("hn_scan_v") == 0
    finally:
        _lib.set_option("hn_scan_v", old)
    with pytest.raises(RuntimeError):
        _lib.set_option("no_such_switch", 1)


def test_library_links_no_vendor_math_library():
    """Every kernel on the path is hand-written (north star: no dual backends): the shared
    library's dynamic dependencies name no vendor BLAS / DNN / GEMM library."""
    import subprocess
    from two_towers_amd import _lib
    out = subprocess.run(["readelf", "-d", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    needed = [ln.split("[")[1].rstrip("]") for ln in out.splitlines() if "(NEEDED)" in ln]
    assert needed, out
    vendor = [n for n in needed if any(v in n for v in ("blas", "MIOpen", "miopen", "rocsparse", "hipsparse", "ck_"))]
    assert not vendor, needed


def test_library_has_no_unprotected_wide_buffer_stores():
    """No 16/12-byte buffer store in the built gfx950 code takes its soffset from a
    register: LLVM inserts no wait states for that form, and a VALU write of the store's
    data right after it corrupted the persistent GRU forward's saved gh_n in round 2
    (tools/check_store_hazard.py)."""
    import importlib.util
    from two_towers_amd import _lib
    if not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"):
        pytest.skip("llvm-objdump not available")
    spec = importlib.util.spec_from_file_location("chk", os.path.join(ROOT, "tools", "check_store_hazard.py"))
    chk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(chk)
    text = chk.disassemble(_lib.LIB_PATH)
    assert "gru_fwd_seq" in text and "buffer_store_dwordx4" in text
    reg_soff, hazards = chk.scan(text)
    assert not hazards, hazards[:3]
    assert not reg_soff, reg_soff[:3]
    # the scanner itself flags the round-2 sequence
    old = ("_Z3fooPv:\n\tbuffer_store_dwordx4 v[0:3], v158, s[40:43], s61 offen\n"
           "\tv_mov_b32_e32 v0, v22\n")
    r, h = chk.scan(old)
    assert len(r) == 1 and len(h) == 1


def test_bad_arguments_are_reported_not_launched():
    from two_towers_amd import _lib
    lib = _lib.load()
    rc = lib.tt_gemm(7, 0, 0, 0, 4, 4, 4, None, 1, 4, 4, 4, 1.0, 0, 0, 0, 0, 0.0, 1, None, None)
    assert rc == _lib.TT_EINVAL
    assert "dtype" in lib.tt_last_error().decode()
    assert lib.tt_adam_multi(None, None, None, None, None, 0, 1e-3, 0.9, 0.999, 1e-8, 0.0, 0, None, None) == _lib.TT_EINVAL


def test_product_path_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    m = tta.EnhancedTwoTowerModel(16, 8)
    with pytest.raises(RuntimeError, match="GPU"):
        m(torch.randn(2, 3, 16), torch.randn(2, 3, 16))
    with pytest.raises(RuntimeError, match="GPU"):
        tta.InfoNCELoss()(torch.randn(4, 8), torch.randn(4, 8))
    with pytest.raises(RuntimeError, match="GPU"):
        tta.get_hard_negatives(torch.randn(8), torch.randn(10, 8), 0)


def test_oracle_is_not_imported_by_the_product():
    import ast
    pkg = os.path.join(ROOT, "two_towers_amd")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            tree = ast.parse(open(os.path.join(pkg, f)).read())
            for node in ast.walk(tree):
                if isinstance(node, (ast.Import, ast.ImportFrom)):
                    mods = [a.name for a in node.names] if isinstance(node, ast.Import) else [node.module or ""]
                    assert not any(m.startswith("oracle") for m in mods), f


def test_embedding_rows_are_padded_to_whole_lines():
    """Gathered embedding rows (and W_ih l0's K) are padded to 128-byte lines, so every
    layer-0 GEMM K-tile starts on a cache line and the padding adds no K-tile."""
    from two_towers_amd import ops
    assert ops.pad_cols(300, torch.bfloat16) == 320 and ops.pad_cols(300, torch.float32) == 320
    assert ops.pad_cols(64, torch.bfloat16) == 64 and ops.pad_cols(65, torch.bfloat16) == 128
    for e in (1, 48, 300, 301, 512):
        for dt in (torch.bfloat16, torch.float32):
            ep = ops.pad_cols(e, dt)
            esz = 2 if dt == torch.bfloat16 else 4
            assert ep >= e and (ep * esz) % 128 == 0 and (ep - e) * esz < 128


def test_split_k_picker_fills_the_chip():
    """Host-side launch heuristics: a small-M/N, long-K weight gradient (the projection
    head's dW, 8 or 32 tiles) must be split over K; big problems are not split."""
    from two_towers_amd import _lib
    lib = _lib.load()
    for m, n, k in [(256, 512, 8192), (512, 1024, 8192), (1536, 1024, 524288)]:
        s = lib.tt_gemm_pick_splits(m, n, k, 1)
        assert s > 1, (m, n, k, s)
        assert k // s >= 64 * 8 or s == 1
    assert lib.tt_gemm_pick_splits(524288, 3072, 1024, 2) == 1
    # one-split calls need no workspace (no library path: every GEMM is hand-written)
    assert lib.tt_gemm_ws_size(524288, 3072, 2, 1) == 0
    assert lib.tt_gemm_ws_size(1536, 1024, 4, 8) == 1536 * 1024 * 4 * 8
    assert lib.tt_gru_fwd_launches(1, 64, 512) == 1 and lib.tt_gru_fwd_launches(0, 64, 512) == 64


def test_margin_dataset_matches_reference_fixture():
    """two_towers_amd.margin.SimpleDataset / margin_ids vs margin_two_tower.SimpleDataset
    (tests/golden/margin_featurize.npz, made by oracle/gen_goldens.py)."""
    import numpy as np

    from two_towers_amd.margin import SimpleDataset, margin_ids
    from two_towers_amd.data import Vocab
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "margin_featurize.npz"), allow_pickle=False)
    words = [str(w) for w in z["words"]]
    vocab = Vocab(words, z["vecs"])
    T = int(z["max_length"])
    for text, emb in zip(z["texts"], z["emb"]):
        text = str(text)
        np.testing.assert_array_equal(SimpleDataset.text_to_embedding(text, vocab, T).numpy(), emb)
        ids = margin_ids(text, vocab, T)
        rows = np.stack([z["vecs"][i] if i >= 0 else np.zeros(z["vecs"].shape[1], np.float32) for i in ids])
        np.testing.assert_array_equal(rows, emb)


def test_margin_model_state_dict_matches_reference_layout():
    import torch

    from oracle import cpu_ref
    from two_towers_amd.margin import TwoTowerModel
    m = TwoTowerModel(300, 512)
    sd = m.state_dict()
    shapes = cpu_ref.margin_param_shapes(300, 512)
    assert {k: tuple(v.shape) for k, v in sd.items()} == shapes
    torch.manual_seed(0)
    a = TwoTowerModel(16, 8).state_dict()
    torch.manual_seed(0)
    b = TwoTowerModel(16, 8).state_dict()
    assert all(torch.equal(a[k], b[k]) for k in a)


def test_search_response_formatting():
    """serving.format_results / snippet / query_to_docs_map restate app.py:30-36,104-115."""
    from two_towers_amd.serving import format_results, query_to_docs_map, snippet
    long = "x" * 250
    assert snippet(long) == "x" * 200 + "..." and snippet("short") == "short" and snippet("y" * 200) == "y" * 200
    docs = ["alpha doc", long, "gamma", "alpha doc"]
    m = query_to_docs_map(["q1", "q2", "q1"], ["alpha doc", "gamma", long])
    assert m == {"q1": ["alpha doc", long], "q2": ["gamma"]}
    res = format_results(docs, m["q1"], [1, 2, 3], [0.9, 0.5, 0.25])
    assert res == [{"text": "x" * 200 + "...", "score": 0.9, "is_ground_truth": True, "rank": 1},
                   {"text": "gamma", "score": 0.5, "is_ground_truth": False, "rank": 2},
                   {"text": "alpha doc", "score": 0.25, "is_ground_truth": True, "rank": 3}]
    # the oracle's restatement agrees on the same ranking
    q = torch.tensor([1.0, 0.0])
    mat = torch.tensor([[0.1, 1.0], [1.0, 0.1], [1.0, 1.0], [-1.0, 0.0]])
    ref = cpu_ref.search_results(q, mat, docs, m["q1"], 3)
    assert [r["rank"] for r in ref] == [1, 2, 3] and [r["text"] for r in ref] == ["x" * 200 + "...", "gamma",
                                                                                  "alpha doc"]


def test_search_http_contract():
    """make_app: POST /search request/response models of app.py:72-123, 500 on errors."""
    from fastapi.testclient import TestClient

    from two_towers_amd.serving import make_app

    class FakeIndex:
        def search(self, query):
            if query == "boom":
                raise RuntimeError("kaput")
            return {"query": query, "results": [{"text": "d", "score": 0.5, "is_ground_truth": False, "rank": 1}]}

    client = TestClient(make_app(FakeIndex()))
    r = client.post("/search", json={"query": "what is a gene"})
    assert r.status_code == 200
    assert r.json() == {"query": "what is a gene",
                        "results": [{"text": "d", "score": 0.5, "is_ground_truth": False, "rank": 1}]}
    r = client.post("/search", json={"query": "boom"})
    assert r.status_code == 500 and r.json()["detail"] == "kaput"
    assert client.post("/search", json={}).status_code == 422


def test_word2vec_binary_and_text_formats(tmp_path):
    """w2v.read_word2vec_format on hand-built word2vec.c layouts (header 'V E', then
    'word ' + E little-endian float32 [+ '\\n'] or 'word v1 .. vE\\n')."""
    import struct

    from two_towers_amd import w2v
    raw = (b"4 2\n" + b"hello " + struct.pack("<2f", 1.0, -2.5) + b"\n" + b"World " + struct.pack("<2f", 0.5, 3.0)
           + b"caf\xc3\xa9 " + struct.pack("<2f", 7.0, 8.0) + b"\n" + b"hello " + struct.pack("<2f", 9.0, 9.0) + b"\n")
    p = tmp_path / "v.bin"
    p.write_bytes(raw)
    v = w2v.read_word2vec_format(str(p))
    assert list(v.index) == ["hello", "World", "café"]  # duplicate: first occurrence wins
    np.testing.assert_array_equal(v.vectors, np.array([[1, -2.5], [0.5, 3], [7, 8]], np.float32))
    assert len(w2v.read_word2vec_format(str(p), limit=2)) == 2
    t = tmp_path / "v.txt"
    t.write_text("2 3\nfoo 1 2 3\nbar -1.5 0 1e-3\n", encoding="utf-8")
    vt = w2v.read_word2vec_format(str(t))
    assert list(vt.index) == ["foo", "bar"]
    np.testing.assert_array_equal(vt.vectors, np.array([[1, 2, 3], [-1.5, 0, 1e-3]], np.float32))
    for binary in (True, False):
        out = tmp_path / f"rt{int(binary)}"
        w2v.write_word2vec_format(v, str(out), binary=binary)
        back = w2v.read_word2vec_format(str(out))
        assert list(back.index) == list(v.index)
        np.testing.assert_array_equal(back.vectors, v.vectors)
    (tmp_path / "bad.bin").write_bytes(b"2 4\nx " + struct.pack("<2f", 1, 2))
    with pytest.raises(ValueError, match="truncated"):
        w2v.read_word2vec_format(str(tmp_path / "bad.bin"), binary=True)


def test_word2vec_store_roundtrip(tmp_path):
    from two_towers_amd import w2v
    rng = np.random.default_rng(0)
    words = [f"w{i}" for i in range(1000)] + ["naïve", "日本"]
    v = tta.Vocab(words, rng.standard_normal((len(words), 12)).astype(np.float32))
    w2v.save_store(v, str(tmp_path / "store"))
    back = w2v.load_store(str(tmp_path / "store"))
    assert back.index == v.index and isinstance(back.vectors, np.memmap)
    np.testing.assert_array_equal(np.asarray(back.vectors), v.vectors)
    tab = back.device_table("cpu")
    assert torch.equal(tab, torch.from_numpy(v.vectors))
    assert "日本" in back and np.array_equal(back["naïve"], v.vectors[1000])


def test_pretokenize_matches_reference_featurization(tmp_path):
    """Offline id files reproduce EnhancedDataset / SimpleDataset rows of the reference
    (the featurize / margin_featurize fixtures), through a fork pool and the id store."""
    import json

    from two_towers_amd import pretok
    for fixture, tok in (("featurize", "enhanced"), ("margin_featurize", "margin")):
        z = np.load(os.path.join(GOLD, fixture + ".npz"), allow_pickle=False)
        vocab = tta.Vocab([str(w) for w in z["words"]], z["vecs"])
        texts = [str(t) for t in z["texts"]] * 3
        T = int(z["max_length"])
        out = tmp_path / tok
        meta = pretok.pretokenize(texts, texts[::-1], vocab, str(out), T, tok, workers=2)
        assert meta["n"] == len(texts) and meta["tokenizer"] == tok
        ds = pretok.PairIds(str(out), vocab)
        emb = np.concatenate([z["emb"]] * 3)
        zero = np.zeros((1, vocab.vector_size), np.float32)
        table = np.concatenate([vocab.vectors, zero])  # row -1 -> zero row
        for i in range(len(ds)):
            q, d = ds[i]
            np.testing.assert_array_equal(table[q.numpy()], emb[i])
            np.testing.assert_array_equal(table[d.numpy()], emb[len(texts) - 1 - i])
        with open(out / "meta.json") as f:
            assert json.load(f)["vocab_sha1"] == pretok.vocab_sha1(vocab)
    other = tta.Vocab(["x"], np.zeros((1, 8), np.float32))
    with pytest.raises(ValueError, match="different vocabulary"):
        pretok.PairIds(str(tmp_path / "enhanced"), other)


def test_pair_id_batches_shard_global_batches(tmp_path):
    from two_towers_amd import pretok
    vocab = tta.Vocab([f"t{i}" for i in range(50)], np.ones((50, 4), np.float32))
    texts = [f"t{i % 50} t{(i * 7) % 50}" for i in range(103)]
    pretok.pretokenize(texts, texts, vocab, str(tmp_path), 4, "enhanced", workers=1)
    ds = pretok.PairIds(str(tmp_path))
    full = [q for q, _ in ds.batches(8, device="cpu", seed=3, world=1)]
    assert len(full) == 103 // 8
    r0 = [q for q, _ in ds.batches(4, device="cpu", seed=3, rank=0, world=2)]
    r1 = [q for q, _ in ds.batches(4, device="cpu", seed=3, rank=1, world=2)]
    assert len(r0) == len(r1) == 103 // 8
    for a, b, g in zip(r0, r1, full):  # the two ranks' rows are exactly the global batch
        assert sorted(map(tuple, torch.cat([a, b]).tolist())) == sorted(map(tuple, g.tolist()))
    assert len({tuple(q.flatten().tolist()) for q in full}) == len(full)  # no aliased batches
    # world > 1: the ragged last global batch is dropped even with drop_last=False, so
    # every rank's slices stay equal (the DP collectives need equal shapes)
    r0 = [q for q, _ in ds.batches(4, device="cpu", seed=3, rank=0, world=2, drop_last=False)]
    r1 = [q for q, _ in ds.batches(4, device="cpu", seed=3, rank=1, world=2, drop_last=False)]
    assert len(r0) == len(r1) == 103 // 8 and all(q.shape[0] == 4 for q in r0 + r1)
    tail = [q for q, _ in ds.batches(8, device="cpu", seed=3, world=1, drop_last=False)]
    assert len(tail) == 103 // 8 + 1 and tail[-1].shape[0] == 103 % 8


def test_read_pairs_formats(tmp_path):
    import json

    from two_towers_amd import pretok
    rows = [{"query": "q1", "passages": {"passage_text": ["a", "b", "c"], "is_selected": [0, 1, 1]}},
            {"query": "", "passages": {"passage_text": ["x"], "is_selected": [1]}},
            {"query": "q3"},
            {"query": "q4", "passages": {"passage_text": ["d"], "is_selected": [1]}}]
    (tmp_path / "p.jsonl").write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    assert pretok.read_pairs(str(tmp_path / "p.jsonl")) == (["q1", "q1", "q4"], ["b", "c", "d"])
    (tmp_path / "p.tsv").write_text("q1\tdoc one\nq2\tdoc\ttwo\n\n")
    assert pretok.read_pairs(str(tmp_path / "p.tsv")) == (["q1", "q2"], ["doc one", "doc\ttwo"])


def test_column_split_publish_waits_cover_the_exchange_store():
    """gru_fwd_xcp publishes a half step after `s_waitcnt vmcnt(6)`: correct only while the
    exchange-image store is followed by exactly the six output stores (Y, S r / z / n /
    gh_n, X1) and nothing else of vector memory. Checked in the built gfx950 code of every
    instance, with the exchange store identified, not just counted: it is the one store
    the kernel issues in two forms (plain where the group shares an XCD, write-through
    `sc1` otherwise, on the two sides of a branch), so the 7th vector-memory op before
    each marked wait must be that `sc1` store, the 8th its plain twin (same address and
    resource registers), and none of the six after it may use its resource (a compiler
    that moved an output store in front of it would leave the exchange store inside the
    six in flight, and the members could read an incomplete image)."""
    import importlib.util
    import re
    from two_towers_amd import _lib
    if not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"):
        pytest.skip("llvm-objdump not available")
    spec = importlib.util.spec_from_file_location("chk", os.path.join(ROOT, "tools", "check_store_hazard.py"))
    chk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(chk)
    text = chk.disassemble(_lib.LIB_PATH)
    funcs = re.split(r"\n(?=[0-9a-f]* ?<[^>]+>:)", text)
    vmem = re.compile(r"^\s*(buffer|global|flat)_(load|store|atomic)\w*")
    store = re.compile(r"^\s*buffer_store_dwordx4 v\[\d+:\d+\], (v\d+), (s\[\d+:\d+\]), 0 offen(.*)$")
    checked = 0
    for f in funcs:
        head = f.split("\n", 1)[0]
        if "gru_fwd_xc" not in head:
            continue
        lines = [ln.split("//")[0].rstrip() for ln in f.split("\n")]
        # the publish waits are the asm pair `s_nop 0; s_waitcnt vmcnt(6)` (s_nop 0 marks them)
        marks = {k + 1 for k in range(len(lines) - 1)
                 if re.match(r"^\s*s_nop 0\b", lines[k]) and "s_waitcnt vmcnt(6)" in lines[k + 1]}
        ops = [(k, ln) for k, ln in enumerate(lines) if vmem.match(ln) or k in marks]
        for i, (k, ln) in enumerate(ops):
            if k not in marks:
                continue
            before = [o for _, o in ops[:i] if vmem.match(o)][-8:]
            assert len(before) == 8, head
            m = [store.match(o) for o in before]
            assert all(m), (head, before)
            plain, wt, outs = m[0], m[1], m[2:]
            assert "sc1" in wt.group(3) and "sc1" not in plain.group(3), (head, before[:2])
            assert (plain.group(1), plain.group(2)) == (wt.group(1), wt.group(2)), (head, before[:2])
            assert all(o.group(2) != wt.group(2) and "sc1" not in o.group(3) for o in outs), (head, before)
            checked += 1
    assert checked >= 8, checked  # 2 half-step publishes per instance, 4 instances
