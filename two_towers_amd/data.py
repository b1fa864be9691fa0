"""Host-side featurisation and data loading (the data formats either side of the path).

  EnhancedDataset(queries, docs, word2vec, max_length=30)
        enhanced_two_tower.py:135-174, same semantics and float [T, E] output, so it
        drops into the reference's DataLoader loops unchanged.
  Vocab / encode_ids / EnhancedIdDataset
        the fast form of the same featurisation: text -> int32 row ids ([T], -1 = zero
        row), gathered on the GPU by tt_embed_gather from a device table. Identical
        embeddings by construction (tests/test_host.py pins it against the reference).
  MSMarcoDataset(word2vec), load_ms_marco_train(), load_word2vec()
        the names train_enhanced.py:9,11,36-37 imports (the reference's own modules do
        not define them: SURVEY.md §0). Network downloads are unavailable offline and
        raise with a clear message; pairs_from_msmarco is the pure pairing rule of
        dataset_ms_marco.py:16-28.
"""
from __future__ import annotations

import os
from typing import Iterable, List, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset


class EnhancedDataset(Dataset):
    def __init__(self, queries: List[str], docs: List[str], word2vec, max_length: int = 30):
        super().__init__()
        self.queries = queries
        self.docs = docs
        self.word2vec = word2vec
        self.max_length = max_length
        self.embedding_dim = word2vec.vector_size

    def text_to_embedding(self, text: str) -> torch.Tensor:
        words = text.lower().split()[: self.max_length]
        rows = []
        for w in words:
            try:
                rows.append(np.asarray(self.word2vec[w], dtype=np.float32))
            except KeyError:
                continue
        out = np.zeros((self.max_length, self.embedding_dim), dtype=np.float32)
        for i, r in enumerate(rows[: self.max_length]):
            out[i] = r
        return torch.from_numpy(out)

    def __len__(self):
        return len(self.queries)

    def __getitem__(self, idx):
        return self.text_to_embedding(self.queries[idx]), self.text_to_embedding(self.docs[idx])


class Vocab:
    """word -> row of a [V, E] float32 table (the on-device Word2Vec store)."""

    def __init__(self, words: Sequence[str], vectors: np.ndarray):
        vectors = np.asarray(vectors, dtype=np.float32)
        if vectors.ndim != 2 or vectors.shape[0] != len(words):
            raise ValueError("vectors must be [len(words), E]")
        self.index = {w: i for i, w in enumerate(words)}
        self.vectors = vectors
        self.vector_size = vectors.shape[1]

    @classmethod
    def from_mapping(cls, word2vec) -> "Vocab":
        """From any mapping-like word2vec (dict, or gensim KeyedVectors via index_to_key)."""
        if hasattr(word2vec, "index_to_key") and hasattr(word2vec, "vectors"):
            return cls(list(word2vec.index_to_key), np.asarray(word2vec.vectors))
        words = list(word2vec.keys())
        return cls(words, np.stack([np.asarray(word2vec[w], dtype=np.float32) for w in words]))

    def __getitem__(self, word):  # KeyedVectors-style lookup for EnhancedDataset
        return self.vectors[self.index[word]]

    def __contains__(self, word):
        return word in self.index

    def __len__(self):
        return len(self.index)

    def save(self, path: str):
        np.savez(path, vectors=self.vectors, words=np.array(list(self.index), dtype=object).astype(str))

    @classmethod
    def load(cls, path: str) -> "Vocab":
        z = np.load(path, allow_pickle=False)
        return cls([str(w) for w in z["words"]], z["vectors"])

    def device_table(self, device="cuda", dtype=torch.float32) -> torch.Tensor:
        """[V, E] table on the device, uploaded in 64 MiB slices (the host array may be a
        read-only memory map of a multi-GB store: w2v.load_store)."""
        V, E = self.vectors.shape
        out = torch.empty(V, E, dtype=dtype, device=device)
        step = max(1, (64 << 20) // max(4 * E, 1))
        for i in range(0, V, step):
            out[i:i + step] = torch.from_numpy(np.array(self.vectors[i:i + step], dtype=np.float32)).to(device, dtype)
        return out


def encode_ids(text: str, vocab, max_length: int = 30) -> List[int]:
    """text_to_embedding as row ids: truncate to max_length words, drop OOV words, a
    single zero row (-1) if nothing is left, pad with -1 at the end."""
    index = vocab.index if isinstance(vocab, Vocab) else vocab
    ids = [index[w] for w in text.lower().split()[:max_length] if w in index]
    if not ids:
        ids = [-1]
    return ids[:max_length] + [-1] * (max_length - len(ids))


def encode_batch(texts: Iterable[str], vocab, max_length: int = 30) -> torch.Tensor:
    return torch.tensor([encode_ids(t, vocab, max_length) for t in texts], dtype=torch.int32)


class EnhancedIdDataset(Dataset):
    """EnhancedDataset returning int32 id rows instead of float embeddings."""

    def __init__(self, queries: List[str], docs: List[str], vocab: Vocab, max_length: int = 30):
        self.queries, self.docs, self.vocab, self.max_length = queries, docs, vocab, max_length

    def __len__(self):
        return len(self.queries)

    def __getitem__(self, idx):
        return (torch.tensor(encode_ids(self.queries[idx], self.vocab, self.max_length), dtype=torch.int32),
                torch.tensor(encode_ids(self.docs[idx], self.vocab, self.max_length), dtype=torch.int32))


def pairs_from_msmarco(samples: Iterable[dict]) -> Tuple[List[str], List[str]]:
    """dataset_ms_marco.py:16-28: one (query, passage) pair per selected passage."""
    queries, docs = [], []
    for sample in samples:
        query = sample.get("query", "")
        if not query or "passages" not in sample:
            continue
        passages = sample["passages"]
        for text, selected in zip(passages.get("passage_text", []), passages.get("is_selected", [])):
            if selected == 1:
                queries.append(query)
                docs.append(text)
    return queries, docs


def load_ms_marco_train(split: str = "train"):
    try:
        from datasets import load_dataset
        ds = load_dataset("ms_marco", "v1.1")[split]
    except Exception as e:  # offline / no cache
        raise RuntimeError(f"MS MARCO v1.1 is not available offline ({e}); build pairs with "
                           "pairs_from_msmarco(samples) from a local copy") from e
    return pairs_from_msmarco(ds)


def load_word2vec(cache_dir: str = "cache") -> Vocab:
    """Word2Vec-300d as a Vocab: cache/word2vec.npz (Vocab.save format) or gensim."""
    path = os.path.join(cache_dir, "word2vec.npz")
    if os.path.exists(path):
        return Vocab.load(path)
    try:
        import gensim.downloader as api
        kv = api.load("word2vec-google-news-300")
    except Exception as e:
        raise RuntimeError(f"Word2Vec is not available offline ({e}); provide {path} "
                           "(Vocab(words, vectors).save(path))") from e
    vocab = Vocab.from_mapping(kv)
    os.makedirs(cache_dir, exist_ok=True)
    vocab.save(path)
    return vocab


class MSMarcoDataset(EnhancedDataset):
    """The MSMarcoDataset(word2vec) train_enhanced.py:37 expects."""

    def __init__(self, word2vec, max_length: int = 30, samples=None):
        queries, docs = pairs_from_msmarco(samples) if samples is not None else load_ms_marco_train()
        super().__init__(queries, docs, word2vec, max_length)
