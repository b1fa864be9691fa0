"""Word2Vec stores on disk (the data format in front of the embedding gather).

The reference loads `word2vec-google-news-300` through gensim and caches the gensim
KeyedVectors object (utils.py:6-23, server/python-api/utils.py:4-21); lookups are
`word2vec[word]` raising KeyError for out-of-vocabulary words. Here the vocabulary is a
Vocab (data.py): a [V, E] float32 table plus a word -> row index, which is what the GPU
gather (tt_embed_gather) consumes. This module converts to and from:

  - the word2vec C formats (what `KeyedVectors.load_word2vec_format` reads): a header
    line "V E", then per word either `word<space>` + E little-endian float32 (binary,
    the GoogleNews-vectors-negative300.bin layout; an optional '\\n' may follow each
    vector) or `word v1 ... vE\\n` (text);
  - a flat directory store made for the GPU path: vectors.npy ([V, E] float32, loadable
    with mmap so a 3.6 GB table is paged straight into the device copy) and words.txt
    (one UTF-8 word per line, row order).

No unpickling: gensim's own .model files are pickles and are not read here.
"""
import json
import mmap
import os
from typing import Optional

import numpy as np

from .data import Vocab


def read_word2vec_format(path: str, binary: Optional[bool] = None, limit: Optional[int] = None,
                         encoding: str = "utf-8", unicode_errors: str = "strict") -> Vocab:
    """Parse a word2vec .bin / .txt file into a Vocab (first occurrence of a repeated
    word wins). binary=None detects the layout from the first entry."""
    with open(path, "rb") as f:
        buf = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    try:
        words, vecs = _parse(buf, path, binary, limit, encoding, unicode_errors)
    finally:
        try:
            buf.close()
        except BufferError:  # a view still referenced by an in-flight exception: GC closes it
            pass
    return Vocab(words, vecs)


def _parse(buf, path, binary, limit, encoding, unicode_errors):
    nl = buf.find(b"\n")
    if nl < 0:
        raise ValueError(f"{path}: missing 'V E' header")
    head = buf[:nl].split()
    if len(head) != 2:
        raise ValueError(f"{path}: bad header {buf[:nl]!r}")
    V, E = int(head[0]), int(head[1])
    if limit is not None:
        V = min(V, int(limit))
    pos = nl + 1
    if binary is None:
        binary = _looks_binary(buf, pos, E)
    vecs = np.empty((V, E), dtype=np.float32)
    words = []
    seen = set()
    for _ in range(V):
        if binary:
            while pos < len(buf) and buf[pos:pos + 1] in (b"\n", b"\r"):
                pos += 1
            sp = buf.find(b" ", pos)
            if sp < 0 or sp + 1 + 4 * E > len(buf):
                raise ValueError(f"{path}: truncated at entry {len(words)}")
            word = buf[pos:sp].decode(encoding, errors=unicode_errors)
            v = np.frombuffer(buf[sp + 1:sp + 1 + 4 * E], dtype="<f4")
            pos = sp + 1 + 4 * E
        else:
            end = buf.find(b"\n", pos)
            end = len(buf) if end < 0 else end
            parts = buf[pos:end].rstrip().split(b" ")
            pos = end + 1
            if len(parts) != E + 1:
                raise ValueError(f"{path}: entry {len(words)} has {len(parts) - 1} values, expected {E}")
            word = parts[0].decode(encoding, errors=unicode_errors)
            v = np.array([float(x) for x in parts[1:]], dtype=np.float32)
        if word in seen:
            continue
        seen.add(word)
        vecs[len(words)] = v
        words.append(word)
    return words, vecs[:len(words)]


def _looks_binary(buf, pos, E) -> bool:
    sp = buf.find(b" ", pos)
    nl = buf.find(b"\n", pos)
    if sp < 0:
        return False
    # text layout: the first line holds exactly E+1 space-separated fields that parse
    line = buf[pos:nl if nl >= 0 else len(buf)].rstrip().split(b" ")
    if len(line) == E + 1:
        try:
            [float(x) for x in line[1:]]
            return False
        except ValueError:
            pass
    return True


def write_word2vec_format(vocab: Vocab, path: str, binary: bool = True):
    words = _words(vocab)
    with open(path, "wb") as f:
        f.write(f"{len(words)} {vocab.vector_size}\n".encode())
        for w, v in zip(words, vocab.vectors):
            if binary:
                f.write(w.encode() + b" " + np.asarray(v, dtype="<f4").tobytes() + b"\n")
            else:
                f.write((w + " " + " ".join(repr(float(x)) for x in v) + "\n").encode())


def _words(vocab: Vocab):
    words = [None] * len(vocab.index)
    for w, i in vocab.index.items():
        words[i] = w
    return words


def save_store(vocab: Vocab, directory: str):
    """vectors.npy + words.txt + meta.json (the flat store of this module's docstring)."""
    words = _words(vocab)
    if any("\n" in w or "\r" in w for w in words):
        raise ValueError("words containing line breaks cannot be stored in words.txt")
    os.makedirs(directory, exist_ok=True)
    np.save(os.path.join(directory, "vectors.npy"), np.ascontiguousarray(vocab.vectors, dtype=np.float32))
    with open(os.path.join(directory, "words.txt"), "w", encoding="utf-8", newline="\n") as f:
        for w in words:
            f.write(w + "\n")
    with open(os.path.join(directory, "meta.json"), "w") as f:
        json.dump({"format": "two_towers_amd.w2v/1", "vocab": len(words), "dim": int(vocab.vector_size)}, f)


def load_store(directory: str, mmap_vectors: bool = True) -> Vocab:
    vecs = np.load(os.path.join(directory, "vectors.npy"), mmap_mode="r" if mmap_vectors else None,
                   allow_pickle=False)
    with open(os.path.join(directory, "words.txt"), encoding="utf-8", newline="\n") as f:
        words = f.read().split("\n")[:-1]
    if len(words) != vecs.shape[0]:
        raise ValueError(f"{directory}: {len(words)} words for {vecs.shape[0]} vectors")
    v = Vocab.__new__(Vocab)  # keep the (possibly memory-mapped) array as is
    v.index = {w: i for i, w in enumerate(words)}
    v.vectors = vecs
    v.vector_size = vecs.shape[1]
    return v


__all__ = ["read_word2vec_format", "write_word2vec_format", "save_store", "load_store"]
