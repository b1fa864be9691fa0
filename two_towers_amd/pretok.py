"""Pre-tokenized pair files: (query, passage) texts -> int32 Word2Vec row ids on disk.

The reference featurises every pair on the host inside the training loop
(EnhancedDataset.__getitem__, enhanced_two_tower.py:144-170, num_workers=0 in
train_enhanced.py:38), shipping [B, T, 300] float32 batches to the model. Here the
pairing rule of dataset_ms_marco.py:16-28 (data.pairs_from_msmarco) and the text ->
row-id rule of the chosen tokenizer (data.encode_ids for the enhanced model,
margin.margin_ids for the margin model) run once, offline, in a process pool; training
then reads [N, T] int32 id matrices (memory-mapped .npy) and uploads 4*T bytes per text
instead of 1200*T, the embedding rows being gathered on the GPU (tt_embed_gather).

Layout of an id store directory:
  q_ids.npy, d_ids.npy   [N, T] int32, -1 = zero row (padding / empty text)
  meta.json              n, max_length, tokenizer, vocab_size, vocab_sha1

CLI:
  python -m two_towers_amd.pretok --vocab W2V --pairs PAIRS --out DIR [--max-length 30]
         [--tokenizer enhanced|margin] [--workers 8]
  W2V: a w2v.save_store directory, a Vocab .npz, or a word2vec .bin/.txt file;
  PAIRS: .jsonl of MS MARCO samples ({"query", "passages": {"passage_text",
  "is_selected"}}) or a .tsv of "query<TAB>passage" lines.
"""
import argparse
import hashlib
import json
import multiprocessing as mp
import os
from typing import Iterator, List, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

from .data import Vocab, encode_ids, pairs_from_msmarco

TOKENIZERS = ("enhanced", "margin")


def _tokenizer(name: str):
    if name == "enhanced":
        return encode_ids
    if name == "margin":
        from .margin import margin_ids
        return margin_ids
    raise ValueError(f"tokenizer must be one of {TOKENIZERS}")


def vocab_sha1(vocab: Vocab) -> str:
    words = [None] * len(vocab.index)
    for w, i in vocab.index.items():
        words[i] = w
    return hashlib.sha1("\n".join(words).encode("utf-8")).hexdigest()


def read_pairs(path: str) -> Tuple[List[str], List[str]]:
    if path.endswith(".tsv"):
        qs, ds = [], []
        with open(path, encoding="utf-8") as f:
            for line in f:
                line = line.rstrip("\n")
                if not line:
                    continue
                q, d = line.split("\t", 1)
                qs.append(q)
                ds.append(d)
        return qs, ds
    with open(path, encoding="utf-8") as f:
        return pairs_from_msmarco(json.loads(line) for line in f if line.strip())


def load_vocab(path: str) -> Vocab:
    from . import w2v
    if os.path.isdir(path):
        return w2v.load_store(path)
    if path.endswith(".npz"):
        return Vocab.load(path)
    return w2v.read_word2vec_format(path)


_G = {}


def _encode_chunk(args):
    texts, = args
    fn, index, T = _G["fn"], _G["index"], _G["T"]
    return np.array([fn(t, index, T) for t in texts], dtype=np.int32).reshape(len(texts), T)


def encode_texts(texts: Sequence[str], vocab: Vocab, max_length: int = 30, tokenizer: str = "enhanced",
                 workers: int = 8, chunk: int = 8192) -> np.ndarray:
    """[len(texts), max_length] int32 ids, computed in a fork pool (the vocabulary index
    is inherited, not pickled)."""
    _G.update(fn=_tokenizer(tokenizer), index=vocab.index, T=max_length)
    jobs = [(list(texts[i:i + chunk]),) for i in range(0, len(texts), chunk)]
    if not jobs:
        return np.zeros((0, max_length), np.int32)
    if workers <= 1 or len(jobs) == 1:
        parts = [_encode_chunk(j) for j in jobs]
    else:
        with mp.get_context("fork").Pool(min(workers, len(jobs))) as pool:
            parts = pool.map(_encode_chunk, jobs)
    return np.concatenate(parts, 0)


def pretokenize(queries: Sequence[str], docs: Sequence[str], vocab: Vocab, out_dir: str, max_length: int = 30,
                tokenizer: str = "enhanced", workers: int = 8) -> dict:
    if len(queries) != len(docs):
        raise ValueError("queries and docs must pair up")
    os.makedirs(out_dir, exist_ok=True)
    q = encode_texts(queries, vocab, max_length, tokenizer, workers)
    d = encode_texts(docs, vocab, max_length, tokenizer, workers)
    np.save(os.path.join(out_dir, "q_ids.npy"), q)
    np.save(os.path.join(out_dir, "d_ids.npy"), d)
    meta = {"format": "two_towers_amd.pairids/1", "n": int(q.shape[0]), "max_length": int(max_length),
            "tokenizer": tokenizer, "vocab_size": len(vocab), "vocab_sha1": vocab_sha1(vocab)}
    with open(os.path.join(out_dir, "meta.json"), "w") as f:
        json.dump(meta, f)
    return meta


class PairIds(Dataset):
    """A pre-tokenized pair store; items are (q_ids, d_ids) int32 [T] tensors."""

    def __init__(self, directory: str, vocab: Vocab = None, mmap: bool = True):
        with open(os.path.join(directory, "meta.json")) as f:
            self.meta = json.load(f)
        mode = "r" if mmap else None
        self.q = np.load(os.path.join(directory, "q_ids.npy"), mmap_mode=mode, allow_pickle=False)
        self.d = np.load(os.path.join(directory, "d_ids.npy"), mmap_mode=mode, allow_pickle=False)
        if self.q.shape != self.d.shape or self.q.shape[0] != self.meta["n"]:
            raise ValueError(f"{directory}: id matrices do not match meta.json")
        if vocab is not None and vocab_sha1(vocab) != self.meta["vocab_sha1"]:
            raise ValueError(f"{directory} was tokenized with a different vocabulary")

    def __len__(self):
        return self.q.shape[0]

    def __getitem__(self, i):
        return torch.from_numpy(np.array(self.q[i])), torch.from_numpy(np.array(self.d[i]))

    def batches(self, batch: int, device="cuda", shuffle: bool = True, seed: int = 0, drop_last: bool = True,
                rank: int = 0, world: int = 1) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        """One epoch of (q, d) [batch, T] int32 device tensors. With world > 1 every rank
        takes its own contiguous slice of each global batch of batch*world pairs (the DP
        sharding of train steps); the ranks' collectives need equal slices, so a ragged
        last global batch is always dropped there. Two pinned host buffers alternate: the
        host fills one while the other's async copy is in flight, and it only waits for
        the copy event of the buffer it is about to overwrite (never for the step)."""
        n = len(self)
        order = np.random.default_rng(seed).permutation(n) if shuffle else np.arange(n)
        gb = batch * world
        stop = (n // gb) * gb if (drop_last or world > 1) else n
        T = self.q.shape[1]
        dev = torch.device(device)
        pin = torch.cuda.is_available() and dev.type == "cuda"
        bufs = [(torch.empty(batch, T, dtype=torch.int32, pin_memory=pin),
                 torch.empty(batch, T, dtype=torch.int32, pin_memory=pin)) for _ in range(2)]
        done = [None, None]  # copy-completion event of each host buffer pair
        for i, g0 in enumerate(range(0, stop, gb)):
            sel = np.sort(order[g0 + rank * batch: min(g0 + (rank + 1) * batch, stop)])
            if len(sel) == 0:
                break
            k = len(sel)
            hq, hd = bufs[i & 1]
            if done[i & 1] is not None:
                done[i & 1].synchronize()  # the copy that last read this pair has finished
            hq[:k].numpy()[:] = self.q[sel]
            hd[:k].numpy()[:] = self.d[sel]
            if dev.type == "cpu":  # a host target would alias the reused buffers
                q, d = hq[:k].clone(), hd[:k].clone()
            else:
                q = hq[:k].to(dev, non_blocking=pin)
                d = hd[:k].to(dev, non_blocking=pin)
            if pin and dev.type == "cuda":
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(dev))
                done[i & 1] = ev
            yield q, d


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--vocab", required=True)
    ap.add_argument("--pairs", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--max-length", type=int, default=30)
    ap.add_argument("--tokenizer", choices=TOKENIZERS, default="enhanced")
    ap.add_argument("--workers", type=int, default=8)
    a = ap.parse_args(argv)
    vocab = load_vocab(a.vocab)
    qs, ds = read_pairs(a.pairs)
    meta = pretokenize(qs, ds, vocab, a.out, a.max_length, a.tokenizer, a.workers)
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
