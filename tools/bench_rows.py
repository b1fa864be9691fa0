#!/usr/bin/env python3
"""Measurements for the widened §8(f) rows (one JSON line each, to stdout):

  margin_train   train_margin.py step: TwoTowerModel(300, 512), InfoNCE(0.1), dropout
                 0.1, Adam, T=30 (SimpleDataset max_length), B pairs/step, bf16 towers
  serve_encode   /search index build: encode_doc over N documents (T=30), docs/s
  serve_query    /search requests against the resident N x 512 matrix: batch-1 latency and
                 batched queries/s, with the top-k kernel's HBM roofline

    python tools/bench_rows.py [--batch 8192] [--docs 1000000] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from two_towers_amd import timing  # noqa: E402
from two_towers_amd.losses import InfoNCELoss  # noqa: E402
from two_towers_amd.margin import TwoTowerModel  # noqa: E402
from two_towers_amd.optim import Adam  # noqa: E402
from two_towers_amd.serving import SearchIndex  # noqa: E402

HBM = 8000.0


def ids(gen, B, T, V, dev):
    x = torch.randint(0, V, (B, T), generator=gen, dtype=torch.int32)
    x[:, T - T // 5:] = -1  # padded tail
    return x.to(dev)


def kernels(steps):
    return {k: {"ms_per_step": round(v["ms_total"] / steps, 3), "gbs": round(v["bytes"] / (v["ms_total"] * 1e-3) / 1e9, 1)}
            for k, v in sorted(timing.summary().items(), key=lambda kv: -kv[1]["ms_total"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--vocab", type=int, default=400_000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    E, H, T = 300, 512, 30
    gen = torch.Generator().manual_seed(0)
    table = torch.randn(a.vocab, E, generator=gen, device="cpu").to(dev) * 0.1
    torch.manual_seed(0)
    model = TwoTowerModel(E, H).to(dev).set_compute_dtype(torch.bfloat16).set_embedding_table(table)
    crit = InfoNCELoss(temperature=0.1, compute_dtype=torch.bfloat16)
    opt = Adam(model.parameters(), lr=1e-3)
    batches = [(ids(gen, a.batch, T, a.vocab, dev), ids(gen, a.batch, T, a.vocab, dev)) for _ in range(2)]

    def step(i):
        q, d = batches[i % 2]
        opt.zero_grad(set_to_none=True)
        loss = crit(*model(q, d))
        loss.backward()
        opt.step()
        return loss

    model.train()
    for i in range(2):
        step(i)
    torch.cuda.synchronize()
    timing.reset()
    timing.enabled = True
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    timing.enabled = False
    print(json.dumps({"row": "margin_train", "value": round(a.batch * a.steps / dt, 1), "unit": "pairs/s",
                      "ms_per_step": round(1e3 * dt / a.steps, 3), "dtype": "bf16",
                      "config": {"model": "margin TwoTowerModel(300, 512)", "batch": a.batch, "seq_len": T,
                                 "loss": "InfoNCE(0.1)", "dropout": 0.1, "optimizer": "Adam(1e-3)"},
                      "loss_last": round(float(loss), 5), "kernel_ms_per_step": kernels(a.steps)}), flush=True)

    # ---- index build: encode_doc over N documents in 8192-row batches
    model.eval()
    nb = 8192
    doc_ids = ids(gen, nb, T, a.vocab, dev)
    with torch.no_grad():
        model.encode_doc(doc_ids)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        outs = []
        for i in range(0, a.docs, nb):
            outs.append(model.encode_doc(doc_ids[: min(nb, a.docs - i)]))
        doc_vecs = torch.cat(outs, 0)
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"row": "serve_encode", "value": round(a.docs / dt, 1), "unit": "docs/s",
                      "config": {"docs": a.docs, "batch": nb, "seq_len": T, "dtype": "bf16"}}), flush=True)

    # ---- queries against the resident matrix
    for sdt in (torch.float32, torch.bfloat16):
        index = SearchIndex(model, None, [""] * a.docs, doc_vectors=doc_vecs, score_dtype=sdt, device=dev)
        esz = 2 if sdt == torch.bfloat16 else 4
        res = {"row": "serve_query", "score_dtype": "bf16" if sdt == torch.bfloat16 else "fp32",
               "config": {"docs": a.docs, "dim": H, "k": 3}}
        for Q in (1, 1024):
            q_ids = ids(gen, Q, T, a.vocab, dev)
            with torch.no_grad():
                for _ in range(3):
                    index.topk(model.encode_query(q_ids), 3)
                torch.cuda.synchronize()
                n = 20 if Q == 1 else 5
                timing.reset()
                timing.enabled = True
                t0 = time.perf_counter()
                for _ in range(n):
                    idx, val = index.topk(model.encode_query(q_ids), 3)
                idx.cpu()
                dt = (time.perf_counter() - t0) / n
                timing.enabled = False
                kt = timing.summary()["search_topk"]
            sec = kt["ms_total"] * 1e-3
            peak_tf = 2500.0 if sdt == torch.bfloat16 else 157.3
            # the binding roofline: the resident matrix stream (HBM) for few queries, the
            # 2 Q N h contraction (MFMA) for many
            if kt["bytes"] / (HBM * 1e9) >= kt["work"] / (peak_tf * 1e12):
                ach = kt["bytes"] / sec / 1e9
                roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM, "unit": "GB/s",
                        "frac": round(ach / HBM, 4), "bytes_per_launch": round(kt["bytes_per_launch"])}
            else:
                ach = kt["work"] / sec / 1e12
                roof = {"bound": "mfma", "achieved": round(ach, 1), "peak": peak_tf, "unit": "TFLOP/s",
                        "frac": round(ach / peak_tf, 4), "flops_per_launch": round(kt["work_per_launch"])}
            res[f"q{Q}"] = {"ms_per_request": round(1e3 * dt, 3), "queries_per_s": round(Q / dt, 1),
                            "topk_ms": round(kt["ms_total"] / kt["calls"], 4), "roofline": roof}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
