"""Generate tests/golden/bench_b1024.npz: one training step of the bench composition at
B 1024 run by the CPU oracle (oracle/cpu_ref.py), for tests/test_gpu_bench_path.py.

TEST INFRASTRUCTURE ONLY. Run in the build container:
    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_b1024.py

Why this size: at B 1024, T 64 the layer GEMMs have M = B*T = 65,536 rows, so the GPU step
runs bench.py's own kernel selection UNFORCED -- the column-split GRU forward (gru_fwd_xs,
auto from B 1024), the B-resident layer-0 projection (gemm_bres), the persistent layer-1
projection, the split-K weight-gradient GEMMs, the row-owning BPTT and the hard-negative
scan -- while one oracle step still takes ~2 minutes of CPU (too long for a GPU test, so it
is computed once here and committed as data).

The step (train_enhanced.py:58-62 with the configs[2] loss):
EnhancedTwoTowerModel(300, 256) from torch.manual_seed(SEED_MODEL), rounded to bf16; one
batch of correlated pairs (oracle/gen_traj.make_batches: q ~ N(0, 0.25), d = q + N(0,
0.0625), bf16-rounded); dropout 0.1 with the per-tower seeds the GPU model draws from
torch.manual_seed(SEED_DROP); get_hard_negatives k 5 over the in-batch documents +
MarginRankingLoss(0.2) (enhanced_two_tower.py:84-133); the backward. Stored: the loss, the
mined indices and each row's k-th / (k+1)-th cosine gap, each row's 16 best negatives and
their cosines (near-tie checks of the GPU's own picks), the tower outputs of ROWS sampled
rows, and for each of the 44 parameters its gradient's norm and its values at up to NSAMP
fixed positions (all of them for smaller tensors).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import cpu_ref, gen_traj  # noqa: E402

E, HID, T, B, K = 300, 256, 64, 1024, 5
SEED_MODEL, SEED_DATA, SEED_DROP, SEED_POS = 61, 62, 63, 64
NSAMP, ROWS = 16384, 128


def setup():
    """bf16-rounded initial weights, the batch and the dropout seeds, as the GPU test builds them."""
    import two_towers_amd as tta
    torch.manual_seed(SEED_MODEL)
    m = tta.EnhancedTwoTowerModel(E, HID)
    with torch.no_grad():
        for prm in m.parameters():
            prm.copy_(gen_traj.bf16(prm))
    p = {k: v.detach().clone() for k, v in m.state_dict().items()}
    q, d = gen_traj.make_batches(B, seed=SEED_DATA, n=1)[0]
    torch.manual_seed(SEED_DROP)
    seeds = [int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) for _ in range(2)]
    return p, q, d, seeds


def positions(p):
    g = np.random.default_rng(SEED_POS)
    return {k: (np.arange(v.numel()) if v.numel() <= NSAMP else
                np.sort(g.choice(v.numel(), size=NSAMP, replace=False))).astype(np.int64) for k, v in p.items()}


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    p, q, d, seeds = setup()
    pos = positions(p)
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    rq, rd = cpu_ref.forward(q, d, pr, drop_p=0.1, seeds=seeds)
    loss, idx = cpu_ref.hardneg_margin(rq, rd, K, 0.2)
    gaps = gen_traj.tie_gaps(rq, rd, K)
    with torch.no_grad():  # the oracle's 16 best negatives per row (near-tie checks of the GPU's picks)
        cos = cpu_ref.normalize(rq.detach(), 1e-8) @ cpu_ref.normalize(rd.detach(), 1e-8).t()
        cos.fill_diagonal_(-1.0)
        top16 = cos.topk(16, dim=1)
    loss.backward()
    rows = np.sort(np.random.default_rng(SEED_POS + 1).choice(B, size=ROWS, replace=False)).astype(np.int64)
    out = {"loss": np.array(float(loss.detach())), "picks": idx.numpy().astype(np.int16),
           "gaps": gaps.astype(np.float32), "seeds": np.array(seeds, dtype=np.int64), "rows": rows,
           "top16_idx": top16.indices.numpy().astype(np.int16), "top16_cos": top16.values.numpy().astype(np.float32),
           "qv": rq.detach()[rows].numpy(), "dv": rd.detach()[rows].numpy(),
           "qv_absmax": np.array(float(rq.detach().abs().max())), "dv_absmax": np.array(float(rd.detach().abs().max()))}
    for k, v in pr.items():
        out[f"pos/{k}"] = pos[k]
        out[f"g/{k}"] = v.grad.reshape(-1)[pos[k]].numpy().astype(np.float32)
        out[f"gnorm/{k}"] = np.array(float(v.grad.norm()))
    print(f"loss {float(loss.detach()):.6f}; k/k+1 gap median {np.median(gaps):.3e}, rows with gap < 5e-3: "
          f"{np.mean(gaps < 5e-3):.3f}", flush=True)
    path = os.path.join(ROOT, "tests", "golden", "bench_b1024.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
