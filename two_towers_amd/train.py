"""Training drivers of the reference (train_enhanced.py, train_margin.py) over pre-tokenized
pair stores, one process per GPU.

    python -m two_towers_amd.train --model enhanced --ids IDS_DIR --vocab W2V [...]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m two_towers_amd.train --model margin --ids IDS_DIR --vocab W2V [...]

Loop body = train_enhanced.py:54-69 / train_margin.py:107-120: zero_grad, forward,
loss, backward, Adam step; per-epoch mean loss; the best epoch's weights saved as the
reference does (enhanced: bare state_dict, train_enhanced.py:75; margin: {'epoch',
'model_state_dict', 'optimizer_state_dict', 'loss'}, train_margin.py:128-134).
Defaults are the reference's (E=300, hidden 512, batch 128, 10 epochs, Adam default
lr / 1e-3, InfoNCE temperature 0.07 / 0.1). With N ranks each step consumes N*batch
pairs (weak scaling); negatives are the global batch (losses all-gather the doc
vectors) and gradients are all-reduced (dist.allreduce_grads).
"""
import argparse
import json
import logging
import os
import time
from datetime import datetime

import torch
import torch.distributed as tdist

from . import dist as tdp
from .losses import HardNegativeMarginLoss, InfoNCELoss
from .margin import TwoTowerModel
from .model import EnhancedTwoTowerModel
from .optim import Adam
from .pretok import PairIds, load_vocab


def parse(argv=None):
    ap = argparse.ArgumentParser(description="two-tower training on MI355X")
    ap.add_argument("--model", choices=("enhanced", "margin"), default="enhanced")
    ap.add_argument("--ids", required=True, help="pretok.PairIds directory")
    ap.add_argument("--vocab", required=True, help="w2v store dir, Vocab .npz or word2vec .bin/.txt")
    ap.add_argument("--output_dir", default="output")
    ap.add_argument("--num_epochs", type=int, default=10)
    ap.add_argument("--batch_size", type=int, default=128, help="per rank")
    ap.add_argument("--hidden_dim", type=int, default=512)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--temperature", type=float, default=None)
    ap.add_argument("--loss", choices=("infonce", "hardneg"), default="infonce")
    ap.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32")
    ap.add_argument("--max_steps", type=int, default=0, help="stop after this many steps (0: full epochs)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--log_every", type=int, default=20)
    return ap.parse_args(argv)


def main(argv=None):
    a = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        tdist.init_process_group("nccl", device_id=dev)
        group = tdist.group.WORLD
    vocab = load_vocab(a.vocab)
    data = PairIds(a.ids, vocab)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    torch.manual_seed(a.seed)  # identical initial weights on every rank
    E = vocab.vector_size
    if a.model == "enhanced":
        model = EnhancedTwoTowerModel(E, a.hidden_dim)
        lr = 1e-3 if a.lr is None else a.lr
        tau = 0.07 if a.temperature is None else a.temperature
    else:
        model = TwoTowerModel(E, a.hidden_dim)
        lr = 1e-3 if a.lr is None else a.lr
        tau = 0.1 if a.temperature is None else a.temperature
    model = model.to(dev).set_compute_dtype(dt).set_process_group(group, overlap_grad_allreduce=world > 1)
    model.set_embedding_table(vocab.device_table(dev))
    if a.loss == "infonce":
        crit = InfoNCELoss(temperature=tau, compute_dtype=dt, process_group=group)
    else:
        crit = HardNegativeMarginLoss(k=5, margin=0.2, compute_dtype=dt, process_group=group)
    opt = Adam(model.parameters(), lr=lr)
    params = list(model.parameters())

    out = None
    if rank == 0:
        out = os.path.join(a.output_dir, f"{a.model}_run_{datetime.now().strftime('%Y%m%d_%H%M%S')}")
        os.makedirs(out, exist_ok=True)
        logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s",
                            handlers=[logging.FileHandler(os.path.join(out, "training.log")), logging.StreamHandler()],
                            force=True)
        logging.info("config %s, world %d", json.dumps(vars(a)), world)
    best = float("inf")
    steps = 0
    for epoch in range(a.num_epochs):
        model.train()
        total = torch.zeros((), device=dev)
        nb = 0
        t0 = time.perf_counter()
        for i, (q, d) in enumerate(data.batches(a.batch_size, dev, shuffle=True, seed=a.seed + epoch, rank=rank,
                                                world=world)):
            opt.zero_grad(set_to_none=True)
            qv, dv = model(q, d)
            loss = crit(qv, dv)
            loss.backward()
            tdp.allreduce_grads(params, group)
            opt.step()
            total += loss.detach()  # no host sync per step
            nb += 1
            steps += 1
            if rank == 0 and i % a.log_every == 0:
                logging.info("Batch %d, Loss: %.4f", i, float(loss.detach()))
            if a.max_steps and steps >= a.max_steps:
                break
        avg = float(total) / max(nb, 1)
        if rank == 0:
            dtm = time.perf_counter() - t0
            logging.info("Epoch %d completed. Average Loss: %.4f (%.1f pairs/s)", epoch + 1, avg,
                         nb * a.batch_size * world / max(dtm, 1e-9))
            if avg < best:
                best = avg
                path = os.path.join(out, "best_model.pt")
                if a.model == "enhanced":
                    torch.save(model.state_dict(), path)
                else:
                    torch.save({"epoch": epoch, "model_state_dict": model.state_dict(),
                                "optimizer_state_dict": opt.state_dict(), "loss": avg}, path)
        if a.max_steps and steps >= a.max_steps:
            break
    if rank == 0:
        logging.info("Training complete. Best model saved to: %s", os.path.join(out, "best_model.pt"))
    if world > 1:
        tdist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
