#!/usr/bin/env python3
"""Training-throughput benchmark of the two-tower step on MI355X (driver contract).

One step = the train_enhanced.py inner loop (train_enhanced.py:54-69) on one batch of
synthetic token ids already resident in HBM: Word2Vec gather -> 2 x 2-layer BiGRU
-> projection heads -> hard-negative mining (k=5) + margin loss (0.2) -> backward ->
gradient all-reduce (N>1) -> Adam. Workload = BASELINE.json configs[2]
(EnhancedTwoTowerModel(300, 256), seq_len 64, batch 8192 per GPU, bf16); with N GPUs
the job is data-parallel with the doc embeddings all-gathered (configs[3] at N=8),
i.e. weak scaling at 8192 pairs per rank.

    python bench.py [--gpus N --steps K --warmup W]     (N > 1: starts N local ranks itself)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line. `roofline` is measured live with HIP events around the
dominant kernel's launches; `cpu_baseline` times the reference's own CPU path (ATen
nn.GRU / nn.Linear / nn.LayerNorm modules, oracle/aten_ref.py) on a bounded sample on
this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.distributed as tdist

METRIC = "training pairs/sec at global batch=8192, 1/2/4/8 GPUs; MRR@10 match"
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_PEAK_TFS = 2500.0    # dense bf16 MFMA (no sparsity)
FP32_PEAK_TFS = 157.3     # fp32 MFMA = vector rate


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8192, help="pairs per GPU")
    ap.add_argument("--seq", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--emb", type=int, default=300)
    ap.add_argument("--vocab", type=int, default=3_000_000)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--loss", default="hardneg_margin", choices=["hardneg_margin", "infonce"])
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: --batch pairs per GPU (configs[3]: 8 x 8192); strong: --batch is the global "
                         "batch, split over the GPUs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=1024, help="pairs per CPU-baseline step (BASELINE.md plan)")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--cpu-warmup", type=int, default=1)
    ap.add_argument("--cpu-only", action="store_true",
                    help="run only the CPU baseline (e.g. --cpu-batch 8192 --cpu-steps 2: the metric's batch) and "
                         "print its JSON; bench lines attach the committed result (profiles/CPU_B8192)")
    ap.add_argument("--timing", action="store_true", help="print the per-kernel HIP-event table to stderr")
    return ap.parse_args()


def make_batches(n, B, T, V, gen, device):
    """Uniform ids in [0, V) with a 10% pad tail per row (-1 -> zero rows), like
    EnhancedDataset padding of short texts (enhanced_two_tower.py:160-162)."""
    out = []
    pad = max(1, T // 10)
    for _ in range(n):
        q = torch.randint(0, V, (B, T), generator=gen, dtype=torch.int64).to(torch.int32)
        d = torch.randint(0, V, (B, T), generator=gen, dtype=torch.int64).to(torch.int32)
        q[:, T - pad:] = -1
        d[:, T - pad:] = -1
        out.append((q.to(device), d.to(device)))
    return out


def workload_name(args, world):
    """The BASELINE.json config the flags describe (configs[2] by default)."""
    std = (args.emb, args.hidden, args.seq, args.batch) == (300, 256, 64, 8192) and args.dtype == "bf16"
    tag = ""
    if std and args.loss == "hardneg_margin" and args.scaling == "strong":
        tag = f"BASELINE metric (global batch 8192 over {world} GPU): " if world > 1 else "BASELINE configs[2]: "
    elif std and args.loss == "hardneg_margin":
        tag = "BASELINE configs[3]: " if world == 8 else "BASELINE configs[2]: "
    elif (args.emb, args.hidden, args.seq, args.batch, args.dtype, args.loss) == (300, 256, 64, 1024, "fp32", "infonce"):
        tag = "BASELINE configs[1]: "
    elif (args.emb, args.hidden, args.seq, args.dtype) == (300, 512, 128, "bf16"):
        tag = "BASELINE configs[4] (per-GPU share): "
    loss = ("hard-negative mining k=5 + margin 0.2" if args.loss == "hardneg_margin" else "in-batch InfoNCE (tau 0.07)")
    per = args.batch // world if args.scaling == "strong" else args.batch
    return (f"{tag}EnhancedTwoTowerModel({args.emb}, {args.hidden}), seq_len {args.seq}, batch {per} per GPU, "
            f"{args.dtype}, {loss}, dropout 0.1, Adam")


def cpu_baseline(args):
    """The reference's CPU step (oracle/aten_ref.py: the same ATen modules and loss
    composition enhanced_two_tower.py / train_enhanced.py run, fp32, pinned to the
    reference's goldens) on a bounded sample of the workload: same model size, seq_len
    and loss, BASELINE.md's planned CPU batch (1024), a few timed steps."""
    import platform

    from oracle import aten_ref

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    torch.set_num_threads(threads)
    E, h, T, B = args.emb, args.hidden, args.seq, args.cpu_batch
    torch.manual_seed(0)
    model = aten_ref.AtenTwoTower(E, h).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    gen = torch.Generator().manual_seed(0)
    table = torch.randn(20000, E, generator=gen) * 0.1

    def batch():
        ids = torch.randint(0, table.shape[0], (2, B, T), generator=gen)
        x = table[ids]  # host gather, as EnhancedDataset does per word
        x[:, :, T - max(1, T // 10):] = 0
        return x[0], x[1]

    def step():
        q, d = batch()
        opt.zero_grad()
        qv, dv = model(q, d)
        loss = aten_ref.infonce(qv, dv) if args.loss == "infonce" else aten_ref.hardneg_margin(qv, dv)
        loss.backward()
        opt.step()

    import sys
    for i in range(args.cpu_warmup):
        step()
        print(f"cpu baseline: warm-up step {i + 1}/{args.cpu_warmup} done", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for i in range(args.cpu_steps):
        step()
        print(f"cpu baseline: step {i + 1}/{args.cpu_steps} done ({time.perf_counter() - t0:.1f} s)", file=sys.stderr,
              flush=True)
    dt = time.perf_counter() - t0
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), cpu)
    except OSError:
        pass
    return {"value": round(B * args.cpu_steps / dt, 2), "unit": "pairs/s", "cores": threads, "kind": "reference",
            "sample": f"reference CPU path (oracle/aten_ref.py: nn.GRU/nn.Linear/nn.LayerNorm + {args.loss} + "
                      f"torch.optim.Adam, fp32), E={E} h={h} T={T}, batch {B} x {args.cpu_steps} timed steps after "
                      f"{args.cpu_warmup} warm-up ({dt:.1f} s), torch {torch.__version__} CPU, {threads} threads "
                      f"on {cpu}"}


# HBM traffic per launch of a timing region, from the committed rocprofv3 PMC summary of
# this build (tools/pmc_bench.sh: separate FETCH_SIZE / WRITE_SIZE passes over bench.py,
# hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1 KiB per dispatch, the gfx950 correction of
# MI355X_MICROARCH.md). A region launch may cover several dispatches (the GRU backward
# runs two chains of step kernels), hence the dispatches-per-step scaling.
_HERE = os.path.dirname(os.path.abspath(__file__))
# the PMC summary of the build this tree ships (tools/pmc_bench.sh), named explicitly
PMC_SUMMARY = os.path.join(_HERE, "profiles", "r06_pmc_summary.json")
# the CPU baseline at the metric's own batch (bench.py --cpu-only --cpu-batch 8192 --cpu-steps 2)
CPU_B8192 = os.path.join(_HERE, "profiles", "r04_cpu_baseline_b8192.json")
REGION_KERNEL = {"gru_bwd": ("gru_bwd_step<", "gru_bwd_big", "gru_bwd_rows<"), "gru_fwd": ("gru_fwd_xs<", "gru_fwd_xcp<", "gru_fwd_seq<"),
                 "embed_gather": ("embed_gather_kernel",)}


def pmc_traffic(region, kernels, launches_per_step, args):
    """HBM bytes per launch of the region's kernels (every instance the region launched,
    e.g. both layers' gru_fwd_xcp<H, DROP>) from the committed PMC summary."""
    key = tuple(kernels) if kernels else REGION_KERNEL.get(region)
    if key is None or not os.path.exists(PMC_SUMMARY):
        return {"traffic": None, "traffic_source": "no PMC summary of this build committed"}
    # the committed PMC passes (tools/pmc_bench.sh) run the default configs[2] workload
    if (args.emb, args.hidden, args.seq, args.batch, args.dtype, args.loss) != (300, 256, 64, 8192, "bf16",
                                                                                 "hardneg_margin"):
        return {"traffic": None, "traffic_source": "no PMC pass for this workload (the committed one is configs[2])"}
    with open(PMC_SUMMARY) as f:
        summ = json.load(f)
    hits = [v for k, v in summ.items()
            if any(k.startswith(s) for s in key) and "hbm_bytes_est" in v and "dispatches_per_step" in v]
    if not hits:
        return {"traffic": None}
    per_step = sum(v["hbm_bytes_est"] * v["dispatches_per_step"] for v in hits)
    return {"traffic": round(per_step / max(launches_per_step, 1)), "traffic_unit": "bytes/launch",
            "traffic_source": f"profiles/{os.path.basename(PMC_SUMMARY)} (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE)"}


def spawn_local_ranks(n: int) -> int:
    """`python bench.py --gpus N` without an external launcher: start N fresh rank
    processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their
    environment, rendezvous on 127.0.0.1) and return the first nonzero exit code. This
    parent never makes a GPU call, so each child initialises HIP itself; if one rank
    fails, the others are terminated instead of waiting in a collective."""
    import signal
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in live:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


def main():
    args = parse()
    if args.cpu_only:
        print(json.dumps(cpu_baseline(args)))
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(spawn_local_ranks(args.gpus))
    # stdout carries exactly the one JSON line: anything the runtime libraries print to it
    # (RCCL's version banner at communicator creation) goes to stderr instead
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # TT_DIST_BACKEND=gloo (rehearsal only): N ranks sharing the box's GPUs over gloo
    backend = os.environ.get("TT_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    # TT_DIST_FORCE=1 under a launcher: a one-rank group whose collectives still run (RCCL
    # rehearsal of the DP path on one GPU)
    forced = os.environ.get("TT_DIST_FORCE", "0") == "1" and "WORLD_SIZE" in os.environ
    if world > 1 or forced:
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=dev)
        else:
            tdist.init_process_group(backend)
    import two_towers_amd as tta
    from two_towers_amd import dist as tdp
    if backend != "nccl" and world > max(torch.cuda.device_count(), 1):
        # ranks sharing one GPU (gloo rehearsal only): the column-split GRU forward needs
        # every CU of the device for one launch, and two processes' cooperative launches are
        # not made co-resident with each other, so the rehearsal runs the row-owning forward
        tta._lib.set_option("gru_fwd_xc", 0)
    from two_towers_amd import timing

    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world} from the launcher")
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    B, T, h, E, V = args.batch, args.seq, args.hidden, args.emb, args.vocab
    if args.scaling == "strong":
        if B % world:
            raise SystemExit(f"--scaling strong: global batch {B} not divisible by {world} GPUs")
        B //= world
    torch.manual_seed(1234)  # same weights on every rank
    # gradients summed inside the backward (head + layer-1 bucket overlapping the layer-0
    # BPTT); allreduce_grads below is then the only other reducer and skips them
    model = (tta.EnhancedTwoTowerModel(E, h).to(dev).set_compute_dtype(dt)
             .set_process_group(group, overlap_grad_allreduce=True).train())
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    table = (torch.randn(V, E, device=dev, generator=gen) * 0.1).to(dt)  # Word2Vec-shaped, resident in HBM
    model.set_embedding_table(table)
    del table
    cpu_gen = torch.Generator().manual_seed(99 + rank)
    batches = make_batches(4, B, T, V, cpu_gen, dev)
    if args.loss == "infonce":
        crit = tta.InfoNCELoss(compute_dtype=dt, process_group=group)
    else:
        crit = tta.HardNegativeMarginLoss(k=5, margin=0.2, compute_dtype=dt, process_group=group)
    opt = tta.Adam(model.parameters(), lr=1e-3)
    params = list(model.parameters())

    def step(i):
        q, d = batches[i % len(batches)]
        opt.zero_grad(set_to_none=True)
        qv, dv = model(q, d)
        loss = crit(qv, dv)
        loss.backward()
        tdp.allreduce_grads(params, group)
        opt.step()
        return loss

    for i in range(args.warmup):
        loss = step(i)
    first_loss = float(loss.detach()) if args.warmup else float("nan")
    if world > 1:
        tdist.barrier()
    torch.cuda.synchronize()
    timing.reset()
    timing.enabled = True
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    timing.enabled = False
    kt = timing.summary()
    final_loss = float(loss.detach())
    # the column-split GRU forward's waits are bounded: a timeout means invalid outputs
    try:
        tta.check_gru_status(wait=True)
    except tta.GruTimeoutError as e:
        raise SystemExit(f"invalid run: {e}")
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    pairs = B * world * args.steps
    value = pairs / elapsed

    # Rooflines from live HIP-event timings. Every region carries its algorithmic FLOPs
    # and algorithmic HBM bytes; the binding roofline is the one whose floor time
    # (FLOPs / MFMA peak vs bytes / HBM peak) is larger. `roofline` = dominant kernel
    # (largest device time per step).
    peak = BF16_PEAK_TFS if dt == torch.bfloat16 else FP32_PEAK_TFS

    def roof(name):
        r = kt[name]
        sec = r["ms_total"] * 1e-3
        if name == "embed_gather":
            flop_floor, byte_floor = 0.0, r["bytes"] / (HBM_PEAK_GBS * 1e9)
        else:
            flop_floor, byte_floor = r["work"] / (peak * 1e12), r["bytes"] / (HBM_PEAK_GBS * 1e9)
        if byte_floor >= flop_floor:
            ach = r["bytes"] / sec / 1e9
            out = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_launch": round(r["bytes_per_launch"])}
        else:
            ach = r["work"] / sec / 1e12
            out = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                   "frac": round(ach / peak, 4), "flops_per_launch": round(r["work_per_launch"])}
        out["ms_per_launch"] = round(r["ms_per_launch"], 5)
        out["launches_per_step"] = r["launches"] // max(args.steps, 1)
        return out

    dom = max(kt, key=lambda k: kt[k]["ms_total"])
    roofline = {"kernel": kt[dom]["kernel"], "region": dom, **roof(dom),
                **pmc_traffic(dom, kt[dom]["kernels"], kt[dom]["launches"] / max(args.steps, 1), args)}
    extra = {k: roof(k) for k in kt if k != dom}
    step_ms = 1e3 * elapsed / args.steps
    kernels = {k: {"kernel": v["kernel"], "ms_per_step": round(v["ms_total"] / args.steps, 3),
                   "tflops": round(v["work"] / (v["ms_total"] * 1e-3) / 1e12, 1) if k != "embed_gather" else None,
                   "gbs": round(v["bytes"] / (v["ms_total"] * 1e-3) / 1e9, 1)}
               for k, v in sorted(kt.items(), key=lambda kv: -kv[1]["ms_total"])}
    if args.timing and rank == 0:
        import sys
        print(json.dumps(kernels, indent=1), file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
        if os.path.exists(CPU_B8192):  # the metric's batch, measured separately (minutes of CPU time)
            with open(CPU_B8192) as f:
                cpu["at_metric_batch"] = {**json.load(f), "source": f"profiles/{os.path.basename(CPU_B8192)}"}
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(step_ms, 3), "higher_is_better": True, "scaling": args.scaling,
            "vs_baseline": None, "dtype": args.dtype,
            "data": f"synthetic: uniform token ids over a {V}x{E} Word2Vec-shaped table resident in HBM, "
                    f"10% pad tail per row, random-init weights (torch seed 1234)",
            "config": {"workload": workload_name(args, world),
                       "global_batch": B * world, "seq_len": T, "hidden": h, "embedding_dim": E,
                       "parallelism": f"dp{world}", "loss": args.loss,
                       "collectives": (("rccl" if backend == "nccl" else backend) + (" (forced at one rank)" if forced else ""))
                       if tdist.is_initialized() else None},
            "roofline": roofline,
            "rooflines_secondary": extra,
            "kernel_ms_per_step": kernels,
            "loss_first_last": [round(first_loss, 5), round(final_loss, 5)],
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), file=out, flush=True)
    if tdist.is_initialized():
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
