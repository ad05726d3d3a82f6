"""Throughput benchmark of the NCF/NeuMF training step on MI355X.

Workload (BASELINE.json metric "train samples/sec (user-item pairs) NeuMF
ml-20m"; config C of SURVEY §8(d)): ml-20m table sizes (138,493 users,
27,278 items), NeuMF with gmf_dim 64 and MLP layers [128, 64, 32, 16],
3 negatives per positive (groups of 4: [neg, neg, neg, pos], user repeated
per group as the data pipeline emits them), batch 65,536 per GPU, Adam
(lr 1e-3) with Keras' dense semantics (every row moves every step), fp32.
Synthetic, seeded ids resident in HBM before the timed region (a fresh
batch per step); random-init weights.

One step = ncf_train_step on 1 GPU (one table, deferred exact decay).  On N
GPUs (one process per GPU, RCCL over xGMI, per-GPU batch fixed = weak
scaling) the default layout is user-partitioned (``--dp user``): rank r trains
the users u % N == r and alone holds their rows and Adam state, the item table
and the dense layers are replicated, and ONE all-reduce per step carries
[item-row gradient | dense-layer gradient | summary].  ``--dp sharded`` (row-
sharded tables, all_to_all of rows) and ``--dp replicated`` (reduce-scatter +
all-gather) are the other layouts.

``python bench.py --gpus N`` with N > 1 and no torchrun environment launches
the N ranks itself (``torch.distributed.run`` as a child process, before any
GPU call) and exits with its status; under torchrun, ``--gpus`` must equal
WORLD_SIZE.

Prints ONE JSON line (rank 0).  ``roofline`` is the step's dominant kernel
(config C: the fused forward/backward, MFMA-bound), ``roofline_emb_update``
the embedding scatter-add + Adam (the HBM-bound kernel the north star's
>= 50 % target names), both timed live with HIP events in the dispatch packets
of the launch stream.  ``traffic`` comes from a committed rocprofv3 PMC
measurement of the same config and batch (profiles/traffic/), else null.
``cpu_baseline`` times the torch-CPU restatement of the reference's Keras step
(oracle/ncf_torch_cpu.py) on rank 0 at N=1 only: BASELINE.md's protocol
(20 warm-up steps, median of 5 timed runs, threads = the host cores this
process may use), the run length bounded by ``--cpu-seconds`` unless
``--cpu-protocol full`` (200 steps per run).
"""

import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "movierecommender-tf-trt_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "train samples/sec (user-item pairs) NeuMF ml-20m at 1/2/4/8 MI355X; HR@10"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFS = 157.3   # dense fp32 MFMA peak (v_mfma_f32_32x32x2_f32), MI355X_MICROARCH.md

CONFIGS = {
    "A": dict(workload="ml-100k GMF-only (config A): 943 users x 1682 items, GMF d=8 (no MLP), 3 neg/pos, "
                       "batch 256 (the reference's CPU plumbing case; generic per-sample kernel)",
              num_users=943, num_items=1682, layers=[], gmf_dim=8, negs=3, batch=256),
    "C": dict(workload="ml-20m NeuMF (config C): 138493 users x 27278 items, gmf 64 + MLP [128,64,32,16], "
                       "3 neg/pos, Adam dense",
              num_users=138493, num_items=27278, layers=[128, 64, 32, 16], gmf_dim=64, negs=3, batch=65536),
    "B": dict(workload="ml-1m NeuMF (config B shape): 6040 users x 3952 items, gmf 8 + MLP [64,32,16,8], 4 neg/pos, "
                       "bf16 MLP operands (fp32 accumulation, master weights and Adam)",
              num_users=6040, num_items=3952, layers=[64, 32, 16, 8], gmf_dim=8, negs=4, batch=4095, precision="bf16"),
    "D": dict(workload="synthetic 10M users x 1M items (config D): gmf 128 + MLP [256,128,64,32], 3 neg/pos, "
                       "Adam dense semantics via deferred exact decay (layer-by-layer hand-written MFMA path)",
              num_users=10000000, num_items=1000000, layers=[256, 128, 64, 32], gmf_dim=128, negs=3, batch=65536),
    "E": dict(workload="ml-20m all-item scoring + top-10 (config E): every one of 138493 users x all 27278 items, "
                       "NeuMF gmf 64 + MLP [128,64,32,16] (config C's model), fp16 MFMA / fp32 accumulate",
              num_users=138493, num_items=27278, layers=[128, 64, 32, 16], gmf_dim=64, negs=3, batch=65536),
}
FP16_MFMA_PEAK_TFS = 2500.0  # dense fp16/bf16 MFMA peak (MI355X_MICROARCH.md), no sparsity


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="strong scaling: a fixed global batch split over the ranks (per-GPU batch = global / N; "
                         "config C's BASELINE configuration is --global-batch 65536 on 8 GPUs); default: weak "
                         "scaling, the per-GPU batch fixed")
    ap.add_argument("--pool", type=int, default=None,
                    help="distinct synthetic batches cycled through (default: one per warmup + timed step, at "
                         "most 1024: every step trains on fresh uniform ids, as epochs over real data do; a "
                         "small pool leaves the users it never draws to owe the Keras dense decay of every step)")
    ap.add_argument("--generic", action="store_true", help="force the generic (non-MFMA) kernel")
    ap.add_argument("--precision", default=None, choices=["fp32", "bf16"],
                    help="MLP operand precision (default: the config's; bf16 = BASELINE config B)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0,
                    help="budget of the timed CPU baseline runs (the 5 runs share it)")
    ap.add_argument("--cpu-protocol", default="bounded", choices=["bounded", "full"],
                    help="full: BASELINE.md's 20 warm-up + 5 x 200 timed steps, whatever it takes")
    ap.add_argument("--selftest-launch", action="store_true",
                    help="launcher self-test (CPU, gloo): ranks start, synchronise and report without any "
                         "GPU work; the JSON line names the rank count")
    ap.add_argument("--e2e", action="store_true",
                    help="end-to-end: each step also samples its batch on the device (ncf_sample_batch) from an "
                         "ml-20m-shaped synthetic ratings set (20M positives)")
    ap.add_argument("--fit-epochs", action="store_true",
                    help="end to end through the reference's API: --steps whole MovierecModel.fit_generator epochs "
                         "(after one warm-up epoch) over an ml-20m-shaped synthetic ratings set with the device "
                         "sampler (trainer params sampler='device'; world_size = --gpus); samples/s of the epochs")
    ap.add_argument("--dense-sweep", action="store_true",
                    help="sweep every embedding row every step instead of the deferred exact decay (same result)")
    ap.add_argument("--id-span", type=float, default=1.0,
                    help="diagnostic (single table): draw user ids from the first FRACTION of the user "
                         "range only (row locality of the gather and the update, e.g. the TLB question "
                         "on config D's 11 GB table); the line's config names it")
    ap.add_argument("--emulate-world", type=int, default=1,
                    help="--dp user at N=1 only: size the local table as rank 0 of this many ranks would "
                         "(per-rank compute of the N-GPU step without its all-reduce; a diagnostic, not a result)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse N ranks sharing one GPU (correctness only, not a measurement)")
    ap.add_argument("--time-every", type=int, default=10,
                    help="kernel durations: HIP events on every k-th step of the timed region (events in the "
                         "dispatch packets lengthen the step they ride on)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no HIP events on the profiled launches (the roofline fields are then null)")
    ap.add_argument("--dp", default="auto", choices=["auto", "user", "sharded", "replicated"],
                    help="multi-GPU layout (auto: single engine at N=1, user-partitioned at N>1)")
    ap.add_argument("--item-optimizer", default="split", choices=["split", "replicated"],
                    help="--dp user: the item rows' Adam split across the ranks (reduce-scatter + all-gather, "
                         "ncf_user_dp_step_split) or replicated on every rank (one all-reduce, ncf_user_dp_step)")
    return ap.parse_args()


def experiment_env(name, default):
    """A kernel-selection switch of the library: only a -DNCF_EXPERIMENT_ENV=1 build reads it
    (csrc/ncf_internal.h experiment_env); the product library runs its default."""
    return os.environ.get(name, default) if os.environ.get("NCF_EXPERIMENT_ENV") == "1" else default


def grad_rows(eng, batch, group):
    """Per-sample gradient rows one batch produces: B item rows plus the user rows — one per
    group when the fused kernel folds a group's user rows (include/movierec_ncf.h "User-row
    folding"; the synthetic batches share the user within a group), else B."""
    fused = bool(eng.fast_path)
    fold = group if (fused and group in (2, 4, 8) and experiment_env("NCF_FOLD_USERS", "1") != "0") else 1
    return batch + batch // fold


def emb_update_bytes(cfg_shape, batch, dense_rows=None, sparse_rows=None, touched_rows=None, contribs=None):
    """Algorithmic HBM bytes of one embedding scatter-add + Adam sweep launch:
    read+write p, m, v of every swept table element (24 B/param), plus the
    gradient.  Single table: the per-sample gradient rows (``contribs`` of them, W floats;
    default 2B) + list (4 B per contribution) + row offsets (4 B/row).  Replicated DP
    (``dense_rows`` = this rank's shard): the reduce-scattered dense gradient
    (4 B/param).  Row-sharded DP (``sparse_rows`` = (shard rows, received
    gradient rows m)): the m received rows + list + offsets of the shard."""
    R, W = cfg_shape.num_rows, cfg_shape.row_width
    c = 2 * batch if contribs is None else contribs
    if touched_rows is not None:
        # deferred exact decay: only the batch's touched rows are read and written
        return 24 * touched_rows * W + c * W * 4 + c * 4 + (R + 1) * 4
    if dense_rows is not None:
        return 28 * dense_rows * W
    if sparse_rows is not None:
        S, m = sparse_rows
        return 24 * S * W + m * W * 4 + m * 4 + (S + 1) * 4
    return 24 * R * W + c * W * 4 + c * 4 + (R + 1) * 4


def replayed_rows(pool, warmup, steps, U, rows, items=True, far=0):
    """Rows the catch-up-ahead blocks of a timed step's update launch replay, averaged over the
    timed steps: those of the next batch that this step does not touch and that some earlier step
    did (a row no step has touched yet is pristine: its zero moments make the zero-gradient steps
    a fixed point, nothing to replay).  ``items``: item rows are under deferred decay too (one
    table; the user layout sweeps its replicated item rows).  ``far`` > 0: only rows owing more than
    that many steps (the one-table step replays the nearer ones in its stats launch, NCF_DEFER_OWED)."""
    seq = [pool[i % len(pool)] for i in range(warmup + steps + 1)]

    def rows_of(b):
        r = torch.unique(b[0].long())
        return torch.cat([r, U + torch.unique(b[1].long())]) if items else r
    seen = torch.zeros(rows, dtype=torch.bool, device=seq[0][0].device)
    last = torch.zeros(rows, dtype=torch.long, device=seq[0][0].device)  # batch index of the last touch
    out = []
    cur = rows_of(seq[0])
    for t in range(len(seq) - 1):
        nxt = rows_of(seq[t + 1])
        if t >= warmup:
            rep = ~torch.isin(nxt, cur) & seen[nxt]
            if far > 0:
                rep &= (t - last[nxt]) > far   # the update of batch t takes the row from step last + 1 to t + 1
            out.append(int(rep.sum()))
        seen[cur] = True
        last[cur] = t
        cur = nxt
    return float(np.mean(out)) if out else 0.0


def deferred_replay_owed(info):
    """The library's NCF_DEFER_OWED (rows owing at most this many steps are replayed in the stats
    launch of a one-table step), from its build defines; 0 when the replays all run in the update."""
    d = (info or {}).get("defines", "") or ""
    if "NCF_REPLAY_IN_SCAN=0" in d:
        return 0
    m = re.search(r"NCF_DEFER_OWED=(\d+)", d)
    return int(m.group(1)) if m else 4   # ncf_update.hip's default


def fwd_bwd_flops(cfg):
    """Algorithmic flops per sample of the fused forward+backward: 2 x MACs of the forward
    (MLP layers, GMF product+dot, output), the backward data chain (dX, G_l) and the
    weight gradients (dW_l, output kernel)."""
    L, G = cfg["layers"], cfg["gmf_dim"]
    mlp = sum(a * b for a, b in zip(L[:-1], L[1:]))
    out = G + (L[-1] if L else 0)
    fwd = mlp + out + G
    bwd_data = mlp + G * 2 + out
    dw = mlp + out
    return 2 * (fwd + bwd_data + dw)


def fwd_bwd_executed_flops(cfg, batch, group, kpath):
    """MFMA-issued flops per launch when they differ from the algorithmic count: the wave kernel's
    group-user form (split form with user-row folding) runs the user half of layer 1,
    of dX and of dW1 once per group of F = group samples, i.e. 3 x 2 x (L0 / 2) x L1 flops per
    sample fewer by a factor F.  None when the kernel does the per-sample work."""
    L = cfg["layers"]
    if (kpath != "fused-mfma-wave" or group not in (2, 4, 8) or experiment_env("NCF_WAVE_SPLIT", "1") == "0"
            or experiment_env("NCF_FOLD_USERS", "1") == "0"):
        return None
    user_half = 3 * 2 * (L[0] // 2) * L[1]
    return fwd_bwd_flops(cfg) * batch - user_half * batch * (group - 1) // group


def fwd_bwd_bytes(shape, batch, contribs=None):
    """Algorithmic HBM bytes of the fused kernel: ids+label (12 B), both gathered rows
    (2W floats), the per-sample gradient rows written (``contribs`` rows of W floats, default
    2B), the probability."""
    c = 2 * batch if contribs is None else contribs
    return batch * (12 + 2 * shape.row_width * 4 + 4) + c * shape.row_width * 4


def cpu_baseline(cfg, budget_s, protocol="bounded"):
    """torch-CPU restatement (oracle/ncf_torch_cpu.py) of the reference's Keras training step,
    timed with BASELINE.md's protocol: 20 warm-up steps, 5 timed runs, median; threads = the
    host cores this process may use.  ``bounded``: the 5 runs share ``budget_s`` seconds (at most
    200 steps each); ``full``: 200 steps each."""
    from oracle import ncf_torch_cpu as T
    full = protocol == "full"
    med, rates, threads, steps = T.time_protocol(cfg["num_users"], cfg["num_items"], cfg["layers"], cfg["gmf_dim"],
                                                 cfg["batch"], cfg["negs"], warmup=20, steps=200, repeats=5,
                                                 budget_s=None if full else budget_s)
    return dict(value=round(med, 1), unit="samples/s", cores=int(threads), kind="port",
                runs=[round(r, 1) for r in rates],
                sample="torch-CPU fp32 Keras-equivalent step (autograd, dense embedding gradient, dense Adam "
                       "over every table row), batch %d: 20 warm-up steps, median of 5 runs of %d steps "
                       "(protocol %s)" % (cfg["batch"], steps, protocol))


def cpu_sampler_baseline(cfg, budget_s):
    """The reference-faithful host sampler (movierec.data_pipeline mirror of data_pipeline.py:99-150:
    one np.random.choice over the user's non-positives per positive, single thread like Keras
    workers=1) on synthetic ratings with the config's user/item counts: samples/s."""
    import pandas as pd
    from movierec.data_pipeline import MovieLensDataGenerator
    from movierec.util import movielens_utils as ml
    rng = np.random.RandomState(5)
    n = 2000000
    df = pd.DataFrame({"userId": rng.randint(0, cfg["num_users"], n).astype(np.int32),
                       "itemId": rng.randint(0, cfg["num_items"], n).astype(np.int32)})
    name = "ml-20m"
    saved = (ml.NUM_USERS[name], ml.NUM_ITEMS[name])
    ml.NUM_USERS[name], ml.NUM_ITEMS[name] = cfg["num_users"], cfg["num_items"]
    try:
        np.random.seed(0)
        bs = 4096 // (cfg["negs"] + 1) * (cfg["negs"] + 1)
        gen = MovieLensDataGenerator(name, df, bs, cfg["negs"])
        gen[0]   # builds the per-user CSR (one-off)
        t0, b = time.perf_counter(), 1
        while time.perf_counter() - t0 < budget_s and b < len(gen):
            gen[b]
            b += 1
        dt = time.perf_counter() - t0
    finally:
        ml.NUM_USERS[name], ml.NUM_ITEMS[name] = saved
    return (b - 1) * bs / dt, "%d batches of %d from 2M synthetic ratings, %.1f s" % (b - 1, bs, dt)


def score_flops(cfg):
    """Algorithmic flops per (user, item) pair of the scorer after the first-layer split
    (ncf_score.hip): layers 2.., output layer and the GMF dot; and of the naive forward."""
    L, G = cfg["layers"], cfg["gmf_dim"]
    rewritten = 2 * (sum(a * b for a, b in zip(L[1:-1], L[2:])) + L[-1] + G)
    naive = 2 * (sum(a * b for a, b in zip(L[:-1], L[1:])) + L[-1] + 2 * G)
    return rewritten, naive


def cpu_score_baseline(cfg, budget_s):
    """numpy restatement (oracle/) of all-item scoring + top-10 for a bounded sample of users."""
    from oracle import ncf_oracle as O
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        threads = 1
    shape = O.NCFShape(cfg["num_users"], cfg["num_items"], cfg["layers"], cfg["gmf_dim"])
    w = O.init_weights(shape, seed=0, dtype=np.float32)
    t_total, n = 0.0, 0
    while t_total < budget_s and n < 200:
        t0 = time.perf_counter()
        O.top_k_items(O.score_all_items(shape, w, [n]), 10)
        t_total += time.perf_counter() - t0
        n += 1
    return dict(value=round(n * cfg["num_items"] / t_total, 1), unit="pairs/s", cores=int(threads), kind="port",
                sample="%d users x all %d items scored + top-10, numpy, %.1f s" % (n, cfg["num_items"], t_total))


def score_main(args, cfg, world, rank):
    """Config E: every user x every item, top-10 per user; users split across ranks (no collective)."""
    from movierec.engine import NCFEngine
    from movierec.model import initial_weights
    from movierec import _native as N
    U, I = cfg["num_users"], cfg["num_items"]
    eng = NCFEngine(U, I, cfg["layers"], cfg["gmf_dim"], max_batch=1024)
    eng.set_keras_weights(initial_weights(U, I, cfg["layers"], cfg["gmf_dim"], seed=0))
    lo, hi = rank * U // world, (rank + 1) * U // world
    users = torch.arange(lo, hi, dtype=torch.int32, device="cuda")
    for _ in range(args.warmup):
        eng.score_topk(users, k=10)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    N.profile_enable([N.K_SCORE], args.steps + 1)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.score_topk(users, k=10)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms, nl = N.profile_read(N.K_SCORE)
    N.profile_enable([], 0)
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    pairs = U * I
    value = args.steps * pairs / elapsed
    kern_ms = ms / max(nl, 1)
    fl, fl_naive = score_flops(cfg)
    my_pairs = (hi - lo) * I
    achieved = fl * my_pairs / (kern_ms * 1e-3) / 1e12
    if rank == 0:
        cpu = None if (world > 1 or args.no_cpu_baseline) else cpu_score_baseline(cfg, args.cpu_seconds)
        emit(json.dumps({
            "metric": "all-item scoring + top-10 (user, item) pairs/s, ml-20m NeuMF (config E)", "value": round(value, 1),
            "unit": "pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "fp16 (fp32 accumulate)", "data": "synthetic (random-init weights)",
            "config": {"workload": cfg["workload"], "users": U, "items": I, "k": 10,
                       "parallelism": "users split across %d ranks" % world},
            "roofline": {"bound": "mfma", "kernel": "k_score_topk (+ k_score_merge)", "achieved": round(achieved, 1),
                         "peak": FP16_MFMA_PEAK_TFS, "unit": "TFLOP/s", "frac": round(achieved / FP16_MFMA_PEAK_TFS, 4),
                         "traffic": pmc_traffic("k_score_topk", "E", U, "all-items") if world == 1 else None,
                         "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/traffic/)",
                         "algorithmic_flops_per_pair": fl, "naive_flops_per_pair": fl_naive,
                         "avg_launch_ms": round(kern_ms, 4)},
            "cpu_baseline": cpu}))
    if dist.is_initialized():
        dist.destroy_process_group()


def fit_main(args, cfg, world, rank):
    """Trainer-style epochs: MovierecModel.fit_generator (the reference's model.py:305-333 loop:
    every batch of the Sequence, on_epoch_end; no validation pass) over DeviceMovieLensDataGenerator
    batches, timed whole — sampling, the H2D-free batch handoff, training steps, per-epoch error
    checks and metric reads included."""
    import tempfile
    from movierec.model import MovierecModel
    B, g = cfg["batch"], cfg["negs"] + 1
    L = cfg["layers"]
    params = dict(num_users=cfg["num_users"], num_items=cfg["num_items"], layers_sizes=L, layers_l2reg=[0] * len(L),
                  optimizer="adam", lr=0.001, batch_size=B * world, num_negs_per_pos=cfg["negs"],
                  batch_size_eval=100 * world, num_negs_per_pos_eval=99, k=min(10, g), seed=0,
                  gmf_dim=cfg["gmf_dim"], world_size=world, precision=args.precision or cfg.get("precision", "fp32"),
                  max_batch=B)
    model = MovierecModel(params, "bench", tempfile.mkdtemp(), verbose=0)
    eng = model.model.engine
    gen = synthetic_device_generator(cfg, B, g, seed=1234 + rank, world=world,
                                     num_users=eng.num_users if world > 1 else None)

    def barrier():
        torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()

    model.fit_generator(gen, None, epochs=1)   # warm-up epoch
    barrier()
    t0 = time.perf_counter()
    model.fit_generator(gen, None, epochs=args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    steps_per_epoch = len(gen)
    if dist.is_initialized():
        from movierec.distributed import all_reduce_min
        steps_per_epoch = all_reduce_min(steps_per_epoch)
    samples = args.steps * steps_per_epoch * B * world
    if rank == 0:
        emit(json.dumps({
            "metric": "fit_generator epoch samples/sec (user-item pairs) NeuMF ml-20m, device sampler",
            "value": round(samples / elapsed, 1), "unit": "samples/s", "n_gpus": world, "epochs": args.steps,
            "warmup_epochs": 1, "steps_per_epoch": steps_per_epoch, "ms_per_step": round(elapsed / (args.steps *
                                                                                               steps_per_epoch) * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "dtype": params["precision"],
            "data": "synthetic ml-20m-shaped ratings (%d positives per rank), negatives sampled on the device"
                    % len(gen.data),
            "config": {"workload": cfg["workload"], "global_batch": B * world, "per_gpu_batch": B,
                       "api": "MovierecModel.fit_generator (trainer params sampler='device', world_size=%d)" % world,
                       "epoch_rule": "len = positives // batch (the reference's data_pipeline.py:97, SURVEY F4)"}}))
    if dist.is_initialized():
        dist.destroy_process_group()


def synthetic_device_generator(cfg, batch, group, seed, num_users=None, world=1):
    """ml-20m-shaped synthetic ratings (20M positives over the config's users x items, uniform)
    behind the on-device sampler: a step = sample one batch + train on it.  User-partitioned
    data parallelism: this rank's 1/world of the ratings over its ``num_users`` (local ids)."""
    import pandas as pd
    from movierec.sampler import DeviceMovieLensDataGenerator
    from movierec.util import movielens_utils as ml
    rng = np.random.RandomState(seed)
    n = 20000263 // world  # ml-20m ratings
    nu = cfg["num_users"] if num_users is None else int(num_users)
    df = pd.DataFrame({"userId": rng.randint(0, nu, n).astype(np.int32),
                       "itemId": rng.randint(0, cfg["num_items"], n).astype(np.int32)})
    name = "ml-20m"
    saved = (ml.NUM_USERS[name], ml.NUM_ITEMS[name])
    ml.NUM_USERS[name], ml.NUM_ITEMS[name] = nu, cfg["num_items"]
    try:
        gen = DeviceMovieLensDataGenerator(name, df, batch, group - 1, seed=seed)
    finally:
        ml.NUM_USERS[name], ml.NUM_ITEMS[name] = saved
    gen[0]
    return gen


def device_glorot_init(eng, w_small, seed):
    """Keras glorot_uniform embedding tables drawn on the device (config D's 11 GB table); dense
    layers from ``w_small`` (initial_weights of the same layers)."""
    from movierec.layout import Layout
    lay = Layout(1, 1, eng.layers, eng.gmf_dim)
    eng.mlp.copy_(torch.from_numpy(lay.to_device(w_small)[1]))
    g = torch.Generator(device="cuda").manual_seed(seed)
    U, G, G4 = eng.num_users, eng.gmf_dim, eng.shape.gmf_stride
    du, di = eng.shape.du, eng.shape.di
    eng.emb.zero_()
    for rows, n, d, col in ((slice(0, U), U, du, G4), (slice(U, eng.num_rows), eng.num_items, di, G4)):
        for width, c0 in ((G, 0), (d, col)):
            if width:
                lim = (6.0 / (n + width)) ** 0.5
                part = eng.emb[rows, c0:c0 + width]
                part.copy_(torch.rand(part.shape, generator=g, device="cuda") * (2 * lim) - lim)
    torch.cuda.synchronize()


def device_glorot_init_shard(eng, w_small, seed):
    """device_glorot_init for one rank's shard of a row-sharded table (local row l = global row
    l * world + rank): each row drawn with its table's (user / item) Keras glorot limits."""
    from movierec.layout import Layout
    lay = Layout(1, 1, eng.layers, eng.gmf_dim)
    eng.mlp.copy_(torch.from_numpy(lay.to_device(w_small)[1]))
    g = torch.Generator(device="cuda").manual_seed(seed + eng.rank)
    U, I, G, G4 = eng.num_users, eng.num_items, eng.gmf_dim, eng.shape.gmf_stride
    du, di = eng.shape.du, eng.shape.di
    eng.emb.zero_()
    chunk = 1 << 20
    for r0 in range(0, eng.shard_rows, chunk):
        r1 = min(eng.shard_rows, r0 + chunk)
        gl = torch.arange(r0, r1, device="cuda", dtype=torch.int64) * eng.world + eng.rank
        user = (gl < U).unsqueeze(1)
        valid = (gl < U + I).unsqueeze(1)
        for wu, wi, c0 in ((G, G, 0), (du, di, G4)):
            width = max(wu, wi)
            if not width:
                continue
            r = torch.rand(r1 - r0, width, generator=g, device="cuda") * 2 - 1
            lim_u = (6.0 / (U + wu)) ** 0.5 if wu else 0.0
            lim_i = (6.0 / (I + wi)) ** 0.5 if wi else 0.0
            cols = torch.arange(width, device="cuda").unsqueeze(0)
            lim = torch.where(user, torch.where(cols < wu, lim_u, 0.0), torch.where(cols < wi, lim_i, 0.0))
            eng.emb[r0:r1, c0:c0 + width].copy_(r * lim * valid)
    torch.cuda.synchronize()


def native_step_check(cfg, world, rank, split):
    """At N > 1 over RCCL, before the measured run: movierec.distributed.native_step_check — the
    library's one-call user-partitioned step against the same step issued call by call with
    torch.distributed's collectives, from identical state, on this config's model with small
    tables; the measured run uses the native step only when the two agree."""
    from movierec.distributed import native_step_check as check
    return check(cfg["layers"], cfg["gmf_dim"], cfg["negs"] + 1, split)


def pmc_mfma_busy(kernel, config, batch):
    """The MFMA-busy fraction of a forward/backward kernel from its committed rocprofv3 PMC pass
    (profiles/mfma/<config>_b<batch>_<kernel>.json, tools/pmc_mfma.sh), or None."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "mfma",
                        "%s_b%d_%s.json" % (config, batch, kernel))
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    return {"mfma_busy_frac": round(float(d["mfma_busy_frac"]), 3), "source": os.path.relpath(path, os.path.dirname(path) + "/../..")}


def pmc_traffic(kernel, config, batch, mode):
    """HBM bytes per launch of ``kernel`` measured by tools/gpu_profile.sh (separate FETCH_SIZE /
    WRITE_SIZE rocprofv3 passes) for exactly this config, per-GPU batch and layout; None when no
    such measurement is committed under profiles/traffic/."""
    path = os.path.join(ROOT, "profiles", "traffic", "%s_b%d_%s_%s.json" % (config, batch, mode, kernel))
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    if (d.get("kernel"), d.get("config"), d.get("batch"), d.get("mode")) != (kernel, config, batch, mode):
        return None
    return d.get("bytes_per_launch")


_RESULT_OUT = None


def _keep_stdout_for_result():
    """stdout carries exactly one line, the result: everything else written to file descriptor 1
    (RCCL's version banner on every rank, gloo's connection chatter) goes to stderr."""
    global _RESULT_OUT
    if _RESULT_OUT is None:
        sys.stdout.flush()
        _RESULT_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)


def emit(text):
    _RESULT_OUT.write(text + "\n")
    _RESULT_OUT.flush()


def _free_port():
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch_ranks(nproc):
    """``--gpus N`` outside torchrun: run this same command as N ranks under
    torch.distributed.run (a child process, started before this process touches the GPU) and
    return its exit status.  The ranks' stdout is this process's stdout: rank 0 prints the one
    JSON line, the others print nothing there."""
    import subprocess
    pre = os.environ.get("LD_PRELOAD", "")
    if os.environ.get("ROCP_TOOL_LIBRARIES") or os.environ.get("ROCPROF_PRELOAD") or "rocprof" in pre:
        # under rocprofv3 the profiler's preloaded library has initialised the GPU in this process:
        # starting the launcher from here would be the forbidden exec of a GPU-initialised process
        sys.stderr.write("bench.py --gpus %d: refusing to launch ranks under a profiler; profile one rank per "
                         "process instead (an outer torch.distributed.run with rocprofv3 -- python bench.py per "
                         "rank)\n" % nproc)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")   # torchrun's default; keeps its warning off stderr
    sys.stdout.flush()
    return subprocess.call(cmd, env=env)


def selftest_main(args, world, rank):
    """Launcher self-test: the process group forms (gloo, CPU), the ranks time a trivial region
    between barriers, the max over ranks reaches rank 0, rank 0 prints the line."""
    if world > 1:
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    x = torch.zeros(1)
    for _ in range(max(args.steps, 1)):
        x += 1
    if dist.is_initialized():
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        emit(json.dumps({"metric": "launcher self-test", "value": None, "n_gpus": world, "ranks": world,
                         "steps": args.steps, "warmup": args.warmup, "elapsed_max_s": float(t.item()),
                         "backend": dist.get_backend() if dist.is_initialized() else None}))
    if dist.is_initialized():
        dist.destroy_process_group()


def _native_build_info():
    from movierec import _native as N
    info = N.build_info()
    try:
        import importlib.util
        spec = importlib.util.spec_from_file_location(
            "ncf_build", os.path.join(os.path.dirname(os.path.abspath(__file__)), "movierecommender-tf-trt_amd",
                                      "csrc", "build.py"))
        b = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(b)
        info["matches_tree"] = info["src_sha256"] == b.source_hash()
    except Exception as exc:  # the sources are always shipped with the tree; report rather than fail
        info["matches_tree"] = "unknown (%s)" % exc
    return info


def main():
    args = parse()
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    _keep_stdout_for_result()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit("--gpus %d but the launcher started %d rank(s) (WORLD_SIZE)" % (args.gpus, world))
    if args.selftest_launch:
        return selftest_main(args, world, rank)
    torch.cuda.set_device(local if args.dist_backend == "nccl" else 0)
    mode = args.dp if args.dp != "auto" else ("single" if world == 1 else "user")
    if world > 1:
        if args.dist_backend == "gloo":   # rehearsal of the multi-rank logic on one GPU (tests)
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    elif mode != "single":
        # one-rank process group: exercises the data-parallel path on one GPU
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                                device_id=torch.device("cuda", local))
    cfg = dict(CONFIGS[args.config])
    if args.config == "E":
        return score_main(args, cfg, world, rank)
    if args.fit_epochs:
        if args.batch:
            cfg["batch"] = args.batch
        return fit_main(args, cfg, world, rank)
    from movierec.engine import NCFEngine
    from movierec.model import initial_weights
    from movierec import _native as N

    if args.batch and args.global_batch:
        raise SystemExit("--batch (per GPU, weak scaling) and --global-batch (strong scaling) exclude each other")
    if args.batch:
        cfg["batch"] = args.batch
    if args.global_batch:
        if args.global_batch % world:
            raise SystemExit("--global-batch %d does not split over %d ranks" % (args.global_batch, world))
        cfg["batch"] = args.global_batch // world
    B, g = cfg["batch"], cfg["negs"] + 1
    prec = args.precision or cfg.get("precision", "fp32")
    if prec == "bf16" and mode == "sharded":
        raise SystemExit("bf16 MLP operands run on the single-table and user-partitioned layouts")
    assert B % g == 0, "batch must be divisible by negs+1"
    big = args.config == "D"   # 11 GB table: initialised on the device, not through host numpy
    if big and mode not in ("single", "sharded"):
        raise SystemExit("config D runs on one table or row-sharded (--dp sharded), as BASELINE names it")
    ew = max(world, args.emulate_world)
    if ew > world and (world > 1 or mode not in ("user", "sharded")):
        raise SystemExit("--emulate-world: one process, --dp user or --dp sharded")
    w0 = initial_weights(1 if big else cfg["num_users"], 1 if big else cfg["num_items"], cfg["layers"],
                         cfg["gmf_dim"], seed=0)
    dp = None
    native_check = None
    if mode == "sharded":
        from movierec.sharded import ShardedNCFEngine
        from movierec.distributed import RowShardedDataParallel
        # the shard's rows under deferred exact decay (its own rows, served when requested)
        eng = ShardedNCFEngine(cfg["num_users"], cfg["num_items"], cfg["layers"], cfg["gmf_dim"], world=ew,
                               rank=rank, max_batch=B, force_generic=args.generic, lazy_adam=not args.dense_sweep)
        if big:
            device_glorot_init_shard(eng, w0, seed=0)
        else:
            eng.set_keras_weights(w0)
        dp = RowShardedDataParallel(eng, emulate=ew > world)
        dp.broadcast_parameters()
    elif mode == "user":
        from movierec.distributed import UserPartitionedDataParallel, partition_keras_weights
        n_loc = (cfg["num_users"] - rank + ew - 1) // ew
        # the own users under deferred exact decay (the replicated item rows are swept every step)
        eng = NCFEngine(n_loc, cfg["num_items"], cfg["layers"], cfg["gmf_dim"], max_batch=B,
                        force_generic=args.generic, precision=prec, lazy_adam=not args.dense_sweep,
                        lazy_rows=n_loc)
        eng.set_keras_weights(partition_keras_weights(w0, ew, rank))
        native = None
        if world > 1 and dist.get_backend() == "nccl" and not args.dense_sweep:
            native_check = native_step_check(cfg, world, rank, args.item_optimizer == "split")
            native = native_check["ok"]
            if not native:
                # the one-call RCCL step disagrees with the call-by-call step: no silent fallback
                # (every rank holds the same all-reduced verdict, so every rank exits)
                msg = json.dumps({"error": "native_step_check failed: the one-call RCCL step (ncf_user_dp_step%s) "
                                           "does not match the call-by-call step" %
                                           ("_split" if args.item_optimizer == "split" else ""),
                                  "native_step_check": native_check, "n_gpus": world})
                print(msg, file=sys.stderr)
                if rank == 0:
                    emit(msg)
                sys.exit(3)
        dp = UserPartitionedDataParallel(eng, native=native, split_items=args.item_optimizer == "split",
                                         emulate_world=ew if ew > world else None)
        dp.broadcast_parameters()
    else:
        eng = NCFEngine(cfg["num_users"], cfg["num_items"], cfg["layers"], cfg["gmf_dim"], max_batch=B,
                        force_generic=args.generic, lazy_adam=(mode == "single" and not args.dense_sweep),
                        precision=prec)
        if big:
            device_glorot_init(eng, w0, seed=0)
        else:
            eng.set_keras_weights(w0)
        if mode == "replicated":
            from movierec.distributed import ReplicatedDataParallel
            dp = ReplicatedDataParallel(eng)
    del w0
    gen = torch.Generator(device="cuda").manual_seed(1234 + rank)
    sampler = None
    if args.e2e:
        if mode in ("user", "single"):
            sampler = synthetic_device_generator(cfg, B, g, seed=1234 + rank, world=world,
                                                 num_users=eng.num_users if mode == "user" else None)
        else:
            raise SystemExit("--e2e supports the single-table and user-partitioned layouts")
    pool = []
    npool = args.pool if args.pool else max(8, min(1024, args.warmup + args.steps + 1))
    own = mode == "sharded" and ew > world   # emulated rank: every row of its batches is its own
    for _ in range(npool):
        # user-partitioned data: this rank's users only, as local ids (u // world)
        if own:
            U, I = cfg["num_users"], cfg["num_items"]
            u = torch.randint(0, (U - rank + ew - 1) // ew, (B // g,), generator=gen, device="cuda",
                              dtype=torch.int32) * ew + rank
            i0 = (rank - U) % ew   # the first item whose table row U + i0 is this rank's
            it = torch.randint(0, (I - i0 + ew - 1) // ew, (B,), generator=gen, device="cuda",
                               dtype=torch.int32) * ew + i0
            u = u.repeat_interleave(g)
            pool.append((u.contiguous(), it.contiguous(),
                         torch.tensor([0.0] * (g - 1) + [1.0], device="cuda").repeat(B // g).contiguous()))
            continue
        u_hi = eng.num_users if mode == "user" else cfg["num_users"]
        if mode == "single" and args.id_span < 1.0:
            u_hi = max(1, int(round(u_hi * args.id_span)))
        u = torch.randint(0, u_hi, (B // g,), generator=gen, device="cuda", dtype=torch.int32)
        u = u.repeat_interleave(g)
        it = torch.randint(0, cfg["num_items"], (B,), generator=gen, device="cuda", dtype=torch.int32)
        y = torch.tensor([0.0] * (g - 1) + [1.0], device="cuda").repeat(B // g)
        pool.append((u.contiguous(), it.contiguous(), y.contiguous()))
    k = 10 if g > 10 else g - 1
    inv = 1.0 / (B * world)

    def step(i):
        if sampler is not None:
            (u, it), y = sampler[i % len(sampler)]
        else:
            u, it, y = pool[i % len(pool)]
        if dp is None and sampler is None:
            nu, ni, _ = pool[(i + 1) % len(pool)]   # the next step's ids: counted inside this step
            eng.train_step(u, it, y, group=g, k=k, inv_batch=inv, next_batch=(nu, ni))
        elif dp is None:
            eng.train_step(u, it, y, group=g, k=k, inv_batch=inv)
        elif mode in ("user", "sharded") and sampler is None:
            nu, ni, _ = pool[(i + 1) % len(pool)]
            dp.train_step(u, it, y, group=g, k=k, next_batch=(nu, ni))
        else:
            dp.train_step(u, it, y, group=g, k=k)

    def barrier():
        torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()
            torch.cuda.synchronize()

    for i in range(args.warmup):
        step(i)
    barrier()
    eng.flush() if hasattr(eng, "flush") else None
    barrier()
    # timed region.  The profiled launch groups carry HIP events in their dispatch packets
    # (hipExtLaunchKernel): per-kernel durations with no marker packets added to the stream.
    if not args.no_kernel_timing:
        N.profile_enable([N.K_EMB_UPDATE, N.K_FWD_BWD, N.K_INDEX, N.K_SAMPLE, N.K_CATCHUP], 2 * args.steps)
    every = max(1, min(args.time_every, args.steps // 6))   # at least 6 sampled steps
    if mode == "user":
        # the collectives as they run inside the step: side-stream spans and the compute stream's
        # waits, on the same sampled steps' schedule (read after the region)
        dp.exchange_timing(every)
    t0 = time.perf_counter()
    # one launch group per sampled step (its events lengthen that step by ~9 us per group): the
    # forward/backward and the embedding update (the two roofline kernels) alternate, the index and
    # the catch-up (and the sampler) take every third turn
    rota = [[N.K_FWD_BWD], [N.K_EMB_UPDATE]]
    minor = [[N.K_INDEX], [N.K_CATCHUP]] + ([[N.K_SAMPLE]] if sampler is not None else [])
    turns = []
    for j in range(args.steps // every + 1):
        turns.append(rota[j % 2] if j % 3 != 2 else minor[(j // 3) % len(minor)])
    for i in range(args.steps):
        if not args.no_kernel_timing and every > 1:
            # mid-interval: the first timed step (after the pre-region flush and sync: clocks and
            # caches cold) is not sampled
            N.profile_pause(i % every != every // 2)
            if i % every == every // 2:
                N.profile_select(turns[i // every])
        step(args.warmup + i)
    t_issue = time.perf_counter() - t0   # host time to issue the K steps (diagnostic, stderr)
    if not args.no_kernel_timing:
        N.profile_pause(True)    # the end-of-region flush is not a step's catch-up
    if hasattr(eng, "flush"):
        eng.flush()   # deferred decay settled inside the timed region: the table ends in the dense state
    t_flush_issued = time.perf_counter() - t0
    barrier()
    if not args.no_kernel_timing:
        N.profile_pause(False)
    elapsed = time.perf_counter() - t0
    print("host issue %.1f us for %d steps (%.1f us/step), flush issued at %.1f us, region %.1f us"
          % (t_issue * 1e6, args.steps, t_issue * 1e6 / max(1, args.steps), t_flush_issued * 1e6, elapsed * 1e6),
          file=sys.stderr)
    # sampled steps per launch group (one group per sampled step when every > 1)
    sampled = [turns[i // every] if every > 1 else None for i in range(every // 2 if every > 1 else 0, args.steps, every)]

    def steps_of(k):
        return max(1, sum(1 for t in sampled if t is None or k in t))
    in_step = None
    if mode == "user":
        xt = dp.read_exchange_timing()
        dp.exchange_timing(0)
        keys = ("rs_ar_ms", "ag_ms", "rs_ar_exposed_ms", "ag_exposed_ms")
        mine = torch.tensor([xt[k_] if xt[k_] is not None else float("nan") for k_ in keys], dtype=torch.float64,
                            device="cuda")
        allr = [torch.zeros_like(mine) for _ in range(world)] if dist.is_initialized() else [mine]
        if dist.is_initialized():
            dist.all_gather(allr, mine)
        allr = torch.stack(allr).cpu().numpy()
        in_step = {"path": xt["path"], "sampled_steps_per_rank": xt["steps"],
                   "note": "ms per sampled step; *_ms: the collective on the communicator's side stream, "
                           "*_exposed_ms: the compute stream's wait for it (max/min over the ranks)"}
        for j, k_ in enumerate(keys):
            col = allr[:, j]
            in_step[k_] = (None if np.isnan(col).all() else
                           {"max": round(float(np.nanmax(col)), 4), "min": round(float(np.nanmin(col)), 4)})
    ms_emb, nl = N.profile_read(N.K_EMB_UPDATE)
    ms_fb, nfb = N.profile_read(N.K_FWD_BWD)
    ms_idx, nidx = N.profile_read(N.K_INDEX)
    ms_smp, nsmp = N.profile_read(N.K_SAMPLE)
    ms_cu, ncu = N.profile_read(N.K_CATCHUP)
    N.profile_enable([], 0)
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = args.steps * B * world / elapsed
    kern_ms = ms_emb / nl if nl else float("nan")
    fb_ms = ms_fb / nfb if nfb else float("nan")
    fb_flops = fwd_bwd_flops(cfg) * B
    contribs = grad_rows(eng, B, g) if mode != "sharded" else 2 * B
    replay_rows = replay_rows_here = 0.0
    fb_bytes = fwd_bwd_bytes(eng.shape, B, contribs)
    fill_bytes = 0
    train_exchange = dp.last_exchange if mode == "sharded" else None
    if mode == "sharded" and getattr(eng, "lazy", False):
        # deferred decay: the m served rows (unique per source) read and written (p, m, v), their
        # m received gradient rows, the owner index entries (list + (offset, count))
        m_srv, W = train_exchange[1], eng.shape.row_width
        nbytes = 24 * m_srv * W + m_srv * W * 4 + m_srv * 12
    elif mode == "sharded":
        nbytes = emb_update_bytes(eng.shape, B, sparse_rows=(eng.shard_rows, train_exchange[1]))
    elif getattr(eng, "lazy", False) and mode == "single":
        touched = float(np.mean([torch.unique(u).numel() + torch.unique(it).numel() for u, it, _ in pool[:16]]))
        nbytes = emb_update_bytes(eng.shape, B, touched_rows=touched, contribs=contribs)
        if sampler is None and eng.kernel_for(B) in ("fused-mfma-wave", "fused-mfma-unit"):
            # the counted batch's index is filled inside the forward/backward launch: per contribution
            # its key's block offset read, cursor atomic and list slot written (the ids are already
            # counted), per touched row its scan-ahead entry read and touched-list entry written
            fill_bytes = contribs * 12 + touched * 24
        if sampler is None:
            nbytes += 2 * B * (4 + 8)   # the launch also counts the next batch: id reads + counter atomics
            # ... and catches the next batch's stale rows up (the rows it touches that this step
            # did not): their p, m, v read and written once more before the next forward pass
            replay_rows = replayed_rows(pool, args.warmup, args.steps, eng.num_users, eng.num_rows, items=True)
            # a replayed row: p, m, v read, p written (the next update re-derives m and v: P-ahead rows);
            # the rows owing few steps are replayed in the stats launch, not in this one
            owed = deferred_replay_owed(N.build_info())
            replay_rows_here = (replayed_rows(pool, args.warmup, args.steps, eng.num_users, eng.num_rows, items=True,
                                              far=owed) if owed else replay_rows)
            nbytes += 16 * replay_rows_here * eng.shape.row_width
        if eng.kernel_for(B) == "fused-mfma-wave" and B >= 16384:
            # the launch's dense-layer blocks reduce the wave kernel's 256 dense-gradient slabs (both
            # levels) and step the dense layers: slab reads + p, m, v of every dense parameter
            nbytes += 256 * eng.mlp_params * 4 + 24 * eng.mlp_params
    elif mode == "user":
        # two launches per step: the own users' scatter-add + Adam over the B user contributions
        # (ncf_update_rows), then Adam over the item rows with the all-reduced dense gradient
        # (ncf_apply_update); bytes per launch = the step's bytes / 2, time per launch = the average
        Uloc, W = eng.num_users, eng.shape.row_width
        cu = contribs - B   # the own users' gradient rows
        if getattr(eng, "lazy", False):
            # deferred decay of the own users: the touched ones only, plus (counting ahead) the next
            # batch's id reads + counter atomics and the replay of its own rows this step missed
            tu = float(np.mean([torch.unique(u).numel() for u, _, _ in pool[:16]]))
            own = 24 * tu * W + cu * W * 4 + cu * 4 + 2 * B * (4 + 8)
            replay_rows = replay_rows_here = replayed_rows(pool, args.warmup, args.steps, eng.num_users, Uloc,
                                                           items=False)
            own += 16 * replay_rows * W   # P-ahead replays: p, m, v read, p written
        else:
            own = 24 * Uloc * W + cu * W * 4 + cu * 4 + (Uloc + 1) * 4
        item_rows = (eng.num_rows - Uloc) if not dp.split else max(0, min(dp.Ic, eng.num_rows - Uloc))
        nbytes = (own + 28 * item_rows * W) / 2.0
    else:
        nbytes = emb_update_bytes(eng.shape, B, dense_rows=(dp.row_count if mode == "replicated" else None),
                                  contribs=contribs)
    achieved = nbytes / (kern_ms * 1e-3) / 1e9

    # HR@10 on a synthetic validation set (1 positive + 99 sampled items per user), per rank
    # evaluation users drawn inside the table (user mode: this rank's own users, as local ids;
    # config A's table has 943 users, so at most that many distinct ones)
    ev_table = eng.num_users if mode == "user" else cfg["num_users"]
    ev_users = min(2000, ev_table)
    eval_ms = None
    ev_u = torch.randperm(ev_table, generator=gen, device="cuda")[:ev_users].to(torch.int32).repeat_interleave(100)
    ev_i = torch.randint(0, cfg["num_items"], (ev_users * 100,), generator=gen, device="cuda", dtype=torch.int32)
    if own:   # the emulated rank evaluates on rows it owns
        U, I = cfg["num_users"], cfg["num_items"]
        i0 = (rank - U) % ew
        ev_u = ((ev_u.long() % ((U - rank + ew - 1) // ew)) * ew + rank).to(torch.int32)
        ev_i = ((ev_i.long() % ((I - i0 + ew - 1) // ew)) * ew + i0).to(torch.int32)
    ev_y = torch.tensor([0.0] * 99 + [1.0], device="cuda").repeat(ev_users)
    if mode == "sharded":
        probs = dp.predict(ev_u, ev_i)
        hit, dcg = eng.group_metrics(probs, ev_y, group=100, k=10)
        hd = torch.stack([hit.double().sum(), dcg.double().sum()])
    else:
        st = eng.val_stats.new_zeros(eng.val_stats.shape)
        eng.evaluate(ev_u, ev_i, ev_y, group=100, k=10, stats=st)
        torch.cuda.synchronize()
        t_ev = time.perf_counter()
        for _ in range(5):
            eng.evaluate(ev_u, ev_i, ev_y, group=100, k=10, stats=eng.val_stats.new_zeros(eng.val_stats.shape))
        torch.cuda.synchronize()
        eval_ms = (time.perf_counter() - t_ev) / 5 * 1e3
        r = NCFEngine.read_stats(st)
        hd = torch.tensor([r["hr"] * ev_users, r["dcg"] * ev_users], dtype=torch.float64, device="cuda")
    if dist.is_initialized():
        dist.all_reduce(hd)
    hr = {"hr": float(hd[0]) / (ev_users * world), "dcg": float(hd[1]) / (ev_users * world)}

    emb_kernel = "k_emb_adam_touched" if getattr(eng, "lazy", False) and mode in ("single", "sharded") else "k_emb_update"
    # the update launch's traffic depends on whether it also counts (and catches up) the next batch:
    # the files are keyed on it (layout "single-ahead" / "single")
    ahead = getattr(eng, "lazy", False) and sampler is None and mode in ("single", "user", "sharded")
    traffic = pmc_traffic(emb_kernel, args.config, B, mode + ("-ahead" if ahead else ""))
    kpath = eng.kernel_for(B) if hasattr(eng, "kernel_for") else ("fused-mfma-tile" if eng.fast_path else "generic")
    fb_kernel = {"fused-mfma-tile": "k_fb_fused", "fused-mfma-unit": "k_fb_unit",
                 "fused-mfma-wave": "k_fb_wave"}.get(kpath)
    fb_traffic = pmc_traffic(fb_kernel, args.config, B, mode) if fb_kernel else None
    par = {"single": "dp1 (one table)",
           "user": ("dp%d user-partitioned data (rank r trains users u %% %d == r and alone holds their rows + "
                    "Adam state); item table replicated, its Adam split across the ranks (reduce-scatter of the "
                    "item-row grad + all-reduce of the dense-layer grad in one RCCL group, Adam on 1/%d of the "
                    "item rows, all-gather of the updated rows)" % (world, world, max(world, ew))
                    if args.item_optimizer == "split" else
                    "dp%d user-partitioned data (rank r trains users u %% %d == r and alone holds their rows + "
                    "Adam state); item table replicated; ONE all-reduce per step of [item-row grad | dense-layer "
                    "grad | summary]" % (world, world)),
           "sharded": "dp%d row-sharded tables (rank r owns rows g %% %d == r + their Adam state; all_to_all of "
                      "unique row ids / rows / row grads, all-reduce of the dense-layer grad)" % (world, world),
           "replicated": "dp%d replicated tables (reduce-scatter of the dense embedding grad, sharded Adam, "
                         "all-gather of the table; all-reduce of the dense-layer grad)" % world}[mode]

    exchange = None
    if mode == "user":
        # the step's one collective, timed alone after the timed region (same buffer size, same
        # communicator): how long the all-reduce the step overlaps with its own-user update takes
        buf = dp.shared.clone()

        def collectives():
            if dp.split and world > 1:
                # reduce-scatter of the item-row grad, all-reduce of the dense part, all-gather of the rows
                ig = buf[:dp.grads[0].numel()]
                part = torch.empty(ig.numel() // world, dtype=buf.dtype, device=buf.device)
                dist.reduce_scatter_tensor(part, ig)
                dist.all_reduce(buf[dp.grads[0].numel():])
                dist.all_gather_into_tensor(ig, part)
            else:
                dist.all_reduce(buf)
        for _ in range(3):
            collectives()
        torch.cuda.synchronize()
        t_ar = time.perf_counter()
        for _ in range(10):
            collectives()
        torch.cuda.synchronize()
        ar_ms = (time.perf_counter() - t_ar) / 10 * 1e3
        exchange = {"allreduce_bytes_per_step": dp.shared.numel() * dp.shared.element_size(),
                    "allreduce_ms_standalone": round(ar_ms, 4),   # the step's collectives, timed alone
                    "collectives_per_step": 3 if dp.split else 1,
                    "item_optimizer": ("split: reduce-scatter of the item-row grad + all-reduce of [dense-layer "
                                       "grad | summary] (one RCCL group), all-gather of the updated item rows"
                                       if dp.split else "replicated: one all-reduce"),
                    "native_step": dp.comm is not None,
                    "native_step_check": native_check,
                    "in_step": in_step,
                    "local_users": eng.num_users}
    elif mode == "sharded":
        W = eng.shape.row_width
        exchange = {"unique_rows_per_rank": train_exchange[0], "rows_served_per_rank": train_exchange[1],
                    "shard_rows": eng.shard_rows,
                    "all_to_all_bytes_per_step": {"row_ids": 4 * train_exchange[0],
                                                  "row_values": 4 * W * train_exchange[0],
                                                  "row_grads": 4 * W * train_exchange[0]},
                    "allreduce_bytes_per_step": eng.dense_buf.numel() * 4,
                    "counts": "planned a step ahead (pinned host copy, no per-step device sync)"}
    if exchange is not None:
        exchange.update(ranks=world, backend=dist.get_backend(),
                        transport="RCCL over xGMI" if dist.get_backend() == "nccl" else dist.get_backend())

    emb_roof = {"bound": "hbm", "kernel": ("embedding scatter-add + Adam on the batch's touched rows "
                                           "(k_emb_adam_touched; deferred exact decay"
                                           + ("; its launch also counts the next batch's index "
                                              "contributions)" if sampler is None else ")")
                                           if getattr(eng, "lazy", False) and mode == "single" else
                                           "embedding Adam, 2 launches per step (k_emb_adam_touched: the "
                                           "touched own-user rows with their scatter-add, deferred exact "
                                           "decay, the next batch counted and its own rows caught up ahead; "
                                           "k_emb_update_mlp: item rows with the all-reduced gradient + the "
                                           "dense layers)" if mode == "user" and getattr(eng, "lazy", False) else
                                           "embedding Adam, 2 launches per step (k_emb_update: own-user "
                                           "rows with their scatter-add; item rows with the all-reduced "
                                           "gradient)" if mode == "user" else
                                           "row-sharded owner update: scatter-add of the received row gradients + Adam "
                                           "on the served rows (k_emb_adam_touched; deferred exact decay)"
                                           if mode == "sharded" and getattr(eng, "lazy", False) else
                                           "embedding scatter-add + Adam sweep (k_emb_update)"),
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": nbytes, "avg_launch_ms": round(kern_ms, 5),
                "gradient_rows_per_step": contribs, "replayed_rows_per_step": replay_rows,
                "replayed_rows_in_launch": replay_rows_here,
                "launches_per_step": round(nl / steps_of(N.K_EMB_UPDATE), 2),
                "timed_steps": "every %d-th step of the timed region, one launch group per sampled step "
                               "(HIP events in the dispatch packets): %d launches timed" % (every, nl),
                "traffic_source": "rocprofv3 --pmc FETCH_SIZE(x2 gfx950) + WRITE_SIZE, profiles/traffic/ "
                                  "(this config, batch, layout and counted-ahead form only; null if not "
                                  "measured)"}
    fb_bytes += fill_bytes
    fb_achieved = fb_flops / (fb_ms * 1e-3) / 1e12
    fb_exec = fwd_bwd_executed_flops(cfg, B, g, kpath)
    # the MLP tower's matrix products run on bf16 MFMA in the bf16 mode (config B): its dense peak
    fb_peak = FP16_MFMA_PEAK_TFS if prec == "bf16" else FP32_MFMA_PEAK_TFS
    fb_roof = {"bound": "mfma", "kernel": {
                   "fused-mfma-tile": "fused NeuMF forward+backward, 128-sample tiles (k_fb_fused, fp32 MFMA "
                                      "32x32x2)",
                   "fused-mfma-unit": "fused NeuMF forward+backward, 32-sample units split by output feature "
                                      "over a workgroup's waves (k_fb_unit, fp32 MFMA 16x16x4)",
                   "fused-mfma-wave": "fused NeuMF forward+backward, 16-sample units, the whole chain in one "
                                      "wave (k_fb_wave, fp32 MFMA 16x16x4)",
                   "layered-mfma": "layer-by-layer forward+backward, every layer on hand-written fp32 MFMA "
                                   "(k_lay_l1f gather + layer 1, k_lay_mid layers 2.. + loss + backward to G1, "
                                   "k_lay_dw1, k_lay_l1b dX + gradient rows)"}.get(kpath, "generic forward+backward"),
               "achieved": round(fb_achieved, 2), "peak": fb_peak, "unit": "TFLOP/s",
               "frac": round(fb_achieved / fb_peak, 4), "traffic": fb_traffic,
               "peak_of": "bf16 dense MFMA (the MLP products; GMF, loss and Adam stay fp32)" if prec == "bf16"
                          else "fp32 dense MFMA",
               "traffic_unit": "HBM bytes per launch",
               "algorithmic_flops_per_launch": fb_flops, "avg_launch_ms": round(fb_ms, 5),
               "executed_flops_per_launch": fb_exec,
               "executed_TFLOPs": round(fb_exec / (fb_ms * 1e-3) / 1e12, 2) if fb_exec else None,
               "frac_executed": round(fb_exec / (fb_ms * 1e-3) / 1e12 / fb_peak, 4) if fb_exec else None,
               "hbm_GBs": round(fb_bytes / (fb_ms * 1e-3) / 1e9, 1), "algorithmic_bytes_per_launch": fb_bytes,
               "index_fill_bytes_in_launch": fill_bytes or None}
    busy = pmc_mfma_busy(fb_kernel, args.config, B) if fb_kernel else None
    if busy is not None:
        # what the counters say limits it: "bound" names the roofline it is priced against
        hbm_frac = fb_roof["hbm_GBs"] / HBM_PEAK_GBS
        fb_roof["mfma_busy_frac"] = busy["mfma_busy_frac"]
        fb_roof["limiter"] = ("mfma" if busy["mfma_busy_frac"] >= 0.6 else "hbm" if hbm_frac >= 0.6 else
                              "issue/latency: MFMA pipe busy %.2f of the kernel's cycles, HBM %.2f of peak "
                              "(%s)" % (busy["mfma_busy_frac"], hbm_frac, busy["source"]))
    # `roofline` = the step's dominant kernel (longest average time per step)
    fb_per_step = fb_ms * nfb / steps_of(N.K_FWD_BWD)
    emb_per_step = kern_ms * nl / steps_of(N.K_EMB_UPDATE)
    dominant_fb = not (emb_per_step > fb_per_step)

    if rank == 0:
        cpu = None
        cpu_e2e = None
        if world == 1 and not args.no_cpu_baseline and not big:
            cpu = cpu_baseline(cfg, args.cpu_seconds, args.cpu_protocol)
            smp, smp_desc = cpu_sampler_baseline(cfg, min(6.0, args.cpu_seconds))
            # model step and sampler back to back on the host (the reference's Keras loop, workers=1)
            cpu_e2e = dict(value=round(1.0 / (1.0 / cpu["value"] + 1.0 / smp), 1), unit="samples/s",
                           cores=cpu["cores"], kind="port", sampler_samples_per_s=round(smp, 1),
                           sample="model step as cpu_baseline + the reference-faithful host sampler "
                                  "(1 thread): " + smp_desc)
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong" if args.global_batch else "weak", "vs_baseline": None,
            "dtype": "bf16 MLP operands, fp32 accumulate/master/Adam" if prec == "bf16" else "fp32",
            "data": ("synthetic ml-20m-shaped ratings (%d positives), negatives sampled on the device each step"
                     % len(sampler.data) if sampler is not None else
                     "synthetic (uniform ids, seeded; %d distinct batches cycled; random-init weights)" % len(pool)),
            "config": {"workload": cfg["workload"], "global_batch": B * world, "per_gpu_batch": B,
                       "negatives_per_positive": cfg["negs"], "parallelism": par,
                       "kernel_path": kpath, **({"id_span": args.id_span} if args.id_span < 1.0 else {})},
            "roofline": fb_roof if dominant_fb else emb_roof,
            "roofline_emb_update" if dominant_fb else "roofline_fwd_bwd": emb_roof if dominant_fb else fb_roof,
            # the north star's gather + scatter bandwidth over both kernels together: the
            # forward/backward's rows in and gradient rows out plus the update's bytes, over the two
            # launches' summed average durations
            "gather_scatter_hbm": {
                "bytes_per_step": int(fb_bytes + nbytes), "ms_per_step": round(fb_ms + kern_ms, 5),
                "achieved": round((fb_bytes + nbytes) / ((fb_ms + kern_ms) * 1e-3) / 1e9, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round((fb_bytes + nbytes) / ((fb_ms + kern_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "index_build_ms": round(ms_idx / max(nidx, 1), 5),
            "sampler_ms": round(ms_smp / nsmp, 5) if nsmp else None,
            "catchup_ms": round(ms_cu / ncu, 5) if ncu else None,
            "adam": ("deferred exact decay (untouched rows replay their zero-gradient steps when next touched; "
                     "flushed inside the timed region; bitwise the dense Keras sweep)"
                     + ("; the replicated item rows are swept every step" if mode == "user" else "")
                     if getattr(eng, "lazy", False) else "dense sweep of every row every step (Keras, F5)"),
            "cpu_baseline": cpu,
            "cpu_baseline_with_sampler": cpu_e2e,
            "hr_at_10": {"value": round(hr["hr"], 4), "ndcg_at_10": round(hr["dcg"], 4),
                         "data": "synthetic eval groups (random ids; ~0.1 expected for an untrained model)",
                         "eval_samples": ev_users * 100,
                         "eval_ms": round(eval_ms, 4) if eval_ms is not None else None},
        }
        if exchange is not None:
            line["exchange"] = exchange
        # provenance of the benched binary: the source hash compiled into it and its -D defines
        # (empty for the product build; csrc/build.py rebuilds whenever the tree's hash differs)
        line["build_info"] = _native_build_info()
        if args.emulate_world > 1 and mode == "sharded":
            line["emulated_world"] = args.emulate_world
            line["note"] = ("diagnostic: rank 0's per-rank compute of the %d-rank row-sharded step on one GPU (a "
                            "1/%d shard of the table; batches drawn from its own rows so that its plan, serve, "
                            "forward/backward and update see the work one rank of %d does; the all_to_all / "
                            "all-reduce exchanges replaced by its own buffers); not a scaling result"
                            % (args.emulate_world, args.emulate_world, args.emulate_world))
        elif args.emulate_world > 1:
            line["emulated_world"] = args.emulate_world
            line["note"] = ("diagnostic: rank 0's per-rank compute of the %d-rank user-partitioned step on one GPU "
                            "(local table of 1/%d of the users, a one-rank communicator); not a scaling result"
                            % (args.emulate_world, args.emulate_world))
        emit(json.dumps(line))
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
