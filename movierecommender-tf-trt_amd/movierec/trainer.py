"""Train and evaluate models (mirror of the reference ``movierec/trainer.py``).

``train()`` keeps the reference's flow (``trainer.py:30-80``): leave-two-out
split, train generator (no extra data, shuffled) and validation generator
(train as extra, not shuffled), table sizes from the dataset constants, build,
``fit_generator``, ``save``.  The CLI keeps ``-m -n -d -o -l``
(``trainer.py:83-102``) and adds ``--gmf-dim``, ``--epochs``, ``--seed``,
``--sampler``, ``--batch-size``, ``--batch-size-eval``, ``--negs``, ``--precision``.

New params keys (optional):
  * ``sampler``: ``"host"`` (default: ``MovieLensDataGenerator``, the reference's numpy RNG
    stream batch for batch) or ``"device"`` (``DeviceMovieLensDataGenerator``: negatives drawn
    on the GPU by ``ncf_sample_batch``, no host sampling or per-batch H2D copy);
  * ``world_size``: data parallelism over that many GPUs, one process each (``python -m
    torch.distributed.run --nproc-per-node N -m movierec.trainer ...``; the CLI takes it from
    WORLD_SIZE).  The ratings are partitioned by user — rank r trains the users u % N == r as
    local ids u // N (``UserPartitionedDataParallel``) — and ``batch_size`` stays the GLOBAL batch
    of one step, split evenly over the ranks; ``batch_size_eval`` is split into whole groups per
    rank (``eval_batch_per_rank``).
"""

import copy
import logging
import os

import numpy as np

from . import data_pipeline
from .model import MovierecModel

DEFAULT_PARAMS = {
    # model ("num_users"/"num_items" come from the data generator)
    "layers_sizes": [64, 32, 16, 8],
    "layers_l2reg": [0, 0, 0, 0],
    # training
    "optimizer": "adam",
    "lr": 0.001,
    "beta_1": 0.9,
    "beta_2": 0.999,
    "batch_size": 100,
    "batch_size_eval": 200,
    "num_negs_per_pos": 9,
    "num_negs_per_pos_eval": 99,
    "k": 5,
    "epochs": 20,
}


def user_partition(df, world, rank):
    """Rank ``rank``'s share of a ratings frame under user-partitioned data parallelism: the rows
    of users u % world == rank, user ids made local (u // world), file order kept."""
    u = np.asarray(df[data_pipeline.COL_USER_ID])
    out = df[u % world == rank].reset_index(drop=True)
    out[data_pipeline.COL_USER_ID] = (np.asarray(out[data_pipeline.COL_USER_ID]) // world).astype(u.dtype)
    out.attrs = dict(df.attrs)
    return out


def _per_rank(batch, negs, world, what):
    if batch % world or (batch // world) % (negs + 1):
        raise ValueError("{} {} does not split into {} rank batches of whole (num_negs + 1)-groups"
                         .format(what, batch, world))
    return batch // world


def eval_batch_per_rank(batch_eval, negs_eval, world):
    """Validation batch of one rank: the global ``batch_size_eval`` split over the ranks, rounded
    down to whole (negs + 1)-groups (at least one group).  Validation metrics are means over
    groups, so the split does not change what a group contributes; it only sizes the batches
    (the reference's default 200 with 99 negatives is 2 groups: one per rank at world 2, one
    group per rank at any larger world)."""
    g = negs_eval + 1
    per = (batch_eval // world) // g * g
    return max(per, g)


def train(model_name, dataset_name, data_dir, output_dir, params=DEFAULT_PARAMS, verbose=1):
    train_df, validation_df, _test_df = data_pipeline.load_ratings_train_test_sets(dataset_name, data_dir)
    world = int(params.get("world_size", 1))
    rank = 0
    bs, bs_eval = params["batch_size"], params["batch_size_eval"]
    if world > 1:
        from .distributed import ensure_process_group
        rank = ensure_process_group(world, params.get("dist_backend"))
        train_df = user_partition(train_df, world, rank)
        validation_df = user_partition(validation_df, world, rank)
        bs = _per_rank(bs, params["num_negs_per_pos"], world, "batch_size")
        bs_eval = eval_batch_per_rank(bs_eval, params["num_negs_per_pos_eval"], world)
    if params.get("sampler", "host") == "device":
        from .sampler import DeviceMovieLensDataGenerator

        def gen(df, b, n, extra, shuffle, salt):
            return DeviceMovieLensDataGenerator(dataset_name, df, b, n, extra_data_df=extra, shuffle=shuffle,
                                                seed=int(params.get("seed") or 0) * 1000003 + 2 * rank + salt)
    elif params.get("sampler", "host") == "host":
        def gen(df, b, n, extra, shuffle, salt):
            return data_pipeline.MovieLensDataGenerator(dataset_name, df, b, n, extra_data_df=extra, shuffle=shuffle)
    else:
        raise ValueError("sampler must be 'host' or 'device', found {}".format(params.get("sampler")))
    # negatives in train may be val/test positives (as in the reference)
    train_gen = gen(train_df, bs, params["num_negs_per_pos"], None, True, 0)
    val_gen = gen(validation_df, bs_eval, params["num_negs_per_pos_eval"], train_df, False, 1)
    # the reference mutates the caller's dict here (trainer.py:72-73); keep that
    params["num_users"] = train_gen.num_users
    params["num_items"] = train_gen.num_items
    model = MovierecModel(params, model_name, output_dir, verbose)
    model.log_summary()
    history = model.fit_generator(train_gen, val_gen, params["epochs"])
    model.save()
    raw = train_df.attrs.get("raw_item_ids")
    if raw is not None and rank == 0:
        # dense item id -> the dataset's movieId - 1 (ml-20m's remap, data_pipeline F6)
        np.save(os.path.join(output_dir, "{}_raw_item_ids.npy".format(model_name)), np.asarray(raw))
    return model, history


def main(argv=None):
    import argparse
    parser = argparse.ArgumentParser(description="Train a movie recommendation (NCF/NeuMF) model on MI355X.")
    parser.add_argument("-m", "--model-name", type=str, required=True,
                        help="Name given to the saved weights, params and checkpoint files.")
    parser.add_argument("-n", "--dataset-name", type=str, required=True,
                        help="One of ml-100k, ml-1m, ml-20m.")
    parser.add_argument("-d", "--data-dir", type=str, default="data/",
                        help="Directory holding the extracted MovieLens folders.")
    parser.add_argument("-o", "--output-dir", type=str, default="models",
                        help="Directory the trained model files are written to.")
    parser.add_argument("-l", "--log-level", type=str, default="INFO",
                        help="Python logging level name, e.g. DEBUG, INFO (the default) or WARNING.")
    parser.add_argument("--gmf-dim", type=int, default=0, help="NeuMF GMF branch width (0 = MLP-only model).")
    parser.add_argument("--epochs", type=int, default=None)
    parser.add_argument("--seed", type=int, default=None)
    parser.add_argument("--sampler", choices=["host", "device"], default="host",
                        help="host: the reference's numpy negative sampling; device: sampled on the GPU.")
    parser.add_argument("--batch-size", type=int, default=None, help="Training batch (global, all ranks).")
    parser.add_argument("--batch-size-eval", type=int, default=None,
                        help="Validation batch (global; each rank takes its share in whole groups).")
    parser.add_argument("--negs", type=int, default=None, help="Negatives per positive in training.")
    parser.add_argument("--precision", choices=["fp32", "bf16"], default=None,
                        help="MLP operand precision (bf16: BASELINE config B).")
    parser.add_argument("--dist-backend", choices=["nccl", "gloo"], default=None,
                        help="Process-group backend under torch.distributed.run (default: nccl = RCCL over xGMI).")
    args = parser.parse_args(argv)
    logging.getLogger().setLevel(logging.getLevelName(args.log_level))
    params = copy.deepcopy(DEFAULT_PARAMS)
    params["gmf_dim"] = args.gmf_dim
    params["sampler"] = args.sampler
    params["world_size"] = int(os.environ.get("WORLD_SIZE", "1"))   # under torch.distributed.run
    if args.dist_backend:
        params["dist_backend"] = args.dist_backend
    for key, val in (("epochs", args.epochs), ("seed", args.seed), ("batch_size", args.batch_size),
                     ("batch_size_eval", args.batch_size_eval),
                     ("num_negs_per_pos", args.negs), ("precision", args.precision)):
        if val is not None:
            params[key] = val
    logging.info("Starting training with params: {}".format(params))
    train(args.model_name, args.dataset_name, args.data_dir, args.output_dir, params, logging.getLogger().level)


if __name__ == "__main__":
    main()
