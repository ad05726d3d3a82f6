"""Train and evaluate models (mirror of the reference ``movierec/trainer.py``).

``train()`` keeps the reference's flow (``trainer.py:30-80``): leave-two-out
split, train generator (no extra data, shuffled) and validation generator
(train as extra, not shuffled), table sizes from the dataset constants, build,
``fit_generator``, ``save``.  The CLI keeps ``-m -n -d -o -l``
(``trainer.py:83-102``) and adds ``--gmf-dim``, ``--epochs``, ``--seed``.
"""

import copy
import logging

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


def train(model_name, dataset_name, data_dir, output_dir, params=DEFAULT_PARAMS, verbose=1):
    train_df, validation_df, _test_df = data_pipeline.load_ratings_train_test_sets(dataset_name, data_dir)
    train_gen = data_pipeline.MovieLensDataGenerator(
        dataset_name, train_df, params["batch_size"], params["num_negs_per_pos"],
        extra_data_df=None,  # negatives in train may be val/test positives (as in the reference)
        shuffle=True)
    val_gen = data_pipeline.MovieLensDataGenerator(
        dataset_name, validation_df, params["batch_size_eval"], params["num_negs_per_pos_eval"],
        extra_data_df=train_df, shuffle=False)
    # the reference mutates the caller's dict here (trainer.py:72-73); keep that
    params["num_users"] = train_gen.num_users
    params["num_items"] = train_gen.num_items
    model = MovierecModel(params, model_name, output_dir, verbose)
    model.log_summary()
    history = model.fit_generator(train_gen, val_gen, params["epochs"])
    model.save()
    return model, history


def main(argv=None):
    import argparse
    parser = argparse.ArgumentParser(description="Train a movie recommendation (NCF/NeuMF) model on MI355X.")
    parser.add_argument("-m", "--model-name", type=str, required=True, help="Name given to the saved weights, params and checkpoint files.")
    parser.add_argument("-n", "--dataset-name", type=str, required=True, help="Movielens dataset name.")
    parser.add_argument("-d", "--data-dir", type=str, default="data/", help="Dataset directory to read ratings from")
    parser.add_argument("-o", "--output-dir", type=str, default="models", help="Directory the trained model files are written to.")
    parser.add_argument("-l", "--log-level", type=str, default="INFO", help="Python logging level name, e.g. DEBUG, INFO (the default) or WARNING.")
    parser.add_argument("--gmf-dim", type=int, default=0, help="NeuMF GMF branch width (0 = MLP-only model).")
    parser.add_argument("--epochs", type=int, default=None)
    parser.add_argument("--seed", type=int, default=None)
    args = parser.parse_args(argv)
    logging.getLogger().setLevel(logging.getLevelName(args.log_level))
    params = copy.deepcopy(DEFAULT_PARAMS)
    params["gmf_dim"] = args.gmf_dim
    if args.epochs is not None:
        params["epochs"] = args.epochs
    if args.seed is not None:
        params["seed"] = args.seed
    logging.info("Starting training with params: {}".format(params))
    train(args.model_name, args.dataset_name, args.data_dir, args.output_dir, params, logging.getLogger().level)


if __name__ == "__main__":
    main()
