"""Recommender model: the reference's ``movierec/model.py`` API on the MI355X path.

``MovierecModel`` keeps the reference's constructor, parameter dict, checks
and error types (``model.py:54-133``), file naming (``:217-223``),
``save`` / ``load_from_dir`` / ``load_from_files`` (``:239-303``) and
``fit_generator`` with early stopping and best-checkpointing on
``val_output_dcg`` (``:305-333``).  ``RankLayer`` (``:336-358``) and the
metric functions ``hit_rate`` / ``discounted_cumulative_gain`` /
``_get_hits_per_user`` (``:361-455``) keep their signatures.

What changed underneath: the Keras graph (``build_mlp_model``, ``:135-195``)
becomes an :class:`NCFNetwork` handle whose parameters live on one MI355X
(``engine.NCFEngine``); training steps, predictions, ranks and metrics run in
the HIP library.  Additions: optional ``gmf_dim`` param (NeuMF GMF branch; 0 =
the reference MLP-only model), ``evaluate(generator, k)`` for full-protocol
HR@k/NDCG@k, and weights stored as safetensors (h5py is not available).

Documented deviations: ``load_from_files`` passes name/dir in the
intended order (the reference swaps them, ``model.py:301``);
checkpoints use the ``.safetensors`` suffix.
"""

import copy
import functools
import json
import logging
import math
import os
import random

import numpy as np

DEFAULT_PARAMS = {  # toy params, as in the reference (model.py:15-34)
    "num_users": 5,
    "num_items": 10,
    "layers_sizes": [5, 4],
    "layers_l2reg": [0.01, 0.01],
    "optimizer": "adam",
    "lr": 0.001,
    "beta_1": 0.9,
    "beta_2": 0.999,
    "batch_size": 6,
    "num_negs_per_pos": 2,
    "batch_size_eval": 12,
    "num_negs_per_pos_eval": 5,
    "k": 3,
}

ADAM_NAME = "adam"
SGD_NAME = "sgd"
OPTIMIZERS = [ADAM_NAME, SGD_NAME]

HIT_RATE = "hr"
DCG = "dcg"

OUTPUT_PRED = "output"
OUTPUT_RANK = "rank"

METRIC_VAL_DCG = "val_{}_{}".format(OUTPUT_PRED, DCG)

WEIGHTS_SUFFIX = "_weights.safetensors"
RUNTIME_KEYS = ("world_size", "dist_backend")


class _Layer(object):
    def __init__(self, name, kind, output_shape, weights=()):
        self.name = name
        self.kind = kind
        self.output_shape = output_shape
        self.weight_names = list(weights)

    def __repr__(self):
        return "<%s %s %s>" % (self.kind, self.name, self.output_shape)


class NCFNetwork(object):
    """Stands where the reference's ``keras.Model`` stood (``model.py:194``):
    two int inputs (user, item), outputs ``[output (B,1), rank (B/(n+1), n+1)]``."""

    def __init__(self, engine, layers_sizes, gmf_dim, num_negs_train, num_negs_eval, name, dp=None):
        self.engine = engine
        self.dp = dp          # UserPartitionedDataParallel when world_size > 1
        self.name = name
        self._negs = (num_negs_train, num_negs_eval)
        self.learning_phase = 0
        self.input_shape = [(None, 1), (None, 1)]
        self.inputs = ["user_input", "item_input"]
        self.output_shape = [(None, 1), (None, None)]
        self.outputs = [OUTPUT_PRED, OUTPUT_RANK]
        self.trainable = True
        L = list(layers_sizes)
        ly = [_Layer("user_input", "InputLayer", (None, 1)), _Layer("item_input", "InputLayer", (None, 1))]
        if L:   # layers_sizes == [] with gmf_dim > 0: the GMF-only model (BASELINE config A)
            du, di = L[0] // 2, L[0] - L[0] // 2
            ly += [_Layer("user_embedding", "Embedding", (None, 1, du), ["user_embedding"]),
                   _Layer("item_embedding", "Embedding", (None, 1, di), ["item_embedding"]),
                   _Layer("flatten", "Flatten", (None, du)), _Layer("flatten_1", "Flatten", (None, di)),
                   _Layer("concatenate", "Concatenate", (None, L[0]))]
        if gmf_dim > 0:
            ly += [_Layer("user_gmf_embedding", "Embedding", (None, 1, gmf_dim), ["user_gmf_embedding"]),
                   _Layer("item_gmf_embedding", "Embedding", (None, 1, gmf_dim), ["item_gmf_embedding"]),
                   _Layer("flatten_2", "Flatten", (None, gmf_dim)), _Layer("flatten_3", "Flatten", (None, gmf_dim)),
                   _Layer("gmf_multiply", "Multiply", (None, gmf_dim))]
        for l in range(1, len(L)):
            ly.append(_Layer("hidden_%d" % l, "Dense", (None, L[l]), ["hidden_%d/kernel" % l, "hidden_%d/bias" % l]))
        if gmf_dim > 0 and L:
            ly.append(_Layer("neumf_concatenate", "Concatenate", (None, gmf_dim + L[-1])))
        ly.append(_Layer(OUTPUT_PRED, "Dense", (None, 1), ["output/kernel", "output/bias"]))
        ly.append(_Layer(OUTPUT_RANK, "RankLayer", (None, None)))
        self.layers = ly
        self.trainable_weights = [w for layer in ly for w in layer.weight_names]
        self.trainable_variables = list(self.trainable_weights)
        self.non_trainable_weights = []
        self.non_trainable_variables = []

    def get_layer(self, name):
        for layer in self.layers:
            if layer.name == name:
                return layer
        raise ValueError("No such layer: " + name)

    def get_weights(self):
        """The whole model's weights.  Data-parallel (world_size > 1): gathered from every rank's
        users (a collective: every rank calls it)."""
        if self.dp is not None:
            return self.dp.keras_weights()
        return self.engine.keras_weights()

    def set_weights(self, w):
        """Load the whole model's weights (data-parallel: this rank keeps its users' rows)."""
        if self.dp is not None:
            from .distributed import partition_keras_weights
            w = partition_keras_weights(w, self.dp.world, self.dp.rank)
        self.engine.set_keras_weights(w)

    def local_user_ids(self, users):
        """Data-parallel: global ids of this rank's users (u % world == rank) -> local rows."""
        if self.dp is None:
            return users
        u = np.asarray(users)
        if u.size and np.any(u % self.dp.world != self.dp.rank):
            raise ValueError("user ids not owned by rank %d of %d (u %% world != rank)" % (self.dp.rank, self.dp.world))
        return u // self.dp.world

    def count_params(self):
        return sum(int(np.prod(a.shape)) for a in self.get_weights().values())

    def summary(self, print_fn=print):
        w = self.get_weights()
        print_fn("Model: %s (MI355X HIP path, fast_path=%s)" % (self.name, self.engine.fast_path))
        for layer in self.layers:
            n = sum(int(np.prod(w[x].shape)) for x in layer.weight_names)
            print_fn("%-22s %-12s %-18s %d" % (layer.name, layer.kind, layer.output_shape, n))
        print_fn("Total params: %d" % self.count_params())

    def predict_on_batch(self, x):
        """``[output (B,1) float32, rank (B/(n+1), n+1) int32]`` in the current
        learning phase (RankLayer group size, model.py:347)."""
        users, items = x
        users = self.local_user_ids(users)
        self.engine.check_ids(users, items)
        p = self.engine.predict(users, items)
        group = self._negs[0 if self.learning_phase else 1] + 1
        rank = self.engine.rank(p, group)
        return [p.cpu().numpy().reshape(-1, 1), rank.cpu().numpy()]

    def save_weights(self, path):
        w = self.get_weights()          # collective when data-parallel
        if self.dp is None or self.dp.rank == 0:
            save_tensors(path, w)

    def load_weights(self, path):
        self.set_weights(load_tensors(path))


def save_tensors(path, arrays):
    from safetensors.numpy import save_file
    save_file({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in arrays.items()}, path)


def load_tensors(path):
    from safetensors.numpy import load_file
    return {k: v.astype(np.float64) for k, v in load_file(path).items()}


class History(object):
    def __init__(self):
        self.history = {}
        self.epoch = []


class MovierecModel(object):
    """Movie Recommendation Model (reference model.py:49-333)."""

    def __init__(self, params=DEFAULT_PARAMS, model_name="movierec", output_dir="models/", verbose=1):
        # Same checks, order and exception types as the reference (model.py:73-112).
        self._num_users = params["num_users"]
        self._num_items = params["num_items"]
        self._layers_sizes = params["layers_sizes"]
        self._layers_l2reg = params["layers_l2reg"]
        if len(self._layers_sizes) != len(self._layers_l2reg):
            raise ValueError("'layers_sizes' length = {}, 'layers_l2reg' length = {}, but must be equal."
                             .format(len(self._layers_sizes), len(self._layers_l2reg)))
        self._num_layers = len(self._layers_sizes)
        self._optimizer = params["optimizer"]
        if self._optimizer not in OPTIMIZERS:
            raise NotImplementedError("Optimizer {} is not implemented.".format(params["optimizer"]))
        self._lr = params["lr"]
        self._beta_1 = params.get("beta_1", 0.9)
        self._beta_2 = params.get("beta_2", 0.999)
        self._batch_size = params["batch_size"]
        self._num_negs_per_pos = params["num_negs_per_pos"]
        if self._num_negs_per_pos <= 0:
            raise ValueError("num_negs_per_pos must be > 0, found {}".format(self._num_negs_per_pos))
        if self._batch_size % (self._num_negs_per_pos + 1):
            raise ValueError("Batch size must be divisible by (num_negs_per_pos + 1). Found: batch_size={}, "
                             "num_negs_per_pos={}".format(self._batch_size, self._num_negs_per_pos))
        self._batch_size_eval = params["batch_size_eval"]
        self._num_negs_per_pos_eval = params["num_negs_per_pos_eval"]
        if self._num_negs_per_pos_eval <= 0:
            raise ValueError("num_negs_per_pos_eval must be > 0, found {}".format(self._num_negs_per_pos_eval))
        if self._batch_size_eval % (self._num_negs_per_pos_eval + 1):
            raise ValueError("Batch size (eval) must be divisible by (num_negs_per_pos_eval + 1). Found: "
                             "batch_size_eval={}, num_negs_per_pos_eval={}".format(self._batch_size_eval,
                                                                                   self._num_negs_per_pos_eval))
        self._k = params.get("k", self._num_negs_per_pos + 1)
        if self._k > (self._num_negs_per_pos + 1):
            raise ValueError("'k' must be lower than (num_negs_per_pos + 1) and lower than (num_negs_per_pos_eval + 1)."
                             "Found: k={}, num_negs_per_pos={}, num_negs_per_pos_eval={}"
                             .format(self._k, self._num_negs_per_pos, self._num_negs_per_pos_eval))
        # NeuMF extension + runtime options (new, optional keys)
        self._gmf_dim = int(params.get("gmf_dim", 0))
        self._seed = params.get("seed", None)
        self._max_batch = int(params.get("max_batch", max(self._batch_size, self._batch_size_eval)))
        # "bf16": the MLP tower's matrix products take bf16 operands (fp32 accumulation, master
        # weights and Adam) — BASELINE config B's precision; default fp32 (the reference's)
        self._precision = params.get("precision", "fp32")
        # data parallelism (new; SURVEY §5 "world_size"): one process per GPU under torchrun, the
        # ratings partitioned by user (rank r trains users u % world == r, as local ids u // world,
        # movierec.distributed.UserPartitionedDataParallel); 1 = the reference's single device
        self._world_size = int(params.get("world_size", 1))
        if self._world_size < 1:
            raise ValueError("world_size must be >= 1, found {}".format(self._world_size))
        self._rank = 0
        if self._world_size > 1:
            from .distributed import ensure_process_group
            self._rank = ensure_process_group(self._world_size, params.get("dist_backend"))

        try:
            os.makedirs(output_dir)
        except FileExistsError:
            pass
        self.name = model_name
        self._model_weights_path = self.get_model_weights_path(output_dir, model_name)
        self._params_path = self.get_params_json_path(output_dir, model_name)
        # the run's layout (world_size, dist_backend) is not part of the model: a saved model loads
        # anywhere, on one device or another rank count
        self._serialized_params = json.dumps({k: v for k, v in params.items() if k not in RUNTIME_KEYS})
        self._output_model_checkpoints = os.path.join(
            output_dir, "{}-checkpoint-{{epoch:02d}}-{{val_loss:.2f}}.safetensors".format(model_name))
        self.verbose = verbose

        self.model = self.build_mlp_model()
        self.compile_model()

    # ---------------------------------------------------------------- build
    def build_mlp_model(self):
        """Allocate the device parameters and initialise them like Keras:
        glorot_uniform embeddings and hidden kernels, lecun_uniform output
        kernel, zero biases (model.py:161-188)."""
        from .engine import NCFEngine
        world, rank = self._world_size, self._rank
        lazy = bool(params_lazy(self._layers_l2reg))
        # data-parallel: this rank's users only (local row u // world), every item
        n_users = self._num_users if world == 1 else (self._num_users - rank + world - 1) // world
        eng = NCFEngine(n_users, self._num_items, self._layers_sizes, self._gmf_dim,
                        max_batch=self._max_batch, optimizer=self._optimizer, lr=self._lr, beta_1=self._beta_1,
                        beta_2=self._beta_2, layers_l2reg=self._layers_l2reg, lazy_adam=lazy,
                        precision=self._precision, lazy_rows=n_users if world > 1 and lazy else None)
        w = initial_weights(self._num_users, self._num_items, self._layers_sizes, self._gmf_dim, self._seed)
        dp = None
        if world > 1:
            from .distributed import UserPartitionedDataParallel, partition_keras_weights
            w = partition_keras_weights(w, world, rank)
            eng.set_keras_weights(w)
            dp = UserPartitionedDataParallel(eng)
            dp.broadcast_parameters()   # one replicated item table and dense layers (unseeded init)
        else:
            eng.set_keras_weights(w)
        return NCFNetwork(eng, self._layers_sizes, self._gmf_dim, self._num_negs_per_pos,
                          self._num_negs_per_pos_eval, self.name, dp=dp)

    def compile_model(self):
        """Optimizer and metrics (model.py:197-215): the optimizer state lives
        on the device; hr/dcg at k are computed by the library per batch."""
        if self._optimizer not in OPTIMIZERS:
            raise NotImplementedError("Optimizer {} is not implemented.".format(self._optimizer))
        self.model.engine.set_hyper(self._optimizer, self._lr, self._beta_1, self._beta_2, self._layers_l2reg)
        hr = functools.partial(hit_rate, k=self._k, pred_rank_idx=None)
        hr.__name__ = HIT_RATE
        dcg = functools.partial(discounted_cumulative_gain, k=self._k, pred_rank_idx=None)
        dcg.__name__ = DCG
        self.metrics = {OUTPUT_PRED: [hr, dcg]}

    @staticmethod
    def get_model_weights_path(output_dir, model_name):
        return os.path.join(output_dir, "{}{}".format(model_name, WEIGHTS_SUFFIX))

    @staticmethod
    def get_params_json_path(output_dir, model_name):
        return os.path.join(output_dir, "{}_params.json".format(model_name))

    def get_pred_rank(self):
        return self.model.get_layer(OUTPUT_RANK)

    def log_summary(self):
        self.model.summary(print_fn=logging.info)

    # ------------------------------------------------------------ persistence
    def save(self):
        self.model.save_weights(self._model_weights_path)   # collective when data-parallel
        if self._rank != 0:
            return
        logging.info("Model weights saved to: {}".format(self._model_weights_path))
        with open(self._params_path, "w") as f_out:
            f_out.write(self._serialized_params)
        logging.info("Model params saved to: {}".format(self._params_path))

    @staticmethod
    def load_from_dir(model_dir, model_name, verbose=1):
        params_path = MovierecModel.get_params_json_path(model_dir, model_name)
        weights_path = MovierecModel.get_model_weights_path(model_dir, model_name)
        return MovierecModel.load_from_files(params_path, weights_path, model_dir, model_name, verbose)

    @staticmethod
    def load_from_files(params_path, weights_path, output_model_dir, output_model_name, verbose=1):
        with open(params_path, "r") as f_in:
            params = json.load(f_in)
        movierec = MovierecModel(params, output_model_name, output_model_dir, verbose)
        movierec.model.load_weights(weights_path)
        return movierec

    # --------------------------------------------------------------- training
    def fit_generator(self, train_data_generator, validation_data_generator, epochs, shuffle=True,
                      patience=5, prefetch=10):
        """Keras-style training loop (model.py:305-333): per epoch, every batch
        of the Sequence (batch order shuffled with python ``random`` when
        ``shuffle``, as Keras' OrderedEnqueuer does), ``on_epoch_end``, then a
        validation pass; EarlyStopping(val_output_dcg, max, patience,
        restore_best_weights) and best-only checkpoints.  Returns a History.

        Batches go to the device one step ahead: each step's launch counts the next batch's
        index (and, under deferred decay, catches its rows up) while it updates the current one.
        Data-parallel (``world_size`` > 1): every rank passes ITS generators (its users' ratings,
        local user ids u // world); each step trains the ranks' batches together as one global
        batch (UserPartitionedDataParallel: one all-reduce), all ranks run the same number of
        steps (the smallest generator's), validation metrics are averaged over every rank's
        batches, and the early-stopping / checkpoint decisions are the same on every rank."""
        eng = self.model.engine
        dp = self.model.dp
        hist = History()
        best, wait, best_w = -math.inf, 0, None
        group_t = self._num_negs_per_pos + 1
        group_v = self._num_negs_per_pos_eval + 1
        n_train = len(train_data_generator)
        n_val = len(validation_data_generator) if validation_data_generator is not None else 0
        if dp is not None:
            from .distributed import all_reduce_min
            n_train = all_reduce_min(n_train, dp.group)
            n_val = all_reduce_min(n_val, dp.group) if validation_data_generator is not None else 0
        for epoch in range(epochs):
            self.model.learning_phase = 1
            eng.stats.zero_()
            order = list(range(n_train))
            if shuffle:
                random.shuffle(order)
            batches = _device_batches(train_data_generator, order, prefetch, eng)
            cur = next(batches, None)
            while cur is not None:
                nxt = next(batches, None)
                (xu, xi), y = cur
                nb = (nxt[0][0], nxt[0][1]) if nxt is not None else None
                if dp is not None:
                    dp.train_step(xu, xi, y, group=group_t, k=self._k, global_batch=xu.numel() * dp.world,
                                  next_batch=nb)
                else:
                    eng.train_step(xu, xi, y, group=group_t, k=self._k, next_batch=nb)
                cur = nxt
            if hasattr(train_data_generator, "check_errors"):
                train_data_generator.check_errors()
            eng.check_errors()
            train_data_generator.on_epoch_end()
            tr = eng.read_stats(eng.stats)
            self.model.learning_phase = 0
            eng.val_stats.zero_()
            for (xu, xi), y in _device_batches(validation_data_generator, list(range(n_val)), prefetch, eng):
                eng.evaluate(xu, xi, y, group=group_v, k=self._k)
            if dp is not None:
                from .distributed import all_reduce_sum_
                all_reduce_sum_(eng.val_stats, dp.group)
            va = eng.read_stats(eng.val_stats)
            # Keras' History keys of this two-output model: `loss` is the total (BCE + the L2
            # regularisers), `output_loss` the BCE of the `output` head alone; batch means averaged
            # over the epoch's batches (all of one size)
            logs = {"loss": tr["loss"], "output_loss": tr["bce"], "output_hr": tr["hr"], "output_dcg": tr["dcg"]}
            if n_val:
                logs.update({"val_loss": va["loss"], "val_output_loss": va["bce"], "val_output_hr": va["hr"],
                             METRIC_VAL_DCG: va["dcg"]})
            hist.epoch.append(epoch)
            for key, val in logs.items():
                hist.history.setdefault(key, []).append(float(val))
            if self.verbose and self._rank == 0:
                logging.info("Epoch %d/%d - %s", epoch + 1, epochs,
                             " - ".join("%s: %.4f" % kv for kv in logs.items()))
            current = logs.get(METRIC_VAL_DCG)
            if current is None:
                continue
            if current > best:
                best, wait = current, 0
                best_w = self.model.get_weights()
                path = self._output_model_checkpoints.format(epoch=epoch + 1, val_loss=logs["val_loss"])
                self.model.save_weights(path)
            else:
                wait += 1
                if wait >= patience:
                    if best_w is not None:
                        self.model.set_weights(best_w)
                    break
        return hist

    def evaluate(self, generator, k=None, batches=None):
        """Full-protocol evaluation (new): mean loss / HR@k / DCG@k (= NDCG@k,
        one relevant item per group) over every batch of ``generator``."""
        eng = self.model.engine
        dp = self.model.dp
        k = self._k if k is None else int(k)
        group = generator.negatives_per_positive + 1
        stats = eng.val_stats.new_zeros(eng.val_stats.shape)
        n = len(generator) if batches is None else batches
        if dp is not None:
            from .distributed import all_reduce_min, all_reduce_sum_
            n = all_reduce_min(n, dp.group)
        for (xu, xi), y in _device_batches(generator, list(range(n)), 10, eng):
            eng.evaluate(xu, xi, y, group=group, k=k, stats=stats)
        if dp is not None:
            all_reduce_sum_(stats, dp.group)   # every rank's batches: the mean over all of them
        return eng.read_stats(stats)

    def recommend(self, user_ids, k=10, precision="fp16"):
        """Top-k recommendations over the whole catalogue (new; BASELINE config E): the
        serving workload of trt_client.py:43-57 — score items for a user with the model's
        sigmoid output and keep the K = 10 best (``np.argsort(output)[-K:][::-1]``) — for
        every user of ``user_ids`` and every item.  Returns numpy ``(items (n, k) int32,
        scores (n, k) float32)``, best first, ties broken by the lower item id."""
        user_ids = np.asarray(user_ids).reshape(-1)
        if user_ids.size and (user_ids.min() < 0 or user_ids.max() >= self._num_users):
            raise ValueError("user id out of range [0, %d)" % self._num_users)
        user_ids = self.model.local_user_ids(user_ids)   # data-parallel: this rank's users
        items, scores = self.model.engine.score_topk(user_ids, k=k, precision=precision)
        return items.cpu().numpy(), scores.cpu().numpy()


def _prefetch(gen, order, depth):
    """Produce ``gen[i]`` for i in order on one background thread (Keras'
    workers=1 enqueuer), so host batch assembly overlaps device steps."""
    if not order:
        return
    import queue
    import threading
    q = queue.Queue(maxsize=max(1, depth))
    sentinel = object()

    def work():
        try:
            for i in order:
                q.put(gen[i])
        except BaseException as e:  # surface in the consumer
            q.put(e)
        q.put(sentinel)

    t = threading.Thread(target=work, daemon=True)
    t.start()
    while True:
        item = q.get()
        if item is sentinel:
            break
        if isinstance(item, BaseException):
            raise item
        yield item
    t.join()


def _device_batches(gen, order, depth, eng):
    """``gen[i]`` for i in order, as device tensors ``([users int32, items int32], labels float32)``:
    host batches are produced on one background thread (``_prefetch``), range-checked against the
    engine's tables (TF's gather raises on out-of-range ids) and uploaded here; batches already on
    the device (DeviceMovieLensDataGenerator) pass through."""
    import torch
    if gen is None:
        return
    dev = eng.device
    for (xu, xi), y in _prefetch(gen, order, depth):
        if not (torch.is_tensor(xu) and xu.is_cuda):
            eng.check_ids(xu, xi)
        up = [torch.as_tensor(np.ascontiguousarray(np.asarray(x).reshape(-1), dtype=np.int32)).to(dev)
              if not (torch.is_tensor(x) and x.is_cuda and x.dtype == torch.int32) else x.reshape(-1).contiguous()
              for x in (xu, xi)]
        yy = y if torch.is_tensor(y) and y.is_cuda else torch.as_tensor(
            np.ascontiguousarray(np.asarray(y).reshape(-1), dtype=np.float32)).to(dev)
        yield up, yy.reshape(-1).to(torch.float32)


def initial_weights(num_users, num_items, layers_sizes, gmf_dim=0, seed=None):
    """Keras initialisers (glorot_uniform / lecun_uniform / zeros) on the host."""
    rng = np.random.RandomState(seed) if seed is not None else np.random.RandomState()
    L = list(layers_sizes)

    def glorot(r, c):
        lim = math.sqrt(6.0 / (r + c))
        return rng.uniform(-lim, lim, size=(r, c)).astype(np.float32)

    w = {}
    if L:   # GMF-only model (layers_sizes == []): no MLP embeddings
        du, di = L[0] // 2, L[0] - L[0] // 2
        w["user_embedding"] = glorot(num_users, du)
        w["item_embedding"] = glorot(num_items, di)
    if gmf_dim > 0:
        w["user_gmf_embedding"] = glorot(num_users, gmf_dim)
        w["item_gmf_embedding"] = glorot(num_items, gmf_dim)
    for l in range(1, len(L)):
        w["hidden_%d/kernel" % l] = glorot(L[l - 1], L[l])
        w["hidden_%d/bias" % l] = np.zeros(L[l], np.float32)
    f = gmf_dim + (L[-1] if L else 0)
    lim = math.sqrt(3.0 / f)
    w["output/kernel"] = rng.uniform(-lim, lim, size=(f, 1)).astype(np.float32)
    w["output/bias"] = np.zeros(1, np.float32)
    return w


class RankLayer(object):
    """Stable descending ranking per user group (model.py:336-358)."""

    def __init__(self, num_negs_per_pos_train, num_negs_per_pos_eval, name, **kwargs):
        self.name = name
        self.num_negs_per_pos_train = num_negs_per_pos_train
        self.num_negs_per_pos_eval = num_negs_per_pos_eval
        self.learning_phase = 0

    def call(self, inputs, **kwargs):
        """Rank on the device (HIP ``ncf_rank``); accepts numpy or device tensors."""
        import torch
        from . import _native as N
        negs = self.num_negs_per_pos_train if self.learning_phase else self.num_negs_per_pos_eval
        group = negs + 1
        t = inputs if torch.is_tensor(inputs) else torch.as_tensor(np.asarray(inputs, dtype=np.float32))
        t = t.reshape(-1).to("cuda", torch.float32).contiguous()
        ng = t.numel() // group
        out = torch.empty(ng, group, dtype=torch.int32, device=t.device)
        N.check(N.lib().ncf_rank(N.ptr(t), ng, group, N.ptr(out), N.stream_handle(t.device)))
        return out.cpu().numpy()

    def get_config(self):
        return {"name": self.name, "num_negs_per_pos_train": self.num_negs_per_pos_train,
                "num_negs_per_pos_eval": self.num_negs_per_pos_eval}


def _get_hits_per_user(y_true, pred_rank_idx, k):
    """Position of each group's label (argmax of y_true) in the ranking and
    whether it lies in the top k (model.py:420-455)."""
    rank = np.asarray(pred_rank_idx)
    y = np.asarray(y_true).reshape(rank.shape)
    lab = np.argmax(y, axis=-1)
    pos = np.argmax(rank == lab[:, None], axis=-1)
    return (pos < k).astype(np.float32), pos


def hit_rate(y_true, _, k, pred_rank_idx):
    hits, _pos = _get_hits_per_user(y_true, pred_rank_idx, k)
    return float(np.mean(hits, axis=-1))


def discounted_cumulative_gain(y_true, _, k, pred_rank_idx):
    hits, pos = _get_hits_per_user(y_true, pred_rank_idx, k)
    dcg = np.float32(math.log(2.0)) / np.log(pos.astype(np.float32) + np.float32(2.0))
    return float(np.mean(dcg * hits, axis=-1))


def params_lazy(layers_l2reg):
    """Deferred exact decay is used whenever the embedding L2 is off (trainer default)."""
    return len(layers_l2reg) == 0 or float(layers_l2reg[0]) == 0.0


def params_copy(params):
    """Deep copy of a params dict (the reference tests mutate shared lists)."""
    return copy.deepcopy(params)
