"""The reference's training API (``MovierecModel.fit_generator``, ``trainer.train``,
``movierec/model.py:305-333``, ``movierec/trainer.py:30-80``) with the new ``world_size`` and
``sampler`` params.

* ``fit_generator`` with ``world_size = 2`` (two processes sharing the box's GPU over gloo, each
  driving the HIP library through ``UserPartitionedDataParallel``) against one process fed the
  concatenated batches: same History (train loss/hr/dcg of every global step, validation metrics
  averaged over every rank's batches) and the same final weights, at the fp32 tolerance of the
  other data-parallel tests (weights |dw| <= 1e-5, loss rel 1e-5, hr/dcg abs 1e-6).
* ``trainer.train`` end to end with ``sampler = "device"`` (on-device negatives), and with
  ``world_size = 2`` launched as torchrun would (RANK / WORLD_SIZE / MASTER_* in the environment).
"""

import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import gpu_available

pytestmark = pytest.mark.gpu

U, I = 60, 50
GROUP = 4
PER = 32          # samples per rank and step
STEPS = 6         # steps per epoch
VAL_GROUP = 10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _params(world):
    return dict(num_users=U, num_items=I, layers_sizes=[16, 8], layers_l2reg=[0, 0], optimizer="adam", lr=0.01,
                batch_size=PER * 2, num_negs_per_pos=GROUP - 1, batch_size_eval=VAL_GROUP * 4,
                num_negs_per_pos_eval=VAL_GROUP - 1, k=3, seed=7, gmf_dim=4, world_size=world,
                dist_backend="gloo")


class ListSeq(object):
    """A Sequence over precomputed batches (the reference's generator contract,
    data_pipeline.py:89-154)."""

    def __init__(self, batches, negs):
        self.batches = batches
        self.negatives_per_positive = negs

    def __len__(self):
        return len(self.batches)

    def __getitem__(self, i):
        return self.batches[i]

    def on_epoch_end(self):
        pass


def _data(seed=3):
    """Per step and rank: groups of rank r's users (u % 2 == r), global ids."""
    rng = np.random.RandomState(seed)
    train, val = [], []
    for _ in range(STEPS):
        parts = []
        for r in range(2):
            users = (rng.randint(0, U // 2, PER // GROUP) * 2 + r).repeat(GROUP).astype(np.int32)
            items = rng.randint(0, I, PER).astype(np.int32)
            y = np.tile([0] * (GROUP - 1) + [1], PER // GROUP).astype(np.int64)
            parts.append((users, items, y))
        train.append(parts)
    for _ in range(2):
        parts = []
        for r in range(2):
            users = (rng.randint(0, U // 2, 2) * 2 + r).repeat(VAL_GROUP).astype(np.int32)
            items = rng.randint(0, I, 2 * VAL_GROUP).astype(np.int32)
            y = np.tile([0] * (VAL_GROUP - 1) + [1], 2).astype(np.int64)
            parts.append((users, items, y))
        val.append(parts)
    return train, val


def _rank_seq(steps, rank, negs):
    return ListSeq([([p[rank][0] // 2, p[rank][1]], p[rank][2]) for p in steps], negs)


def _global_seq(steps, negs):
    return ListSeq([([np.concatenate([p[0][0], p[1][0]]), np.concatenate([p[0][1], p[1][1]])],
                     np.concatenate([p[0][2], p[1][2]])) for p in steps], negs)


def _fit_worker(rank, world, port, out_dir, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    from movierec.model import MovierecModel
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    train, val = _data()
    model = MovierecModel(_params(world), "dp", out_dir, verbose=0)
    random.seed(11)
    hist = model.fit_generator(_rank_seq(train, rank, GROUP - 1), _rank_seq(val, rank, VAL_GROUP - 1), epochs=3)
    w = model.model.get_weights()        # collective: every rank
    q.put((rank, hist.history, w if rank == 0 else None))
    dist.barrier()
    dist.destroy_process_group()


def test_fit_generator_world2_matches_single_process(tmp_path):
    from movierec.model import MovierecModel
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fit_worker, args=(r, world, port, str(tmp_path / "dp"), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, h, w = q.get(timeout=300)
        res[r] = (h, w)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    train, val = _data()
    ref = MovierecModel(_params(1), "one", str(tmp_path / "one"), verbose=0)
    random.seed(11)
    rh = ref.fit_generator(_global_seq(train, GROUP - 1), _global_seq(val, VAL_GROUP - 1), epochs=3).history
    rw = ref.model.get_weights()
    for r in range(world):
        h = res[r][0]
        assert sorted(h) == sorted(rh)
        for key in rh:
            tol = dict(rel=1e-5) if "loss" in key else dict(abs=1e-6)
            assert h[key] == pytest.approx(rh[key], **tol), key
    w = res[0][1]
    for name in rw:
        np.testing.assert_allclose(w[name], rw[name], rtol=0, atol=1e-5, err_msg=name)
    # best-only checkpoints: written once, by rank 0
    assert len(os.listdir(str(tmp_path / "dp"))) == len(os.listdir(str(tmp_path / "one")))
    assert gpu_available()


def _write_ml100k(data_dir, seed=0):
    from test_trainer_gpu import _write_ml100k as w
    w(data_dir, seed)


def test_trainer_device_sampler(tmp_path):
    """trainer.train with sampler='device': batches sampled on the GPU (ncf_sample_batch), the
    reference flow otherwise (split, validation, early stopping, save)."""
    from movierec import trainer
    from movierec.model import MovierecModel
    data_dir, out_dir = str(tmp_path / "data"), str(tmp_path / "models")
    _write_ml100k(data_dir)
    np.random.seed(0)
    random.seed(0)
    params = dict(trainer.DEFAULT_PARAMS)
    params.update(layers_sizes=[16, 8], layers_l2reg=[0, 0], batch_size=240, num_negs_per_pos=3,
                  batch_size_eval=200, num_negs_per_pos_eval=99, k=4, epochs=3, gmf_dim=8, seed=1, sampler="device")
    model, history = trainer.train("dev", "ml-100k", data_dir, out_dir, params, verbose=0)
    h = history.history
    assert h["loss"][-1] < h["loss"][0]
    assert all(np.isfinite(h["val_output_hr"]))
    assert os.path.exists(MovierecModel.get_model_weights_path(out_dir, "dev"))


def _trainer_worker(rank, world, port, data_dir, out_dir, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from movierec import trainer
    np.random.seed(rank)
    random.seed(5)
    params = dict(trainer.DEFAULT_PARAMS)
    params.update(layers_sizes=[16, 8], layers_l2reg=[0, 0], batch_size=480, num_negs_per_pos=3,
                  batch_size_eval=400, num_negs_per_pos_eval=99, k=4, epochs=2, gmf_dim=8, seed=1,
                  sampler="device", world_size=world, dist_backend="gloo")
    model, history = trainer.train("dp2", "ml-100k", data_dir, out_dir, params, verbose=0)
    q.put((rank, history.history, model.model.engine.num_users))
    dist.barrier()
    dist.destroy_process_group()


def test_trainer_world2_device_sampler(tmp_path):
    """trainer.train under a two-rank launch (the environment torchrun sets, gloo): the ratings
    split by user, each rank samples its own batches on the device, one all-reduce per step; both
    ranks see the same History and rank 0 saves the whole model."""
    from movierec.model import MovierecModel
    data_dir, out_dir = str(tmp_path / "data"), str(tmp_path / "models")
    _write_ml100k(data_dir, seed=2)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_worker, args=(r, world, port, data_dir, out_dir, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, h, nu = q.get(timeout=300)
        res[r] = (h, nu)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0]
    assert res[0][1] + res[1][1] == 943
    assert all(np.isfinite(res[0][0]["loss"]))
    loaded = MovierecModel.load_from_dir(out_dir, "dp2", verbose=0)
    assert loaded.model.get_weights()["user_embedding"].shape[0] == 943
    assert gpu_available()


def _trainer_main_worker(rank, world, port, data_dir, out_dir, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from movierec import trainer
        np.random.seed(rank)
        random.seed(5)
        # the reference's DEFAULT_PARAMS (batch_size_eval 200 with 99 negatives: 2 groups) at 4 ranks;
        # only the training batch is given (100 does not split into 4 ranks of whole 10-groups)
        trainer.main(["-m", "w4", "-n", "ml-100k", "-d", data_dir, "-o", out_dir, "--epochs", "1", "--batch-size",
                      "120", "--sampler", "device", "--dist-backend", "gloo", "-l", "WARNING"])
        q.put((rank, "ok"))
    except BaseException as e:
        import traceback
        q.put((rank, "worker failed:\n" + traceback.format_exc()))
        raise
    dist.barrier()
    dist.destroy_process_group()


def test_trainer_main_world4_default_params(tmp_path):
    """The CLI (trainer.main) under a four-rank launch with the reference's default params: the
    validation batch (200 samples = 2 groups of 100) is split per rank in whole groups
    (trainer.eval_batch_per_rank) instead of raising."""
    from movierec.model import MovierecModel
    data_dir, out_dir = str(tmp_path / "data"), str(tmp_path / "models")
    _write_ml100k(data_dir, seed=3)
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_main_worker, args=(r, world, port, data_dir, out_dir, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for _ in range(world):
        r, msg = q.get(timeout=300)
        assert msg == "ok", msg
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert os.path.exists(MovierecModel.get_model_weights_path(out_dir, "w4"))
