"""On-device negative sampling: a ``MovieLensDataGenerator`` whose batches are assembled by
the HIP library (``ncf_sample_batch``).

Same constructor, ``__len__`` (the F4 quirk included), ``on_epoch_end`` and batch layout as
the reference generator (``data_pipeline.py:17-154``); ``__getitem__`` returns device tensors
``([x_user, x_item], y)`` (int32, int32, float32) ready for ``NCFEngine.train_step`` — no host
sampling and no H2D copy per batch.  The epoch order (``:152-154``) is a device permutation
(``torch.randperm``, seeded by (seed, epoch)); the negatives come from the library's
counter-based Philox stream (seed, epoch, batch), so batches are reproducible but NOT numpy's
stream: reference-exact batches remain available from the host ``MovieLensDataGenerator``.
"""

import ctypes

import numpy as np
import torch

from . import _native as N
from .data_pipeline import COL_ITEM_ID, COL_USER_ID, MovieLensDataGenerator


def excluded_csr(num_users, frames):
    """Per-user ascending unique excluded items (the positives of every frame), as CSR."""
    us = [np.asarray(f[COL_USER_ID].values, dtype=np.int64) for f in frames if f is not None]
    its = [np.asarray(f[COL_ITEM_ID].values, dtype=np.int64) for f in frames if f is not None]
    u = np.concatenate(us) if us else np.zeros(0, np.int64)
    it = np.concatenate(its) if its else np.zeros(0, np.int64)
    ok = (u >= 0) & (u < num_users)
    key = np.unique(u[ok] * (np.int64(1) << 32) + it[ok])  # sorted by user, then item; deduplicated
    uu = key >> 32
    ii = key & 0xFFFFFFFF
    ptr = np.zeros(num_users + 1, dtype=np.int64)
    np.add.at(ptr, uu + 1, 1)
    return np.cumsum(ptr).astype(np.int32), ii.astype(np.int32)


class DeviceMovieLensDataGenerator(MovieLensDataGenerator):
    """Reference-compatible generator whose batches are sampled on the GPU."""

    def __init__(self, dataset_name, data_df, batch_size, negatives_per_positive, extra_data_df=None,
                 shuffle=True, seed=0, device=None):
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.seed = int(seed)
        self.epoch = -1  # on_epoch_end (also called by the constructor) advances it
        self._dev = None
        super(DeviceMovieLensDataGenerator, self).__init__(dataset_name, data_df, batch_size,
                                                           negatives_per_positive, extra_data_df, shuffle)

    def _upload(self):
        dev = self.device
        ptr, items = excluded_csr(self.num_users, [self.data, self.extra_data])
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev)
        self._dev = dict(users=t(self._users), items=t(self._items), ptr=t(ptr), excl=t(items if len(items) else [0]),
                         err=torch.zeros(1, dtype=torch.int32, device=dev))
        d = self._dev
        self._data = N.NcfSamplerData(d["users"].data_ptr(), d["items"].data_ptr(), len(self._users),
                                      d["ptr"].data_ptr(), d["excl"].data_ptr(), self.num_users, self.num_items)

    def on_epoch_end(self):
        # the epoch's positive order (data_pipeline.py:152-154) is drawn on the device: numpy's
        # shuffle of ml-20m's 20M positives takes about a second per epoch on the host (the
        # batches are not the numpy stream anyway; the host generator keeps the exact mode)
        self.epoch += 1
        n = len(self.indexes)
        if self.shuffle:
            g = torch.Generator(device=self.device).manual_seed((self.seed * 1000003 + self.epoch) & 0x7FFFFFFFFFFF)
            self._order = torch.randperm(n, generator=g, device=self.device).to(torch.int32)
        else:
            self._order = torch.arange(n, dtype=torch.int32, device=self.device)

    def __getitem__(self, idx):
        if self._dev is None:
            self._upload()
        n = self.negatives_per_positive
        P = self.num_positives_per_batch
        first = idx * P
        npos = max(0, min(P, len(self.indexes) - first))
        B = npos * (n + 1)
        dev = self.device
        xu = torch.empty(B, dtype=torch.int32, device=dev)
        xi = torch.empty(B, dtype=torch.int32, device=dev)
        y = torch.empty(B, dtype=torch.float32, device=dev)
        stream = (self.epoch << 32) | (idx & 0xFFFFFFFF)
        N.check(N.lib().ncf_sample_batch(ctypes.byref(self._data), N.ptr(self._order), int(first), int(npos), int(n),
                                         ctypes.c_uint64(self.seed), ctypes.c_uint64(stream), N.ptr(xu), N.ptr(xi),
                                         N.ptr(y), N.ptr(self._dev["err"]), N.stream_handle(dev)))
        return [xu, xi], y

    def check_errors(self):
        """Raise if any batch so far met a user id out of range or without candidates."""
        e = int(self._dev["err"].item()) if self._dev is not None else 0
        if e & 1:
            raise ValueError("user id out of range [0, %d)" % self.num_users)
        if e & 2:
            raise ValueError("a user has no negative candidates (every item is a positive)")
