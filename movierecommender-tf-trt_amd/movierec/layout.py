"""Host-side description of the device parameter layout (include/movierec_ncf.h).

Pure numpy: converts between the reference's Keras weights (names from
movierec/model.py:161-188 — ``user_embedding``, ``item_embedding``,
``hidden_<l>`` kernel/bias, ``output`` kernel/bias — plus the NeuMF GMF
tables) and the device layout: one combined embedding table (users then
items; each row [GMF part | MLP part], 16-byte padded) and one flat vector of
dense parameters.  The formulas mirror ``ncf_shape_init``.
"""

import numpy as np


def _round4(x):
    return (x + 3) // 4 * 4


class Layout(object):
    def __init__(self, num_users, num_items, layers, gmf_dim=0):
        self.num_users = int(num_users)
        self.num_items = int(num_items)
        self.layers = [int(x) for x in layers]
        self.gmf_dim = int(gmf_dim)
        # model.py:159-160; no MLP (layers_sizes == []) = the GMF-only model (BASELINE config A)
        self.du = self.layers[0] // 2 if self.layers else 0
        self.di = self.layers[0] - self.du if self.layers else 0
        self.gmf_stride = _round4(self.gmf_dim)
        self.row_width = self.gmf_stride + _round4(max(self.du, self.di))
        self.num_rows = self.num_users + self.num_items
        self.out_features = self.gmf_dim + (self.layers[-1] if self.layers else 0)
        self.mlp_params = sum(a * b + b for a, b in zip(self.layers[:-1], self.layers[1:])) + self.out_features + 1

    def weight_names(self):
        names = ["user_embedding", "item_embedding"] if self.layers else []
        if self.gmf_dim > 0:
            names += ["user_gmf_embedding", "item_gmf_embedding"]
        for l in range(1, len(self.layers)):
            names += ["hidden_%d/kernel" % l, "hidden_%d/bias" % l]
        return names + ["output/kernel", "output/bias"]

    def to_device(self, w, dtype=np.float32):
        """Keras-layout dict -> (emb [num_rows x row_width], flat dense vector)."""
        U, G, G4 = self.num_users, self.gmf_dim, self.gmf_stride
        emb = np.zeros((self.num_rows, self.row_width), dtype=dtype)
        if self.layers:
            emb[:U, G4:G4 + self.du] = w["user_embedding"]
            emb[U:, G4:G4 + self.di] = w["item_embedding"]
        if G > 0:
            emb[:U, :G] = w["user_gmf_embedding"]
            emb[U:, :G] = w["item_gmf_embedding"]
        parts = []
        for l in range(1, len(self.layers)):
            parts += [np.asarray(w["hidden_%d/kernel" % l]).ravel(), np.asarray(w["hidden_%d/bias" % l]).ravel()]
        parts += [np.asarray(w["output/kernel"]).ravel(), np.asarray(w["output/bias"]).ravel()]
        flat = np.concatenate(parts).astype(dtype)
        assert flat.size == self.mlp_params
        return emb, flat

    def from_device(self, emb, flat):
        """(emb, flat) -> Keras-layout dict (copies)."""
        U, G, G4 = self.num_users, self.gmf_dim, self.gmf_stride
        e = np.asarray(emb)[:self.num_rows]
        f = np.asarray(flat)
        w = {}
        if self.layers:
            w["user_embedding"] = e[:U, G4:G4 + self.du].copy()
            w["item_embedding"] = e[U:, G4:G4 + self.di].copy()
        if G > 0:
            w["user_gmf_embedding"] = e[:U, :G].copy()
            w["item_gmf_embedding"] = e[U:, :G].copy()
        off = 0
        for l in range(1, len(self.layers)):
            a, b = self.layers[l - 1], self.layers[l]
            w["hidden_%d/kernel" % l] = f[off:off + a * b].reshape(a, b).copy()
            off += a * b
            w["hidden_%d/bias" % l] = f[off:off + b].copy()
            off += b
        F = self.out_features
        w["output/kernel"] = f[off:off + F].reshape(F, 1).copy()
        w["output/bias"] = f[off + F:off + F + 1].copy()
        return w
