"""CPU oracle (numpy) for the NCF / NeuMF training hot path.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``): the checker for the HIP
path and the timed ``cpu_baseline`` of ``bench.py``.  Never shipped, never a
fallback.

What it restates (citations are ``/root/reference`` file:line):

* model graph — ``movierec/model.py:135-195``: user/item ``Embedding`` of widths
  ``L0//2`` and ``L0-L0//2`` (``:159-170``), ``concatenate`` (``:171-172``),
  ``Dense(relu)`` for ``layers_sizes[1:]`` (``:175-181``), ``Dense(1, sigmoid)``
  (``:184-188``).  The reference is MLP-only; the GMF branch (``gmf_dim > 0``)
  is the NeuMF extension named by BASELINE.json (He et al. 2017, eq. 11:
  ``y = sigmoid(h^T [phi_GMF ; phi_MLP])``).  With ``gmf_dim == 0`` this is
  exactly the reference model.
* loss — ``model.py:213-214`` ``binary_crossentropy`` (TF 1.x Keras backend):
  ``clip(p, eps, 1-eps)`` → ``logit = log(p/(1-p))`` →
  ``sigmoid_cross_entropy_with_logits``, mean over the batch, plus the L2
  regularisers of ``model.py:163,168,178`` (``l2(x) = x * sum(w**2)`` over the
  WHOLE variable).  Gradient wrt the output pre-activation is ``p - y`` where
  the clip is inactive and 0 where it clips (TF ``clip_by_value`` gradient).
* optimizer — ``model.py:199-202``: Keras v1 ``Adam(lr, beta_1, beta_2)``
  (``epsilon = K.epsilon() = 1e-7``, ``t`` = iterations after increment,
  ``lr_t = lr*sqrt(1-b2^t)/(1-b1^t)``, dense update of EVERY element — the
  IndexedSlices embedding gradient is densified, duplicates summed) and
  ``SGD(lr)`` (momentum 0).
* ranking/metrics — ``RankLayer.call`` ``model.py:344-352`` (``top_k`` sorted,
  ties → lower index first), ``hit_rate`` ``:361-385``,
  ``discounted_cumulative_gain`` ``:388-417``, ``_get_hits_per_user``
  ``:420-455``.

Parity pinning: the rank/metric functions are pinned by the reference's own
known-answer tests (``test/test_model.py:69-190``), reproduced in
``tests/test_oracle_kats.py``.  Loss, gradients, initialisation and optimizer
semantics live in third-party TF/Keras, which is not installed here: they are
restated from the TF 1.x sources' published algorithm and are **parity
unpinned** by reference fixtures; the gradients are
self-checked against finite differences in ``tests/test_oracle_kats.py``.
"""

import math

import numpy as np

KERAS_EPSILON = 1e-7  # K.epsilon() default


# ---------------------------------------------------------------------------
# shapes and weights
# ---------------------------------------------------------------------------

class NCFShape(object):
    """Model dimensions; ``layers`` = ``layers_sizes`` (``model.py:75``)."""

    def __init__(self, num_users, num_items, layers, gmf_dim=0):
        self.num_users = int(num_users)
        self.num_items = int(num_items)
        self.layers = [int(x) for x in layers]
        self.gmf_dim = int(gmf_dim)
        # model.py:159-160; layers == [] is the GMF-only model (BASELINE config A, an extension:
        # p = sigmoid(w . (u_gmf * i_gmf) + b), He et al. 2017 eq. 10)
        self.du = self.layers[0] // 2 if self.layers else 0
        self.di = self.layers[0] - self.du if self.layers else 0
        self.n = len(self.layers)

    @property
    def out_features(self):
        return self.gmf_dim + (self.layers[-1] if self.layers else 0)


def init_weights(shape, seed=0, dtype=np.float64):
    """Keras initialisers: glorot_uniform embeddings/kernels (limit
    sqrt(6/(fan_in+fan_out)), model.py:163,168,178), lecun_uniform output
    kernel (sqrt(3/fan_in), model.py:186), zero biases."""
    rng = np.random.RandomState(seed)

    def glorot(rows, cols):
        lim = math.sqrt(6.0 / (rows + cols))
        return rng.uniform(-lim, lim, size=(rows, cols)).astype(dtype)

    w = {}
    if shape.n > 0:
        w["user_embedding"] = glorot(shape.num_users, shape.du)
        w["item_embedding"] = glorot(shape.num_items, shape.di)
    if shape.gmf_dim > 0:
        w["user_gmf_embedding"] = glorot(shape.num_users, shape.gmf_dim)
        w["item_gmf_embedding"] = glorot(shape.num_items, shape.gmf_dim)
    for l in range(1, shape.n):
        w["hidden_%d/kernel" % l] = glorot(shape.layers[l - 1], shape.layers[l])
        w["hidden_%d/bias" % l] = np.zeros(shape.layers[l], dtype=dtype)
    f = shape.out_features
    lim = math.sqrt(3.0 / f)
    w["output/kernel"] = rng.uniform(-lim, lim, size=(f, 1)).astype(dtype)
    w["output/bias"] = np.zeros(1, dtype=dtype)
    return w


def weight_names(shape):
    names = ["user_embedding", "item_embedding"] if shape.n > 0 else []
    if shape.gmf_dim > 0:
        names += ["user_gmf_embedding", "item_gmf_embedding"]
    for l in range(1, shape.n):
        names += ["hidden_%d/kernel" % l, "hidden_%d/bias" % l]
    names += ["output/kernel", "output/bias"]
    return names


def l2_of(shape, name, layers_l2reg):
    """Which l2 factor applies to a weight (model.py:163,168,178; the output
    layer and all biases carry none, model.py:184-187)."""
    if name.endswith("embedding"):
        # the GMF-only model has no layers_l2reg entries: no embedding L2
        return float(layers_l2reg[0]) if len(layers_l2reg) else 0.0
    if name.startswith("hidden_") and name.endswith("/kernel"):
        return float(layers_l2reg[int(name.split("_")[1].split("/")[0])])
    return 0.0


# ---------------------------------------------------------------------------
# forward / loss / backward
# ---------------------------------------------------------------------------

def bf16_round(x):
    """Round to bfloat16 (round-to-nearest-even on the float32 value, v_cvt_pk_bf16_f32), back
    as float64: the operand rounding of the bf16 MLP mode (include/movierec_ncf.h mlp_bf16)."""
    b = np.ascontiguousarray(np.asarray(x, dtype=np.float32)).view(np.uint32).astype(np.uint64)
    r = ((b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32).astype(np.float64)


def _identity(x):
    return x


def forward(shape, w, users, items, mm_round=_identity):
    """Per-sample forward; returns probabilities (B,) and a cache.  ``mm_round`` is applied to
    both operands of every hidden-layer matrix product (bf16_round: the bf16 MLP mode)."""
    users = np.asarray(users).reshape(-1).astype(np.int64)
    items = np.asarray(items).reshape(-1).astype(np.int64)
    if shape.n > 0:
        dt = w["user_embedding"].dtype
        h = [np.concatenate([w["user_embedding"][users], w["item_embedding"][items]], axis=1)]
    else:
        dt = w["user_gmf_embedding"].dtype
        h = [np.zeros((len(users), 0), dtype=dt)]
    for l in range(1, shape.n):
        z = mm_round(h[-1]) @ mm_round(w["hidden_%d/kernel" % l]) + w["hidden_%d/bias" % l]
        h.append(np.maximum(z, 0))
    if shape.gmf_dim > 0:
        gu = w["user_gmf_embedding"][users]
        gi = w["item_gmf_embedding"][items]
        feat = np.concatenate([gu * gi, h[-1]], axis=1)
    else:
        gu = gi = None
        feat = h[-1]
    z = feat @ w["output/kernel"][:, 0] + w["output/bias"][0]
    p = 1.0 / (1.0 + np.exp(-z))
    cache = dict(users=users, items=items, h=h, gu=gu, gi=gi, feat=feat, z=z, p=p)
    return p.astype(dt), cache


def clip_bounds(eps=KERAS_EPSILON):
    """The clip range as TF builds it in the model's float32 dtype:
    ``eps_ = cast(K.epsilon(), float32)``, ``1 - eps_`` evaluated in float32."""
    lo = np.float32(eps)
    return float(lo), float(np.float32(1.0) - lo)


def bce_per_sample(p, y, eps=KERAS_EPSILON):
    """Keras binary_crossentropy (TF 1.x backend): clip → logit → sigmoid xent."""
    p = np.asarray(p, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    lo, hi = clip_bounds(eps)
    pc = np.clip(p, lo, hi)
    logit = np.log(pc / (1.0 - pc))
    return np.maximum(logit, 0) - logit * y + np.log1p(np.exp(-np.abs(logit)))


def reg_loss(shape, w, layers_l2reg):
    tot = 0.0
    for name in weight_names(shape):
        lam = l2_of(shape, name, layers_l2reg)
        if lam != 0.0:
            tot += lam * float(np.sum(np.asarray(w[name], dtype=np.float64) ** 2))
    return tot


def loss_and_grads(shape, w, users, items, labels, layers_l2reg, batch_norm=None, mm_round=_identity):
    """Total loss (mean BCE + L2) and dense gradients for every weight.

    ``batch_norm`` overrides the divisor of the mean (data-parallel global
    batch); default = this batch's size.  ``mm_round``: as ``forward``, also on the
    backward's matrix products.
    """
    p, c = forward(shape, w, users, items, mm_round)
    y = np.asarray(labels, dtype=np.float64).reshape(-1)
    B = p.shape[0]
    nb = float(B if batch_norm is None else batch_norm)
    lo, hi = clip_bounds()
    mask = (c["p"] >= lo) & (c["p"] <= hi)
    bce = bce_per_sample(c["p"], y)
    loss = float(np.sum(bce) / nb) + reg_loss(shape, w, layers_l2reg)
    dz = np.where(mask, (c["p"] - y) / nb, 0.0)

    g = {}
    feat = c["feat"]
    g["output/kernel"] = (feat.T @ dz)[:, None]
    g["output/bias"] = np.array([dz.sum()])
    wout = w["output/kernel"][:, 0]
    dfeat = dz[:, None] * wout[None, :]
    gd = shape.gmf_dim
    if gd > 0:
        dg = dfeat[:, :gd]
        g["user_gmf_embedding"] = _segment_sum(c["users"], dg * c["gi"], shape.num_users)
        g["item_gmf_embedding"] = _segment_sum(c["items"], dg * c["gu"], shape.num_items)
    dh = dfeat[:, gd:]
    h = c["h"]
    for l in range(shape.n - 1, 0, -1):
        dzl = dh * (h[l] > 0)
        g["hidden_%d/kernel" % l] = mm_round(h[l - 1]).T @ mm_round(dzl)
        g["hidden_%d/bias" % l] = dzl.sum(axis=0)
        dh = mm_round(dzl) @ mm_round(w["hidden_%d/kernel" % l]).T
    if shape.n > 0:
        g["user_embedding"] = _segment_sum(c["users"], dh[:, :shape.du], shape.num_users)
        g["item_embedding"] = _segment_sum(c["items"], dh[:, shape.du:], shape.num_items)
    for name in weight_names(shape):
        lam = l2_of(shape, name, layers_l2reg)
        if lam != 0.0:
            g[name] = g[name] + 2.0 * lam * w[name]
    return loss, g, p


def _segment_sum(ids, rows, n):
    """Dense conversion of an IndexedSlices gradient: duplicates summed in
    ascending sample order (TF CPU unsorted_segment_sum iterates in order)."""
    out = np.zeros((n, rows.shape[1]), dtype=rows.dtype)
    np.add.at(out, ids, rows)
    return out


# ---------------------------------------------------------------------------
# optimizers (Keras v1 semantics, model.py:199-202)
# ---------------------------------------------------------------------------

def adam_lr_t(lr, beta_1, beta_2, t):
    return lr * math.sqrt(1.0 - beta_2 ** t) / (1.0 - beta_1 ** t)


def adam_update(w, g, m, v, t, lr, beta_1=0.9, beta_2=0.999, eps=KERAS_EPSILON):
    """One dense Adam step on every weight; ``t`` is the 1-based iteration."""
    lr_t = adam_lr_t(lr, beta_1, beta_2, t)
    for k in w:
        m[k] = beta_1 * m[k] + (1.0 - beta_1) * g[k]
        v[k] = beta_2 * v[k] + (1.0 - beta_2) * g[k] * g[k]
        w[k] = w[k] - lr_t * m[k] / (np.sqrt(v[k]) + eps)


def sgd_update(w, g, lr):
    for k in w:
        w[k] = w[k] - lr * g[k]


def train_step(shape, w, opt, users, items, labels, hyper):
    """One Keras ``train_on_batch``: loss, grads, optimizer update.

    ``opt`` holds ``m``, ``v`` dicts and ``t`` (iterations so far);
    ``hyper``: optimizer, lr, beta_1, beta_2, layers_l2reg.
    Returns (loss, probs).
    """
    loss, g, p = loss_and_grads(shape, w, users, items, labels, hyper["layers_l2reg"],
                                hyper.get("batch_norm"))
    if hyper["optimizer"] == "adam":
        opt["t"] += 1
        adam_update(w, g, opt["m"], opt["v"], opt["t"], hyper["lr"],
                    hyper.get("beta_1", 0.9), hyper.get("beta_2", 0.999))
    else:
        sgd_update(w, g, hyper["lr"])
    return loss, p


def new_opt_state(w):
    return dict(m={k: np.zeros_like(a) for k, a in w.items()},
                v={k: np.zeros_like(a) for k, a in w.items()}, t=0)


# ---------------------------------------------------------------------------
# ranking and metrics (model.py:336-455)
# ---------------------------------------------------------------------------

def rank_layer(pred, group):
    """RankLayer.call: reshape (-1, group) then stable descending order
    (tf.nn.top_k sorted=True puts the lower index first on ties)."""
    x = np.asarray(pred).reshape(-1, group)
    # stable sort on -x keeps index order among ties
    return np.argsort(-x, axis=1, kind="stable").astype(np.int32)


def hits_per_user(y_true, pred_rank_idx, k):
    """_get_hits_per_user (model.py:420-455): label = argmax(y) per row,
    its position in the ranking, hit = position < k."""
    rank = np.asarray(pred_rank_idx)
    y = np.asarray(y_true).reshape(rank.shape)
    lab = np.argmax(y, axis=-1)
    pos = np.argmax(rank == lab[:, None], axis=-1)
    hits = (pos < k).astype(np.float32)
    return hits, pos


def hit_rate(y_true, k, pred_rank_idx):
    hits, _ = hits_per_user(y_true, pred_rank_idx, k)
    return float(np.mean(hits))


def discounted_cumulative_gain(y_true, k, pred_rank_idx):
    hits, pos = hits_per_user(y_true, pred_rank_idx, k)
    dcg = np.float32(math.log(2.0)) / np.log(pos.astype(np.float32) + np.float32(2.0))
    return float(np.mean(dcg * hits))


def group_metrics(pred, labels, group, k):
    """(mean HR@k, mean DCG@k) over the groups of one batch."""
    rank = rank_layer(pred, group)
    return (hit_rate(labels, k, rank), discounted_cumulative_gain(labels, k, rank))


# ---------------------------------------------------------------------------
# all-item scoring + top-k (BASELINE config E)
# ---------------------------------------------------------------------------

def score_all_items(shape, w, users):
    """Logits z (n_users, num_items) of every (user, item) pair: the forward of
    ``model.py:154-188`` without the sigmoid, the workload ``trt_client.py:43-57``
    sends to the served model for one user and NUM_ITEMS_PREDICT random items."""
    users = np.asarray(users).reshape(-1).astype(np.int64)
    items = np.arange(shape.num_items)
    out = np.empty((users.size, shape.num_items))
    for q, u in enumerate(users):
        _, c = forward(shape, w, np.full(shape.num_items, u), items)
        out[q] = c["z"]
    return out


def top_k_items(scores, k):
    """Per row: the k best columns, best first, ties broken by the lower column index
    (``trt_client.py:55-57`` takes ``np.argsort(output)[-K:][::-1]``, whose tie order numpy
    leaves unspecified; the build fixes it to the stable order).  Returns (items, scores)."""
    scores = np.asarray(scores)
    idx = np.argsort(-scores, axis=1, kind="stable")[:, :k]
    return idx.astype(np.int32), np.take_along_axis(scores, idx, axis=1)


# ---------------------------------------------------------------------------
# on-device negative sampler (ncf_sample.hip), restated
# ---------------------------------------------------------------------------

_M32 = 0xFFFFFFFF


def philox_u32(a, b, c, d, k0, k1):
    """First word of Philox4x32-10 (Salmon et al., SC'11) of counter (a, b, c, d) and key
    (k0, k1) — the generator ncf_sample.hip draws from."""
    for _ in range(10):
        p0 = 0xD2511F53 * a
        p1 = 0xCD9E8D57 * c
        a, b, c, d = ((p1 >> 32) ^ b ^ k0) & _M32, p1 & _M32, ((p0 >> 32) ^ d ^ k1) & _M32, p0 & _M32
        k0 = (k0 + 0x9E3779B9) & _M32
        k1 = (k1 + 0xBB67AE85) & _M32
    return a


def kth_candidate(excluded, c):
    """The c-th item (0-based) absent from the ascending array ``excluded``."""
    excluded = np.asarray(excluded, dtype=np.int64)
    return int(c + np.count_nonzero(excluded - np.arange(len(excluded)) <= c))


def sample_batch(pos_users, pos_items, excluded, num_items, order, first, n_pos, negs, seed, stream):
    """Batch assembly of ``MovieLensDataGenerator.__getitem__`` (``data_pipeline.py:115-150``:
    groups ``[neg_1 .. neg_n, pos]``, users repeated, labels ``[0]*n + [1]``; negatives uniform
    over the user's items absent from data + extra (``:103-108``), without replacement unless
    fewer than n candidates (``:111-112``)) with the device sampler's random stream: candidate
    index = Lemire(Philox(k, attempt, slot_lo, slot_hi ^ stream_hi; seed_lo ^ stream_lo,
    seed_hi)).  ``excluded[u]`` = ascending unique excluded items of user u."""
    k0, k1 = seed & _M32, (seed >> 32) & _M32
    s0, s1 = stream & _M32, (stream >> 32) & _M32
    xu, xi, y = [], [], []
    for g in range(n_pos):
        slot = first + g
        pidx = int(order[slot])
        u, ip = int(pos_users[pidx]), int(pos_items[pidx])
        ex = np.asarray(excluded.get(u, []), dtype=np.int64)
        C = num_items - len(ex)
        replace = C < negs
        thresh = ((1 << 32) - C) % C
        sl, sh = slot & _M32, ((slot >> 32) ^ s1) & _M32
        group = []
        for k in range(negs):
            a = 0
            while True:
                r = philox_u32(k, a, sl, sh, k0 ^ s0, k1)
                a += 1
                m = r * C
                if (m & _M32) < thresh:
                    continue
                cand = kth_candidate(ex, m >> 32)
                if not replace and cand in group:
                    continue
                group.append(cand)
                break
        xu += [u] * (negs + 1)
        xi += group + [ip]
        y += [0.0] * negs + [1.0]
    return np.array(xu, np.int32), np.array(xi, np.int32), np.array(y, np.float32)


# ---------------------------------------------------------------------------
# conversion helpers to / from the device layout used by the HIP library
# ---------------------------------------------------------------------------

def mlp_flat(shape, w):
    """Flat dense-parameter vector in the device order: for each hidden layer
    kernel (row-major, Keras layout) then bias; output kernel then bias."""
    parts = []
    for l in range(1, shape.n):
        parts += [np.asarray(w["hidden_%d/kernel" % l]).ravel(), np.asarray(w["hidden_%d/bias" % l]).ravel()]
    parts += [np.asarray(w["output/kernel"]).ravel(), np.asarray(w["output/bias"]).ravel()]
    return np.concatenate(parts)
