"""User-row folding (include/movierec_ncf.h, "User-row folding"): the fused kernels (and, since
round 6, the layered path's backward k_lay_l1b at config D's widths) sum the user-row gradients of
a group's samples that share the group head's user and write one row;
the index lists that one contribution.  The reference's batches always share the user within a
group (data_pipeline.py:141), but the device path must stay exact for any batch: a sample whose
user differs from its head's keeps its own contribution.

Checked against the oracle (reference model.py:154-214 restated) on batches that mix folded and
unfolded samples, for every fold width (2..32: DPP and ds_swizzle butterfly steps), through the
dense-gradient path (ncf_forward_backward), the touched-row step (ncf_train_step, deferred decay)
and the row-sharded plan; and the device flag for an index built ahead with another group.
Tolerances as tests/test_native_gpu.py.
"""

import numpy as np
import pytest

from conftest import gpu_available
from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from movierec.engine import NCFEngine

CONFIG_C = (200, 150, [128, 64, 32, 16], 64)
CONFIG_D_SMALL = (160, 120, [256, 128, 64, 32], 128)   # config D's widths: the layered path (k_lay_l1b folds)
KERNELS = [None, "wave", "layered"]
KERNEL_IDS = ["default", "wave", "layered"]
HYPER = dict(optimizer="adam", lr=0.001, beta_1=0.9, beta_2=0.999, layers_l2reg=[0.0] * 4)


def _weights(shape, seed):
    from test_native_gpu import _weights as w
    return w(shape, seed)


def _dims(kernel):
    return CONFIG_D_SMALL if kernel == "layered" else CONFIG_C


def _engine(shape, kernel, max_batch, **kw):
    if kernel == "layered":
        eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=max_batch,
                        force_layered=True, **kw)
        assert eng.kernel_for(max_batch) == "layered-mfma"
    else:
        eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=max_batch,
                        fb_kernel=kernel, **kw)
    return eng


def _mixed_batch(shape, B, group, seed, w=None):
    """Groups of `group` samples sharing a user, then: ~25% of the non-head samples get another
    user, ~10% of the heads get another user (the rest of that group still shares one), and one
    group whose samples all differ.  With the weights ``w``: samples on a ReLU kink (a hidden
    pre-activation within rounding of 0, where fp32 and fp64 may take different sides, and two fp32
    summation orders too) draw another item until none is left."""
    rng = np.random.RandomState(seed)
    users = rng.randint(0, shape.num_users, B // group).repeat(group)
    items = rng.randint(0, shape.num_items, B)
    y = np.tile([0] * (group - 1) + [1], B // group).astype(np.float32)
    pos = np.arange(B) % group
    swap = (pos != 0) & (rng.rand(B) < 0.25)
    users[swap] = rng.randint(0, shape.num_users, int(swap.sum()))
    heads = (pos == 0) & (rng.rand(B) < 0.10)
    users[heads] = rng.randint(0, shape.num_users, int(heads.sum()))
    users[group:2 * group] = rng.permutation(shape.num_users)[:group]
    if w is not None:
        from test_headline_parity_gpu import kink_samples
        for _ in range(50):
            k = kink_samples(shape, w, users, items)
            if not k.any():
                break
            items[k] = rng.randint(0, shape.num_items, int(k.sum()))
    return users.astype(np.int32), items.astype(np.int32), y


@pytest.mark.parametrize("kernel", KERNELS, ids=KERNEL_IDS)
@pytest.mark.parametrize("group", [2, 4, 8, 16, 32])
def test_mixed_groups_grads_match_oracle(group, kernel):
    shape = O.NCFShape(*_dims(kernel))
    w = _weights(shape, 60 + group)
    B = 1024
    users, items, y = _mixed_batch(shape, B, group, 61 + group, w)
    eng = _engine(shape, kernel, B)
    eng.set_keras_weights(w)
    grads = eng.alloc_grads()
    probs = torch.empty(B, dtype=torch.float32, device="cuda")
    eng.forward_backward(users, items, y, group=group, k=2, inv_batch=1.0 / B, grads=grads, probs_out=probs)
    _, g, _ = O.loss_and_grads(shape, w, users, items, y, [0.0] * len(shape.layers))
    got = eng.keras_weights(grads[0], grads[1])
    for name in O.weight_names(shape):
        scale = np.max(np.abs(g[name])) + 1e-12
        err = np.max(np.abs(got[name] - g[name]))
        assert err <= 1e-5 * scale + 1e-9, (name, err, scale)
    pref, _ = O.forward(shape, w, users, items)
    assert np.max(np.abs(probs.cpu().numpy() - pref)) <= 2e-6


@pytest.mark.parametrize("kernel", KERNELS, ids=KERNEL_IDS)
@pytest.mark.parametrize("lazy", [False, True], ids=["dense", "deferred"])
def test_mixed_groups_train_steps_match_oracle(lazy, kernel):
    shape = O.NCFShape(*_dims(kernel))
    w = _weights(shape, 70)
    eng = _engine(shape, kernel, 512, lazy_adam=lazy)
    eng.set_keras_weights(w)
    ref = {k: v.copy() for k, v in w.items()}
    st = O.new_opt_state(ref)
    batches = [_mixed_batch(shape, 512, 4, 71 + s, w) for s in range(3)]
    dev = [tuple(torch.from_numpy(x).cuda() for x in b) for b in batches]
    for s, (u, it, yy) in enumerate(dev):
        nxt = (dev[s + 1][0], dev[s + 1][1]) if lazy and s + 1 < len(dev) else None
        eng.train_step(u, it, yy, group=4, k=2, next_batch=nxt)
        O.train_step(shape, ref, st, *batches[s], dict(HYPER, layers_l2reg=[0.0] * len(shape.layers)))
    eng.check_errors()
    got = eng.keras_weights()
    for name in O.weight_names(shape):
        tol = 3 * 2e-6 + 2e-6 * np.max(np.abs(ref[name]))
        err = np.max(np.abs(got[name] - ref[name]))
        assert err <= tol, (name, err, tol)


@pytest.mark.parametrize("kernel", KERNELS, ids=KERNEL_IDS)
def test_folded_step_is_deterministic(kernel):
    shape = O.NCFShape(*_dims(kernel))
    w = _weights(shape, 80)
    users, items, y = _mixed_batch(shape, 2048, 4, 81)
    outs = []
    for _ in range(2):
        eng = _engine(shape, kernel, 2048)
        eng.set_keras_weights(w)
        for _ in range(2):
            eng.train_step(users, items, y, group=4, k=2)
        torch.cuda.synchronize()
        outs.append((eng.emb.clone(), eng.mlp.clone(), eng.emb_m.clone(), eng.emb_v.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("kernel", [None, "wave"], ids=["default", "wave"])
def test_index_built_with_another_group_is_flagged(kernel):
    """An index built ahead (ncf_build_index) with group 4 (fold 4) used by a step with group 2
    (fold 2): the step's fold check sets NCF_WSERR_FOLD and check_errors raises."""
    shape = O.NCFShape(*CONFIG_C)
    w = _weights(shape, 90)
    users, items, y = [torch.from_numpy(x).cuda() for x in _mixed_batch(shape, 256, 4, 91)]
    eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=256, fb_kernel=kernel)
    eng.set_keras_weights(w)
    U = shape.num_users
    grads = (torch.zeros(shape.num_items, eng.row_width, device="cuda"), torch.zeros(eng.mlp_params, device="cuda"),
             torch.zeros(8, device="cuda"))
    eng.build_index(users, items, 4)
    eng._prebuilt = eng._prebuilt[:5] + (2,)   # make the host-side guard accept it
    eng.forward_backward_part(users, items, y, group=2, k=2, inv_batch=1.0 / 256, shared_row_begin=U, grads=grads)
    with pytest.raises(RuntimeError, match="sample group"):
        eng.check_errors()
    # the same index with the matching group passes
    eng.build_index(users, items, 4)
    eng.forward_backward_part(users, items, y, group=4, k=2, inv_batch=1.0 / 256, shared_row_begin=U, grads=grads)
    eng.check_errors()
    assert gpu_available()
