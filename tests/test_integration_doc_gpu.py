"""INTEGRATION.md §1's drop-in example, executed as written (the first ```python block of the
section), on synthetic ml-1m-shaped ratings: a script written against the reference's
MovierecModel / MovieLensDataGenerator API runs unchanged on the MI355X path."""

import os
import re

import numpy as np
import pandas as pd
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _section_code():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 1."):text.index("## 2.")]
    return re.search(r"```python\n(.*?)```", sec, re.S).group(1)


def test_integration_example_runs(tmp_path):
    code = _section_code().replace('"/tmp/out"', repr(str(tmp_path)))
    rng = np.random.RandomState(0)
    n = 60000
    ratings = pd.DataFrame({"userId": rng.randint(0, 6040, n).astype(np.int32),
                            "itemId": rng.randint(0, 3952, n).astype(np.int32)})
    ratings = ratings.drop_duplicates().reset_index(drop=True)
    val = ratings.groupby("userId").tail(1)
    train = ratings.drop(val.index).reset_index(drop=True)
    ns = {"train_df": train, "validation_df": val.reset_index(drop=True)}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    h = ns["history"].history
    assert len(h["loss"]) == 2 and np.isfinite(h["loss"]).all()
    assert np.isfinite(h["val_output_hr"]).all()
    assert gpu_available()


def test_integration_ctypes_stub_runs():
    """INTEGRATION.md §2's ctypes stub, as written (the library path aside): one training step
    through the bare C ABI, Keras `iterations` bumped, a finite BCE near log(2) for near-zero
    initial weights."""
    import torch
    from movierec import _native as N
    from test_integration_doc import stub_code
    code = stub_code().replace('ctypes.CDLL("libmovierec_ncf.so")', "ctypes.CDLL(%r)" % N.LIB_PATH)
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    torch.cuda.synchronize()
    assert int(ns["state"][4].item()) == 1
    assert np.isfinite(ns["loss"]) and 0.3 < ns["loss"] < 1.0, ns["loss"]
    assert torch.isfinite(ns["emb"]).all()
