"""Guards for two code-generation workarounds of the in-kernel index.

Both were found on the GPU from their symptoms (tools/dbg_scan.py, tools/dbg_rows.py) and fixed by
reordering source; no reduced reproducer was isolated, so these CPU checks keep the orderings from
being undone unnoticed:

1. scan_local_apply (ncf_internal.h, the scan body): the `zero_at_end` store — `blk == 0 && threadIdx.x == 0` — must
   come after every use of threadIdx.x.  With a `blockIdx.x == 1 && threadIdx.x == 0` store ahead of
   the scan body, the later workgroups read back garbage block totals (the scan was wrong for
   workgroups >= 2 on ROCm 7.2).
2. fill_wave (ncf_internal.h): the scan-block count and prefixes are read with v_readlane while every
   lane is active, before the lane-divergent `if (j < ub)` branch: v_readlane takes the named lane's
   register whatever the exec mask, and inside the branch that lane may be inactive (its register then
   holds whatever the allocator put there; a first version wrote a row at another block's position).
"""

import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "movierecommender-tf-trt_amd", "csrc", "ncf_internal.h")


def _function(text, name):
    i = text.index(name + "(")
    j = text.index(") {", i) + 2   # the body's brace (a default argument may hold braces too)
    depth, k = 0, j
    while True:
        if text[k] == "{":
            depth += 1
        elif text[k] == "}":
            depth -= 1
            if depth == 0:
                return text[j:k + 1]
        k += 1


@pytest.mark.parametrize("fn", ["__device__ inline void scan_local_apply"])
def test_scan_zero_store_comes_last(fn):
    body = _function(open(SRC).read(), fn)
    store = body.index("*zero_at_end = 0")
    # no use of threadIdx after the store, and the store is the body's last statement
    assert "threadIdx" not in body[store + len("*zero_at_end = 0"):]
    assert body[store:].count(";") == 1


def test_fill_readlanes_hoisted_out_of_the_divergent_branch():
    body = _function(open(SRC).read(), "__device__ inline void fill_wave")
    branch = body.index("if (j < ub) {")
    reads = [m.start() for m in re.finditer(r"__builtin_amdgcn_readlane", body)]
    assert len(reads) == 3
    assert all(r < branch for r in reads)
    # and the chunk skip before the branch is wave-uniform (compares only readlane results)
    assert re.search(r"if \(\(int\)\(ch % \(kScanBlock / 64\)\) \* 64 >= ub\) continue;", body)
