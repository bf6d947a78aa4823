"""CPU: the order model of torch.dot (AS:335, EDEN's scale; MKL sdot on the fixtures' host)
in both oracles -- oracle/uq_eden.py:torch_dot (NumPy) and oracle/uq_oracle.c uqo_torch_dot
(C, exact fmaf) -- against torch.dot's own bits recorded in tests/golden/dot_vectors.json
(make_golden_dot.py): n = 1 .. 2^22 at powers of two for four input kinds, and ragged n."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

from oracle import uq_eden as E
from oracle import uq_oracle_c as C

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, HERE)
from make_golden_dot import inputs  # noqa: E402


@pytest.fixture(scope="module")
def cases():
    return json.load(open(os.path.join(HERE, "dot_vectors.json")))["cases"]


def test_c_oracle_matches_torch_dot(cases):
    for c in cases:
        x, y = inputs(c["kind"], c["n"], c["seed"])
        assert hashlib.sha256(x.tobytes() + y.tobytes()).hexdigest()[:16] == c["in_sha"], c
        got = C.torch_dot(x, y)
        assert int(got.view(np.uint32)) == c["dot_bits"], (c["kind"], c["n"])


def test_numpy_oracle_matches_torch_dot(cases):
    for c in cases:
        if c["n"] > (1 << 16) and c["n"] != (1 << 20):
            continue                            # the C form covers every size; NumPy's loop is slow
        x, y = inputs(c["kind"], c["n"], c["seed"])
        got = E.torch_dot(x, y)
        assert int(np.float32(got).view(np.uint32)) == c["dot_bits"], (c["kind"], c["n"])
