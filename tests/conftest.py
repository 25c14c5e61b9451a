import json
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")
for p in (REPO, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def load_fixture(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def state_layout(which):
    with open(os.path.join(GOLDEN, "state_layout.json")) as f:
        return [(k, tuple(s)) for k, s in json.load(f)[which]]


def fixture_params(which, fx):
    """Parameter dict (reference state_dict names) for a fixture: stored for
    the reduced config, closed-form for the full-width one."""
    from formula import formula_state_dict
    if which == "small":
        return {k: torch.from_numpy(fx["param_" + k].copy()) for k, _ in state_layout("small")}
    return formula_state_dict(dict(state_layout("full")))


@pytest.fixture(scope="session")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
