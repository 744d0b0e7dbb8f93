"""Shared test setup.

* ``gpu`` marker: tests that need an MI355X (run with ``-m gpu``); everything
  else runs on CPU (``-m "not gpu"``).
* Import paths: the product package (``ofdm-based-systems_amd``), the oracle
  (``oracle/``, test infrastructure only) and the repo root.
"""

import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ofdm-based-systems_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
CHANNELS = os.path.join(ROOT, "config", "channel_models")

DEFAULT_4TAP = np.array(
    [
        0.7767824138452235072 + 0.4560896742466611919j,
        -0.06669848996328063551 + 0.2839935704583463338j,
        0.1398968327715586490 - 0.1591963958343969865j,
        0.02229949514514480494 + 0.2409945439452868821j,
    ],
    dtype=np.complex128,
)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) and libofdm_hip.so")


def channel(name):
    """CIR by fixture name; None / FLAT_DEFAULT = the reference's hard-coded 4-tap channel."""
    if name is None or name == "FLAT_DEFAULT":
        return DEFAULT_4TAP.copy()
    return np.load(os.path.join(CHANNELS, name + ".npy"))


def load_runs():
    with open(os.path.join(GOLDEN, "runs.json")) as f:
        return json.load(f)


def load_stages():
    with open(os.path.join(GOLDEN, "stages.json")) as f:
        return json.load(f)


def stage_arrays(name):
    return np.load(os.path.join(GOLDEN, f"stage_{name}.npz"))


@pytest.fixture(scope="session")
def gpu():
    """Skip-free GPU guard: a gpu-marked test fails loudly when the HIP path is missing."""
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no GPU is visible")
    from ofdm_based_systems import _backend as B

    B.load_library()
    return torch.device("cuda", 0)
