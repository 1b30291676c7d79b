import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

importlib.import_module("stuttering-speech-representation_amd")   # registers `ssr_amd`

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through libsse.so)")
    config.addinivalue_line("markers", "slow: large shapes (minutes)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_wavlm():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "wavlm_base.npz"))


@pytest.fixture(scope="session")
def golden_manifest():
    import json
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def wavlm_sd():
    from ssr_amd import config as C, synth
    return synth.synth_wavlm_state_dict(C.WAVLM_BASE, seed=7)


@pytest.fixture(scope="session")
def wavlm_clips():
    from ssr_amd import synth
    return synth.synth_clips(16, 48000, seed=1234)
