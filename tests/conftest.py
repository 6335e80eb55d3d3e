import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "f-lite_amd"))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libflite_hip.so)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden():
    from safetensors.torch import load_file

    return load_file(str(ROOT / "tests" / "golden" / "golden.safetensors"))


@pytest.fixture(scope="session")
def golden_meta():
    import json

    return json.loads((ROOT / "tests" / "golden" / "golden_meta.json").read_text())


@pytest.fixture(scope="session")
def golden_nobias():
    """Reference outputs of the released-checkpoint layout (train_bias_and_rms=False, pt.py:31)."""
    from safetensors.torch import load_file

    return load_file(str(ROOT / "tests" / "golden" / "golden_nobias.safetensors"))
