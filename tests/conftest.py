import os
import subprocess
import sys
import warnings

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "matrix-factorization_amd")
ORACLE_DIR = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG_DIR, ORACLE_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

warnings.filterwarnings("ignore", category=FutureWarning)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmf_hip.so)")


@pytest.fixture(scope="session", autouse=True)
def _built_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz")))


def golden_hp(d):
    import ast

    return ast.literal_eval(str(d["hp_json"]))


@pytest.fixture
def golden():
    return load_golden
