"""Pickle contract on a GPU-less host.

The reference's train CLI pickles the fitted model
(project_template/pipeline/train.py:46-48) and its serving app unpickles it
(app/api.py:38-40) and calls predict inside ``try/except Exception: return
zeros`` (:49-52).  tests/golden/kernelmf_tiny_linear_gpu.pkl was written on
an MI355X by tools/make_pickle_fixture.py (KernelMF fitted through
libmf_hip.so on the tiny_linear golden inputs).  Here it is loaded with
plain ``pickle`` in a fresh process that has no GPU and never loads
libmf_hip.so; the behaviour this build chooses:

* the load succeeds and every attribute is a plain NumPy / Python value,
  pinned to the reference's golden vectors (<= 1e-10, as the GPU parity
  tests), ``get_params`` intact;
* the load warns (RuntimeWarning) that predict / recommend need a HIP
  device -- a serving wrapper that swallows predict's exception would
  otherwise silently serve default scores;
* predict raises MFLibraryError: there is no host scoring path.
"""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, PKG_DIR, golden_hp, load_golden

PKL = os.path.join(GOLDEN, "kernelmf_tiny_linear_gpu.pkl")

_CHILD = r"""
import json, pickle, sys, warnings
sys.path.insert(0, {pkg!r})
import numpy as np
with warnings.catch_warnings(record=True) as caught:
    warnings.simplefilter("always")
    with open({pkl!r}, "rb") as f:
        m = pickle.load(f)
with open("/proc/self/maps") as f:
    hip_loaded = "libmf_hip.so" in f.read()
import pandas as pd
err = None
try:
    m.predict(pd.DataFrame({{"user_id": [next(iter(m.user_id_map))],
                             "item_id": [next(iter(m.item_id_map))]}}))
except Exception as e:
    err = type(e).__name__ + ": " + str(e)
np.savez({npz!r}, P=m.user_features, Q=m.item_features, bu=m.user_biases,
         bi=m.item_biases, rmse=np.asarray(m.train_rmse),
         uids=np.asarray(list(m.user_id_map)), iids=np.asarray(list(m.item_id_map)))
print(json.dumps({{
    "cls": type(m).__name__,
    "params": {{k: (v if isinstance(v, (int, float, str, type(None))) else repr(v))
                for k, v in m.get_params().items()}},
    "types": [type(a).__name__ for a in (m.user_features, m.item_features,
                                         m.user_biases, m.item_biases)],
    "global_mean": float(m.global_mean),
    "warnings": [str(w.message) for w in caught if w.category is RuntimeWarning],
    "hip_loaded_at_load": hip_loaded,
    "predict_error": err,
}}))
"""


@pytest.mark.skipif(not os.path.exists(PKL), reason="GPU-trained pickle fixture not generated")
def test_gpu_trained_pickle_loads_without_gpu(tmp_path):
    npz = str(tmp_path / "attrs.npz")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="",
               ROCR_VISIBLE_DEVICES="")
    out = subprocess.run([sys.executable, "-c", _CHILD.format(pkg=PKG_DIR, pkl=PKL, npz=npz)],
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    d = load_golden("tiny_linear")
    hp = golden_hp(d)
    assert res["cls"] == "KernelMF"
    for key, val in hp.items():
        if key != "verbose":
            assert res["params"][key] == val, key
    assert res["params"]["dtype"] == "float64" and res["params"]["schedule"] == "exact"
    assert res["types"] == ["ndarray"] * 4
    assert res["global_mean"] == float(d["global_mean"])
    assert not res["hip_loaded_at_load"]
    assert any("predict() and recommend() will raise" in w for w in res["warnings"])
    assert res["predict_error"] and res["predict_error"].startswith("MFLibraryError")
    a = np.load(npz)
    for name, ref in (("P", "user_features"), ("Q", "item_features"), ("bu", "user_biases"),
                      ("bi", "item_biases")):
        scale = max(1.0, float(np.max(np.abs(d[ref]))))
        assert float(np.max(np.abs(a[name] - d[ref]))) <= 1e-10 * scale, name
    assert float(np.max(np.abs(a["rmse"] - d["train_rmse"]))) <= 1e-12
    assert a["uids"].tolist() == d["user_ids"].tolist()
    assert a["iids"].tolist() == d["item_ids"].tolist()
