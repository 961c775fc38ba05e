"""Write the GPU-trained pickle fixture of tests/test_pickle_cpu.py (run on
the GPU box: `gpurun -- bash tools/gpu.sh TAG py:tools/make_pickle_fixture.py`).

KernelMF is fitted on the tiny_linear golden inputs with the golden's seed
and hyper-parameters (schedule 'exact', FP64, libmf_hip.so on cuda:0) and
pickled exactly as project_template/pipeline/train.py:46-48 of the reference
dumps its model.  The CPU test unpickles it in a process that never loads
libmf_hip.so and pins the attributes to the golden vectors.
"""
import os
import pickle
import sys

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "matrix-factorization_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import golden_hp, load_golden  # noqa: E402

import matrix_factorization as mf  # noqa: E402

d = load_golden("tiny_linear")
hp = golden_hp(d)
hp["verbose"] = 0
np.random.seed(int(d["seed"]))
X = pd.DataFrame({"user_id": d["user_id"], "item_id": d["item_id"]})
m = mf.KernelMF(**hp).fit(X, pd.Series(d["rating"]))
out = os.path.join(ROOT, "gpurun_out", "pickle")
os.makedirs(out, exist_ok=True)
with open(os.path.join(out, "kernelmf_tiny_linear_gpu.pkl"), "wb") as f:
    pickle.dump(m, f)
print("wrote", os.path.join(out, "kernelmf_tiny_linear_gpu.pkl"),
      "max|P - golden| =", float(np.max(np.abs(m.user_features - d["user_features"]))))
