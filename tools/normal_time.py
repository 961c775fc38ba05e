"""Host-only timing of fit()'s initial draws at C3: np.random.normal of P
(1M x 64) and Q (100K x 64) from the global legacy RandomState."""
import json
import time

import numpy as np

np.random.seed(0)
t = time.perf_counter()
np.random.normal(0, 0.1, (1_000_000, 64))
np.random.normal(0, 0.1, (100_000, 64))
print(json.dumps({"normals": 70_400_000, "s": round(time.perf_counter() - t, 3)}))
