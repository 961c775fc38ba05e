"""matrix_factorization -- MI355X-native drop-in for the SGD path of
SHEEPididoo/matrix-factorization.

Same public names as the reference package for the path this build covers
(matrix_factorization/__init__.py:1-16 of the reference): KernelMF and
BaselineModel train on the GPU through libmf_hip.so (hand-written gfx950
kernels behind a C ABI, include/mf_hip.h); RecommenderBase and
train_update_test_split are the host-side surface around them.  ALSMF (no
reference counterpart: BASELINE config 5) fits the same linear factor model
by alternating least squares with an MFMA Gramian.  The
neighbourhood and content-based models of the reference are outside this
build's scope.
"""

from .als_matrix_factorization import ALSMF
from .baseline_model import BaselineModel
from .kernel_matrix_factorization import KernelMF
from .recommender_base import RecommenderBase
from .utils import train_update_test_split

__all__ = [
    "ALSMF",
    "BaselineModel",
    "KernelMF",
    "RecommenderBase",
    "train_update_test_split",
]

__version__ = "0.1.0"
