"""Writes the bench's C2 coefficients (resonant_coefficients(4096, 0.999, 1.0)) as raw doubles,
4096 x (3 fwd + 2 back), for scripts/probe/stream_cpp.cpp."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from golden.spec_numpy import resonant_coefficients  # noqa: E402

f, b = resonant_coefficients(4096, 0.999, 1.0)
np.concatenate([np.asarray(f, np.float64), np.asarray(b, np.float64)], axis=1).tofile(sys.argv[1])
