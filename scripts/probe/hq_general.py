"""(probe) block-engine accuracy on a high-Q bank (R = 0.9999, centre 1.0: the last band's double
pole at -R) over long calls, per engine, against the restatement, per 1024-sample block"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from golden.spec_numpy import resonant_coefficients  # noqa: E402
from oracle import OracleFilterbank  # noqa: E402
from test_c2_pinned_gpu import block_errors  # noqa: E402
from huygens_amd import Filterbank  # noqa: E402

R = float(os.environ.get("RAD", "0.9999"))
CENTRE = float(os.environ.get("CENTRE", "1.0"))
N = int(os.environ.get("NB", "64"))
CALLS = int(os.environ.get("CALLS", "6"))
fwd, back = resonant_coefficients(64, R, CENTRE)
fwd, back = fwd[64 - N:], back[64 - N:]
KP, KG = float(os.environ.get("KP", "0.01")), float(os.environ.get("KG", "0.01"))
if os.environ.get("FWD"):
    fwd = np.tile(np.array([float(v) for v in os.environ["FWD"].split(",")]), (N, 1))
CONFIGS = os.environ.get("CONFIGS", "auto,auto resp off,auto 4 groups,general,general 4 groups").split(",")
rng = np.random.default_rng(31)
xs = [rng.uniform(-1, 1, 200_000).astype(np.float32).astype(np.float64) for _ in range(CALLS)]
o = OracleFilterbank(2, N, KP, KG)
for n in range(N):
    o.coefficients(n, fwd[n], back[n])
o.boost(np.ones(N))
o.open()
ycs = [o.process(x) for x in xs]
ALL = {"auto": (0, 0, None), "auto resp off": (0, 0, 0), "auto 4 groups": (4, 0, 0),
       "general": (0, 1, None), "general 4 groups": (4, 1, None), "general 1 group": (1, 1, None)}
for label in CONFIGS:
    groups, path, resp = ALL[label]
    g = Filterbank(2, N, KP, KG)
    for n in range(N):
        g.coefficients(n, fwd[n], back[n])
    g.boost(np.ones(N))
    g.open()
    if groups:
        g.set_target_groups(groups)
    if path:
        g.set_path(path)
    if resp is not None:
        g.set_response(resp)
    out = []
    for x, yc in zip(xs, ycs):
        yg = g.process(x)
        err, _ = block_errors(yg, yc)
        np.save(os.path.join(ROOT, 'gpurun_out', f'hq_{label.replace(" ", "_")}.npy'), yg) if os.environ.get('SAVE') else None
        out.append(f"{g.last_path()}:{err.max():.1e}")
        if os.environ.get("PROFILE") and len(out) == 1:
            am = int(err.argmax())
            print("argmax", am, "peaks", " ".join(f"{v:.2e}" for v in _[max(0, am - 4):am + 4]),
                  "errs", " ".join(f"{v:.1e}" for v in err[max(0, am - 4):am + 4]))
            print("blocks", " ".join(f"{e:.1e}" for e in err[int(os.environ.get("B0", "0")):int(os.environ.get("B0", "0")) + 48]), flush=True)
    print(f"{label:18s} N {N} R {R} centre {CENTRE} k {KP},{KG} fwd {fwd[-1]}: " + " ".join(out), flush=True)
    g.close()
