"""(diagnostic) repeat tests/test_filterbank_resp_gpu.py::test_stream_and_per_sample_after_stationary
in one process and count failures, optionally with the modal states off (HZ_FLAKE_NOMODAL=1)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import huygens_amd._lib as L  # noqa: E402
import test_filterbank_resp_gpu as T  # noqa: E402

if os.environ.get("HZ_FLAKE_NOMODAL"):
    orig = T.make

    def make(*a, **k):
        g, o = orig(*a, **k)
        g.tune_modal(False)
        return g, o
    T.make = make
fails = 0
n = int(os.environ.get("HZ_FLAKE_N", "12"))
poison = os.environ.get("HZ_FLAKE_POISON")
for i in range(n):
    if poison:   # device memory full of a large finite value, freed: later allocations may reuse it
        import torch
        t = torch.full((int(poison) << 17,), 3.0e3, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        del t
        torch.cuda.empty_cache()
    for lazy in (False, True):
        try:
            T.test_stream_and_per_sample_after_stationary(None, lazy)
        except AssertionError as e:
            fails += 1
            print("fail", i, lazy, str(e).split("\n")[0][:100])
print(f"{fails} failures in {2 * n} runs")
