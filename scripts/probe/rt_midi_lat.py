"""Per-sample latency of tests/cpp/rt_midi.cpp around the setters (which samples are slow)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
exe = os.path.join(ROOT, "tests", "cpp", "rt_midi")
lib = os.path.join(ROOT, "huygens_amd", "lib")
r = subprocess.run(["g++", "-std=c++17", "-O2", "-pthread", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "rt_midi.cpp"), "-o", exe, "-L", lib, "-lhuygens_hip",
                    f"-Wl,-rpath,{lib}", "-Wl,-rpath-link,/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib"],
                   capture_output=True, text=True)
assert r.returncode == 0, r.stderr[-2000:]
out = sys.argv[1]
os.makedirs(out, exist_ok=True)
N, S = 4096, 20000
p = subprocess.run([exe, out, str(N), str(S), sys.argv[2] if len(sys.argv) > 2 else "500"], capture_output=True,
                   text=True, timeout=120)
print(p.stdout.strip())
lat = np.fromfile(os.path.join(out, "lat.bin"), dtype=np.int64)[200:] * 1e-3
log = np.fromfile(os.path.join(out, "log.bin")).reshape(-1, 4)
seqs = set(int(v) - 200 for v in log[:, 0])
at = np.array([i in seqs for i in range(len(lat))])
print(f"all: median {np.median(lat):.2f} p99 {np.percentile(lat, 99):.2f} p99.9 {np.percentile(lat, 99.9):.2f} "
      f"worst {lat.max():.2f} us over {len(lat)} samples")
print(f"first sample after a setter ({at.sum()}): median {np.median(lat[at]):.2f} worst {lat[at].max():.2f}")
print(f"others: median {np.median(lat[~at]):.2f} p99 {np.percentile(lat[~at], 99):.2f} worst {lat[~at].max():.2f}")
top = np.argsort(lat)[-10:][::-1]
print("slowest samples (index, us, setter-at):", [(int(i), round(float(lat[i]), 1), bool(at[i])) for i in top])
