"""Host check of the FMA-corrected quotients in the HIP kernels (tests/cpp/divcheck.c):
cdiv_one (hz_fb_tv.hip, the resonant gain's complex divide from one reciprocal) and div_sr
(x / 48000) equal the IEEE quotients bit for bit on random and targeted hard inputs.
(An empirical check: the one-step correction is not proven exact for q0 = RN(ratio RN(1/den)).)"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fma_corrected_quotients_bit_exact(tmp_path):
    exe = tmp_path / "divcheck"
    subprocess.run(["gcc", "-O2", "-march=native", "-ffp-contract=off",
                    os.path.join(ROOT, "tests", "cpp", "divcheck.c"), "-o", str(exe), "-lm"], check=True)
    r = subprocess.run([str(exe), "4000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    rows = {" ".join(l.split()[:2]): [int(v) for v in l.split()[2:]] for l in r.stdout.splitlines()
            if l.startswith(("cdiv_one", "div_sr"))}
    assert set(rows) == {"cdiv_one hard", "cdiv_one resonant", "cdiv_one generic", "div_sr generic"}
    for name, (trials, bad) in rows.items():
        assert trials > 1_000_000 and bad == 0, (name, trials, bad)
