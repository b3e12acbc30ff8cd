"""CPU: the offline Audio stand-in (include/soundmath/audio.h) for src/audio.h -- the
reference's process(const float*, float*) callback driven over WAV files, headless."""
import os
import subprocess
import wave

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = r'''
#include "soundmath/audio.h"
using namespace soundmath;
#define BSIZE 32
static int process(const float* in, float* out) {   // 2 in -> 3 out, tests/*.cpp style callback
    for (int i = 0; i < BSIZE; i++) {
        out[3 * i] = 0.5f * in[2 * i];
        out[3 * i + 1] = in[2 * i] - in[2 * i + 1];
        out[3 * i + 2] = 0.25f;
    }
    return 0;
}
int main(int argc, char** argv) {
    Audio A(process, BSIZE);
    if (argc > 2) Audio::offline(argv[1], argv[2]);
    A.startup(2, 3, false);
    A.shutdown();
    return A.finished() ? 0 : 1;
}
'''


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    d = tmp_path_factory.mktemp("audio")
    src, out = d / "a.cpp", d / "a"
    src.write_text(PROG)
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                        str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return str(out)


def read_f32(path):
    raw = open(path, "rb").read()
    assert raw[:4] == b"RIFF" and raw[8:12] == b"WAVE"
    assert int.from_bytes(raw[20:22], "little") == 3   # IEEE float
    ch = int.from_bytes(raw[22:24], "little")
    rate = int.from_bytes(raw[24:28], "little")
    n = int.from_bytes(raw[40:44], "little")
    return np.frombuffer(raw[44:44 + n], dtype="<f4").reshape(-1, ch), rate


def test_int16_stereo_in(exe, tmp_path):
    x = (np.random.default_rng(0).uniform(-1, 1, (1000, 2)) * 32767).astype("<i2")
    p_in, p_out = tmp_path / "in.wav", tmp_path / "out.wav"
    with wave.open(str(p_in), "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(48000)
        w.writeframes(x.tobytes())
    r = subprocess.run([exe, str(p_in), str(p_out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    y, rate = read_f32(p_out)
    assert rate == 48000 and y.shape == (1000, 3)   # frames kept; 1000 = 31 blocks + 8
    xf = x.astype(np.float32) / np.float32(32768)
    assert np.array_equal(y[:, 0], np.float32(0.5) * xf[:, 0])
    assert np.array_equal(y[:, 1], xf[:, 0] - xf[:, 1])
    assert np.all(y[:, 2] == np.float32(0.25))


def test_silence_without_input(exe, tmp_path):
    p_out = tmp_path / "s.wav"
    env = dict(os.environ, HZ_AUDIO_OUT=str(p_out), HZ_AUDIO_SECONDS="0.01")
    r = subprocess.run([exe], capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stderr
    y, _ = read_f32(p_out)
    assert y.shape == (480, 3) and not y[:, :2].any() and np.all(y[:, 2] == np.float32(0.25))
