"""GPU parity: a Bowl<float> block into a Delaybank<float> in one launch (hz_bowl_fill_delaybank,
SURVEY.md 8(d) C5: `bowl.fill(buf, 1024); bank.process(buf, out, 1024)` per block).

* the bank's part is bit-exact: the fused outputs equal a separate Delaybank fed the fused fill
  buffer, block by block (the rings carry the feedback across blocks);
* the fill buffer is the Bowl model with the mode sum in a different (fixed) order than the
  separate fill's: within 1e-6 of the separate path, and the chain within north_star's 1e-5 of
  the restatement (OracleBowl -> OracleDelaybank);
* banks whose taps make samples of a block depend on each other run the two block calls (the
  bank then counts its own launches) and equal them exactly."""
import numpy as np
import pytest

from oracle import rel_err
from oracle_bowl import OracleBowl
from oracle_delay import OracleDelaybank

pytestmark = pytest.mark.gpu
SR = 48000


def _model(M, seed=5):
    rng = np.random.default_rng(seed)
    return (np.exp(rng.uniform(np.log(20.0), np.log(16000.0), M)), rng.uniform(1e-4, 5e-2, M),
            rng.uniform(0.05, 15.0, M))


def _c5_taps(k, short=False):
    if short:
        return [(0, 1.0)], [(300 + 7 * k, 0.5), (2000 + 53 * k, 0.25)]
    return [(0, 1.0)], [(10000 + 37 * k, 0.5), (20000 + 53 * k, 0.5)]


def _pair(torch, M, L, short=False):
    from huygens_amd import Bowl, Delaybank
    f, a, d = _model(M)
    bowl = Bowl(M, f, a, d, np.float32)
    bank = Delaybank(L, 3, 2 * SR, np.float32)
    for k in range(L):
        bank.coefficients(k, *_c5_taps(k, short))
    s = torch.cuda.Stream()   # one stream for both (torch's default stream is the null stream)
    bowl.set_stream(s.cuda_stream)
    bank.set_stream(s.cuda_stream)
    bowl._keep_stream = s
    return bowl, bank


def _run(torch, M, L, blocks, B=1024, fused=True, short=False, mix=True):
    bowl, bank = _pair(torch, M, L, short)
    buf = torch.zeros(blocks * B, dtype=torch.float32, device="cuda")
    out = torch.zeros(blocks * B * (1 if mix else L), dtype=torch.float32, device="cuda")
    bank.profile(True)
    bowl.trigger()
    for i in range(blocks):
        bp = buf.data_ptr() + 4 * B * i
        op = out.data_ptr() + 4 * B * i * (1 if mix else L)
        if fused:
            bowl.fill_delaybank(bank, bp, op, B, mix)
        else:
            bowl.fill_device(bp, B)
            bank.process_device(bp, op, B, False, mix)
    torch.cuda.synchronize()
    bank_launches = bank.profile_read()[1]
    bank.profile(False)
    return buf.cpu().numpy(), out.cpu().numpy(), bank_launches


def test_c5_fused_vs_separate_and_oracle():
    torch = pytest.importorskip("torch")
    M, L, blocks, B = 2048, 64, 30, 1024   # 30 blocks: both feedback taps of every line live
    bf, of, lf = _run(torch, M, L, blocks)
    bs, os_, ls = _run(torch, M, L, blocks, fused=False)
    assert lf == 0 and ls == blocks          # the fused path launched nothing on the bank
    assert rel_err(bf, bs) < 1e-6
    assert rel_err(of, os_) < 1e-6
    # the bank's arithmetic is the separate engine's, bit for bit, on the same input
    from huygens_amd import Delaybank
    bank = Delaybank(L, 3, 2 * SR, np.float32)
    for k in range(L):
        bank.coefficients(k, *_c5_taps(k))
    ref = np.concatenate([bank.process(bf[i * B:(i + 1) * B], mix=True) for i in range(blocks)])
    assert np.array_equal(of, ref)
    # the restatement: Bowl<float>::fill -> Delaybank<float,64>, lines mixed / 64
    f, a, d = _model(M)
    ob = OracleBowl(M, f, a, d, np.float32)
    ob.trigger()
    ox = np.concatenate([ob.fill(B) for _ in range(blocks)])
    od = OracleDelaybank(L, 3, 2 * SR, np.float32)
    for k in range(L):
        od.coefficients(k, *_c5_taps(k))
    oy = od.process(ox, mix=True)
    assert rel_err(bf, ox) < 1e-5
    assert rel_err(of, oy) < 1e-5


def test_line_outputs_and_ragged_block():
    """mix = 0 (line-major outputs) and a block length that is not a multiple of the
    workgroup's 4 samples."""
    torch = pytest.importorskip("torch")
    M, L, blocks = 300, 5, 12
    for B in (1021, 64):
        bowl, bank = _pair(torch, M, L)
        buf = torch.zeros(blocks * B, dtype=torch.float32, device="cuda")
        out = torch.zeros(blocks * B * L, dtype=torch.float32, device="cuda")
        bowl.trigger()
        for i in range(blocks):
            bowl.fill_delaybank(bank, buf.data_ptr() + 4 * B * i, out.data_ptr() + 4 * B * L * i, B, False)
        torch.cuda.synchronize()
        bf, of = buf.cpu().numpy(), out.cpu().numpy()
        from huygens_amd import Delaybank
        ref_bank = Delaybank(L, 3, 2 * SR, np.float32)
        for k in range(L):
            ref_bank.coefficients(k, *_c5_taps(k))
        ref = np.concatenate([ref_bank.process(bf[i * B:(i + 1) * B]).reshape(-1) for i in range(blocks)])
        assert np.array_equal(of, ref)


def test_dependent_taps_fall_back():
    """A feedback tap shorter than the block: the two block calls run (the bank counts its
    launches) and the outputs equal the separate calls'."""
    torch = pytest.importorskip("torch")
    bf, of, lf = _run(torch, 256, 8, 6, short=True)
    bs, os_, ls = _run(torch, 256, 8, 6, fused=False, short=True)
    assert lf == ls == 6
    assert np.array_equal(bf, bs) and np.array_equal(of, os_)
