"""Decryption-failure characterisation at the radix layer's noise limit: >= 10^6
bootstraps on the GPU, every one fed at the maximum noise the radix layer admits, zero decode
failures, and the measured noise against the analytic model of the pipeline.

Inputs.  The radix layer bounds a PBS input at kMaxNoise = 25 fresh-bootstrap variances
(csrc/radix.h).  Its two extreme shapes are exercised:
  * type A, 22 units: the carry prefix's lookup input 4 s0 + 2 s1 + s2 + c (csrc/radix.cpp
    carry_prefix), s in {0, 1, 2}, c in {0, 1}, bootstrapped through f(x) = x mod 3 -> a new s;
  * type B, 25 units: 4 s + 3 c, bootstrapped through g(x) = x mod 2 (= c) -> a new c.
Each round forms C combinations of each type from the previous round's outputs (random
permutations, so every combination's four / two inputs are distinct blocks of unit noise) on the
device (torch int64 arithmetic = u64 mod 2^64), bootstraps all 2C through the engine's raw device
boundary (fhe_pbs_batch_device: MFMA keyswitch + throughput blind rotate), and decrypts every
output on the device.  Round 0 starts from 4096 fresh encryptions tiled over the pool (its combos
are distinct tuples, not independent ones) and is counted separately; rounds 1.. are the sample.

Model (printed beside the measurement): per CMUX the external product adds
2 N var(digit) var(GGSW) = 2 * 2048 * (2^44/3) * (2^34/3) plus, when s_i = 1, the gadget rounding
(2^80/3) (1 + N/2); the factored CMUX multiplies both by ||X^a - 1||^2 = 2; n CMUX.  That gives the output sigma before f64 rounding; the measured excess is
the f64-accumulator/transform rounding.  The decode margin is set by the modulus switch (sigma =
2^54.6 at 22 units, tests/test_oracle.py) against the 2^58 half box."""
import math

import numpy as np
import pytest

from fhe_sign import Context, default_params, generate_keys, multi_bit_params

pytestmark = pytest.mark.gpu

C = 1 << 17          # combinations of each type per round -> 2C = 262,144 bootstraps per round
ROUNDS = 4           # measured rounds: 4 * 2C = 1,048,576 bootstraps at 22 / 25 units
DELTA = 1 << 59      # 2^63 / (message * carry)


def _model_sigma_log2(n, multibit=False):
    var_digit = 2.0 ** 44 / 3
    var_ggsw = 2.0 ** 34 / 3
    var_dec = (2.0 ** 80 / 3) * (1 + 1024)  # gadget rounding of one digit through the key polynomial
    if not multibit:  # n factored CMUX (acc += (X^a - 1) ExtProd(GGSW(s_i), acc)): the GGSW(s_i) noise
        # and, when s_i = 1, the rounding of acc's digits, both through ||X^a - 1||^2 = 2
        return 0.5 * math.log2(n * (2 * 2048 * var_digit * var_ggsw * 2 + 0.5 * 2 * var_dec))
    # n/2 groups: the key bundle sum_B (X^m_B - 1) GGSW(f_B) carries 3 GGSW noises, each through
    # ||X^m - 1||^2 = 2; the rounding of acc's digits enters through (X^m(s) - 1) unless s = 00 (3/4)
    return 0.5 * math.log2(n / 2 * (2 * 2048 * var_digit * var_ggsw * 3 * 2 + 0.75 * 2 * var_dec))


@pytest.mark.parametrize("lwe_bound", [44, 45])
@pytest.mark.parametrize("kind", ["classic", "multibit"])
def test_million_bootstraps_at_the_noise_limit(kind, lwe_bound):
    """lwe_bound: the small key's TUniform bound (KSK noise) -- 44 and 45 (tfhe 0.10's recalled
    new_t_uniform for this parameter set; neither can be verified offline), so the budget
    is shown to hold at both"""
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    dev = torch.device("cuda:0")
    mb = kind == "multibit"
    P = multi_bit_params() if mb else default_params()
    P.lwe_noise_log2 = lwe_bound
    ck, sk = generate_keys(P, seed=0x7E57)
    ctx = Context(0)
    ctx.set_server_key(sk)
    n = sk.params.lwe_dimension
    lid_f = ctx.lut([x % 3 for x in range(16)])
    lid_g = ctx.lut([x % 2 for x in range(16)])
    _, glwe = ck.export()
    S = torch.from_numpy(glwe.astype(np.int64)).to(dev)

    def decrypt(ct):  # phase and decoded value of every row (torch int64 wraps like u64)
        ph = torch.empty(ct.shape[0], dtype=torch.int64, device=dev)
        for i in range(0, ct.shape[0], 16384):
            blk = ct[i:i + 16384]
            ph[i:i + 16384] = blk[:, 2048] - (blk[:, :2048] * S).sum(dim=1)
        val = torch.remainder(torch.div(ph + (DELTA // 2), DELTA, rounding_mode="floor"), 32)
        return ph, val

    def torus_err(ph, m):  # signed phase error in units of 2^-64 (float64)
        return (ph - m * DELTA).to(torch.float64)

    # ---- round 0 inputs: 4096 fresh encryptions tiled over the pools
    rs = np.random.default_rng(0xF00D)
    sv0 = rs.integers(0, 3, 4096)
    cv0 = rs.integers(0, 2, 4096)
    ck.seed_encryption(0xA11, 100)
    fresh_s = torch.from_numpy(ck.encrypt_blocks(sv0).view(np.int64)).to(dev)
    fresh_c = torch.from_numpy(ck.encrypt_blocks(cv0).view(np.int64)).to(dev)
    tile = torch.arange(C, device=dev) % 4096
    pool_s, pool_c = fresh_s[tile].contiguous(), fresh_c[tile].contiguous()
    val_s = torch.from_numpy(sv0).to(dev)[tile]
    val_c = torch.from_numpy(cv0).to(dev)[tile]

    lut = torch.cat([torch.full((C,), lid_f, dtype=torch.int32), torch.full((C,), lid_g, dtype=torch.int32)]).to(dev)
    out = torch.empty((2 * C, 2049), dtype=torch.int64, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0xBEEF)
    fails, total = 0, 0
    errs_out, errs_a, errs_b = [], [], []
    for rnd in range(ROUNDS + 1):
        p = [torch.randperm(C, generator=g, device=dev) for _ in range(5)]
        combo = torch.empty((2 * C, 2049), dtype=torch.int64, device=dev)
        combo[:C] = 4 * pool_s[p[0]] + 2 * pool_s[p[1]] + pool_s[p[2]] + pool_c[p[3]]
        combo[C:] = 4 * pool_s[p[1]] + 3 * pool_c[p[4]]
        m_a = 4 * val_s[p[0]] + 2 * val_s[p[1]] + val_s[p[2]] + val_c[p[3]]
        m_b = 4 * val_s[p[1]] + 3 * val_c[p[4]]
        assert int(m_a.max()) <= 15 and int(m_b.max()) <= 15
        if rnd > 0:  # input noise of the combinations (one sample of each type per round suffices)
            ph, _ = decrypt(combo[:4096])
            errs_a.append(torus_err(ph, m_a[:4096]).cpu())
            ph, _ = decrypt(combo[C:C + 4096])
            errs_b.append(torus_err(ph, m_b[:4096]).cpu())
        torch.cuda.synchronize()
        ctx.pbs_device(combo.data_ptr(), 2 * C, lut.data_ptr(), out.data_ptr())
        ctx.sync()
        want = torch.cat([m_a % 3, m_b % 2])
        ph, got = decrypt(out)
        bad = int((got != want).sum())
        if rnd > 0:
            fails += bad
            total += 2 * C
            errs_out.append(torus_err(ph, want)[::16].cpu())
        else:
            assert bad == 0, f"round 0: {bad} decode failures"
        pool_s, pool_c = out[:C].clone(), out[C:].clone()
        val_s, val_c = want[:C], want[C:]
        del combo

    eo = torch.cat(errs_out).numpy()
    ea, eb = torch.cat(errs_a).numpy(), torch.cat(errs_b).numpy()
    s_out, s_a, s_b = (math.log2(x.std()) for x in (eo, ea, eb))
    model = _model_sigma_log2(n, mb)
    print(f"\nnoise [{kind}, lwe TUniform 2^{lwe_bound}]: {total} bootstraps at 22/25 units, {fails} decode failures; output sigma 2^{s_out:.2f} "
          f"(model without f64 rounding 2^{model:.2f}); inputs: 22-unit sigma 2^{s_a:.2f} "
          f"(22 x output: 2^{s_out + 0.5 * math.log2(22):.2f}), 25-unit 2^{s_b:.2f} "
          f"(2^{s_out + 0.5 * math.log2(25):.2f}); max |output err| = 2^{math.log2(np.abs(eo).max()):.2f}")
    ctx.close()
    assert total >= 1_000_000 and fails == 0
    # the measured output noise is the model's plus the f64 rounding: within a factor 2 in sigma
    assert model - 0.5 < s_out < model + 1.0
    # inputs carry 22 / 25 output variances (linear combination of independent blocks)
    assert abs(s_a - (s_out + 0.5 * math.log2(22))) < 0.15
    assert abs(s_b - (s_out + 0.5 * math.log2(25))) < 0.15
