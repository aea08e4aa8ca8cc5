"""CPU tests of the oracle (test infrastructure) -- pins it before it is trusted.

1. SURVEY.md §8(c) known answers, produced by the reference's own
   cpu_attention (flash_attention.cu:668-697) at H=2, S=64, causal, srand(42).
2. Independent re-implementations: glibc rand() (TYPE_3 additive feedback) in
   Python for the generator, numpy's IEEE float16 for the conversions, and a
   float64 numpy attention for the math.
3. The committed golden fixtures (tests/golden/) bit-for-bit.
"""
import json
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_survey_known_answers():
    # "Result at H=2, S=64, causal, srand(42): o[0]=0.190674,
    # q[0]=-0.466553, sum=-5.014025" (reference cpu_attention compiled at survey time)
    q, k, v = oracle.gen_inputs(1, 2, 64, 128, 42)
    o = oracle.attention(q, k, v, True)
    qf, of = oracle.f16_bits_to_f32(q).ravel(), oracle.f16_bits_to_f32(o).ravel()
    assert f"{qf[0]:.6f}" == "-0.466553"
    assert f"{of[0]:.6f}" == "0.190674"
    s = np.float32(0)
    for x in of:  # the survey summed the fp16 outputs in float
        s = np.float32(s + x)
    assert f"{s:.6f}" == "-5.014025"


def _glibc_rand_stream(seed, n):
    """glibc random() TYPE_3 (x^31 + x^3 + 1), as srand()/rand() use it."""
    r = [0] * (34 + 310 + n)
    r[0] = seed
    for i in range(1, 31):
        hi, lo = divmod(r[i - 1], 127773)
        word = 16807 * lo - 2836 * hi
        if word < 0:
            word += 2147483647
        r[i] = word
    for i in range(31, 34):
        r[i] = r[i - 31]
    for i in range(34, len(r)):
        r[i] = (r[i - 31] + r[i - 3]) & 0xFFFFFFFF
    return [x >> 1 for x in r[344:344 + n]]


def test_generator_matches_independent_glibc_rand():
    n = 3000
    qs, ks, vs = oracle.gen_inputs(1, 1, n, 1, 42)
    stream = _glibc_rand_stream(42, 3 * n)
    RAND_MAX = 2147483647
    vals = [np.float16(np.float32(np.float32(x) / np.float32(RAND_MAX)) - np.float32(0.5))
            for x in stream]
    exp = np.array(vals, dtype=np.float16).view(np.uint16)
    np.testing.assert_array_equal(qs.ravel(), exp[0::3])
    np.testing.assert_array_equal(ks.ravel(), exp[1::3])
    np.testing.assert_array_equal(vs.ravel(), exp[2::3])


def test_f16_to_f32_exhaustive():
    lib = oracle.load()
    bits = np.arange(65536, dtype=np.uint32)
    ref = bits.astype(np.uint16).view(np.float16).astype(np.float32)
    got = np.array([lib.fa_oracle_f16_to_f32(int(b)) for b in bits], dtype=np.float32)
    finite = np.isfinite(ref)
    np.testing.assert_array_equal(got[finite].view(np.uint32), ref[finite].view(np.uint32))
    assert np.all(np.isnan(got[np.isnan(ref)]))
    assert np.array_equal(got[np.isinf(ref)], ref[np.isinf(ref)])


def test_f32_to_f16_rne():
    lib = oracle.load()
    rng = np.random.default_rng(0)
    xs = np.concatenate([
        rng.uniform(-1, 1, 20000).astype(np.float32),
        (rng.standard_normal(5000) * 1e4).astype(np.float32),
        (rng.standard_normal(5000) * 1e-6).astype(np.float32),  # fp16 subnormals
        np.array([0.0, -0.0, 65504.0, 65519.99, 65520.0, 1e9, -1e9, 2.0 ** -24, 2.0 ** -25,
                  3 * 2.0 ** -26, 5.960464477539063e-08, np.inf, -np.inf], dtype=np.float32),
    ])
    # exact ties (x.5 ulp) in the normal range
    ties = (np.arange(1, 2000, dtype=np.float32) * np.float32(2.0 ** -11) + np.float32(1.0)
            + np.float32(2.0 ** -12))
    xs = np.concatenate([xs, ties.astype(np.float32)])
    got = np.array([lib.fa_oracle_f32_to_f16(float(x)) for x in xs], dtype=np.uint16)
    with np.errstate(over="ignore"):
        ref = xs.astype(np.float16).view(np.uint16)
    np.testing.assert_array_equal(got, ref)


def _np_attention_f64(q, k, v, causal):
    qf, kf, vf = (oracle.f16_bits_to_f32(x).astype(np.float64) for x in (q, k, v))
    d = qf.shape[-1]
    s = qf @ np.swapaxes(kf, -1, -2) / np.sqrt(d)
    if causal:
        n = s.shape[-1]
        s = np.where(np.tril(np.ones((n, n), bool)), s, -np.inf)
    s = s - s.max(-1, keepdims=True)
    p = np.exp(s)
    p /= p.sum(-1, keepdims=True)
    return p @ vf


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("scale", [1.0, 8.0])
def test_oracle_vs_float64(causal, scale):
    q, k, v = oracle.gen_inputs(2, 3, 97, 128, 5)
    if scale != 1.0:
        f = lambda a: (oracle.f16_bits_to_f32(a) * scale).astype(np.float16).view(np.uint16)
        q, k = f(q), f(k)
    o = oracle.f16_bits_to_f32(oracle.attention(q, k, v, causal))
    ref = _np_attention_f64(q, k, v, causal)
    # oracle is fp32 then rounded to fp16: within one fp16 ulp of |o| <= 0.5
    assert np.max(np.abs(o - ref)) <= 3e-4


def test_thread_count_invariance():
    q, k, v = oracle.gen_inputs(2, 4, 130, 128, 9)
    a = oracle.attention(q, k, v, True, threads=1)
    b = oracle.attention(q, k, v, True, threads=4)
    np.testing.assert_array_equal(a, b)


def test_heads_subset_matches_full():
    q, k, v = oracle.gen_inputs(2, 3, 64, 128, 1)
    full = oracle.attention(q, k, v, False)
    part = oracle.attention_heads(q, k, v, 2, 5, False)
    np.testing.assert_array_equal(part.reshape(6, -1)[2:5], full.reshape(6, -1)[2:5])
    assert not part.reshape(6, -1)[:2].any()


@pytest.mark.parametrize("causal", [False, True])
def test_rows_subset_matches_full(causal):
    # the row-sampled entry (maximum-size GPU tests) is the same per-row code
    q, k, v = oracle.gen_inputs(1, 1, 300, 128, 5)
    full = oracle.attention(q, k, v, causal)[0, 0]
    rows = [0, 1, 63, 64, 150, 298, 299, 7]
    got = oracle.attention_rows(q[0, 0], k[0, 0], v[0, 0], rows, causal)
    np.testing.assert_array_equal(got, full[rows])


@pytest.mark.parametrize("name", ["attn_h2_s64_causal", "attn_h2_s64_noncausal",
                                  "attn_h2_s256_causal", "attn_h2_s256_noncausal"])
def test_golden_fixtures(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    h, s = (int(x[1:]) for x in name.split("_")[1:3])
    causal = name.endswith("_causal")
    q, k, v = oracle.gen_inputs(1, h, s, 128, 42)
    np.testing.assert_array_equal(q, z["q"])
    np.testing.assert_array_equal(k, z["k"])
    np.testing.assert_array_equal(v, z["v"])
    np.testing.assert_array_equal(oracle.attention(q, k, v, causal), z["o"])


def test_reference_check_hashes_small():
    """The s256 reference check (flash_attention.cu:757-788) vs its committed hash."""
    import hashlib

    with open(os.path.join(GOLDEN, "ref_checks.json")) as fh:
        checks = json.load(fh)
    c = checks["s256_h32_causal"]
    q, k, v = oracle.gen_inputs(1, c["heads"], c["seq_len"], 128, 42)
    o = oracle.attention(q, k, v, c["causal"])
    assert hashlib.sha256(o.tobytes()).hexdigest() == c["sha256_o"]
    assert o.reshape(-1, 128)[0].tolist() == c["o_row0_bits"]


def test_max_abs_diff_metric():
    a = np.array([0x3C00, 0x0000], np.uint16)  # 1.0, 0.0
    b = np.array([0x3C01, 0xB800], np.uint16)  # 1.0009765625, -0.5
    assert oracle.max_abs_diff(a, b) == pytest.approx(0.5)
