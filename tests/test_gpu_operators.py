"""GPU operators vs the oracle and the reference's stage fixtures (bit-exact for integer
outputs, 1e-12 absolute for complex128 stages, 2e-5 for complex64 FFTs)."""

import io

import numpy as np
import pytest
import torch
from conftest import load_stages, stage_arrays

import ofdm_oracle as O
from ofdm_based_systems import _backend as B
from ofdm_based_systems.channel.models import ChannelModel
from ofdm_based_systems.constellation.adaptive import AdaptiveConstellationMapper
from ofdm_based_systems.constellation.models import NNClassifier, PSKConstellationMapper, QAMConstellationMapper
from ofdm_based_systems.equalization.models import MMSEEqualizator, NoEqualizator, ZeroForcingEqualizator
from ofdm_based_systems.modulation.models import OFDMModulator, SingleCarrierOFDMModulator
from ofdm_based_systems.noise.models import AWGNoiseModel, NoNoiseModel
from ofdm_based_systems.prefix.models import CyclicPrefixScheme, NoPrefixScheme, ZeroPaddingPrefixScheme

pytestmark = pytest.mark.gpu
EQ = {"MMSE": MMSEEqualizator, "ZF": ZeroForcingEqualizator, "NONE": NoEqualizator}


@pytest.mark.parametrize("precision", [B.OFDM_F64, B.OFDM_F32])
@pytest.mark.parametrize("logn", list(range(0, 13)))
def test_fft_matches_numpy(gpu, logn, precision):
    n = 1 << logn
    rng = np.random.default_rng(logn)
    x = rng.normal(size=(7, n)) + 1j * rng.normal(size=(7, n))
    plan = B.Plan(n_fft=n, precision=precision)
    dt = plan.cdtype
    tol = 1e-12 if precision == B.OFDM_F64 else 3e-5
    for inverse in (0, 1):
        d = torch.from_numpy(x).to(dt).to(gpu)
        B.check(B.lib().ofdm_fft(plan.handle, B.stream_ptr(), B.ptr(d), 7, inverse))
        ref = np.fft.ifft(x, axis=1, norm="ortho") if inverse else np.fft.fft(x, axis=1, norm="ortho")
        np.testing.assert_allclose(d.cpu().numpy(), ref, rtol=0, atol=tol * max(1.0, np.sqrt(logn)))


@pytest.mark.parametrize("m", [4, 16, 64, 256])
def test_qam_encode_decode_vs_oracle(gpu, m):
    rng = np.random.default_rng(m)
    b = int(np.log2(m))
    data = rng.integers(0, 256, size=3 * 1000 + 1, dtype=np.uint8).tobytes()  # ragged tail
    mapper = QAMConstellationMapper(m)
    sym = mapper.encode(io.BytesIO(data))
    idx = O.bits_to_indices(O.bytes_to_bits(data), b)
    assert np.array_equal(sym, O.qam_lut(m)[idx])
    z = sym + 0.08 * (rng.normal(size=len(sym)) + 1j * rng.normal(size=len(sym)))
    got = mapper.decode(z).read()
    assert got == O.indices_to_bytes(O.nn_demap(z, O.qam_lut(m)), b)
    # encode from a bit list (no padding path) and scalar decode
    bits = rng.integers(0, 2, size=5 * b).tolist()
    assert np.array_equal(mapper.encode(bits), O.qam_lut(m)[O.bits_to_indices(np.array(bits), b)])
    assert mapper.decode(complex(sym[0])).read() == O.indices_to_bytes(idx[:1], b)


@pytest.mark.parametrize("m", [2, 4, 8, 16])
def test_psk_encode_decode_vs_oracle(gpu, m):
    rng = np.random.default_rng(100 + m)
    b = int(np.log2(m))
    data = rng.integers(0, 256, size=96, dtype=np.uint8).tobytes()
    mapper = PSKConstellationMapper(m)
    sym = mapper.encode(io.BytesIO(data))
    idx = O.bits_to_indices(O.bytes_to_bits(data), b)
    assert np.array_equal(sym, O.psk_lut(m)[idx])
    z = sym + 0.05 * (rng.normal(size=len(sym)) + 1j * rng.normal(size=len(sym)))
    assert mapper.decode(z).read() == O.indices_to_bytes(O.nn_demap(z, O.psk_lut(m)), b)


def test_nn_classifier_ties_take_first_index(gpu):
    lut = O.qam_lut(16)
    z = np.array([0, 1e-3, lut[3], (lut[0] + lut[1]) / 2], dtype=np.complex128)
    got = NNClassifier().classify(lut, z)
    assert np.array_equal(got, lut[O.nn_demap(z, lut)])


@pytest.mark.parametrize("st", load_stages(), ids=lambda s: s["name"])
def test_stage_operators_match_reference(gpu, st):
    a = stage_arrays(st["name"])
    N, M, cp, snr = st["N"], st["M"], st["cp"], st["snr_db"]
    mapper = QAMConstellationMapper(M)
    X = mapper.encode(io.BytesIO(a["tx_bytes"].tobytes())).reshape(-1, N)
    assert np.array_equal(X, a["X"])
    prefix = CyclicPrefixScheme(cp) if st["prefix"] == "CP" else NoPrefixScheme(cp)
    eq = EQ[st["eq"]](channel_frequency_response=a["H"], snr_db=snr)
    mod = OFDMModulator(N, prefix, eq)
    x = mod.modulate(X)
    np.testing.assert_allclose(x, a["x"], rtol=0, atol=1e-12)
    s = a["x"].ravel()
    y_clean = ChannelModel(a["h_raw"], snr, NoNoiseModel()).transmit(s)
    np.testing.assert_allclose(y_clean, a["y_clean"], rtol=0, atol=1e-12)
    np.random.seed(st["seed"])
    y = ChannelModel(a["h_raw"], snr, AWGNoiseModel()).transmit(s)
    np.testing.assert_allclose(y, a["y"], rtol=0, atol=1e-12)
    Z = mod.demodulate(a["y"].reshape(-1, N + cp))
    np.testing.assert_allclose(Z, a["Z"], rtol=1e-9, atol=1e-9)
    assert mapper.decode(a["Z"].ravel()).read() == a["rx_bytes"].tobytes()
    # per-row equaliser operator (the reference's call granularity)
    Y = np.fft.fft(a["y"].reshape(-1, N + cp)[:, cp:], axis=1, norm="ortho")
    np.testing.assert_allclose(eq.equalize(Y[0]), a["Z"][0], rtol=1e-9, atol=1e-9)


def test_channel_response_and_gains(gpu):
    from conftest import channel

    h = channel("severe_multipath")
    cm = ChannelModel(h, 10.0)
    for n in (8, 64, 1024):
        H = cm.get_frequency_response(n)
        np.testing.assert_allclose(H, np.fft.fft(cm.impulse_response, n), rtol=0, atol=1e-13)
        np.testing.assert_allclose(cm.get_gains(n), np.abs(np.fft.fft(cm.impulse_response, n)) ** 2,
                                   rtol=1e-13, atol=1e-15)


def test_zero_padding_and_sc_ofdm_vs_oracle(gpu):
    rng = np.random.default_rng(7)
    N, cp = 64, 3
    X = O.qam_lut(16)[rng.integers(0, 16, size=(5, N))]
    H = np.fft.fft(np.array([1, 0.3j, 0.1, -0.05]), N)
    eq = MMSEEqualizator(H, 20.0)
    zp = OFDMModulator(N, ZeroPaddingPrefixScheme(cp), eq)
    x = zp.modulate(X)
    ref_x = np.concatenate([np.fft.ifft(X, axis=1, norm="ortho"), np.zeros((5, cp))], axis=1)
    np.testing.assert_allclose(x, ref_x, atol=1e-12)
    y = x + 0.01 * (rng.normal(size=x.shape) + 1j * rng.normal(size=x.shape))
    folded = y[:, :N].copy()
    folded[:, :cp] += y[:, N:]
    ref_Z = O.equalize(np.fft.fft(folded, axis=1, norm="ortho"), H, "MMSE", 20.0)
    np.testing.assert_allclose(zp.demodulate(y), ref_Z, atol=1e-12)
    sc = SingleCarrierOFDMModulator(CyclicPrefixScheme(cp), ZeroForcingEqualizator(H), N)
    xs = sc.modulate(X)
    np.testing.assert_array_equal(xs, O.add_cp(X, cp))
    ref = np.fft.ifft(O.equalize(np.fft.fft(xs[:, cp:], axis=1, norm="ortho"), H, "ZF", 0), axis=1, norm="ortho")
    np.testing.assert_allclose(sc.demodulate(xs), ref, atol=1e-12)


def test_adaptive_mapper_vs_oracle(gpu):
    rng = np.random.default_rng(3)
    N = 64
    orders = rng.choice([0, 4, 16, 64, 256], size=N)
    orders[0] = 16
    m = AdaptiveConstellationMapper(orders, QAMConstellationMapper, N)
    bps = int(m.get_bits_per_subcarrier().sum())
    S = 8 * 3
    data = rng.integers(0, 256, size=S * bps // 8, dtype=np.uint8).tobytes()
    sym = m.encode(io.BytesIO(data)).reshape(S, N)
    res = O.run_adaptive(data, orders, N, np.array([1.0 + 0j]), 0, "NONE", 40.0, None)
    assert res.bit_errors == 0
    bits = O.bytes_to_bits(data).reshape(S, bps)
    offs = np.concatenate([[0], np.cumsum(m.get_bits_per_subcarrier())[:-1]])
    for k in range(N):
        if orders[k] == 0:
            assert np.all(sym[:, k] == 0)
            continue
        b = int(np.log2(orders[k]))
        idx = bits[:, offs[k]:offs[k] + b] @ (1 << np.arange(b - 1, -1, -1))
        assert np.array_equal(sym[:, k], O.qam_lut(int(orders[k]))[idx])
    noisy = sym.ravel() + 0.02 * (rng.normal(size=S * N) + 1j * rng.normal(size=S * N))
    out = m.decode(noisy).read()
    # oracle decode: per-subcarrier NN, subcarrier-major bits, whole bytes only
    rb = []
    z2 = noisy.reshape(S, N)
    for s in range(S):
        for k in range(N):
            if orders[k]:
                b = int(np.log2(orders[k]))
                i = O.nn_demap(z2[s, k:k + 1], O.qam_lut(int(orders[k])))[0]
                rb += [(i >> (b - 1 - j)) & 1 for j in range(b)]
    rb = np.array(rb[: len(rb) // 8 * 8], np.uint8)
    assert out == np.packbits(rb).tobytes()


@pytest.mark.parametrize("precision", [B.OFDM_F64, B.OFDM_F32])
@pytest.mark.parametrize("st", load_stages(), ids=lambda s: s["name"])
def test_demap_count_matches_reference_counts(gpu, st, precision):
    """ofdm_demap_count (fused decode + XOR/popcount) on the reference's own equalised symbols Z
    gives the reference's bit_errors / symbol_errors (constellation/models.py:251-295,
    simulation/models.py:596-606); complex64: Z rounded to float32, same decisions here."""
    a = stage_arrays(st["name"])
    N, M = st["N"], st["M"]
    plan = B.Plan(n_fft=N, precision=precision, luts=[O.qam_lut(M)])
    Z = torch.from_numpy(a["Z"]).to(plan.cdtype).to(gpu)
    tx = torch.from_numpy(a["tx_bytes"].copy()).to(gpu)
    cnt = torch.zeros(2, dtype=torch.int64, device=gpu)
    B.check(B.lib().ofdm_demap_count(plan.handle, B.stream_ptr(), B.ptr(Z), B.ptr(tx), Z.shape[0], B.ptr(cnt)))
    assert tuple(cnt.cpu().tolist()) == (st["bit_errors"], st["symbol_errors"])


def test_demap_count_adaptive_vs_oracle(gpu):
    """CAPACITY_BASED decode + count: per-subcarrier orders, unused subcarriers, the trailing
    partial byte of the run not compared (constellation/adaptive.py:259-263)."""
    rng = np.random.default_rng(11)
    N, S = 64, 7
    orders = rng.choice([0, 4, 16, 64, 256], size=N)
    orders[0] = 4
    m = AdaptiveConstellationMapper(orders, QAMConstellationMapper, N)
    bps = int(m.get_bits_per_subcarrier().sum())
    data = rng.integers(0, 256, size=(S * bps + 7) // 8, dtype=np.uint8).tobytes()
    bits = O.bytes_to_bits(data)[: S * bps].reshape(S, bps)
    offs = np.concatenate([[0], np.cumsum(m.get_bits_per_subcarrier())[:-1]])
    X = np.zeros((S, N), complex)
    idx = np.zeros((S, N), np.int64)
    for k in range(N):
        if orders[k]:
            b = int(np.log2(orders[k]))
            idx[:, k] = bits[:, offs[k]:offs[k] + b] @ (1 << np.arange(b - 1, -1, -1))
            X[:, k] = O.qam_lut(int(orders[k]))[idx[:, k]]
    Z = X + 0.06 * (rng.normal(size=X.shape) + 1j * rng.normal(size=X.shape))
    ridx = np.zeros_like(idx)
    for k in range(N):
        if orders[k]:
            ridx[:, k] = O.nn_demap(Z[:, k], O.qam_lut(int(orders[k])))
    import philox_streams as P
    be, se = P.adaptive_counts((ridx ^ idx).astype(np.int64), m.get_bits_per_subcarrier().astype(np.int64), S)
    luts, sc = m.lut_tables()
    plan = B.Plan(n_fft=N, precision=B.OFDM_F64, luts=luts, sc_lut=sc)
    Zd = torch.from_numpy(Z).to(gpu)
    tx = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to(gpu)
    cnt = torch.zeros(2, dtype=torch.int64, device=gpu)
    B.check(B.lib().ofdm_demap_count(plan.handle, B.stream_ptr(), B.ptr(Zd), B.ptr(tx), S, B.ptr(cnt)))
    assert be > 0 and tuple(cnt.cpu().tolist()) == (be, se)
