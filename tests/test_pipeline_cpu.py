"""simulate_CZ_gate_batch's chunked pipeline (simulation.py): the derivation of a slice
of a call (physics.slice_inputs) equals those rows of the whole call's derivation, bit for
bit, for every argument kind -- per-point apparatus arrays, species by name, per-point
overrides, shared and per-point bang-bang schedules, length-1 arrays that broadcast -- and
physics.concat_batches reassembles the whole DerivedBatch."""
import warnings

import numpy as np
import pytest

from noisyquantumsimulator_amd import configurations as CF
from noisyquantumsimulator_amd import physics as PH
from noisyquantumsimulator_amd import sweeps as SW


def _same(a, b):
    assert a.n == b.n and a.protocol == b.protocol and a.pulse_shape == b.pulse_shape
    assert set(a.cols) == set(b.cols)
    for k in a.cols:
        np.testing.assert_array_equal(a.cols[k], b.cols[k], err_msg=k)
    for f in ("bangbang_times", "bangbang_phases", "status_bits"):
        x, y = getattr(a, f), getattr(b, f)
        assert (x is None) == (y is None), f
        if x is not None:
            np.testing.assert_array_equal(x, y, err_msg=f)
    assert sorted(a.warnings) == sorted(b.warnings)


def _chunked(si, n, kw, bounds):
    parts = [PH.derive_batch(si, hi - lo, **PH.slice_inputs(kw, n, lo, hi)) for lo, hi in zip(bounds[:-1], bounds[1:])]
    return PH.concat_batches(parts)


def _cases():
    rng = np.random.default_rng(3)
    n = 997
    exc = SW.medium_excitation()
    yield "c2", *SW.omega_delta_call()
    kw = dict(temperature=np.logspace(-6, -4, n), tweezer_power=rng.uniform(1e-3, 0.1, n),
              species=np.array(["Rb87", "Cs133"])[rng.integers(0, 2, n)], B_field=np.array([2e-4]),
              spacing_factor=rng.uniform(2.0, 5.0, n), n_rydberg=rng.integers(50, 100, n).astype(float))
    yield "apparatus", CF.LPSimulationInputs(excitation=exc), n, kw
    yield "shared_bangbang", CF.JPSimulationInputs(excitation=exc), n, dict(
        overrides=dict(switching_times=np.array([1.0, 2.0, 3.0]), phases=np.array([0.0, 1.0, 2.0, 0.5]),
                       laser_2_power=rng.uniform(0.05, 1.0, n)))
    yield "per_point_bangbang", CF.JPSimulationInputs(excitation=exc), n, dict(
        overrides=dict(switching_times=np.sort(rng.uniform(0, 20, (n, 4)), axis=1),
                       phases=rng.uniform(-np.pi, np.pi, (n, 5))))
    yield "smooth_jp", CF.SmoothJPSimulationInputs(excitation=exc), n, dict(
        hilbert_space_dim=4, overrides=dict(A=rng.uniform(0.5, 1.5, n), delta_over_omega=rng.uniform(-0.05, 0.05, n)))


@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_chunked_derivation_is_the_whole_derivation(case):
    warnings.simplefilter("ignore")
    _, si, n, kw = case
    whole = PH.derive_batch(si, n, **kw)
    for bounds in ([0, n], [0, n // 4, n // 2, 3 * n // 4, n], [0, 1, 2, 515, n - 1, n]):
        _same(whole, _chunked(si, n, kw, bounds))


def test_batch_size_is_derive_batch_inference():
    warnings.simplefilter("ignore")
    si, n, kw = SW.omega_delta_call()
    assert PH.batch_size(**{k: v for k, v in kw.items() if k in PH.POINT_ARGS or k == "overrides"}) == n
    assert PH.batch_size(temperature=2e-6) == 1
    assert PH.batch_size(species=["Rb87"] * 5, overrides=dict(switching_times=np.zeros(7))) == 5
