"""Edge cases of the device path (empty and ragged batches, k > m, one-param
spaces, extreme float ranges, all-duplicate batches, argument errors) against
the oracle.  Needs a GPU."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import de as ode  # noqa: E402
from oracle import hashing as oh  # noqa: E402
from oracle import select as osel  # noqa: E402
from oracle.space import BOOL, ENUM, FLOAT, INT, Param, features, row_values  # noqa: E402


def _engine(space, seed=0):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from _spaces import to_manip
    from uptune_amd.engine import BatchEngine
    return BatchEngine(to_manip(space), device=0, seed=seed)


def _hex(d):
    from uptune_amd.engine import digests_to_hex
    return digests_to_hex(d)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_empty_batches():
    space = [Param("x", FLOAT, 0.0, 1.0), Param("n", INT, 1, 9)]
    e = _engine(space)
    e.population_init(16)
    assert e.propose_de(0).shape == (2, 0)
    empty = torch.zeros((2, 0), dtype=torch.float64, device="cuda")
    assert e.hash(empty).shape == (0, 8)
    assert e.dedup(torch.zeros((0, 8), dtype=torch.int32, device="cuda")).numel() == 0
    assert e.encode(empty).shape == (2, 0)
    idx, top = e.topk(torch.zeros(0, dtype=torch.float64, device="cuda"), 4)
    assert idx.cpu().tolist() == [-1, -1, -1, -1]


def test_single_candidate_round_and_k_above_m():
    space = [Param("x", FLOAT, -1.0, 1.0), Param("y", FLOAT, -1.0, 1.0)]
    e = _engine(space, seed=4)
    e.population_init(8)
    rng = np.random.default_rng(0)
    X = rng.uniform(size=(20, 2))
    e.gp_fit(X, np.sum(X ** 2, axis=1), lengthscale=0.5, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    e.history_reset(0)
    pop = e.population_get().cpu().numpy()
    for m in (1, 3, 257):
        idx, top, dig, vals = e.score_round_de(m, 300, round_=m)
        got = idx.cpu().numpy()
        # every distinct trial is selected once (clamped trials of a tiny population repeat),
        # the first occurrence of each, and the remaining slots are empty
        trial = ode.propose_de_vec(space, pop, 4, m, 0, m, 0.2, 1)
        hx = [oh.hash_config(space, row_values(space, trial, j)) for j in range(m)]
        first = [j for j in range(m) if hx[j] not in hx[:j]]
        valid = got[got >= 0].tolist()
        assert sorted(valid) == first and (got[len(first):] == -1).all()


def test_one_param_and_extreme_float_ranges():
    for space in ([Param("only", FLOAT, -1e300, 1e300)], [Param("tiny", FLOAT, 0.0, 1e-300)],
                  [Param("b", BOOL)], [Param("e", ENUM, options=list(range(300)))],
                  [Param("i", INT, -(2 ** 40), 2 ** 40)]):
        e = _engine(space, seed=5)
        e.population_init(700)
        pop = e.population_get().cpu().numpy()
        np.testing.assert_array_equal(pop, ode.population_init(space, 700, seed=5))
        got = e.propose_de(900, round_=1, cr=0.9).cpu().numpy()
        np.testing.assert_array_equal(got, ode.propose_de_vec(space, pop, 5, 1, 0, 900, 0.9, 1))
        assert _hex(e.hash(_dev(got))) == [oh.hash_config(space, row_values(space, got, j)) for j in range(900)]
        np.testing.assert_array_equal(e.encode(_dev(got)).cpu().numpy(), features(space, got))


def test_all_duplicate_batch():
    space = [Param("a", INT, 0, 5), Param("f", BOOL)]
    e = _engine(space)
    vals = np.tile(np.array([[3.0], [1.0]]), (1, 5000))
    d = e.hash(_dev(vals))
    e.history_reset(0)
    dup = e.dedup(d).cpu().numpy()
    assert dup[0] == 0 and dup[1:].all()
    e.history_add(_hex(d[:1]))
    assert e.dedup(d).cpu().numpy().all()          # now seen in the history as well
    s = np.zeros(5000)
    idx, _ = e.topk(_dev(s), 3, dup=_dev(np.zeros(5000, np.uint8)))
    assert idx.cpu().tolist() == osel.topk(list(s), 3)


def test_argument_errors_raise():
    from uptune_amd._lib import UthotError
    space = [Param("x", FLOAT, 0.0, 1.0)]
    e = _engine(space)
    with pytest.raises(UthotError):
        e.propose_de(10)                            # no population yet
    e.population_init(16)
    with pytest.raises(UthotError):
        e.propose_de(10, n_cross=5)                 # n_cross must be <= 4
    with pytest.raises(UthotError):
        e.score_round_de(10, 2)                     # no GP fitted
    with pytest.raises(UthotError):
        e.propose_ga(10, max_retries=0)
    with pytest.raises(ValueError):
        e.propose_pso(np.zeros(1), 4, crossover="op3_cross_XX")
