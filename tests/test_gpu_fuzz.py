"""GPU parity on randomised cases: a slice of the seeded generators of tools/fuzz_parity.py (extraction: frame
size, nfeatures, scale factor, 1-12 levels, FAST thresholds, OpenCV variant bits, noise / scene content) and
tools/fuzz_matcher.py (SearchByBoW both forms, single and batched, SearchForTriangulation single and batched, with
random FeatureVectors, map-point / stereo masks, ratio, orientation check, F12 and epipoles) against the oracle.
The full runs (400 and 150 cases, 0 mismatches) are recorded in profiles/r06/fuzz_parity_*.log; these seeds keep
a sample of them in the suite.  Bit-exact; a refusal must be the oracle's too, or the LDS bound orbgpu.h
documents for ORB_ERR_GEOMETRY."""
import pytest

pytestmark = pytest.mark.gpu

# seeds of the recorded runs: 0..63 of the extraction run hold equal cases, both-side refusals, the LDS bound (10, 16)
# and a variant mix;
# matcher seeds 16..39 include seed 24's both-side refusal (a 348 x 595 portrait frame)
EXTRACT_SEEDS = list(range(0, 64))
MATCHER_SEEDS = list(range(16, 40))


@pytest.fixture(scope="module")
def fuzz_extract(orbgpu_mod, oracle_mod):
    from tools import fuzz_parity
    return fuzz_parity


@pytest.fixture(scope="module")
def fuzz_matcher(orbgpu_mod, oracle_mod):
    from tools import fuzz_matcher
    return fuzz_matcher


@pytest.mark.parametrize("seed", EXTRACT_SEEDS)
def test_fuzz_extract_case(fuzz_extract, seed):
    st, cfg, nk = fuzz_extract.extract_case(seed)
    assert st in ("equal", "refused", "refused_bound"), (st, cfg, nk)


@pytest.mark.parametrize("seed", MATCHER_SEEDS)
def test_fuzz_matcher_case(fuzz_matcher, seed):
    st, info, bad = fuzz_matcher.matcher_case(seed)
    assert st in ("equal", "refused"), (st, info, bad)
