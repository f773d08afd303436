"""Device uniform item sampler (rg_uniform.hip through the C-ABI):
``sample_items(..., device=)`` / ``sample_items_device`` against NumPy's legacy
``RandomState.randint(0, num_items, shape)`` itself -- the reference's
``spotlight/sampling.py:9-35`` calls exactly that, so NumPy is the oracle here.
Checked bit-exact: the values, the generator state afterwards (key, position and the
cached Gaussian NumPy keeps beside them), and the next draws continuing from it.
Ranges cover NumPy's three cases: one value (no words drawn), masked rejection
(acceptance from just above 1/2 to 1) and the full 32-bit range."""
import numpy as np
import pytest
import torch

from recommendation_gans_amd.spotlight.sampling import sample_items, sample_items_device

pytestmark = pytest.mark.gpu

CASES = [
    (0, 20108, (5, 8192)),       # ML-20M items, n_neg x batch
    (1, 3, 1000),                # mask 3: acceptance 3/4
    (2, 2, 777),                 # mask 1: every word accepted
    (3, 1025, (7, 13)),          # mask 2047: acceptance just above 1/2
    (4, 2 ** 31 + 5, 5000),      # 32-bit words, mask 2^32 - 1
    (5, 2 ** 32, 3000),          # the full 32-bit range (no rejection)
    (6, 1, 10),                  # one value: NumPy draws nothing
    (7, 65537, 0),               # empty
    (8, 100, 300_000),           # many blocks
]


def states_equal(a, b):
    sa, sb = a.get_state(), b.get_state()
    return sa[0] == sb[0] and np.array_equal(sa[1], sb[1]) and sa[2:] == sb[2:]


@pytest.mark.parametrize("seed,num_items,shape", CASES)
def test_sample_items_device_matches_numpy(seed, num_items, shape):
    ref_rs, dev_rs = np.random.RandomState(seed), np.random.RandomState(seed)
    # move both generators to a mid-block position with a cached Gaussian
    ref_rs.random_sample(101), dev_rs.random_sample(101)
    ref_rs.standard_normal(), dev_rs.standard_normal()
    ref = ref_rs.randint(0, num_items, shape, dtype=np.int64)
    got = sample_items_device(num_items, shape, dev_rs, device="cuda")
    assert got.dtype == torch.int64 and tuple(got.shape) == tuple(np.shape(ref))
    assert np.array_equal(got.cpu().numpy(), ref)
    assert states_equal(ref_rs, dev_rs), "generator state after the draw"
    # the streams continue identically (the cached Gaussian included)
    assert ref_rs.standard_normal() == dev_rs.standard_normal()
    assert np.array_equal(ref_rs.randint(0, 97, 50), dev_rs.randint(0, 97, 50))


def test_sample_items_dropin_device_keyword():
    """The reference signature with the additive ``device`` keyword; consecutive calls
    continue one stream as consecutive NumPy calls do."""
    ref_rs, dev_rs = np.random.RandomState(11), np.random.RandomState(11)
    for _ in range(3):
        ref = ref_rs.randint(0, 20108, (3, 64), dtype=np.int64)
        got = sample_items(None, None, 20108, (3, 64), random_state=dev_rs, device="cuda")
        assert np.array_equal(got.cpu().numpy(), ref)
    assert states_equal(ref_rs, dev_rs)
    host = sample_items(None, None, 20108, (3, 64), random_state=dev_rs)   # default: NumPy, as the reference
    assert isinstance(host, np.ndarray) and np.array_equal(host, ref_rs.randint(0, 20108, (3, 64), dtype=np.int64))
