"""Parity with every work buffer pre-filled with a pattern (RF_AMD_POISON, read at batch
creation): a kernel that read memory it did not write in the current build (stale results
of an earlier batch that happened to occupy the same memory) would fail here."""
import pytest

from tests import test_gpu_fuzz as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("pattern", ["165", "255", "0"])
@pytest.mark.parametrize("seed", sorted(set(range(0, 150, 5)) | {59}))
def test_fuzz_parity_poisoned(oracle, monkeypatch, pattern, seed):
    monkeypatch.setenv("RF_AMD_POISON", pattern)
    F.test_random_geometry_parity(oracle, seed)
