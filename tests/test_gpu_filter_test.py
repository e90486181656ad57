"""The reference's own filter tests, unmodified, against the drop-in.

tests/functional/filter_test.c is the reference's only direct test of the routing filter
(SURVEY §4). oracle/ref_filter_test.c #includes it unmodified and exports its two test
bodies; oracle/Makefile links that unit once with the reference's src/routing_filter.c
(_ref/libfilter_test_ref.so) and once with shim/routing_filter_amd.c -- the MI355X engine --
in its place (_ref/libfilter_test_shim.so), each on the reference's page stack. Both must
return STATUS_OK and print the same numbers: per step num_unique and the unique-key
estimate, the estimate across filters (routing_filter_estimate_unique_fp) and the false
positive rate.
"""
import re

import pytest

from oracle import refimpl as R

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not (R.available(R.FT_REF_PATH) and R.available(R.FT_SHIM_PATH)),
                                 reason="oracle/_ref filter_test libraries not built")]

RFLIMIT = 8_388_607  # routing_filter_max_fingerprints at the test config (fp 26, lis 8)
FANOUT = 8  # tests/config.c:31


def run_both(fn):
    out = []
    for path in (R.FT_REF_PATH, R.FT_SHIM_PATH):
        with R.Stack(path=path, cache_mib=2048, disk_mib=16384) as s:
            out.append(fn(s))
            assert s.device_writes() == 0
    return out


# the four configurations of filter_test() (filter_test.c:383-410)
@pytest.mark.timeout(900)
@pytest.mark.parametrize("num_fingerprints,num_values", [
    (RFLIMIT // FANOUT, FANOUT), (100, FANOUT), (1, FANOUT), (1, 2 * FANOUT)])
def test_filter_basic_reference_vs_shim(num_fingerprints, num_values):
    (rc_r, log_r), (rc_s, log_s) = run_both(lambda s: s.filter_test_basic(num_fingerprints, num_values))
    assert rc_r == 0 and rc_s == 0, (rc_r, rc_s, log_s)
    assert log_s == log_r
    assert "false positive rate" in log_s


def _numbers(log):
    """the perf test's non-timing lines (its timing lines differ by construction)"""
    return [ln for ln in log.splitlines() if ln.startswith("filter_basic_test: false positive rate")]


@pytest.mark.timeout(900)
def test_filter_perf_reference_vs_shim():
    """test_filter_perf (filter_test.c:150-273) scaled to 2 trees of 8 x 65,535 fingerprints
    (the reference runs 100 trees of 8 x 1,048,575): chains of incremental adds, then a
    synchronous routing_filter_lookup of every key and of as many unused keys"""
    (rc_r, log_r), (rc_s, log_s) = run_both(lambda s: s.filter_test_perf(65_535, FANOUT, 2))
    assert rc_r == 0 and rc_s == 0
    assert _numbers(log_s) == _numbers(log_r) and len(_numbers(log_r)) == 1
    assert re.search(r"filter insert time per key \d+", log_s)
