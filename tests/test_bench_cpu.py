"""CPU checks of bench.py's bookkeeping (no GPU): the committed profiles it
reads beside its live measurement belong to the kernels it names."""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

import bench  # noqa: E402


def test_rocprof_summary_names_the_bench_kernels():
    """profiles/bench_kernel_stats.rocprof (the rocprofv3 --stats CSV of
    `bench.py --steps 10`) holds every kernel the roofline reports, with a
    plausible mean launch time."""
    prof = REPO / "profiles"
    for k in ("k_step_sell2", "k_dots_nc", "k_cgs_update_nc"):
        ms = bench.rocprof_avg_ms(prof, k)
        assert ms is not None and 0.001 < ms < 0.1, (k, ms)


def test_rocprof_summary_absent_is_none(tmp_path):
    assert bench.rocprof_avg_ms(tmp_path, "k_step_sell2") is None


def test_pmc_traffic_has_the_bench_kernels():
    t = bench.pmc_traffic(REPO / "profiles")
    for k in ("k_step_sell2:fold", "k_dots_nc", "k_cgs_update_nc"):
        assert t.get(k) and t[k] > 1e7, (k, t.get(k))
    # the FETCH_SIZE x2 correction is recorded with the numbers
    d = json.loads((REPO / "profiles" / "pmc_traffic.json").read_text())
    assert "x2" in d["_fetch_correction"]
