"""GPU: BASELINE config 4's per-GPU workloads at full size.

* the strong-scaling base: the 9.6M x 80 mesh as one partition on this GPU (about 100 GB of HBM),
  the direction-split pass with the plan's automatic settings;
* rank 3 of the 8-way strong split: an interior 3200 x 375 strip (1.2M nodes, two neighbours) built
  from global ids, i.e. one GPU's share of the N = 8 point.

Both run through bench.py's own legs (the exact commands of the driver's bench: ``--scaling strong``
and ``--emulate-rank 3/8``), in a child process, which checks every owned cell and local edge with
the oracle: the strip-parallel check (16 worker processes, each the oracle on a row strip widened by
one row, exact without an exchange); for the emulated rank the halo rows' plus/minus come from the
oracle's pass over the two halo rows alone (``bench.oracle_halo_plus_minus``, tested against the
single-domain pass in tests/test_bench.py).  A mismatch makes bench.py exit with status 1.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def run_bench(*extra, timeout=540):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--scaling", "strong", "--extras", "none",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines, f"bench.py printed no record (rc {r.returncode}):\n{r.stderr[-3000:]}"
    rec = json.loads(lines[-1])
    assert r.returncode == 0, f"rc {r.returncode}: {rec.get('check')}\n{r.stderr[-3000:]}"
    return rec


@pytest.mark.timeout(600)
def test_config4_strong_base_9p6m_x_80_on_one_gpu():
    rec = run_bench()
    assert rec["config"]["nodes_per_gpu"] == 3200 * 3000 and rec["config"]["levels"] == 80, rec["config"]
    chk = rec["check"]
    assert chk["exact"] and chk["max_abs"] == 0.0 and not chk["mismatched_cells"], chk
    assert chk["cells_compared"] >= 9_600_000 * 80, chk  # every owned wet cell at least once


@pytest.mark.timeout(300)
def test_config4_rank3_of_8_strip_with_the_oracles_halo_rows():
    rec = run_bench("--emulate-rank", "3/8")
    assert rec["config"]["nodes_per_gpu"] == 3200 * 375, rec["config"]
    chk = rec["check"]
    assert chk["exact"] and chk["max_abs"] == 0.0 and not chk["mismatched_cells"], chk
    assert chk["ranks"] == 8 and "halo" in chk, chk
