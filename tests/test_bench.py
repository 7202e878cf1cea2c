"""CPU: bench.py's byte model and helpers (no GPU).

The roofline's `achieved` divides bench.kernel_bytes() by the measured launch time, so the model is
checked here against its definition on a real synthetic mesh.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import bench
from fesom2_amd import synth


@pytest.fixture(scope="module")
def stats():
    m = synth.config_mesh("8k x 20", full_depth=True)
    return m, bench.mesh_stats(m)


def test_mesh_stats_counts(stats):
    m, s = stats
    assert s["N"] == m.N and s["E"] == m.E and s["T"] == m.T
    assert s["cn"] == int((m.nlev_nod[: m.N].astype(np.int64) - 1).sum()) == m.N * m.L  # full depth
    assert s["ce"] == m.edge_cells
    assert s["ring"] == 7 * m.N - 4 * 128  # 6 neighbours + self; 2 fewer on the two non-periodic rows


def test_survey_bytes_match_the_survey_formula(stats):
    _, s = stats
    for ntr in (1, 6):
        kb = bench.kernel_bytes(s, ntr)
        assert kb["survey_pass"] == 32 * s["cn"] + ntr * (120 * s["cn"] + 24 * s["ce"])


def test_split_model_moves_internal_edges_from_b3h_to_p1v(stats):
    """With ice edge cells limited inside p1v: p1v writes their limited flux (+8 B per cell, +16 B
    of list per edge), b3h no longer reads and writes it (-16 B per cell, -16 B of index per edge)."""
    _, s = stats
    base = bench.kernel_bytes(dict(s), 1, split=True)
    with_int = bench.kernel_bytes(dict(s, ice=1000, nie=40), 1, split=True)
    assert with_int["fct_ale_p1v"] - base["fct_ale_p1v"] == 8 * 1000 + 16 * 40
    assert base["fct_ale_b3_horizontal"] - with_int["fct_ale_b3_horizontal"] == 16 * 1000 + 16 * 40
    # the unsplit paths ignore it
    assert bench.kernel_bytes(dict(s, ice=1000, nie=40), 1)["fct_ale_b3_horizontal"] == \
        bench.kernel_bytes(dict(s), 1)["fct_ale_b3_horizontal"]


def test_split_pass_bytes_close_to_survey_minimum(stats):
    """The direction-split pass moves (without internal edges) the survey minimum plus b3h's extra
    read of fct_adf_h and plus/minus, and the index arrays."""
    _, s = stats
    kb = bench.kernel_bytes(s, 1, split=True)
    extra = kb["pass_split"] - kb["survey_pass"]
    assert 0 < extra < 0.25 * kb["survey_pass"]


def test_stream_ceiling_without_a_gpu_is_none():
    """On a machine without a GPU the probe fails and the bench reports no ceiling (no exception)."""
    class A:
        config = "8k x 20"
    assert bench.stream_ceiling(A()) is None


def test_bench_help_runs_on_cpu():
    out = subprocess.run([sys.executable, os.path.join(bench.ROOT, "bench.py"), "--help"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0 and "--graph" in out.stdout
