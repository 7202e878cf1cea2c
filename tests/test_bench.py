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


# ----------------------------------------------------------------------------- parity check (verify)

class _Args:
    fct_iter = 1
    vlimit = 1


def test_compare_local_flags_one_changed_cell():
    """bench.py's check counts every differing cell and reports the largest difference."""
    import oracle as O
    m = synth.make_mesh(16, 12, 9, seed=3)
    f = synth.make_fields(m)
    want = [O.full_pass(m, f)]
    got = {k: want[0][k].copy().reshape(1, -1) for k in ("plus", "minus", "del_v", "del_h", "adf_v", "adf_h")}
    bad, max_abs, cells = bench.compare_local(m, got, want)
    assert not bad and max_abs == 0.0 and cells > 0
    got["del_h"][0, 5] += 1e-13
    got["adf_h"][0, -1] = np.nan
    bad, max_abs, _ = bench.compare_local(m, got, want)
    assert bad == {"del_h": 1, "adf_h": 1} and max_abs == float("inf")


def _verify_worker(rank, world, port, q):
    """One rank of bench.py's N > 1 check: oracle_local on its strip with the gloo halo."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fesom2_amd import partition
        g = synth.make_mesh(24, 16, 9, seed=11)
        m, lists = partition.local_mesh(g, partition.strip_parts(24, 16, world), rank)
        fields = synth.make_tracer_fields(m, 2)
        want = bench.oracle_local(m, fields, _Args(), dist, lists)
        q.put((rank, m.node_gid[: m.N].copy(), m.edge_gid.copy(),
               [{k: w[k] for k in ("plus", "minus", "del_v", "del_h", "adf_v", "adf_h")} for w in want], m.N))
    finally:
        dist.destroy_process_group()


def test_per_rank_oracle_with_gloo_halo_equals_single_domain():
    """bench.py's multi-GPU check runs the oracle per rank on its local mesh with the plus/minus halo
    exchanged over gloo; on every owned cell and local edge that equals the single-domain pass."""
    import socket
    import oracle as O
    mp = pytest.importorskip("torch.multiprocessing")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_verify_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = synth.make_mesh(24, 16, 9, seed=11)
    L = g.L
    for k, fk in enumerate(synth.make_tracer_fields(g, 2)):
        want = O.full_pass(g, fk)
        for rank, gid, egid, outs, n in res:
            o = outs[k]
            for name, w in (("plus", L), ("minus", L), ("del_v", L), ("del_h", L), ("adf_v", g.nl)):
                assert np.array_equal(o[name].reshape(-1, w)[:n], want[name].reshape(-1, w)[gid]), (rank, k, name)
            assert np.array_equal(o["adf_h"].reshape(-1, L), want["adf_h"].reshape(-1, L)[egid]), (rank, k)
