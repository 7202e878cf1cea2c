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
from fesom2_amd import partition, synth


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
    assert bench.stream_ceiling("8k x 20") is None
    assert bench.stream_ceiling("8k x 20", 6) is None


def test_pass_roofline_against_the_copy_rate():
    """pass_roofline: SURVEY.md 8(d)'s pass bytes per second against 8 TB/s (frac) and against the
    same run's flat-copy rate (frac_of_copy): the cross-round figure of the driver line."""
    r = bench.pass_roofline(21.5e9, 4.0, {"copy_GBps": 6250.0, "p1v_pattern_GBps": 5400.0})
    assert r["GBps"] == pytest.approx(5375.0) and r["frac"] == pytest.approx(5375.0 / 8000.0, abs=1e-4)
    assert r["copy_GBps"] == 6250.0 and r["frac_of_copy"] == pytest.approx(0.86, abs=1e-4)
    assert "frac_of_copy" not in bench.pass_roofline(21.5e9, 4.0, None)


@pytest.mark.parametrize("world,rank,full", [(4, 1, True), (4, 3, False), (3, 0, False)])
def test_emulated_rank_check_halo_is_the_single_domain_pass(world, rank, full):
    """The emulated-rank leg (one strip of the strong split on one GPU, no exchange) checks its pass
    with the halo plus/minus bench.oracle_halo_plus_minus computes from the halo rows alone: with
    them, phase 2 on the strip equals the single-domain pass on every owned cell and local edge."""
    import oracle as O
    nx, ny, nl = 20, 16, 11
    g = synth.make_mesh(nx, ny, nl, full_depth=full)
    want = O.full_pass(g, synth.make_fields(g))
    y0, y1 = partition.strip_rows(ny, world, rank)
    m, _ = partition.strip_local_mesh(nx, ny, nl, y0, y1, full_depth=full)
    f = synth.make_fields(m)
    st, p1 = O.pre_comm(m, f)
    assert st == 5
    hp, hm = bench.oracle_halo_plus_minus(nx, ny, nl, full, 1, world, rank)
    L = m.L
    assert hp.shape == (m.H, L)
    plus, minus = p1["plus"].reshape(-1, L).copy(), p1["minus"].reshape(-1, L).copy()
    gid = m.node_gid
    wet = np.arange(L)[None, :] < (m.nlev_nod[m.N:, None].astype(np.int64) - 1)
    assert np.array_equal(hp[wet], want["plus"].reshape(-1, L)[gid[m.N:]][wet])
    assert np.array_equal(hm[wet], want["minus"].reshape(-1, L)[gid[m.N:]][wet])
    plus[m.N:], minus[m.N:] = hp, hm
    r = O.post_comm(m, f, plus.reshape(-1), minus.reshape(-1))
    for name, w in (("del_v", L), ("del_h", L), ("adf_v", nl)):
        assert np.array_equal(r[name].reshape(-1, w)[: m.N], want[name].reshape(-1, w)[gid[: m.N]]), name
    assert np.array_equal(r["adf_h"].reshape(-1, L), want["adf_h"].reshape(-1, L)[m.edge_gid])


def test_cpu_baseline_host_counts_physical_cores():
    """The CPU baseline states what it represents: the host's physical cores (for the per-GPU share
    and the full-host estimate) beside nproc."""
    h = bench.host_info()
    assert h["nproc"] >= 1 and (h["physical_cores"] is None or 1 <= h["physical_cores"] <= h["nproc"])


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


# ----------------------------------------------------------------------------- parallel strip check

def _rank_outputs(g, m, ntr):
    """What the GPU of rank-local mesh m would hold after a pass: the single-domain oracle's values
    on its owned nodes / local edges (halo parts arbitrary), laid out as the handles (tracer-slowest)."""
    import oracle as O
    L, nl = g.L, g.nl
    out = {k: [] for k, _ in bench.OUTPUTS}
    NT = m.N + m.H
    for f in synth.make_tracer_fields(g, ntr):
        w = O.full_pass(g, f)
        for name, width in bench.OUTPUTS:
            wd = L if width == "L" else nl
            if name == "adf_h":
                a = w[name].reshape(-1, wd)[m.edge_gid]
            else:
                a = np.full((NT, wd), 7.0)
                a[: m.N] = w[name].reshape(-1, wd)[m.node_gid[: m.N]]
            out[name].append(a.reshape(-1))
    return {k: np.stack(v) for k, v in out.items()}


@pytest.mark.parametrize("mode", ["files", "data"])
@pytest.mark.parametrize("world,ntr,full", [(1, 1, False), (2, 2, False), (3, 1, True)])
def test_parallel_strip_check_is_exact_and_counts_each_cell_once(tmp_path, world, ntr, full, mode):
    """bench.py's parallel check: the oracle on row strips widened by one ring equals the
    single-domain pass on the strip's rows and edges (no exchange), every local edge is compared by
    exactly one strip, and a changed cell is reported once."""
    nx, ny, nl = 24, 17, 9
    g = synth.make_mesh(nx, ny, nl, full_depth=full)
    for rank in range(world):
        R0, R1 = partition.strip_rows(ny, world, rank)
        m, _ = partition.strip_local_mesh(nx, ny, nl, R0, R1, full_depth=full)
        got = _rank_outputs(g, m, ntr)
        s = bench.mesh_stats(m)
        wet = int(s["cn"])

        def run(arrs):
            files = {}
            for name, a in arrs.items():
                p = tmp_path / f"{rank}_{name}"
                mm = np.memmap(p, dtype=np.float64, mode="w+", shape=a.shape)
                mm[:] = a
                mm.flush()
                files[name] = (str(p), a.shape)
            cuts = [R0, R0 + (R1 - R0) // 3, R0 + 2 * (R1 - R0) // 3, R1]
            res = []
            for k in range(3):
                a_, b_ = cuts[k], cuts[k + 1]
                if b_ <= a_:
                    continue
                if mode == "files":
                    src = files
                else:  # the strip's slices, as verify_parallel sends them without /dev/shm room
                    e0, e1 = bench.strip_edge_range(nx, ny, R0, R1, a_, b_)
                    src = {name: (arr[:, e0 * g.L:e1 * g.L] if name == "adf_h" else
                                  arr[:, (a_ - R0) * nx * (g.L if w == "L" else nl):(b_ - R0) * nx * (g.L if w == "L" else nl)])
                           for (name, w), arr in zip(bench.OUTPUTS, [arrs[n] for n, _ in bench.OUTPUTS])}
                res.append(bench._check_strip((nx, ny, nl, full, 1, (R0, R1), (a_, b_), ntr, (mode, src))))
            bad, cells = {}, 0
            for b_, _, c in res:
                for k_, v in b_.items():
                    bad[k_] = bad.get(k_, 0) + v
                cells += c
            return bad, cells

        bad, cells = run(got)
        assert not bad, (rank, bad)
        assert cells == ntr * (2 * wet + 2 * m.N * m.L + m.N * nl + m.E * m.L), (rank, cells)
        got["adf_h"][ntr - 1, 5 * m.L + 1] += 1.0
        got["del_v"][0, 3] = np.nan
        bad, _ = run(got)
        assert bad == {"adf_h": 1, "del_v": 1}, bad


def test_kernel_bytes_min_is_the_survey_minimum(stats):
    """alg_bytes_min of p1v = phase 1 (48 Cn + 8 Ce) + the vertical half of phase 2 (48 Cn) at one
    tracer, mesh fields once per batch."""
    _, s = stats
    one = bench.kernel_bytes_min(s, 1)
    assert one["fct_ale_p1v"] == 96 * s["cn"] + 8 * s["ce"]
    assert one["fct_ale_p1"] == 48 * s["cn"] + 8 * s["ce"]
    six = bench.kernel_bytes_min(s, 6)
    assert six["fct_ale_p1v"] == 32 * s["cn"] + 6 * (64 * s["cn"] + 8 * s["ce"])
    # the kernel's own model counts halo columns, index arrays and internal-edge writes on top
    assert bench.kernel_bytes(s, 1, split=True)["fct_ale_p1v"] > one["fct_ale_p1v"]


def test_watchdog_exits_with_the_stage_on_stderr():
    """A stalled stage ends the rank (status 3) and names the stage."""
    code = ("import sys, time; sys.path.insert(0, %r); import bench; w = bench.Watchdog(5); "
            "w.arm('RCCL communicator setup', 1.0); time.sleep(30)") % bench.ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 3
    assert "rank 5: watchdog: stage 'RCCL communicator setup' not done within 1 s" in out.stderr


def test_reference_byte_models_follow_the_scripts_loops():
    """reference_byte_models evaluates the reference's kernel_tuner byte counters in closed form;
    here they are recounted with the scripts' own loops (kernels/fct_ale_a3.py:116-149,
    fct_ale_b1_horizontal.py:70-88, fct_ale_a2.py:102-111) on a small mesh with variable depth."""
    m = synth.config_mesh("tiny", full_depth=False)
    got = bench.reference_byte_models(m)
    levels = m.nlev_nod.astype(int)
    nelem = m.nie_num.astype(int)
    a3 = 0
    for node in range(m.N):
        a3 += 4
        for _ in range(levels[node] - 1):
            a3 += 4 + 16 + nelem[node] * (4 + 16)
        a3 += 4 * 8 + max(0, levels[node] - 3) * 4 * 8 + 4 * 8
    assert got["fct_ale_a3"] == a3
    b1h = 0
    t = m.edge_tri.reshape(-1, 2)
    le = m.nlev_elem.astype(int)
    for e in range(m.E):
        b1h += 12
        one = t[e, 0] - 1
        if t[e, 1] <= 0:
            b1h += 4
            n = max(le[one] - 1, 0)
        else:
            b1h += 8
            n = max(le[one] - 1, le[t[e, 1] - 1] - 1)
        b1h += n * 5 * 8
    assert got["fct_ale_b1_horizontal"] == b1h
    a2 = 16 * m.T
    for el in range(m.T):
        a2 += max(le[el] - 1, 0) * 8 * 8
        if le[el] <= m.nl - 1:
            a2 += (m.nl - 1 - le[el]) * 2 * 8
    assert got["fct_ale_a2"] == a2
    used = int((levels[: m.N] - 1).sum())
    assert got["fct_ale_b2"] == 4 * m.N + 7 * 8 * used
    assert got["fct_ale_c_vertical"] == 4 * m.N + 9 * 8 * used


def test_extra_legs_cover_every_baseline_config_and_select():
    """The default N = 1 run measures configs 1 (1 and 6 tracers), 3, 4's strong base and one rank
    of its 8-way split, and the two transfer-inclusive modes; N > 1 the strong leg only; --legs
    picks by name and refuses unknown names."""
    import argparse
    a = argparse.Namespace(strong_config="9.6M x 80", steps=20, warmup=5)
    one = dict(bench.extra_legs(a, 1))
    assert set(one) == {"config1_127kx47", "config1_127kx47_6tracers", "config3_1p2Mx80_6tracers",
                        "config4_strong_9p6Mx80", "config4_strong_rank3of8_9p6Mx80",
                        "config2_transfers_reference", "config2_transfers_producer_2tracers"}
    assert one["config4_strong_rank3of8_9p6Mx80"]["emulate"] == (3, 8)
    assert one["config2_transfers_producer_2tracers"]["tracers"] == 2
    assert [n for n, _ in bench.extra_legs(a, 8)] == ["config4_strong_9p6Mx80"]
    legs = bench.extra_legs(a, 1)
    assert bench.select_legs(legs, None) == legs
    assert [n for n, _ in bench.select_legs(legs, "config3_1p2Mx80_6tracers,config1_127kx47")] == \
        ["config1_127kx47", "config3_1p2Mx80_6tracers"]
    with pytest.raises(SystemExit):
        bench.select_legs(legs, "config9")


def test_compact_record_carries_transfers_and_the_emulated_rank():
    import argparse
    m = synth.make_mesh(16, 12, 9)
    rec = {"m": m, "s": bench.mesh_stats(m), "value": 1.0, "ms_per_step": 2.0, "roofline": None,
           "pass_roofline": {}, "kernels": {"fct_ale_p1v": {"avg_ms": 1.0}}, "check": {"exact": True},
           "setup_s": 0.1, "pass_order": 0, "transfers": {"h2d_GBps": 30.0}}
    a = argparse.Namespace(parity_levels=False, mesh="structured", scaling="strong", tracers=1, config="9.6M x 80",
                           steps=5, warmup=1, emulate=(3, 8))
    out = bench.compact(rec, a, 1)
    assert out["transfers"] == {"h2d_GBps": 30.0}
    assert out["emulated_rank"]["rank"] == 3 and out["emulated_rank"]["of"] == 8
    assert "single_passes" not in out
    # a batched leg: the same tracers timed as single-tracer passes ride along
    sp = {"ms_per_step": 2.2, "batch_gain": round(2.0 / 2.2 - 1, 4)}
    b = argparse.Namespace(**dict(vars(a), tracers=6, scaling="weak", config="127k x 47", emulate=None))
    out = bench.compact(dict(rec, single_passes=sp), b, 1)
    assert out["single_passes"] == sp and out["unit"] == "tracer-cell-updates/s"


def test_traffic_is_reported_only_for_the_library_it_measured(tmp_path):
    """profiles/traffic*.json carry the code-object hash of the library their PMC passes ran: a
    matching stamp yields the bytes, a mismatched (or missing) one no traffic and traffic_stale, and
    the emulated-rank leg matches only its own rank's file."""
    import argparse
    import json
    from fesom2_amd import _paths
    code = _paths.code_object_hash()
    assert len(code) == 16 and code == _paths.code_object_hash()  # deterministic per build
    doc = {"workload": "1.2M x 80", "tracers": 1, "bytes_per_launch": {"fct_ale_p1v": 123}, "code_object": code}
    path = tmp_path / "traffic.json"
    path.write_text(json.dumps(doc))
    a = argparse.Namespace(config="1.2M x 80", tracers=1, mesh="structured", parity_levels=False, vlimit=1,
                           fct_iter=1, transfers=None, scaling="weak", traffic=str(path))
    got, info = bench.find_traffic(a, 1, "fct_ale_p1v")
    assert got == 123 and info["traffic_code_object"] == code and "traffic_stale" not in info
    path.write_text(json.dumps(dict(doc, code_object="0" * 16)))
    got, info = bench.find_traffic(a, 1, "fct_ale_p1v")
    assert got is None and info["traffic_stale"] is True and info["code_object"] == code
    path.write_text(json.dumps({k: v for k, v in doc.items() if k != "code_object"}))
    assert bench.find_traffic(a, 1, "fct_ale_p1v")[0] is None  # unstamped: stale
    # another workload, tracer count or kernel: no match at all
    path.write_text(json.dumps(doc))
    six = bench.find_traffic(argparse.Namespace(**dict(vars(a), tracers=6)), 1, "fct_ale_p1v")
    assert six[0] is None or six[1]["traffic_source"] != str(path)  # (the repo's own 6-tracer file may match)
    assert bench.find_traffic(a, 1, "fct_ale_p2h")[1].get("traffic_source") != str(path)
    # the emulated rank: only a file stamped with its rank/world
    e = argparse.Namespace(**dict(vars(a), config="9.6M x 80", scaling="strong", emulate=(3, 8)))
    path.write_text(json.dumps(dict(doc, workload="9.6M x 80")))
    mine = os.path.relpath(str(path), bench.ROOT)
    assert bench.find_traffic(e, 1, "fct_ale_p1v")[1].get("traffic_source") != mine  # (the repo's own rank file may)
    path.write_text(json.dumps(dict(doc, workload="9.6M x 80", emulate="3/8")))
    assert bench.find_traffic(e, 1, "fct_ale_p1v")[0] == 123
    assert bench.traffic_paths(e)[-1].endswith("traffic_9p6Mx80_rank3of8.json")


def test_committed_traffic_files_match_the_built_library():
    """Every profiles/traffic*.json is stamped with the code object of the library built from this
    tree: a kernel change without a new PMC pass (tools/profile.sh, TRAFFIC_OUT) fails here instead
    of leaving the round-end bench line with traffic_stale."""
    import glob
    import json
    from fesom2_amd import _paths
    try:
        code = _paths.code_object_hash()
    except (OSError, ValueError):
        pytest.skip("engine library not built")
    files = sorted(glob.glob(os.path.join(bench.ROOT, "profiles", "traffic*.json")))
    assert files
    stale = [os.path.basename(p) for p in files if json.load(open(p)).get("code_object") != code]
    assert not stale, f"stamped with another build than {code}: {stale}"
