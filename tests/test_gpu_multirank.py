"""GPU: the N > 1 bench path with several ranks on this one GPU.

RCCL refuses two ranks on one device, so the ranks here exchange fct_plus/fct_minus through host
memory and gloo (``--exchange host``: the Fortran's exchange_nod round trip); everything else is the
driver's multi-GPU command -- ``torch.distributed.run`` with one process per rank, the weak-scaling
headline on y-strips of the global mesh, the barrier and max-over-ranks timing, one JSON line from
rank 0 -- and every rank checks its owned cells with the oracle.  127k x 47 per rank: the union plans
of FESOM2's per-GPU depth class, whose unions hold halo columns; with 3 ranks the middle strip has two
neighbours.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(420)
@pytest.mark.parametrize("nranks", [2, 3])
def test_weak_headline_with_a_host_exchange(nranks):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(nranks), "--exchange", "host", "--config", "127k x 47", "--extras", "none",
           "--steps", "5", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines, f"no record (rc {r.returncode}):\n{r.stderr[-3000:]}"
    rec = json.loads(lines[-1])
    assert r.returncode == 0, f"rc {r.returncode}: {rec.get('check')}\n{r.stderr[-3000:]}"
    assert rec["n_gpus"] == nranks and rec["scaling"] == "weak"
    c = rec["check"]
    assert c["exact"] and c["max_abs"] == 0.0 and c["ranks"] == nranks, c
    ranks = rec["ranks"]
    assert len(ranks["ms_per_step"]) == nranks and rec["ms_per_step"] >= max(ranks["ms_per_step"]) * 0.999
