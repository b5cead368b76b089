"""bench.py's N>1 path (independent shards, no data-path
collective) on CPU: two ranks under torch.distributed.run with gloo and a fake
verifier (tests/dist_bench_worker.py).  Checks that only rank 0 prints, that the
timing is the max over ranks, and that value aggregates all ranks' items."""
import json
import os
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_bench_aggregation():
    n, steps = 4096, 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "tests", "dist_bench_worker.py"),
           "--gpus", "2", "--steps", str(steps), "--warmup", "1", "--items", str(n),
           "--no-cpu-baseline", "--no-latency", "--no-extras"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout                     # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == steps and out["scaling"] == "weak"
    assert out["config"]["global_batch"] == 2 * n
    # rank 1 sleeps 20 ms per step: the reported step time is the slower rank's
    assert out["ms_per_step"] >= 20.0
    assert abs(out["value"] - 2 * n / (out["ms_per_step"] * 1e-3)) / out["value"] < 0.01
    par = out["parity"]
    assert par["checked"] == 2 * n and par["mismatches"] == 0
    assert par["adversarial_checked"] == 2 * n and par["adversarial_mismatches"] == 0
    assert 0.2 * 2 * n < par["adversarial_rejects_expected"] < 0.5 * 2 * n
    assert set(out["roofline"]["kernels"]) == {"k_scalar_inv", "k_prep", "k_ecmult"}
