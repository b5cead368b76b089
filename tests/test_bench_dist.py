"""bench.py's N>1 path (independent shards, no data-path
collective) on CPU: two ranks under torch.distributed.run with gloo and a fake
verifier (tests/dist_bench_worker.py).  Checks that only rank 0 prints, that the
timing is the max over ranks, and that value aggregates all ranks' items."""
import json
import os
import socket
import subprocess
import sys

import numpy as np

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


class _FakeMultiDevice:
    """gpuverify.Verifier's host-buffer calls over `nd` fake devices: the batch
    is cut into contiguous slices like gv_runtime's run_host."""

    def __init__(self, devs):
        self.nd = len(devs) if devs else 3
        self._slices = []

    @property
    def num_devices(self):
        return self.nd

    def verify_batch_digests_bits(self, pub, sig, dig):
        n = len(pub)
        ok = ((pub[:, 0] == 2) & ((dig[:, 31] & 1) == 0)).astype(np.uint8)
        per = -(-n // self.nd)
        self._slices = [(0.5, min(n, (k + 1) * per) - min(n, k * per)) for k in range(self.nd)]
        packed = np.packbits(ok, bitorder="little").tobytes().ljust(((n + 63) // 64) * 8, b"\0")
        return np.frombuffer(packed, np.uint64)

    def last_slices(self):
        return self._slices

    def close(self):
        pass


def test_inproc_mode_is_one_process_over_all_devices():
    """bench.py --inproc: one context over every device (the Go node's shape),
    host buffers in, per-device slice rates out; refuses a torchrun launch."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import bench
    import dist_bench_worker as W
    n = 2048
    res = bench.main(["--inproc", "--gpus", "0", "--items", str(n), "--steps", "2", "--warmup", "1"],
                     verifier_factory=_FakeMultiDevice, workload_fn=W.workload)
    assert res["mode"] == "inproc" and res["n_gpus"] == 3 and res["config"]["global_batch"] == 3 * n
    assert res["parity"]["mismatches"] == 0
    assert [d["items"] for d in res["per_device"]] == [n, n, n]
    assert all(d["verifies_per_s"] == n / 0.5e-3 for d in res["per_device"])
