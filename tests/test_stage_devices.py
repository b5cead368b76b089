"""Host staging with several devices (csrc/gv_stage.h): the
runtime's own Pool / Worker / par_copy_segs / run_sliced, driven by the CPU
harness tests/stage/stage_harness.cpp with fake devices (a sleep stands in
for H2D + kernels).  A host batch's slices must all be in flight at once
(each slice waits at a barrier for the others), every device must stage
through its own pool (no thread shared between devices), every staged byte
must match the caller's, and the ThreadSanitizer build must be clean.  The
asynchronous host-batch queue (csrc/gv_async.h) runs over the same fake
devices (tests/stage/async_harness.cpp)."""
import json
import os
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stage")


@pytest.fixture(scope="module")
def harness():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return os.path.join(HERE, "stage_harness"), os.path.join(HERE, "stage_harness_tsan")


@pytest.mark.parametrize("nd,subs,per,tsan", [(4, 3, 12, False), (8, 4, 8, False), (4, 3, 6, True)])
def test_async_queue_over_fake_devices(harness, nd, subs, per, tsan):
    """gv_submit_* / gv_wait's queue (csrc/gv_async.h) over >= 4
    fake devices: the first batch's slices all in flight at once, ragged
    batches from several submitter threads waited out of order with every
    verdict byte right, tickets waited once, a quiescing key loader that never
    sees a pending batch or a running slice, a failing device failing only the
    batches it holds -- and, built with ThreadSanitizer, no data race."""
    exe = os.path.join(HERE, "async_harness_tsan" if tsan else "async_harness")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66") if tsan else None
    out = run(exe, nd, subs, per, 100 if tsan else 200, env=env)
    assert out["ok"] and out["concurrent"] and out["bad_bytes"] == 0, out
    assert out["waited"] == subs * per and out["quiesces"] > 0 and out["quiesce_violations"] == 0, out
    assert out["failed_device_rc"] != 0 and out["other_devices_rc"] == 0 and out["tickets_left"] == 0, out


def run(exe, *args, env=None):
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout)


@pytest.mark.parametrize("nd,tpd", [(2, 2), (4, 2), (8, 1)])
def test_slices_stage_concurrently_on_their_own_pools(harness, nd, tpd):
    out = run(harness[0], nd, 600_000, 65_536, tpd, 300)
    assert out["rc"] == 0 and out["concurrent"], out
    assert all(d["ok"] for d in out["devs"])
    seen = set()
    for d in out["devs"]:
        ts = set(d["threads"])
        assert 1 <= len(ts) <= tpd
        assert not (ts & seen), "a staging thread served two devices"
        seen |= ts
    # items split in contiguous 256-aligned slices: every device got work
    assert all(len(d["stage"]) >= 1 for d in out["devs"])


def test_staging_budget_per_device(harness):
    exe = harness[0]

    def threads(cpus, nd):
        r = subprocess.run([exe, "--threads", str(cpus), str(nd)], capture_output=True, text=True, check=True)
        return int(r.stdout)
    assert threads(16, 1) == 8          # one GPU on the 16-CPU box: the round-3 pool
    assert threads(16, 8) == 1          # eight GPUs on 16 CPUs: each slice stages on its own thread
    assert threads(256, 8) == 8         # a full node's CPUs: 8 per device
    assert threads(2, 4) == 1


def test_tsan_clean(harness):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    out = run(harness[1], 4, 200_000, 32_768, 2, 100, env=env)
    assert out["rc"] == 0 and out["concurrent"] and all(d["ok"] for d in out["devs"])
