"""Worker for tests/test_bench_dist.py: runs bench.main under torch.distributed.run
(gloo, CPU) with a fake verifier, so the multi-rank timing / max-over-ranks /
aggregation logic of bench.py is exercised without a GPU.  Not a test module."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


class FakeVerifier:
    """Device-memory and verify calls of gpuverify.Verifier, on host numpy arrays.
    A signature is 'valid' iff its pubkey prefix byte is 0x02 and bit 0 of its
    digest's last byte is clear (the workload keeps it clear); rank r sleeps
    (r+1)*10 ms per batch so max-over-ranks is observable."""

    def __init__(self, rank):
        self.rank = rank
        self.mem = {}
        self.next = 1

    def dev_alloc(self, nbytes, slot=0):
        p = self.next
        self.next += 1
        self.mem[p] = np.zeros(nbytes, np.uint8)
        return p

    def dev_free(self, p, slot=0):
        self.mem.pop(p)

    def dev_upload(self, p, arr, slot=0):
        self.mem[p][:arr.nbytes] = arr.reshape(-1).view(np.uint8)

    def dev_download(self, arr, p, slot=0):
        arr.reshape(-1).view(np.uint8)[:] = self.mem[p][:arr.nbytes]

    def dev_verify_digests(self, slot, n, d_pub, d_sig, d_dig, d_bits, stream=None):
        ok = ((self.mem[d_pub].reshape(-1, 33)[:n, 0] == 2) &
              ((self.mem[d_dig].reshape(-1, 32)[:n, 31] & 1) == 0)).astype(np.uint8)
        packed = np.packbits(ok, bitorder="little")
        self.mem[d_bits][:] = 0
        self.mem[d_bits][:packed.size] = packed
        time.sleep((self.rank + 1) * 0.01)

    def dev_sync(self, slot=0):
        pass

    def set_option(self, key, val):
        pass

    def stage_stats(self, slot=0):
        return 1, 0.1, 0.2, 0.3

    def stage_stats4(self, slot=0):
        return 1, [0.1, 0.05, 0.15, 0.3]

    def close(self):
        pass


def workload(n, seed, keys, adv, threads):
    rng = np.random.default_rng(seed)
    pub = rng.integers(0, 256, (n, 33), dtype=np.uint8)
    pub[:, 0] = np.where(rng.random(n) < 0.75, 2, 4)
    sig = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    dig = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    dig[:, 31] &= 0xFE
    exp = (pub[:, 0] == 2).astype(np.uint8)
    return pub, sig, dig, exp


if __name__ == "__main__":
    bench.main(sys.argv[1:], verifier_factory=FakeVerifier, workload_fn=workload)
