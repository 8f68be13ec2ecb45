"""Host model of the work queue the register and mixed-decode kernels share
(hdfs-native_amd/csrc/ec_kernels.hip, gf_matmul_v16 next_tile /
gf_decode_mixed WQ loop): min(grid, 8) launch counters, block b on counter
b % n, WQ rounds of tiles (tile = round * n + counter) per atomic, each wave
fetching its next batch while it codes the current one, and the register
kernel's self-reset -- the wave that reads a counter's last value (its
in-range batches + its waves - 1) stores zero.  Waves are interleaved at
random at every fetch latency point.  Checked: every tile is coded exactly
once, every counter in use is reset exactly once and only after its last
fetch, and all counters end at zero (the stream's next launch starts clean).
"""
import random

import pytest

QUEUES = 8


def run(total, grid, wq, waves_per_block, seed):
    rnd = random.Random(seed)
    n = min(grid, QUEUES)
    ctr = [0] * QUEUES
    fetches = [0] * QUEUES
    coded, resets = [], []
    waves = []
    for b in range(grid):
        q = b % n
        rounds = (total - 1 - q) // n + 1 if total > q else 0
        blocks = (grid - 1 - q) // n + 1
        last = (rounds + wq - 1) // wq + blocks * waves_per_block - 1
        waves += [dict(q=q, last=last, left=0, round=0, pending=[]) for _ in range(waves_per_block)]

    def fetch(w):
        q = w["q"]
        w["pending"].append(ctr[q])
        ctr[q] += 1
        fetches[q] += 1

    def wave(w):  # the kernel's loop: for (tile = next_tile(); tile < total; tile = next_tile())
        q = w["q"]
        fetch(w)
        while True:
            while True:  # next_tile
                if w["left"] == 0:
                    yield  # the fetch is in flight
                    v = w["pending"].pop(0)
                    w["round"], w["left"] = v * wq, wq
                    if w["round"] * n + q >= total:
                        if v == w["last"]:
                            assert fetches[q] == w["last"] + 1, "reset before the counter's last fetch"
                            resets.append(q)
                            ctr[q] = 0
                        return
                    fetch(w)
                else:
                    w["round"] += 1
                w["left"] -= 1
                t = w["round"] * n + q
                if t < total:
                    break
                w["left"] = 0
            coded.append(t)
            yield

    gens = [wave(w) for w in waves]
    live = list(range(len(gens)))
    while live:
        i = rnd.choice(live)
        try:
            next(gens[i])
        except StopIteration:
            live.remove(i)
    assert sorted(coded) == list(range(total))
    assert sorted(resets) == sorted({w["q"] for w in waves})
    assert ctr == [0] * QUEUES


@pytest.mark.parametrize("wq", [1, 2, 4])
@pytest.mark.parametrize("waves_per_block", [1, 4, 8])
def test_work_queue_model(wq, waves_per_block):
    for total in [1, 2, 3, 7, 8, 9, 16, 17, 100, 257, 1031]:
        for grid in [1, 2, 3, 7, 8, 9, 33, 256]:
            for seed in range(2):
                # the launcher caps the grid at the tile count
                run(total, min(grid, total), wq, waves_per_block, seed)
