"""Host model of the work queue of wave-tiles the coding, fused, decode +
verify and checksum kernels take their tiles from.

Device code modelled:
  * gf_matmul_v16's batched form (hdfs-native_amd/csrc/ec_kernels.hip,
    next_tile): min(grid, 8) launch counters, block b on counter b % n, WQ
    rounds of tiles per atomic (tile = round * n + counter), each wave
    fetching its next batch while it codes the current one;
  * WaveQueue (csrc/work_queue.hpp init / peek / next), one round per
    atomic, as the fused encode + CRC and decode + verify kernels use it
    (peek() at the end of a tile to prefetch the next tile's inputs) and as
    the checksum kernel uses it (units of consecutive tasks);
  * the counter sets of a stream (ec_kernels.hip queue_lease): two sets per
    stream, launch i counts on set i % 2 and zeroes the other one for launch
    i + 1 (queue_zero_next); nothing in a kernel resets its own counters.

Waves are interleaved at random at every fetch-latency point.  Checked:
every tile is coded exactly once in every launch, and a launch is correct
whatever state an earlier launch left its counters in (junk written into a
finished launch's set, waves that quit early).

test_round5_self_reset_signature replays the round-5 protocol (the wave that
reads a counter's computed last value stores zero) with the blocks-per-
counter term credited to every counter as ceil(grid / n): it reproduces the
r05u / r05v failure exactly (RS(2,1), 8208-B cells, 3 stripes: the encode
correct, then the decode on the same stream writing only tiles 0 and 8).
"""
import random

import pytest

QUEUES = 8


def interleave(gens, rnd):
    live = list(range(len(gens)))
    while live:
        i = rnd.choice(live)
        try:
            next(gens[i])
        except StopIteration:
            live.remove(i)


# ---- the kernels' fetch loops, current protocol (no self-reset) -----------

def batched_waves(ctr, total, grid, wq, waves_per_block, coded, quit_after=None):
    """gf_matmul_v16 next_tile over counter list `ctr` (modified in place)."""
    n = min(grid, QUEUES)
    gens = []
    for b in range(grid):
        for w in range(waves_per_block):
            gens.append(_batched_wave(ctr, b % n, n, total, wq, coded,
                                      quit_after if (b, w) == (0, 0) else None))
    return gens


def _batched_wave(ctr, q, n, total, wq, coded, quit_after):
    pending = [ctr[q]]
    ctr[q] += 1
    left = rnd_round = 0
    done = 0
    while True:
        # next_tile
        while True:
            if left == 0:
                yield  # the fetch is in flight
                v = pending.pop(0)
                rnd_round, left = v * wq, wq
                if rnd_round * n + q >= total:
                    return
                pending.append(ctr[q])
                ctr[q] += 1
            else:
                rnd_round += 1
            left -= 1
            t = rnd_round * n + q
            if t < total:
                break
            left = 0
        coded.append(t)
        done += 1
        if quit_after is not None and done >= quit_after:
            return  # a wave that leaves early (a fault model): its fetched batch is lost
        yield


class WaveQueue:
    """csrc/work_queue.hpp WaveQueue."""

    def __init__(self, ctr, total, grid, block):
        self.ctr, self.total = ctr, total
        self.n = min(grid, QUEUES)
        self.q = block % self.n
        self.peeked = False
        self.pend = self._fetch()

    def _fetch(self):
        v = self.ctr[self.q]
        self.ctr[self.q] += 1
        return v

    def tile_of(self, v):
        t = v * self.n + self.q
        return t if t < self.total else self.total

    def peek(self):
        if not self.peeked:
            self.peek_v, self.peeked = self.pend, True
        return self.tile_of(self.peek_v)

    def next(self):
        v = self.peek_v if self.peeked else self.pend
        self.peeked = False
        t = self.tile_of(v)
        if t < self.total:
            self.pend = self._fetch()
        return t


def fused_wave(ctr, total, grid, block, coded):
    """gf_fused_crc<..., WQ = true>: for (tile = next(); tile < total; tile =
    next()), peeking the next tile before the tile's outputs."""
    wq = WaveQueue(ctr, total, grid, block)
    yield
    tile = wq.next()
    while tile < total:
        yield
        nt = wq.peek()  # the next tile's inputs are loaded from here
        assert nt == total or nt != tile
        coded.append(tile)
        yield
        tile = wq.next()


def checksum_wave(ctr, tasks, unit, grid, block, coded):
    """checksum_chunks512<..., WQ = unit>: units of `unit` consecutive tasks."""
    units = (tasks + unit - 1) // unit
    wq = WaveQueue(ctr, units, grid, block)

    def task_of(u):
        return u * unit if u < units else tasks

    yield
    task = task_of(wq.next())
    while task < tasks:
        unit_end = task % unit == unit - 1 or task + 1 >= tasks
        nxt = task_of(wq.peek()) if unit_end else task + 1
        coded.append(task)
        yield
        task = task_of(wq.next()) if unit_end else nxt


class Stream:
    """ec_kernels.hip queue_lease: two counter sets, both zero when the stream
    is first seen; launch i counts on cur and zeroes cur ^ 1."""

    def __init__(self):
        self.sets = [[0] * QUEUES, [0] * QUEUES]
        self.cur = 0

    def launch(self, make_gens, rnd):
        use, zero = self.sets[self.cur], self.sets[self.cur ^ 1]
        gens = make_gens(use)
        # block 0 zeroes the other set while the waves run (any order: it is
        # not this launch's set)
        zeroer = [self._zero(zero)]
        interleave(gens + zeroer, rnd)
        self.cur ^= 1
        return use

    @staticmethod
    def _zero(s):
        yield
        for i in range(QUEUES):
            s[i] = 0


# ---- tests: current protocol ----------------------------------------------

@pytest.mark.parametrize("wq", [1, 2, 4])
@pytest.mark.parametrize("waves_per_block", [1, 4, 8])
def test_batched_queue_every_tile_once(wq, waves_per_block):
    for total in [1, 2, 3, 7, 8, 9, 16, 17, 100, 257, 1031]:
        for grid in [1, 2, 3, 7, 8, 9, 33, 256]:
            for seed in range(2):
                g = min(grid, total)  # the launcher caps the grid at the tile count
                ctr, coded = [0] * QUEUES, []
                interleave(batched_waves(ctr, total, g, wq, waves_per_block, coded), random.Random(seed))
                assert sorted(coded) == list(range(total)), (total, g)


@pytest.mark.parametrize("waves_per_block", [4, 8])
def test_wave_queue_fused_every_tile_once(waves_per_block):
    for total in [1, 2, 3, 7, 8, 9, 16, 17, 100, 257, 1031]:
        for grid in [1, 3, 8, 9, 33, 512]:
            for seed in range(2):
                g = min(grid, total)
                ctr, coded = [0] * QUEUES, []
                gens = [fused_wave(ctr, total, g, b, coded) for b in range(g) for _ in range(waves_per_block)]
                interleave(gens, random.Random(seed))
                assert sorted(coded) == list(range(total)), (total, g)


@pytest.mark.parametrize("unit", [1, 2, 4, 16])
def test_wave_queue_checksum_every_task_once(unit):
    for tasks in [1, 2, 5, 16, 17, 100, 1000]:
        for grid in [1, 3, 8, 9, 64]:
            units = (tasks + unit - 1) // unit
            g = min(grid, units)
            ctr, coded = [0] * QUEUES, []
            gens = [checksum_wave(ctr, tasks, unit, g, b, coded) for b in range(g) for _ in range(4)]
            interleave(gens, random.Random(tasks * 131 + grid))
            assert sorted(coded) == list(range(tasks)), (tasks, g)


def test_stream_launches_independent_of_previous_state():
    """Back-to-back launches of every kernel form on one stream, random
    geometries; after some launches junk is written into the set they used
    (any miscount) and some launches lose a wave early: every launch whose
    waves all finish still codes every tile exactly once."""
    rnd = random.Random(1234)
    st = Stream()
    for i in range(400):
        kind = rnd.choice(["batched", "fused", "crc"])
        total = rnd.choice([1, 3, 9, 17, 64, 257, 1000])
        grid = min(rnd.choice([1, 5, 8, 9, 13, 256]), total)
        faulty = rnd.random() < 0.1
        coded = []
        if kind == "batched":
            wq = rnd.choice([1, 2])
            make = lambda use: batched_waves(use, total, grid, wq, 4, coded, 1 if faulty else None)  # noqa: E731
        elif kind == "fused":
            make = lambda use: [fused_wave(use, total, grid, b, coded) for b in range(grid) for _ in range(4)]  # noqa: E731
            faulty = False
        else:
            make = lambda use: [checksum_wave(use, total, 4, grid, b, coded) for b in range(grid) for _ in range(4)]  # noqa: E731
            faulty = False
        used = st.launch(make, rnd)
        if not faulty:
            assert sorted(coded) == list(range(total)), (i, kind, total, grid)
        if rnd.random() < 0.2:  # an earlier launch's counters left in any state
            for q in range(QUEUES):
                used[q] = rnd.randrange(1 << 20)


# ---- round 5: the self-resetting protocol and its failure ------------------

def round5_launch(ctr, total, grid, wq, waves_per_block, blocks_term, rnd):
    """The round-5 gf_matmul_v16: counters zero at rest; the wave that reads
    counter q's last value (rounds/wq + blocks(q) * waves - 1) stores zero.
    blocks_term(grid, n, q) is the blocks-per-counter formula."""
    n = min(grid, QUEUES)
    coded, resets = [], []
    gens = []
    for b in range(grid):
        q = b % n
        rounds = (total - 1 - q) // n + 1 if total > q else 0
        last = (rounds + wq - 1) // wq + blocks_term(grid, n, q) * waves_per_block - 1
        for _ in range(waves_per_block):
            gens.append(_round5_wave(ctr, q, n, total, wq, last, coded, resets))
    interleave(gens, rnd)
    return coded, resets


def _round5_wave(ctr, q, n, total, wq, last, coded, resets):
    pending = [ctr[q]]
    ctr[q] += 1
    left = r = 0
    while True:
        while True:
            if left == 0:
                yield
                v = pending.pop(0)
                r, left = v * wq, wq
                if r * n + q >= total:
                    if v == last:
                        resets.append(q)
                        ctr[q] = 0
                    return
                pending.append(ctr[q])
                ctr[q] += 1
            else:
                r += 1
            left -= 1
            t = r * n + q
            if t < total:
                break
            left = 0
        coded.append(t)
        yield


def exact_blocks(grid, n, q):  # the committed round-5 term: blocks b < grid with b % n == q
    return (grid - 1 - q) // n + 1


def ceil_blocks(grid, n, q):  # every counter credited with ceil(grid / n) blocks
    return (grid + n - 1) // n


def r05u_geometry():
    # test_bitsliced_encode_kernels[8208-2-1-0-1]: RS(2,1), 8208-B cells = 513
    # 16-B chunks, wave-tiles of 64 x 4 chunks -> 3 per stripe, 3 stripes;
    # grid = min(256 CUs, 9 tiles); k = 2 takes 2 rounds per atomic; 4 waves
    # per 256-thread block.  Tile-order group = 3 stripes (stripes < 4):
    # tile t -> stripe t % 3, column t // 3.
    return dict(total=9, grid=9, wq=2, waves_per_block=4)


def test_round5_self_reset_signature():
    g = r05u_geometry()
    # the committed formula: both launches correct, every counter back at zero
    ctr = [0] * QUEUES
    for seed in range(20):
        coded, _ = round5_launch(ctr, g["total"], g["grid"], g["wq"], g["waves_per_block"], exact_blocks,
                                 random.Random(seed))
        assert sorted(coded) == list(range(9))
        assert ctr == [0] * QUEUES
    # ceil(grid / n): counters 1..7 (one block each) wait for a last value
    # they never draw and keep their count; counter 0 (blocks 0 and 8) resets
    ctr = [0] * QUEUES
    enc, resets = round5_launch(ctr, g["total"], g["grid"], g["wq"], g["waves_per_block"], ceil_blocks,
                                random.Random(0))
    assert sorted(enc) == list(range(9))  # the encode: parity matched the oracle
    assert resets == [0] and ctr[0] == 0 and all(c > 0 for c in ctr[1:8])
    dec, _ = round5_launch(ctr, g["total"], g["grid"], g["wq"], g["waves_per_block"], ceil_blocks,
                           random.Random(1))
    assert sorted(dec) == [0, 8]
    # tiles 0 and 8 = stripe 0 column 0 and stripe 2 column 2: the r05u output
    # (stripe 0 right at its start, zero at its end; stripe 1 all zero;
    # stripe 2 zero at its start, right at its end)
    assert sorted((t % 3, t // 3) for t in dec) == [(0, 0), (2, 2)]
    # the same geometry through the current protocol: no state carried over
    st = Stream()
    for seed in range(3):
        coded = []
        st.launch(lambda use: batched_waves(use, 9, 9, 2, 4, coded), random.Random(seed))
        assert sorted(coded) == list(range(9))
