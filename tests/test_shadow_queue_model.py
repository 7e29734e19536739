"""Host model of the bundle kernel's shadow-queue bookkeeping (rt_kernel.hip shadow_queue_step /
shadow_chunk, built with RT_SHADOW_QUEUE=1; measured and off by default,
profiles/ab/r03_shadow_queue_rejected.txt).  The wave's 64 lanes are restated lane by lane: ballot,
mbcnt ranks, the ds_permute push to lane dst / 4, the first/second selects and the chunk loop.  The
properties the kernel relies on: the 64 destinations form a permutation, every queued record is
resolved exactly once, in arrival order, in chunks of at most 64 held by lanes 0..n-1, and its result
reaches its owner lane's word at bit 4 * level (reference loops it regroups: RayTracer.cs:573-582,
:851-870)."""
import random

import pytest

LANES = 64


def mbcnt(mask, lane):
    return bin(mask & ((1 << lane) - 1)).count("1")


class Wave:
    def __init__(self):
        self.q_item = [None] * LANES  # lane j: queued item j (hp stand-in: an item id), tag
        self.q_tag = [0] * LANES
        self.len = 0
        self.res = [0] * LANES  # the LDS words
        self.chunks = []

    def chunk(self, n, blocked):
        assert 1 <= n <= LANES
        items = self.q_item[:n]
        assert None not in items and len(set(items)) == n
        self.chunks.append(items)
        for lane in range(n):
            tag = self.q_tag[lane]
            owner, level = tag & 63, tag >> 6
            b = blocked[items[lane]]
            assert self.res[owner] >> (4 * level) & 0xF == 0  # each (owner, level) resolved once
            self.res[owner] |= b << (4 * level)

    def step(self, add, item_of, level, flush, blocked):
        m = sum(1 << i for i in range(LANES) if add[i])
        cnt = bin(m).count("1")
        r = [None] * LANES
        rt = [0] * LANES
        second = [False] * LANES
        if cnt > 0:
            dst = []
            for lane in range(LANES):
                rank = mbcnt(m, lane) if add[lane] else cnt + mbcnt(~m & ((1 << LANES) - 1), lane)
                dst.append(((self.len + rank) & 63) << 2)
            assert sorted(d >> 2 for d in dst) == list(range(LANES))  # a permutation: no lane written twice
            for lane in range(LANES):  # ds_permute: lane's value lands in lane dst / 4
                r[dst[lane] >> 2] = item_of[lane] if add[lane] else ("junk", lane)
                rt[dst[lane] >> 2] = lane | (level[lane] << 6)
            for lane in range(LANES):
                got = ((lane - self.len) & 63) < cnt
                first = got and lane >= self.len
                second[lane] = got and lane < self.len
                if first:
                    self.q_item[lane], self.q_tag[lane] = r[lane], rt[lane]
        total = self.len + cnt
        wrapped = total > 64
        n = 64 if total >= 64 else (total if flush else 0)
        while n > 0:
            self.chunk(n, blocked)
            total -= n
            n = 0
            if wrapped:
                for lane in range(LANES):
                    if second[lane]:
                        self.q_item[lane], self.q_tag[lane] = r[lane], rt[lane]
                wrapped = False
                n = total if flush else 0
        assert 0 <= total < 64
        self.len = total


@pytest.mark.parametrize("seed", range(40))
def test_queue_resolves_every_record_once_in_order(seed):
    rng = random.Random(seed)
    w = Wave()
    depth = [0] * LANES  # records pushed per lane (the level of the next one)
    alive = [True] * LANES
    order, blocked = [], {}
    p_add = rng.choice([0.05, 0.3, 0.7, 1.0])
    for step in range(rng.randint(1, 9)):
        last = step == 8 or rng.random() < 0.15
        add = [alive[i] and depth[i] < 8 and rng.random() < p_add for i in range(LANES)]
        item_of, level = [None] * LANES, [0] * LANES
        for i in range(LANES):
            level[i] = depth[i]
            if add[i]:
                item_of[i] = (i, depth[i])
                order.append(item_of[i])
                blocked[item_of[i]] = rng.randrange(16)
                depth[i] += 1
            if rng.random() < 0.2:
                alive[i] = False
        w.step(add, item_of, level, last, blocked)
        if last:
            break
    else:
        w.step([False] * LANES, [None] * LANES, [0] * LANES, True, blocked)
    assert w.len == 0
    flat = [it for c in w.chunks for it in c]
    assert flat == order  # every record once, in arrival order
    assert all(len(c) == 64 for c in w.chunks[:-1])
    for (lane, lvl), b in blocked.items():
        assert (w.res[lane] >> (4 * lvl)) & 0xF == b


def test_queue_exact_multiples_and_empty_wave():
    w = Wave()
    blocked = {(i, 0): 5 for i in range(LANES)}
    w.step([True] * LANES, [(i, 0) for i in range(LANES)], [0] * LANES, False, blocked)
    assert len(w.chunks) == 1 and w.len == 0  # exactly 64: resolved at once, nothing left
    w.step([False] * LANES, [None] * LANES, [0] * LANES, True, blocked)
    assert len(w.chunks) == 1  # flushing an empty queue runs no chunk
    e = Wave()
    e.step([False] * LANES, [None] * LANES, [0] * LANES, True, {})
    assert e.chunks == [] and e.res == [0] * LANES
