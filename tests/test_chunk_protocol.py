"""The pre-allocated chunk protocol of k_chunk_codes_pipe (csrc/phj_partition.h),
restated in Python and run under random interleavings of many workgroups
(CPU; the kernel's own GPU tests are the parity suites, which all run it).

What is checked, for every interleaving: no workgroup waits forever (a run's
wait always points at a strictly earlier claim of its chain), every chunk of a
chain has ONE id that all runs writing to it agree on, no two chunks share an
id, ids stay inside the shard's pool, and every claimed slot is written exactly
once. The layout: chunks 0 and 1 of chain d are static (2d, 2d + 1); the run
holding chunk j's first slot ("starter" of j) takes chunk j + 1's id (from the
tile's kPipeRes reserved chunks, then the pool counter) and publishes it in the
chain's table and hint {j, id_j, id_j+1}; a run is resolved one iteration after
its claim (publishes first, then waits for ids it could not read from the hint
it loaded with its claim). Reference: the scatter this replaces,
src/RadixCluster/HashJoin.hpp:394-412.
"""
import random

import pytest

RES = 3   # kPipeRes


class Shard:
    def __init__(self, nb, T, per):
        self.nb, self.T, self.per = nb, T, per
        self.cursor = [0] * nb
        self.hint = [None] * nb          # (j, id_j, id_j1) or None (= (0, static0, static1))
        self.tab = [dict() for _ in range(nb)]
        self.pool = 0
        self.dyn_base = 2 * nb + RES * per
        self.stride = 2 * nb + RES * per + per + nb + 1
        self.writes = [dict() for _ in range(nb)]   # slot -> (chunk id, offset)
        self.chunk_ids = [dict() for _ in range(nb)]  # chunk index -> id (every run's view must agree)


class WG:
    def __init__(self, shard, tiles):
        self.s, self.tiles = shard, tiles   # tiles: list of (tile index, [count per digit])
        self.i = 0
        self.pending = None                 # (tile index, [(v0, c, hint)])
        self.phase = 0                      # 0: claim next tile, 1: resolve the pending one
        self.res_used = {}
        self.late_hints = False

    def done(self):
        return self.i >= len(self.tiles) and self.pending is None

    def step(self):
        """One action; False when blocked."""
        S = self.s
        if self.phase == 0:
            if self.i < len(self.tiles):
                t, counts = self.tiles[self.i]
                claims = []
                for d, c in enumerate(counts):
                    v0 = S.cursor[d]
                    S.cursor[d] += c
                    claims.append([v0, c, S.hint[d]])
                    if self.late_hints:   # the hint load lands after other workgroups' updates
                        claims[-1][2] = "late"
                self.i += 1
                self.new = (t, claims)
            else:
                self.new = None
            self.phase = 1
            return True
        # resolve the pending tile (if any), then the new one becomes pending
        if self.pending is not None:
            if not self.resolve(*self.pending):
                return False
        self.pending = self.new
        self.phase = 0
        return True

    def resolve(self, t, claims):
        S, T = self.s, self.s.T
        if not hasattr(self, "st"):   # phase 1, done once per tile (publishes, no waits)
            self.st = {}
            for d, (v0, c, _h) in enumerate(claims):
                if c == 0:
                    continue
                off, k0, k1 = v0 % T, v0 // T, (v0 + c - 1) // T
                s = k0 if off == 0 else (k1 if k1 != k0 else None)
                if s is None:
                    continue
                if s == 0:
                    S.tab[d][0] = 2 * d
                    S.tab[d][1] = 2 * d + 1
                    self.st[d] = (0, 2 * d + 1)
                else:
                    r = self.res_used.get(t, 0)
                    self.res_used[t] = r + 1
                    nid = 2 * S.nb + RES * t + r if r < RES else S.dyn_base + S.pool
                    if r >= RES:
                        S.pool += 1
                    S.tab[d][s + 1] = nid
                    self.st[d] = (s, nid)
        # phase 2: resolve (may block); a late hint is read now (any value the
        # chain's hint held between the claim and the resolution)
        for d, cl in enumerate(claims):
            if cl[2] == "late":
                cl[2] = S.hint[d]
        ids = {}
        for d, (v0, c, h) in enumerate(claims):
            if c == 0:
                continue
            k0, k1 = v0 // T, (v0 + c - 1) // T
            hk, hid, hid1 = h if h is not None else (0, 2 * d, 2 * d + 1)

            def id_of(k):
                if k == 0:
                    return 2 * d
                if k == 1:
                    return 2 * d + 1
                if k == hk:
                    return hid
                if k == hk + 1:
                    return hid1
                return S.tab[d].get(k)
            i0, i1 = id_of(k0), id_of(k1)
            if i0 is None or i1 is None:
                return False   # spin: retried later
            ids[d] = (i0, i1)
        for d, (v0, c, h) in enumerate(claims):
            if c == 0:
                continue
            i0, i1 = ids[d]
            k0, k1 = v0 // T, (v0 + c - 1) // T
            if d in self.st and self.st[d][0] != 0:
                s, nid = self.st[d]
                ent = (s, i0 if s == k0 else i1, nid)
                if S.hint[d] is None or ent[0] > S.hint[d][0]:
                    S.hint[d] = ent   # atomicMax on the packed word
            for k, i in ((k0, i0), (k1, i1)):
                assert S.chunk_ids[d].setdefault(k, i) == i, ("two ids for one chunk", d, k)
                assert 0 <= i < S.stride
            for pos in range(v0, v0 + c):
                k = pos // T
                assert pos not in S.writes[d]
                S.writes[d][pos] = (i0 if k == k0 else i1, pos % T)
        del self.st
        return True


def run(seed, nb=6, T=16, W=5, ntiles=60, skew=False, late=False):
    rng = random.Random(seed)
    per = ntiles
    S = Shard(nb, T, per)
    tiles = []
    for t in range(ntiles):
        n = rng.randint(1, T)
        if skew:
            counts = [0] * nb
            counts[0] = n
        else:
            counts = [0] * nb
            for _ in range(n):
                counts[rng.randrange(nb)] += 1
        tiles.append((t, counts))
    wgs = [WG(S, tiles[w::W]) for w in range(W)]
    for g in wgs:
        g.late_hints = late and rng.random() < 0.5
    stuck = 0
    while not all(g.done() for g in wgs):
        live = [g for g in wgs if not g.done()]
        g = rng.choice(live)
        if g.step():
            stuck = 0
        else:
            stuck += 1
            assert stuck < 10_000, "deadlock: every live workgroup waits"
    # every claimed slot written once; chunk ids unique across the chains
    seen = {}
    for d in range(nb):
        assert sorted(S.writes[d]) == list(range(S.cursor[d]))
        for k, i in S.chunk_ids[d].items():
            assert seen.setdefault(i, (d, k)) == (d, k), "one id for two chunks"
    return S


@pytest.mark.parametrize("seed", range(40))
def test_protocol_random(seed):
    run(seed)


@pytest.mark.parametrize("seed", range(20))
def test_protocol_late_hints(seed):
    run(seed, late=True)
    run(seed, skew=True, late=True, W=7, ntiles=80)


@pytest.mark.parametrize("seed", range(20))
def test_protocol_skewed(seed):
    # every tile's codes in one digit: each claim spans a whole chunk
    run(seed, skew=True, W=7, ntiles=80)


@pytest.mark.parametrize("seed", range(10))
def test_protocol_many_workgroups(seed):
    run(seed, nb=3, T=8, W=16, ntiles=200)
