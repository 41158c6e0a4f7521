"""A model of the tile kernel's group grabs (kernels.hip UnitGrab, round 5), run under random
interleavings on the CPU: workgroups of waves take ordinals from their LDS counter, read the
published slot of their group, and the taker of a group's first unit issues the next global
grab (an atomic whose value arrives later, in arrival order), waits for it and publishes it
before it runs its unit.  Checked: every dynamic unit is run exactly once, no wave waits forever (every schedule
drains), and each workgroup's global grabs increase.  The model follows UnitGrab.next /
publish statement by statement; it needs no device.

Round 6: groups hold at least 16 units (tile_units clamps gshift to 4), and a wave
that finds a LATER tag in its slot -- it lagged a whole ring of 16 groups -- takes the fail-safe
stop at once (its group index is lost) instead of spinning ~1 s.  A parked wave models that lag:
the schedule still drains, no unit runs twice, and a lost unit is always reported as a fault."""
import random

import pytest

SLOTS = 16  # kGrabSlots


class Sim:
    def __init__(self, rnd, n_wg, waves, n_units, gshift, park=0):
        self.rnd = rnd
        self.park = park      # steps the first wave to take an ordinal stays parked after it
        self.parked = None
        self.fault = False
        self.K = 1 << gshift
        self.gshift = gshift
        self.n_units = n_units
        self.n_groups = (n_units + self.K - 1) >> gshift
        self.ctr = 0
        self.pending = []  # outstanding atomics: [wave, value or None]
        self.ran = []
        self.wgs = []
        for w in range(n_wg):
            # thread 0's grab for slot 0, waited for before the barrier
            g0 = self.ctr
            self.ctr += 1
            wg = {'ord': 0, 'slot': {i: (None, None) for i in range(SLOTS)}, 'grabs': [g0]}
            wg['slot'][0] = (0, g0)
            self.wgs.append(wg)
        self.waves = [{'wg': w, 'pub_k': None, 'issued': False, 'atom': None, 'state': 'need',
                       'work': 0, 'k': None, 'sub': None}
                      for w in range(n_wg) for _ in range(waves)]

    def issue(self, wv):
        a = [wv, None]
        self.pending.append(a)
        wv['atom'] = a

    def arrive(self):
        a = self.rnd.choice(self.pending)
        self.pending.remove(a)
        a[1] = self.ctr
        self.ctr += 1

    def publish(self, wv):
        """Returns False while the wave waits for its atomic (vmcnt)."""
        if wv['pub_k'] is None:
            return True
        if wv['issued']:
            if wv['atom'][1] is None:
                return False
            g = wv['atom'][1]
        else:
            g = 1 << 32  # past the end
        wg = self.wgs[wv['wg']]
        k = wv['pub_k']
        wg['slot'][k % SLOTS] = (k, g)
        if g < (1 << 32):
            wg['grabs'].append(g)
        wv['pub_k'] = None
        return True

    def step(self, wv):
        """Advance one wave by one action; False when it is blocked."""
        st = wv['state']
        if st == 'work':
            wv['work'] -= 1
            if wv['work'] <= 0:
                wv['state'] = 'need'
            return True
        if st == 'need':  # next(): publish, then take an ordinal
            if not self.publish(wv):
                return False
            wg = self.wgs[wv['wg']]
            o = wg['ord']
            wg['ord'] += 1
            wv['k'], wv['sub'] = o >> self.gshift, o & (self.K - 1)
            wv['state'] = 'spin'
            if self.park and self.parked is None and wv['sub'] != 0:
                self.parked = [wv, self.park]
            return True
        if st == 'spin':
            if self.parked is not None and self.parked[0] is wv and self.parked[1] > 0:
                self.parked[1] -= 1  # parked: its time passes (not a deadlock)
                return True
            wg = self.wgs[wv['wg']]
            tag, g = wg['slot'][wv['k'] % SLOTS]
            if tag != wv['k']:
                if tag is None or tag < wv['k']:
                    return False  # not published yet: wait
                # a later group in the slot: the fail-safe stop (the flag; no group index)
                self.fault = True
                g = 1 << 32
            live = g < self.n_groups
            if wv['sub'] == 0:  # grab slot k + 1 now, wait for it, publish it at once
                wv['pub_k'] = wv['k'] + 1
                wv['issued'] = live
                if live:
                    self.issue(wv)
                wv['state'] = 'publish'
                wv['u'] = (g << self.gshift) + wv['sub'] if live else self.n_units
                return True
            u = (g << self.gshift) + wv['sub'] if live else self.n_units
            if u >= self.n_units:
                wv['state'] = 'exit'
                return True
            self.ran.append(u)
            wv['state'] = 'work'
            wv['work'] = self.rnd.randint(1, 6)
            return True
        if st == 'publish':  # waits for its atomic (vmcnt), publishes, then runs its unit
            if not self.publish(wv):
                return False
            if wv['u'] >= self.n_units:
                wv['state'] = 'done'
                return True
            self.ran.append(wv['u'])
            wv['state'] = 'work'
            wv['work'] = self.rnd.randint(1, 6)
            return True
        if st == 'exit':  # publish at once, then the wave is done
            if not self.publish(wv):
                return False
            wv['state'] = 'done'
            return True
        return False

    def run(self):
        for _ in range(10_000_000):
            if self.parked is not None and self.parked[1] > 0 and self.rnd.random() < 0.5:
                self.parked[1] -= 1  # the parked wave's time passes while others run
            live = [w for w in self.waves if w['state'] != 'done']
            if not live and not self.pending:
                return
            moved = False
            if self.pending and self.rnd.random() < 0.3:
                self.arrive()
                moved = True
            order = self.rnd.sample(live, len(live))
            for w in order[:self.rnd.randint(1, max(1, len(order)))]:
                moved |= self.step(w)
                break
            if not moved:
                if self.pending:
                    self.arrive()
                elif not any(self.step(w) for w in live):
                    raise AssertionError('deadlock: every wave waits, no atomic in flight')
        raise AssertionError('did not drain')


@pytest.mark.parametrize("seed", range(200))
def test_group_grabs_run_every_unit_once(seed):
    rnd = random.Random(seed)
    n_wg = rnd.choice([1, 2, 3, 7])
    waves = rnd.choice([1, 2, 4, 16])
    gshift = rnd.choice([4, 5, 6])  # tile_units: at least 2^kGrabMinShift units per group
    n_units = rnd.choice([0, 1, 5, 31, 32, 33, 97, 300, 2000])
    sim = Sim(rnd, n_wg, waves, n_units, gshift)
    sim.run()
    assert not sim.fault
    assert sorted(sim.ran) == list(range(n_units))
    for wg in sim.wgs:
        assert wg['grabs'] == sorted(wg['grabs']), 'a workgroup\'s grabs must increase'


@pytest.mark.parametrize("seed", range(60))
def test_parked_wave_faults_instead_of_hanging(seed):
    """One wave parks right after taking its ordinal while 15 others of its workgroup run on:
    short parks change nothing; a park long enough for the ring to come round (16 groups of
    16+ units) ends in the fail-safe stop at once -- never a hang, never a unit run twice, and a
    unit is missing only when the fault was reported."""
    rnd = random.Random(1000 + seed)
    gshift = 4
    park = rnd.choice([5, 50, 20_000, 200_000])
    sim = Sim(rnd, 1, 16, 3000, gshift, park=park)
    sim.run()
    assert len(sim.ran) == len(set(sim.ran)), 'a unit ran twice'
    if not sim.fault:
        assert sorted(sim.ran) == list(range(3000))
    else:
        assert len(sim.ran) < 3000
