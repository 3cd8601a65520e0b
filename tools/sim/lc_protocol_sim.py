"""Randomised interleaving check of the loader/consumer hand-off protocol of bf_wide_i8lc.hip (CPU model).

Agents are generators that yield a predicate to wait on (or None to just take a step); the scheduler advances a
random runnable agent each tick and reports a deadlock if none can run.  Counters mirror the kernel: full[3],
free[3] (ring slots), tready[2], tfree[2] (table buffers).  Run: python tools/sim/lc_protocol_sim.py"""
import random
import sys

RING, LOADERS = 3, 4


def simulate(count, S, NQ, nact, E=None, upt=None, seed=0, max_ticks=10_000_000):
    rng = random.Random(seed)
    per_item = NQ * S
    nsteps = count * per_item
    E = E or 2 * S
    upt = upt or -(-E // per_item)
    c = dict(full=[0] * RING, free=[0] * RING, tready=[0, 0], tfree=[0, 0])

    def consumer():
        yield lambda: c["full"][0] >= LOADERS
        t = 0
        for k in range(count):
            yield lambda k=k: c["tready"][k & 1] >= LOADERS * ((k >> 1) + 1)
            for _ in range(per_item):
                if t > 0:
                    c["free"][(t - 1) % RING] += 1
                tn = t + 1 if t + 1 < nsteps else t
                yield lambda tn=tn: c["full"][tn % RING] >= LOADERS * (tn // RING + 1)
                yield None  # MFMAs
                t += 1
            c["tfree"][k & 1] += 1

    def loader():
        T = dict(k=0, e=0, done=False)

        def tstart(k):
            T.update(k=k, e=0, done=k >= count)

        def try_table():
            if T["done"]:
                return False
            buf = T["k"] & 1
            if T["e"] == 0 and not c["tfree"][buf] >= nact * (T["k"] >> 1):
                return False
            T["e"] += 1
            if T["e"] == E:
                c["tready"][buf] += 1
                T["done"] = True
            return True

        tstart(0)
        while not T["done"]:
            try_table()
            yield None
        tstart(1)
        for t in range(nsteps):
            slot = t % RING
            budget = upt
            while True:
                if T["done"] and T["k"] + 1 < count:
                    tstart(T["k"] + 1)
                did = try_table()
                yield None
                if did:
                    budget -= 1
                    if budget > 0:
                        continue
                if c["free"][slot] >= nact * (t // RING):
                    break
            c["full"][slot] += 1
            yield None
        while True:
            if T["done"]:
                if T["k"] + 1 >= count:
                    break
                tstart(T["k"] + 1)
            try_table()
            yield None

    agents = [consumer() for _ in range(nact)] + [loader() for _ in range(LOADERS)]
    waits = [None] * len(agents)
    alive = set(range(len(agents)))
    for tick in range(max_ticks):
        if not alive:
            return tick
        runnable = [i for i in alive if waits[i] is None or waits[i]()]
        if not runnable:
            return f"DEADLOCK at tick {tick}: counters {c}"
        i = rng.choice(runnable)
        try:
            waits[i] = next(agents[i])
        except StopIteration:
            alive.discard(i)
    return "TIMEOUT"


if __name__ == "__main__":
    bad = 0
    for count, S, NQ, nact in [(16, 8, 4, 4), (5, 8, 4, 4), (3, 1, 1, 1), (7, 2, 1, 2), (9, 3, 2, 3), (1, 8, 4, 4),
                               (2, 1, 1, 4), (6, 4, 1, 4)]:
        for seed in range(20):
            r = simulate(count, S, NQ, nact, seed=seed)
            if not isinstance(r, int):
                print(count, S, NQ, nact, seed, r)
                bad += 1
    print("protocol simulation:", "OK" if not bad else f"{bad} failures")
    sys.exit(1 if bad else 0)
