#!/usr/bin/env python3
"""Debug probe (tool, not product): fold small operand sets through the engine and print mismatches
against Python ints, to localise tree-path failures by modulus shape and operand size."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]
import ddshe  # noqa: E402


def main():
    eng = ddshe.Engine(0)
    rng = random.Random(5)
    mods = {"rand1024": rng.getrandbits(1024) | (1 << 1023) | 1, "rand1100": rng.getrandbits(1100) | (1 << 1099) | 1,
            "rand600": rng.getrandbits(600) | (1 << 599) | 1, "q4094": (1 << 4094) - 1, "rand4094": rng.getrandbits(4094) | (1 << 4093) | 1,
            "rand4095": rng.getrandbits(4095) | (1 << 4094) | 1, "rand2048": rng.getrandbits(2048) | (1 << 2047) | 1}
    for name, Q in mods.items():
        for desc, xs in (("small2", [rng.randrange(Q) for _ in range(2)]),
                         ("small3", [rng.randrange(Q) for _ in range(3)]),
                         ("2Q+5", [2 * Q + 5, 5, 7]),
                         ("big1", [rng.getrandbits(Q.bit_length() + 40), 3]),
                         ("big2", [rng.getrandbits(Q.bit_length() + 40), rng.getrandbits(Q.bit_length() + 40)]),
                         ("big3", [rng.getrandbits(Q.bit_length() + 40) for _ in range(3)]),
                         ("big9", [rng.getrandbits(Q.bit_length() + 40) for _ in range(9)]),
                         ("ones", [1, 1, 1]),
                         ("Q-1", [Q - 1, Q - 1, Q - 1])):
            want = 1
            for x in xs:
                want = want * x % Q
            try:
                got = eng.modmul_fold(Q, xs)
            except Exception as e:  # noqa: BLE001
                got = repr(e)
            print(name, desc, "OK" if got == want else "BAD", flush=True)
    # result-structure probes on the all-ones modulus and neighbours
    for name, Q in (("q4094", (1 << 4094) - 1), ("q4094m2", (1 << 4094) - 3), ("q4000", (1 << 4000) - 1),
                    ("q2000", (1 << 2000) - 1), ("r4094", mods["rand4094"])):
        a = rng.randrange(2, Q) | 1
        try:
            ainv = pow(a, -1, Q)
        except ValueError:
            a = ainv = 1
        for desc, xs in (("1x2", [1, 1]), ("1x3", [1, 1, 1]), ("1x4", [1] * 4), ("2x2", [2, 3]),
                         ("inv2", [a, ainv]), ("inv3", [a, ainv, 1]), ("Qm1x2", [Q - 1, Q - 1]),
                         ("half", [Q // 2, 2]), ("r3", [rng.randrange(Q) for _ in range(3)])):
            want = 1
            for x in xs:
                want = want * x % Q
            got = eng.modmul_fold(Q, xs)
            print(name, desc, "OK" if got == want else "BAD %x %x" % (got, want), flush=True)


if __name__ == "__main__":
    main()
