#!/usr/bin/env python
"""Chain model of the persistent strata sweep's neighbour waits.

B workgroups walk U user ranges (U = B today): at position t workgroup w
takes range (s_t + w * U / B) mod U and may start once (a) it finished
position t-1 and (b) the range's previous holder released it.  Block times
are drawn from N(mean, sd) (the phase probe at C3: block mean 30.3 us, p90
36.6 us), plus a fixed signal cost.  Prints the modelled epoch for U = B
and for U = 2B with half-size blocks (the prologue does not halve).
Usage: python tools/chain_model.py"""
import numpy as np


def epoch_us(B, U, mean, sd, signal=1.2, reps=3, seed=0):
    rs = np.random.RandomState(seed)
    out = []
    for _ in range(reps):
        done = np.zeros(B)
        free = np.zeros(U)
        if U == 2 * B:     # alternate the parity of s: a range's last holder is 2 positions back
            seq = np.empty(U, np.int64)
            seq[0::2] = rs.permutation(np.arange(0, U, 2))
            seq[1::2] = rs.permutation(np.arange(1, U, 2))
        else:
            seq = rs.permutation(U)
        for s in seq:
            r = (s + np.arange(B) * (U // B)) % U
            start = np.maximum(done, free[r])
            fin = start + np.maximum(rs.normal(mean, sd, B), 0.3 * mean) + signal
            free[r] = fin
            done = fin
        out.append(done.max())
    return float(np.mean(out))


def main():
    B, mean = 256, 30.3
    for sd in (4.0, 5.7, 7.0):
        print(f"U = B   block sd {sd:4.1f} us: {epoch_us(B, B, mean, sd) / 1e3:.2f} ms")
        for pro in (0.0, 1.5, 2.5):
            half = (mean - pro) / 2 + pro
            print(f"  U = 2B prologue {pro:3.1f} us: "
                  f"{epoch_us(B, 2 * B, half, sd / np.sqrt(2)) / 1e3:.2f} ms (sd / sqrt 2), "
                  f"{epoch_us(B, 2 * B, half, sd) / 1e3:.2f} ms (same sd)")


if __name__ == "__main__":
    main()
