#!/usr/bin/env python3
"""N2 analysis (measurement aid): what would ballot/prefix compaction of the
reset work buy in a volume wave?

Inside-volume wave-steps of the benchmark (tools/march_stats.py, C oracle on
C3): every wave-step has at least one terminating lane (any_term = 1.000) and
lanes terminate with p ~ 0.25 (exit 0.115 + absorb 0.132). Within one step
compaction therefore skips nothing. The only way to batch resets is across
steps: a terminating lane parks (pending) until the wave runs one reset batch
for all parked lanes, and keeps its own step count, so the wave loops until its
slowest lane has done N steps. Model: per iteration the active lanes cost M
(the step without the reset candidate) and a batch costs Rc, M + Rc = 1 being
today's speculative step (Rc ~ 0.20 measured by knock-out).
Usage: python tools/n2_deferral_model.py [p_term] [Rc]
"""
import sys

import numpy as np


def simulate(p, Rc, thresh, N=256, lanes=64, waves=400, seed=1):
    rng = np.random.default_rng(seed)
    M = 1.0 - Rc
    costs = []
    for _ in range(waves):
        done = np.zeros(lanes, int)
        pending = np.zeros(lanes, bool)
        cost = 0.0
        while (done < N).any():
            act = (~pending) & (done < N)
            if act.any():
                cost += M
                term = act & (rng.random(lanes) < p)
                done[act] += 1
                pending |= term
            if pending.sum() >= thresh or (pending.any() and not ((~pending) & (done < N)).any()):
                cost += Rc
                pending[:] = False
        costs.append(cost / N)
    return float(np.mean(costs))


def main():
    p = float(sys.argv[1]) if len(sys.argv) > 1 else 0.25
    Rc = float(sys.argv[2]) if len(sys.argv) > 2 else 0.20
    print(f"p_term {p}, reset share {Rc}: speculative (today) = 1.000 per lane-step")
    for t in (1, 4, 8, 16, 24, 32, 48):
        print(f"  deferred batches at >= {t:2d} parked lanes: {simulate(p, Rc, t):.3f}")


if __name__ == "__main__":
    main()
